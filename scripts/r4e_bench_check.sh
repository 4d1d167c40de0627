#!/bin/bash
# Round 4: the bench's `configs` object and the multi-rank rehearsals (bench launcher GPU tests), then one default
# bench line (short) with its configs entries summarised.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4e}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread ${TESTS:-tests/test_abc_gpu.py tests/test_gpu_fuzz_abc.py tests/test_gpu_debug.py tests/test_bench_launcher.py} -m gpu > $OUT/launcher.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $OUT/launcher.log; exit 1; }
grep -E "passed|failed" $OUT/launcher.log | tail -2
timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 --cpu-baseline-seconds ${CPUS:-3} > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
python3 - $OUT/bench.json << 'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("headline", f"{d['value']:.4e}", "ms/step", round(d['ms_per_step'], 1), "acc", d["proposal"]["acceptance_rate"],
      "single", f"{d.get('single_chain_value', 0):.3e}", "pf16", f"{d['single_chain_prefetch']['value']:.3e}",
      "pfauto", f"{d['single_chain_prefetch_auto']['value']:.3e}", d['single_chain_prefetch_auto']['slots_used'],
      "rhat", d["gathered_rhat"])
for k, e in d["configs"].items():
    ft = e.get("fixed_theta", {})
    print(k, e["workload"][:40], f"{e['value']:.4e}", "ms/step", round(e["ms_per_step"], 2), "lanes", e["lanes_per_particle"],
          "acc", round(e["acceptance_rate"], 3), "h", e["h"], "fixed_theta", f"{ft.get('value', 0):.4e}",
          "frac", e["roofline"]["frac"], "prefetch_auto", e.get("prefetch_auto", {}).get("value"),
          e.get("prefetch_auto", {}).get("slots_used"))
PY
echo done
