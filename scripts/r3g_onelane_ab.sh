#!/bin/bash
# One-lane subgroup loop on wave masks: parity tests on the one-lane kernel, then an alternating A/B of the config-5
# bench (256 chains, one lane per particle) against ab_old (the previous build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3g; mkdir -p $OUT
ROOT=$(pwd)
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_xcd.py tests/test_gpu_path.py > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
for i in ${ROUNDS:-1 2 3}; do
  for d in ab_old .; do
    n=$(basename $d)
    (cd $ROOT/$d && timeout -k 10 300 python bench.py --config ${CFG:-5} --steps 4 --warmup 1 --no-cpu-baseline --no-single-chain) > $OUT/c${CFG:-5}_${n}_$i.log 2>&1 || { echo "STOP $n $i"; tail -5 $OUT/c${CFG:-5}_${n}_$i.log; exit 1; }
    tail -1 $OUT/c${CFG:-5}_${n}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c${CFG:-5}_${n}_$i', f\"{d['value']:.4e}\", f\"ms/step={d['ms_per_step']:.1f}\", f\"launch_us={r['avg_launch_us']:.1f}\")"
  done
done
echo done
