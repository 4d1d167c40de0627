#!/bin/bash
# Lane-group kernel change: lane/parity tests, then A/B vs lib_old (one and few
# chains, configs 2 and 5).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/stochastic-epidemic-modelling_amd
mkdir -p gpurun_out/r2r
timeout -k 10 500 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_fuzz.py tests/test_gpu_xcd.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2r/tests.log 2>&1; rc=$?; tail -1 gpurun_out/r2r/tests.log; [ $rc -ne 0 ] && exit $rc
for side in old new old new; do
  if [ $side = old ]; then export EPIPF_LIBRARY=$L/lib_old/libepipf.so; else unset EPIPF_LIBRARY; fi
  timeout -k 10 300 python -u scripts/lanes_sweep.py --cfg 2 5 --chains 1 2 8 --lanes 4 --reps 3 --out gpurun_out/r2r/lanes_$side.jsonl > gpurun_out/r2r/lanes_$side.log 2>&1 || { echo "STOP lanes $side"; exit 1; }
done
python3 - <<'PY'
import json, collections
for side in ("old", "new"):
    r = collections.defaultdict(list)
    for l in open(f"gpurun_out/r2r/lanes_{side}.jsonl"):
        d = json.loads(l); r[(d["cfg"], d["chains"])].append(d["particle_steps_per_s"])
    print(side, {k: ["%.4e" % x for x in v] for k, v in sorted(r.items())})
PY
