#!/bin/bash
# Round 4 A/B of this tree against ab_old/ (the previous commit's build).  Parity first (lane-group tests, ABC
# lane tests, the random fuzz sweep), then lanes sweeps of ab_old/ (previous commit) vs this tree, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4ae}; mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_lanes.py tests/test_gpu_fuzz.py tests/test_abc_gpu.py} > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for i in ${ROUNDS:-1 2}; do
  for v in old new; do
    if [ $v = old ]; then LIB=$ROOT/ab_old/stochastic-epidemic-modelling_amd/lib/libepipf.so; else LIB=$ROOT/stochastic-epidemic-modelling_amd/lib/libepipf.so; fi
    EPIPF_LIBRARY=$LIB timeout -k 10 600 python scripts/lanes_sweep.py --cfg ${CFGS:-2 3 5} --chains ${CHAINS:-1 2 4} --lanes ${LANES:-8 16} --reps 3 --out $OUT/sweep_${v}_$i.jsonl > $OUT/sweep_${v}_$i.log 2>&1 || { echo "STOP sweep $v $i"; tail -5 $OUT/sweep_${v}_$i.log; exit 1; }
  done
done
python3 - $OUT << 'PY'
import json, sys, glob, collections
O = sys.argv[1]
r = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{O}/sweep_*_*.jsonl"):
    v = f.split("/")[-1].split("_")[1]
    for l in open(f):
        d = json.loads(l)
        r[(d["cfg"], d["chains"], d["lanes"])][v].append(d["particle_steps_per_s"])
for k in sorted(r):
    o, n = max(r[k]["old"]), max(r[k]["new"])
    print(*k, f"old={o:.3e} new={n:.3e} x{n / o:.3f}")
PY
echo done
