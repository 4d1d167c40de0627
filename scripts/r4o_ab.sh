#!/bin/bash
# Round 4: the certified lane-group clock (FASTCLK) and the 16-particle weight blocks.  Parity first (lane-group tests
# with the default layout and with EPIPF_GROUP_BLOCK=16, the random fuzz sweep with 16-particle blocks), then lanes
# sweeps of ab_old/ (previous commit) vs this tree, each with 64- and 16-particle blocks, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4o}; mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lanes.py > $OUT/pytest64.log 2>&1 || { echo "TESTS (64) FAILED"; tail -40 $OUT/pytest64.log; exit 1; }
  tail -1 $OUT/pytest64.log
  EPIPF_GROUP_BLOCK=16 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lanes.py tests/test_gpu_fuzz.py > $OUT/pytest16.log 2>&1 || { echo "TESTS (16) FAILED"; tail -40 $OUT/pytest16.log; exit 1; }
  tail -1 $OUT/pytest16.log
fi
for i in ${ROUNDS:-1 2}; do
  for v in old new; do
    if [ $v = old ]; then LIB=$ROOT/ab_old/stochastic-epidemic-modelling_amd/lib/libepipf.so; else LIB=$ROOT/stochastic-epidemic-modelling_amd/lib/libepipf.so; fi
    for b in 64 16; do
      EPIPF_GROUP_BLOCK=$b EPIPF_LIBRARY=$LIB timeout -k 10 600 python scripts/lanes_sweep.py --cfg ${CFGS:-2 3 5} --chains ${CHAINS:-1 2} --lanes ${LANES:-8:1 16:1} --reps 3 --out $OUT/sweep_${v}${b}_$i.jsonl > $OUT/sweep_${v}${b}_$i.log 2>&1 || { echo "STOP sweep $v $b $i"; tail -5 $OUT/sweep_${v}${b}_$i.log; exit 1; }
    done
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
    base = max(r[k]["old64"])
    print(*k, " ".join(f"{v}={max(r[k][v]):.3e}(x{max(r[k][v]) / base:.3f})" for v in ("old64", "new64", "old16", "new16") if r[k][v]))
PY
echo done
