#!/bin/bash
# Round 4: lane-group runs on smaller particle blocks (EPIPF_GROUP_BLOCK=$TEST_BLOCK, default 16) -- parity (lane tests,
# bench-scale reference replay and the random fuzz sweep with the layout forced), then a lanes sweep over the layouts
# $BLOCKS (default 64 16), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4n}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  EPIPF_GROUP_BLOCK=${TEST_BLOCK:-16} timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_lanes.py tests/test_gpu_ref_replay.py tests/test_gpu_fuzz.py} > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for i in ${ROUNDS:-1 2}; do
  for b in ${BLOCKS:-64 16}; do
    EPIPF_GROUP_BLOCK=$b timeout -k 10 600 python scripts/lanes_sweep.py --cfg ${CFGS:-2 3 5} --chains ${CHAINS:-1 2 4} --lanes ${LANES:-8:1 16:1} --reps 3 --out $OUT/sweep_b${b}_$i.jsonl > $OUT/sweep_b${b}_$i.log 2>&1 || { echo "STOP sweep $b $i"; tail -5 $OUT/sweep_b${b}_$i.log; exit 1; }
  done
done
python3 - $OUT << 'PY'
import json, sys, glob, collections
O = sys.argv[1]
r = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{O}/sweep_b*_*.jsonl"):
    b = f.split("/")[-1].split("_")[1]
    for l in open(f):
        d = json.loads(l)
        r[(d["cfg"], d["chains"], d["lanes"], d["lane_events"])][b].append(d["particle_steps_per_s"])
for k in sorted(r):
    bs = sorted(r[k], key=lambda b: -int(b[1:]))
    o = max(r[k][bs[0]])
    print(*k, " ".join(f"{b}={max(r[k][b]):.3e}(x{max(r[k][b]) / o:.3f})" for b in bs))
PY
echo done
