#!/bin/bash
# Lane-group tests, then an alternating A/B of the one-chain config-5 bench against ab_old, then a lanes sweep at one
# and two chains (W = 4, 8) of configs 2, 3, 5 on this tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3i; mkdir -p $OUT
ROOT=$(pwd)
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lanes.py tests/test_abc_gpu.py tests/test_gpu_fuzz.py > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for i in ${ROUNDS:-1 2 3}; do
  for d in ab_old .; do
    n=$(basename $d)
    (cd $ROOT/$d && timeout -k 10 300 python bench.py --config 5 --chains 1 --steps 6 --warmup 2 --no-cpu-baseline --no-single-chain) > $OUT/c5x1_${n}_$i.log 2>&1 || { echo "STOP $n"; tail -5 $OUT/c5x1_${n}_$i.log; exit 1; }
    tail -1 $OUT/c5x1_${n}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5x1_${n}_$i', f\"{d['value']:.4e}\")"
  done
done
timeout -k 10 500 python scripts/lanes_sweep.py --cfg 2 3 5 --chains 1 2 --lanes 4 8 --reps 3 --out $OUT/sweep.jsonl > $OUT/sweep.log 2>&1 || { echo "STOP sweep"; tail -5 $OUT/sweep.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/sweep.jsonl'):
    d=json.loads(l); print(d['cfg'], d['chains'], d['lanes'], f\"{d['particle_steps_per_s']:.3e}\")"
echo done
