#!/bin/bash
# Round 4: the lane groups' fixed-point decision pass.  Lane-group parity tests (and ABC, which runs lane groups), then
# an alternating A/B of the one-chain config-5 bench (EPIPF_GROUP_DECIDE=seq: the sequential pass of round 3), then a
# lanes sweep at 1, 2, 4, 8 chains (W = 4, 8, 16) of configs 2, 3, 5 in both modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4a}; mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lanes.py tests/test_abc_gpu.py > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for i in ${ROUNDS:-1 2}; do
  for mode in seq fp; do
    if [ $mode = seq ]; then export EPIPF_GROUP_DECIDE=seq; else unset EPIPF_GROUP_DECIDE; fi
    timeout -k 10 300 python bench.py --config 5 --chains 1 --steps 8 --warmup 2 --no-cpu-baseline --no-single-chain > $OUT/c5x1_${mode}_$i.log 2>&1 || { echo "STOP $mode"; tail -5 $OUT/c5x1_${mode}_$i.log; exit 1; }
    tail -1 $OUT/c5x1_${mode}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5x1_${mode}_$i', f\"{d['value']:.4e}\", d['lanes_per_particle'])"
  done
done
for mode in seq fp; do
  if [ $mode = seq ]; then export EPIPF_GROUP_DECIDE=seq; else unset EPIPF_GROUP_DECIDE; fi
  timeout -k 10 600 python scripts/lanes_sweep.py --cfg 2 3 5 --chains ${CHAINS:-1 2 4 8} --lanes ${LANES:-4:1 8:1 16:1 4:2 8:2 16:2} --reps 3 --out $OUT/sweep_$mode.jsonl > $OUT/sweep_$mode.log 2>&1 || { echo "STOP sweep"; tail -5 $OUT/sweep_$mode.log; exit 1; }
done
python3 -c "
import json
r = {}
for mode in ('seq', 'fp'):
    for l in open('$OUT/sweep_%s.jsonl' % mode):
        d = json.loads(l); r.setdefault((d['cfg'], d['chains'], d['lanes'], d['lane_events']), {})[mode] = d['particle_steps_per_s']
for k in sorted(r):
    v = r[k]; print(*k, ' '.join(f'{m}={v[m]:.3e}' for m in v), f\"x{v.get('fp', 0) / v.get('seq', 1):.3f}\")"
echo done
