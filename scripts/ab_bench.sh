#!/bin/bash
# A/B of the default bench: the tree in $AB_DIR (a worktree of another commit, built in place) against this tree,
# alternating, same box.  One JSON summary line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
ROOT=$(pwd)
for i in ${ROUNDS:-1 2}; do
  for side in A B; do
    dir=$ROOT; [ $side = A ] && dir=$ROOT/${AB_DIR:-ab_old}
    (cd $dir && timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-single-chain ${BENCH_ARGS:-}) > gpurun_out/ab/$side$i.log 2>&1 || { echo "STOP $side$i rc=$?"; tail -5 gpurun_out/ab/$side$i.log; exit 1; }
    tail -1 gpurun_out/ab/$side$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$side$i', f\"{d['value']:.4e}\", f\"ms/step={d['ms_per_step']:.1f}\", f\"launch_us={r['avg_launch_us']:.1f}\", f\"wall_us={r['step_wall_us']:.1f}\")"
  done
done
