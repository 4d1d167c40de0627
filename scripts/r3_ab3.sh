#!/bin/bash
# A/B/C of the default bench over sibling trees (DIRS, built in place), alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab3
ROOT=$(pwd)
for i in ${ROUNDS:-1 2}; do
  for d in ${DIRS:-ab_old . ab_c}; do
    tag=$(basename $d)_$i
    (cd $ROOT/$d && timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-single-chain ${BENCH_ARGS:-}) > gpurun_out/ab3/$tag.log 2>&1 || { echo "STOP $tag"; tail -5 gpurun_out/ab3/$tag.log; exit 1; }
    tail -1 gpurun_out/ab3/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', f\"{d['value']:.4e}\", f\"ms/step={d['ms_per_step']:.1f}\", f\"launch_us={r['avg_launch_us']:.1f}\")"
  done
done
