#!/bin/bash
# rocprofv3 kernel traces of the bench for the A tree ($AB_DIR) and this tree (B), for per-stream timelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
mkdir -p gpurun_out/abt
for side in A B; do
  dir=$ROOT; [ $side = A ] && dir=$ROOT/${AB_DIR:-ab_old}
  (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace -d $ROOT/gpurun_out/abt/$side -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-chain) > gpurun_out/abt/$side.log 2>&1 || { echo "STOP $side rc=$?"; tail -5 gpurun_out/abt/$side.log; exit 1; }
  tail -1 gpurun_out/abt/$side.log | cut -c1-200
done
