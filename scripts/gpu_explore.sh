#!/bin/bash
# Exploration on the GPU box: counter list, SSA microbench, chains/WG sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || echo "rocprofv3 -L rc=$?"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o /tmp/ssa_mb scripts/ssa_microbench.hip || exit 1
timeout -k 10 120 /tmp/ssa_mb > gpurun_out/microbench.log 2>&1; rc=$?; cat gpurun_out/microbench.log
[ $rc -ne 0 ] && exit $rc
bash scripts/sweep.sh
