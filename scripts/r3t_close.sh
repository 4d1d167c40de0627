#!/bin/bash
# Round-3 closing measurement of the build with ABC early rejection: rocprofv3 trace + PMC passes of the default bench
# (TAG=r3t; the PMC summary records the library's build id), the default bench line with that profile in place, and the
# ABC bench at the reference's setting.  Each step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r3t bash scripts/profile.sh || exit $?
cp gpurun_out/prof_r3t/pmc_step_kernel.json profiles/pmc_step_kernel.json
mkdir -p gpurun_out/r3t
cp gpurun_out/prof_r3t/pmc_step_kernel.json gpurun_out/r3t/pmc_step_kernel.json
echo "== bench ($(date +%T))"
timeout -k 10 600 python bench.py > gpurun_out/r3t/bench.log 2>&1 || { tail -5 gpurun_out/r3t/bench.log; exit 1; }
tail -1 gpurun_out/r3t/bench.log | cut -c1-900
echo "== abc bench ($(date +%T))"
timeout -k 10 300 python scripts/abc_bench.py --runs 10 --cpu-seconds 10 > gpurun_out/r3t/abc_bench.log 2>&1 || { tail -5 gpurun_out/r3t/abc_bench.log; exit 1; }
tail -1 gpurun_out/r3t/abc_bench.log | cut -c1-600
echo "== done"
