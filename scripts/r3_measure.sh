#!/bin/bash
# Round-3 closing measurement: rocprofv3 kernel trace + PMC passes of the default bench (scripts/profile.sh, TAG=r3;
# the PMC summary records the library's build id), the default bench line with that profile in place (as the driver
# runs it), every BASELINE config, and config 5 at one chain per GPU.  Each step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
TAG=r3 bash scripts/profile.sh || exit $?
cp gpurun_out/prof_r3/pmc_step_kernel.json profiles/pmc_step_kernel.json
echo "== bench ($(date +%T))"
timeout -k 10 600 python bench.py > gpurun_out/r3_bench.log 2>&1 || { tail -5 gpurun_out/r3_bench.log; exit 1; }
tail -1 gpurun_out/r3_bench.log | cut -c1-600
echo "== configs ($(date +%T))"
CFGS="1 3 4 5" STEPS=8 bash scripts/configs.sh > gpurun_out/r3_configs.txt 2>&1 || { cat gpurun_out/r3_configs.txt; exit 1; }
cat gpurun_out/r3_configs.txt
timeout -k 10 300 python bench.py --config 5 --chains 1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/bench_5_chains1.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/bench_5_chains1.log | cut -c1-200
echo "== done"
