#!/bin/bash
# Round-2 final measurement session: rocprofv3 kernel trace + PMC passes of the default bench, one bench line per
# BASELINE config (1..5), config 5 at one chain per GPU, a kernel trace of one lane-group filter (config 2, one chain),
# and the 2-rank rehearsal of the driver's N>1 bench.  Each step has its own limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r2g bash scripts/profile.sh || exit $?
CFGS="1 2 3 4 5" STEPS=5 bash scripts/configs.sh > gpurun_out/configs.txt 2>&1 || { cat gpurun_out/configs.txt; exit 1; }
cat gpurun_out/configs.txt
timeout -k 10 300 python bench.py --config 5 --chains 1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/bench_5_chains1.log 2>&1 || exit $?
mkdir -p gpurun_out/prof_r2g_lanes
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2g_lanes/trace -o run --output-format csv -- python3 scripts/lanes_sweep.py --reps 3 --cfg 2 --chains 1 --lanes 4 --out gpurun_out/prof_r2g_lanes/sweep.jsonl > gpurun_out/prof_r2g_lanes/trace.log 2>&1 || exit $?
bash scripts/multirank_check.sh || exit $?
echo "== done"
