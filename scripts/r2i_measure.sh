#!/bin/bash
# Round-2 closing numbers: one bench line per BASELINE config (1..5) and config 5 at one chain per GPU, current code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFGS="1 2 3 4 5" STEPS=8 bash scripts/configs.sh > gpurun_out/configs.txt 2>&1 || { cat gpurun_out/configs.txt; exit 1; }
cat gpurun_out/configs.txt
timeout -k 10 300 python bench.py --config 5 --chains 1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/bench_5_chains1.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/bench_5_chains1.log | cut -c1-200
echo "== done"
