#!/bin/bash
# Round-2 measurement session: rocprofv3 kernel trace + PMC passes of the default bench (scripts/profile.sh), one bench
# line per BASELINE config (scripts/configs.sh), and config 5 at the north star's layout (one chain per GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r2} bash scripts/profile.sh || exit $?
STEPS=5 bash scripts/configs.sh > gpurun_out/configs.txt 2>&1 || { cat gpurun_out/configs.txt; exit 1; }
cat gpurun_out/configs.txt
timeout -k 10 300 python bench.py --config 5 --chains 1 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/cfg/bench_5_chains1.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/bench_5_chains1.log | cut -c1-400
