#!/bin/bash
# Round 3: rocprofv3 marker + kernel trace of the debug library's roctx ranges (no counters in this pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/roctx
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/roctx -o run --output-format csv \
    -- python3 scripts/roctx_demo.py > gpurun_out/roctx/run.log 2>&1 || { echo "STOP rc=$?"; tail -20 gpurun_out/roctx/run.log; exit 1; }
tail -2 gpurun_out/roctx/run.log
find gpurun_out/roctx -name "*.csv" | head -20
echo "== done"
