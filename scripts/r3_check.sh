#!/bin/bash
# Round 3: the full -m gpu suite, then an A/B of the default bench against the tree in ab_old/ (a worktree of the
# round-2 commit, built in place).  Every GPU step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest_gpu ($(date +%T))"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/r3_pytest_gpu.log 2>&1 || { echo "STOP pytest rc=$?"; tail -30 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r3_pytest_gpu.log
if [ -d ab_old ]; then ROUNDS="${ROUNDS:-1 2}" STEPS=8 bash scripts/ab_bench.sh || exit 1; fi
echo "== done"
