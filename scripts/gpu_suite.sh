#!/bin/bash
# One GPU session: smoke -> full -m gpu suite -> default bench (+ optional ABC bench).  Every GPU step has its own time
# limit and output file under gpurun_out/; a crash, abort or timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu ${PYTEST_T:-900} python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
step bench 400 python bench.py --steps ${STEPS:-10} --warmup 2
if [ -n "${ABC:-}" ]; then step abc_bench 300 python scripts/abc_bench.py --runs 3 --cpu-seconds 2; fi
echo "== done"
