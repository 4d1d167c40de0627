#!/bin/bash
# Lane-group session: full -m gpu suite, default bench (single chain now on lane groups), config 5 at one chain per GPU,
# speculative-MH slot sweeps for configs 2 and 5 (slots x lanes interplay).  Each GPU step has its own limit; stop on
# the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r2e
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/r2e/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 3 "gpurun_out/r2e/$name.log" | cut -c1-600
    if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread
step bench 400 python bench.py --steps 10 --warmup 2
step bench_cfg5_chain1 300 python bench.py --config 5 --chains 1 --steps 20 --warmup 2 --no-cpu-baseline
step prefetch_cfg2 400 env SLOTS="0 2 4 8 16" ITERS=60 CFG=2 python -u scripts/prefetch_sweep.py
step prefetch_cfg5 400 env SLOTS="0 2 4 8 16" ITERS=60 CFG=5 python -u scripts/prefetch_sweep.py
echo "== done"
