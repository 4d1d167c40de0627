#!/bin/bash
# One GPU session: smoke -> parity tests -> short bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout (rc other than 0/1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
    return 0
}
what=${1:-all}
if [[ $what == all || $what == smoke ]]; then step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; fi
if [[ $what == all || $what == tests ]]; then step pytest_gpu 900 python -m pytest tests -m gpu -q -rf; fi
if [[ $what == all || $what == bench ]]; then step bench 600 python bench.py --steps 5 --warmup 1 --single-chain; fi
if [[ $what == all || $what == prof ]]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-single-chain
fi
echo "== done"
