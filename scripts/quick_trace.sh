#!/bin/bash
# GPU parity tests, one bench line, and a kernel-trace pass of the bench (per-launch duration spread).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/qt
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && { echo "STOP pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log
[ $rc -ne 0 ] && { echo "STOP bench rc=$rc"; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/trace.log 2>&1; rc=$?
[ $rc -ne 0 ] && { echo "STOP trace rc=$rc"; tail -5 $OUT/trace.log; exit $rc; }
python3 scripts/parse_rocprof.py $OUT 2>&1 | grep -v '^ "\|^{\|^}\|^  "' | head -20
