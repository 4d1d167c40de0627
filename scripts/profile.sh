#!/bin/bash
# rocprofv3 session on the GPU box: kernel-trace stats of the bench, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; SQ counters in their own pass).
# Every step has its own time limit; a crash or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
rm -f $OUT/count_*.txt
BENCH="bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-single-chain --configs none ${BENCH_ARGS:-}"
K=${PMC_KERNEL:-pf_step_kernel}
step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
}
# Every pass also records the particle-steps its bench process ran, counted as the bench line counts them (chains that
# proposed a negative theta run no filter and count nothing: at h = 1 the initial-draw loop repeats with few pending
# chains), in count_<pass>.txt (EPIPF_PMC_COUNT, epipf/engine.py); scripts/parse_rocprof.py divides the pass's counter
# totals over all its launches by it.
export EPIPF_PMC_COUNT=$OUT/count_trace.txt
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH
export EPIPF_PMC_COUNT=$OUT/count_fetch.txt
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex $K -d $OUT/fetch -o run --output-format csv -- python3 $BENCH
export EPIPF_PMC_COUNT=$OUT/count_write.txt
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex $K -d $OUT/write -o run --output-format csv -- python3 $BENCH
export EPIPF_PMC_COUNT=$OUT/count_sq.txt
step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex $K -d $OUT/sq -o run --output-format csv -- python3 $BENCH
export EPIPF_PMC_COUNT=$OUT/count_valu.txt
step pmc_valu 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex $K -d $OUT/valu -o run --output-format csv -- python3 $BENCH
unset EPIPF_PMC_COUNT
python3 scripts/parse_rocprof.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
echo "== done"
