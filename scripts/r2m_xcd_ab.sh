#!/bin/bash
# XCD-aware block placement of the step launches (EPIPF_XCD_MAP): GPU suite, then A/B (0 = 2-D grid, 1 = XCD map) on
# the bench (configs 2, 4, 5), the lane-group filters (one chain) and PMC FETCH_SIZE / WRITE_SIZE of pf_step_kernel.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/r2m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
EPIPF_XCD_MAP=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "full_size or oracle" --timeout 300 --timeout-method thread > $OUT/tests_map0.log 2>&1; rc=$?
tail -1 $OUT/tests_map0.log; [ $rc -ne 0 ] && exit $rc
for cfg in 2 4 5; do
  rm -f gpurun_out/ab/b_*.log
  CFG=$cfg STEPS=5 ENVS="EPIPF_XCD_MAP=0 EPIPF_XCD_MAP=1 EPIPF_XCD_MAP=0 EPIPF_XCD_MAP=1" bash scripts/ab_env.sh >> $OUT/ab.jsonl || exit 1
done
cat $OUT/ab.jsonl
for m in 0 1; do
  EPIPF_XCD_MAP=$m timeout -k 10 300 python -u scripts/lanes_sweep.py --cfg 2 5 --chains 1 --lanes 4 --reps 3 --out $OUT/lanes_$m.jsonl > $OUT/lanes_$m.log 2>&1 || { echo "STOP lanes"; exit 1; }
done
cat $OUT/lanes_0.jsonl $OUT/lanes_1.jsonl
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-single-chain"
for m in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    EPIPF_XCD_MAP=$m timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex pf_step_kernel -d $OUT/pmc_${m}_$c -o run --output-format csv -- python3 $BENCH > $OUT/pmc_${m}_$c.log 2>&1 || { echo "STOP pmc $m $c"; tail -3 $OUT/pmc_${m}_$c.log; exit 1; }
  done
done
echo "== done"
