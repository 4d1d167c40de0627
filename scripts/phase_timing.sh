#!/bin/bash
# Phase timing of the lane-group kernel at one chain (configs 2 and 5, W = 4 and 8) with the s_memtime build
# (make -C stochastic-epidemic-modelling_amd/csrc phase -> lib/libepipf_phase.so, EPIPF_PHASE_TIMING; diagnostic only).
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-phase}; mkdir -p $OUT
for cfg in ${CFGS:-5 2}; do for W in ${WS:-4 8}; do
  EPIPF_LIBRARY=$PWD/stochastic-epidemic-modelling_amd/lib/${PHLIB:-libepipf_phase.so} timeout -k 10 120 python scripts/lanes_sweep.py --cfg $cfg --chains 1 --lanes $W --reps 1 --out $OUT/sw.jsonl > $OUT/ph_${cfg}_$W.log 2>&1 || { echo "STOP $cfg $W"; tail -5 $OUT/ph_${cfg}_$W.log; exit 1; }
  python3 scripts/phase_report.py $OUT/ph_${cfg}_$W.log
done; done
