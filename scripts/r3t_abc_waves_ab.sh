#!/bin/bash
# Round 3: ABC trial kernel with early rejection at 8 waves/SIMD (launch bound, 64 VGPRs + 3 spills outside the loop;
# the shipped build) vs 7 waves (65 VGPRs, no bound; lib/libepipf_ab7.so), early rejection on, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc_w
for v in 8 7 8 7; do
  if [ $v = 7 ]; then export EPIPF_LIBRARY=$PWD/stochastic-epidemic-modelling_amd/lib/libepipf_ab7.so; else unset EPIPF_LIBRARY; fi
  timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 > gpurun_out/abc_w/w$v.log 2>&1 || { echo STOP; tail -5 gpurun_out/abc_w/w$v.log; exit 1; }
  tail -1 gpurun_out/abc_w/w$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('waves $v', round(d['value']/1e6,2), 'M/s kernel', round(d['kernel_trials_per_s']/1e6,2), 'kernel_ms/launch', round(d['kernel_ms']/d['launches'],2))"
done
echo "== done"
