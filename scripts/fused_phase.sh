#!/bin/bash
# Per-phase cycles of the one-workgroup filter (make phase -> lib/libepipf_phase.so, EPIPF_PHASE_TIMING): config 1, one
# and 256 chains; the kernel's block 0 prints its phase sums once per launch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ch in 1 256; do
  EPIPF_LIBRARY=$PWD/stochastic-epidemic-modelling_amd/lib/libepipf_phase.so timeout -k 10 120 \
    python scripts/mh_iteration_probe.py --cfg ${CFG:-1} --chains $ch --iters 5 > gpurun_out/fused_phase_$ch.log 2>&1 || { tail -5 gpurun_out/fused_phase_$ch.log; exit 1; }
  grep FUSED gpurun_out/fused_phase_$ch.log | tail -3
done
