#!/bin/bash
# One MH iteration's wall / filter / device time (scripts/mh_iteration_probe.py) with the one-workgroup filter on and off
# (EPIPF_FUSED=0), at BASELINE config 1 (N = 100) for one and 256 chains.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-fused_probe}.jsonl
: > $OUT
for ch in ${CHAINS:-1 256}; do for f in 1 0; do
  EPIPF_FUSED=$f timeout -k 10 120 python scripts/mh_iteration_probe.py --cfg ${CFG:-1} --chains $ch --iters ${ITERS:-200} \
      --tag fused=$f >> $OUT 2>gpurun_out/fused_probe.err || { tail -5 gpurun_out/fused_probe.err; exit 1; }
done; done
cat $OUT
