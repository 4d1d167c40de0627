#!/bin/bash
# Rehearsal of the driver's N>1 bench on a 1-GPU box: 2 ranks (gloo for the collectives) sharing cuda:0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
EPIPF_DIST_BACKEND=gloo EPIPF_BENCH_CHAINS=${CH:-32} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/multirank.log 2>&1
rc=$?; tail -3 gpurun_out/multirank.log; exit $rc
