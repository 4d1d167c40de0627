#!/bin/bash
# The driver's N-GPU bench path on a one-GPU box: torch.distributed.run with one rank, backend nccl (= RCCL), and
# EPIPF_BENCH_DIST=1 so that the process group, the max/sum timing reductions and the RCCL all-gather of the draws run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
EPIPF_BENCH_DIST=1 EPIPF_BENCH_CHAINS=${CH:-64} timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-single-chain \
  > gpurun_out/rccl_bench.log 2>&1
rc=$?; tail -2 gpurun_out/rccl_bench.log | cut -c1-600; exit $rc
