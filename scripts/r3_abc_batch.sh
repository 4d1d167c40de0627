#!/bin/bash
# Round 3: ABC end-to-end throughput over batch size x lane groups (reference setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc3
for b in ${BATCHES:-131072 196608 262144}; do
  for cfg in ${CFGS:-1:0.25 4:0.5}; do
    set -- ${cfg/:/ }
    EPIPF_ABC_LANES=$1 EPIPF_ABC_GROUP_FRAC=$2 timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 --batch $b \
        > gpurun_out/abc3/bb_${b}_$1_$2.log 2>&1 || { echo "STOP $b $cfg"; tail -5 gpurun_out/abc3/bb_${b}_$1_$2.log; exit 1; }
    tail -1 gpurun_out/abc3/bb_${b}_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch $b lanes $1 frac $2', round(d['value']/1e6,2), 'M/s kernel', round(d['kernel_trials_per_s']/1e6,2), 'launches', d['launches'], 'kernel_ms/launch', round(d['kernel_ms']/d['launches'],2))"
  done
done
echo "== done"
