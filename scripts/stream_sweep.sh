#!/bin/bash
# bench value against chain-group streams (EPIPF_STREAMS) and chains per GPU; one JSON line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/streams
for ch in ${CHAINS:-128 256}; do
  for s in ${STREAMS:-2 4 8}; do
    EPIPF_STREAMS=$s timeout -k 10 200 python bench.py --chains $ch --steps 5 --warmup 1 --no-cpu-baseline --no-single-chain > gpurun_out/streams/b_${ch}_${s}.log 2>&1 || { echo "STOP chains=$ch streams=$s rc=$?"; exit 1; }
    tail -1 gpurun_out/streams/b_${ch}_${s}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'chains': $ch, 'streams': $s, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'avg_launch_us': d['roofline']['avg_launch_us'], 'step_wall_us': d['roofline']['step_wall_us']}))"
  done
done
