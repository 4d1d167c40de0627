#!/bin/bash
# Throughput sweep over chains/GPU (each config a fresh process, own time limit).  Blocks are one wave at every N.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/sweep.jsonl; : > $out
for ch in ${CHAINS:-1 8 16 32 48 64 128 256}; do
  echo "== chains=$ch"
  timeout -k 10 300 python bench.py --chains $ch --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-single-chain --detail gpurun_out/sweep_one.json > gpurun_out/sweep_one.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 gpurun_out/sweep_one.log; exit $rc; fi
  python3 -c "import json; print(json.dumps(json.load(open('gpurun_out/sweep_one.json'))))" >> $out
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_one.json')); print(f\"  value={d['value']:.3e} ms/step={d['ms_per_step']:.1f} kernel_us={d['roofline']['avg_launch_us']:.1f} ev/s={d['events_per_s']:.3e} lane_use={d['ssa_lane_utilisation']:.3f}\")"
done
