#!/bin/bash
# Round 3: ABC early rejection -- parity tests, then end-to-end A/B (EPIPF_ABC_EARLY=0/1) over batch sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc_early
timeout -k 10 600 python3 -u -m pytest tests/test_abc_gpu.py tests/test_gpu_fuzz_abc.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/abc_early/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/abc_early/tests.log; exit 1; }
tail -2 gpurun_out/abc_early/tests.log
for b in ${BATCHES:-0 196608 131072}; do
  for early in 0 1 0 1; do
    EPIPF_ABC_EARLY=$early timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 --batch $b \
        > gpurun_out/abc_early/b_${b}_${early}.log 2>&1 || { echo "STOP $b $early"; tail -5 gpurun_out/abc_early/b_${b}_${early}.log; exit 1; }
    tail -1 gpurun_out/abc_early/b_${b}_${early}.log >> gpurun_out/abc_early/all.jsonl
    tail -1 gpurun_out/abc_early/b_${b}_${early}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch $b early $early', round(d['value']/1e6,2), 'M/s kernel', round(d['kernel_trials_per_s']/1e6,2), 'launches', d['launches'], 'kernel_ms/launch', round(d['kernel_ms']/d['launches'],2), 'ev/trial', round(d['events_per_trial']), 'lane_use', round(d['lane_use'],3))"
  done
done
echo "== done"
