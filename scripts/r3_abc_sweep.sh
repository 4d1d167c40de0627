#!/bin/bash
# Round 3: ABC parity tests (lane groups), then end-to-end ABC throughput over the lane-group width and share.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc3
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
echo "== abc tests ($(date +%T))"
timeout -k 10 600 python -u -m pytest tests/test_abc_gpu.py tests/test_gpu_fuzz_abc.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/abc3/tests.log 2>&1 || { echo "STOP tests rc=$?"; tail -30 gpurun_out/abc3/tests.log; exit 1; }
tail -2 gpurun_out/abc3/tests.log
fi
# CFGS: lanes:share pairs, e.g. "1:0.25 4:0.6"
for cfg in ${CFGS:-1:0.25 4:0.1 4:0.25 4:0.4 2:0.25 8:0.25 1:0.25 4:0.25}; do
  set -- ${cfg/:/ }
  EPIPF_ABC_LANES=$1 EPIPF_ABC_GROUP_FRAC=$2 timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 ${ABC_ARGS:-} \
      > gpurun_out/abc3/b_$1_$2.log 2>&1 || { echo "STOP bench $cfg rc=$?"; tail -5 gpurun_out/abc3/b_$1_$2.log; exit 1; }
  tail -1 gpurun_out/abc3/b_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $1 frac $2', {k: d[k] for k in d if k in ('value','kernel_trials_per_s','kernel_ms','launches')})"
done
echo "== done"
