#!/bin/bash
# Round 4: with the round-4 lane-group kernel (fixed-point decisions, early rejection on groups) and W = 16, do lane
# groups for the longest share of the default 256k ABC launch pay now?  Parity first (ABC lane tests incl. W = 16),
# then an env sweep of (lanes, share), the one-lane baseline first and last.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r4q}; mkdir -p $O
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_abc_gpu.py -k lane > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for cfg in ${CFGS:-1:0 4:0.01 8:0.01 16:0.01 8:0.03 16:0.03 16:0.1 16:0.25 1:0}; do
  set -- ${cfg/:/ }
  EPIPF_ABC_LANES=$1 EPIPF_ABC_GROUP_FRAC=$2 timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 \
      > $O/g_$1_$2.log 2>&1 || { echo "STOP $cfg"; tail -5 $O/g_$1_$2.log; exit 1; }
  tail -1 $O/g_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $1 frac $2', round(d['value']/1e6,2), 'M/s kernel', round(d['kernel_trials_per_s']/1e6,2), 'kernel_ms/launch', round(d['kernel_ms']/d['launches'],2), 'ev/trial', round(d['events_per_trial']))"
done
echo "== done"
