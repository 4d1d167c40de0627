#!/bin/bash
# Round 3: with early rejection on, do lane groups for the longest share of a 256k launch pay now? (env sweep)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abc_ge
for cfg in 1:0 4:0.02 4:0.1 4:0.25 2:0.1 1:0; do
  set -- ${cfg/:/ }
  EPIPF_ABC_LANES=$1 EPIPF_ABC_GROUP_FRAC=$2 timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 \
      > gpurun_out/abc_ge/g_$1_$2.log 2>&1 || { echo "STOP $cfg"; tail -5 gpurun_out/abc_ge/g_$1_$2.log; exit 1; }
  tail -1 gpurun_out/abc_ge/g_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $1 frac $2', round(d['value']/1e6,2), 'M/s kernel', round(d['kernel_trials_per_s']/1e6,2), 'kernel_ms/launch', round(d['kernel_ms']/d['launches'],2), 'ev/trial', round(d['events_per_trial']))"
done
echo "== done"
