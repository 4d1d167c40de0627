#!/bin/bash
# Round 4: ABC at the reference's setting (scripts/abc_bench.py), the current library vs ab_old/ (the previous
# commit), interleaved; the lane-use figure of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4j}; mkdir -p $OUT
ROOT=$(pwd)
for v in old new old new; do
  if [ $v = old ]; then export EPIPF_LIBRARY=$ROOT/ab_old/stochastic-epidemic-modelling_amd/lib/libepipf.so; else export EPIPF_LIBRARY=$ROOT/stochastic-epidemic-modelling_amd/lib/libepipf.so; fi
  timeout -k 10 300 python3 scripts/abc_bench.py --runs 10 --cpu-seconds 0.5 > $OUT/abc_$v.log 2>&1 || { echo STOP; tail -5 $OUT/abc_$v.log; exit 1; }
  tail -1 $OUT/abc_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e6,2), 'M/s kernel', round(d['kernel_trials_per_s']/1e6,2), 'kernel_ms/launch', round(d['kernel_ms']/d['launches'],2), 'lane_use', d.get('lane_use'))"
done
echo "== done"
