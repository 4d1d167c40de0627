#!/bin/bash
# A/B of environment settings on one bench config: ENVS="A B ..." where each entry is VAR=VAL[,VAR=VAL...]
# ("-" = defaults).  One JSON summary line per entry.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
i=0
for e in ${ENVS:--}; do
  i=$((i+1))
  envs=(); [ "$e" != "-" ] && IFS=, read -ra envs <<< "$e"
  env "${envs[@]}" timeout -k 10 300 python bench.py --config ${CFG:-2} --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-single-chain --detail gpurun_out/ab/d_$i.json ${BENCH_ARGS:-} > gpurun_out/ab/b_$i.log 2>&1 || { echo "STOP $e rc=$?"; tail -5 gpurun_out/ab/b_$i.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/d_$i.json')); print(json.dumps({'env': '$e', 'cfg': ${CFG:-2}, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'lane_use': d['ssa_lane_utilisation'], 'ev_per_s': d['events_per_s'], 'exact_wave_frac': d['ssa_exact_wave_frac']}))"
done
