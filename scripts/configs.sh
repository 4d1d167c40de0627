#!/bin/bash
# One bench line per BASELINE config (2..5) at the default chains/GPU, CPU baseline included.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
for c in ${CFGS:-2 3 4 5}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-5} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/cfg/bench_$c.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "STOP cfg $c rc=$rc"; tail -5 gpurun_out/cfg/bench_$c.log; exit $rc; }
  tail -1 gpurun_out/cfg/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['cpu_baseline'] or {}; print(f\"cfg $c: value={d['value']:.4e} ms/step={d['ms_per_step']:.1f} kernel_us={d['roofline']['avg_launch_us']:.1f} ev/ps={d['events_per_particle_step']:.1f} ev/s={d['events_per_s']:.3e} lane_use={d['ssa_lane_utilisation'] or 0:.3f} lanes={d.get('lanes_per_particle', 1)} cpu={b.get('value', 0):.3e} x{d.get('speedup_vs_cpu_baseline', 0):.0f}\")"
done
