set -u
mkdir -p gpurun_out/r4t
for s in 4 8 1 2 4 8; do
  EPIPF_STREAMS=$s timeout -k 10 300 python bench.py --config 5 --steps 4 --warmup 1 --no-single-chain --configs none --no-cpu-baseline > gpurun_out/r4t/c5_s$s.log 2>&1 || { tail -5 gpurun_out/r4t/c5_s$s.log; exit 1; }
  tail -1 gpurun_out/r4t/c5_s$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams $s', f\"{d['value']:.4e}\", 'lane_use', d.get('ssa_lane_utilisation'), 'exact_p', d.get('ssa_exact_particle_frac'), 'exact_w', d.get('ssa_exact_wave_frac'), 'ev/ps', d.get('events_per_particle_step'), 'acc', d['proposal'].get('acceptance_rate'))"
done
