#!/bin/bash
# Round-4 closing measurement of the final build: rocprofv3 trace + PMC passes of the headline (config 2, 256 chains,
# one lane per particle -> profiles/pmc_step_kernel.json) and of config 5 at one chain per GPU (the lane-group kernel ->
# profiles/pmc_group_cfg5_c1.json) and of configs 3 / 4 / 5 at 256 chains (profiles/pmc_step_cfg{3,4,5}.json), each
# recording the library's build id; then the default bench line with those
# profiles in place, the ABC bench at the reference's setting, and a fixed-width prefetch sweep at config 5 (the
# adaptive width's yardstick).  Each step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r4z}
PMC_CONFIG=2 PMC_CHAINS=256 TAG=${T}_c2 bash scripts/profile.sh || exit $?
cp gpurun_out/prof_${T}_c2/pmc_step_kernel.json profiles/pmc_step_kernel.json
PMC_CONFIG=5 PMC_CHAINS=1 PMC_LANES=${LANES5:-16} PMC_KERNEL=pf_step_group_kernel PMC_NAME=pmc_group_cfg5_c1.json \
  BENCH_ARGS="--config 5 --chains 1" STEPS=20 TAG=${T}_c5 bash scripts/profile.sh || exit $?
cp gpurun_out/prof_${T}_c5/pmc_group_cfg5_c1.json profiles/pmc_group_cfg5_c1.json
# configs 3, 4, 5 at 256 chains per GPU (the bench line's `configs` entries; one lane per particle)
for cfg in 3 4 5; do
  PMC_CONFIG=$cfg PMC_CHAINS=256 PMC_NAME=pmc_step_cfg$cfg.json BENCH_ARGS="--config $cfg" TAG=${T}_c${cfg}x256 \
    bash scripts/profile.sh || exit $?
  cp gpurun_out/prof_${T}_c${cfg}x256/pmc_step_cfg$cfg.json profiles/
done
mkdir -p gpurun_out/$T
cp profiles/pmc_step_kernel.json profiles/pmc_group_cfg5_c1.json profiles/pmc_step_cfg[345].json gpurun_out/$T/
echo "== bench ($(date +%T))"
timeout -k 10 600 python bench.py > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
tail -1 gpurun_out/$T/bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('headline', f\"{d['value']:.4e}\", 'frac', r['frac'], 'hbm', r['hbm']['frac'], 'single', f\"{d['single_chain_value']:.3e}\", 'pfauto', f\"{d['single_chain_prefetch_auto']['value']:.3e}\")
for k, e in d['configs'].items(): print(k, f\"{e['value']:.4e}\", 'frac', e['roofline']['frac'], 'lanes', e['lanes_per_particle'], 'fixed', f\"{e.get('fixed_theta', {}).get('value', 0):.3e}\", 'pf', e.get('prefetch_auto', {}).get('value'))"
echo "== abc bench ($(date +%T))"
timeout -k 10 300 python scripts/abc_bench.py --runs 10 --cpu-seconds 10 > gpurun_out/$T/abc_bench.log 2>&1 || { tail -5 gpurun_out/$T/abc_bench.log; exit 1; }
tail -1 gpurun_out/$T/abc_bench.log | cut -c1-300
if [ -z "${NO_PREFETCH:-}" ]; then
  echo "== prefetch sweep config 5 ($(date +%T))"
  CFG=5 H=config SLOTS="0 2 4 8 16 auto" ITERS=60 timeout -k 10 600 python scripts/prefetch_sweep.py > gpurun_out/$T/prefetch_cfg5.log 2>&1 || { tail -5 gpurun_out/$T/prefetch_cfg5.log; exit 1; }
  tail -12 gpurun_out/$T/prefetch_cfg5.log
fi
echo "== done"
