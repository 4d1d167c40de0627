#!/bin/bash
# Closing measurement of a build: rocprofv3 trace + PMC passes (scripts/profile.sh) of every workload the bench line
# reports -- the headline (config 2, 256 chains -> profiles/pmc_step_kernel.json), config 1 at 6,144 chains in four host
# pipelines (pmc_fused_cfg1.json: the one-workgroup filter), configs 3, 4, 5 at 256 chains
# (pmc_step_cfg{3,4,5}.json) and config 5 at one chain per GPU (pmc_group_cfg5_c1.json) -- each
# recording the library's build id, so the bench line's rooflines are those of the library it times; the SSA loop's
# ceiling (scripts/loop_ceiling.sh -> loop_ceiling.json, the rooflines' peak); then the default bench line and the ABC
# bench.  Each step has its own time limit; a failure ends the script.
#   TAG=r6z bash scripts/close.sh            (WHAT="c2 c1 c3 c4 c5 c5x1 ceiling bench rccl abc" selects steps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-close}
WHAT=${WHAT:-c2 c1 c3 c4 c5 c5x1 ceiling bench abc}
mkdir -p gpurun_out/$T
has() { [[ " $WHAT " == *" $1 "* ]]; }
prof() {  # prof <tag> <json name> <env...>
    local tag=$1 name=$2; shift 2
    env "$@" PMC_NAME=$name TAG=${T}_$tag bash scripts/profile.sh || exit $?
    cp gpurun_out/prof_${T}_$tag/$name gpurun_out/$T/
}
has c2 && prof c2 pmc_step_kernel.json PMC_CONFIG=2 PMC_CHAINS=256
has c1 && prof c1 pmc_fused_cfg1.json PMC_CONFIG=1 PMC_CHAINS=6144 PMC_LANES=1 PMC_KERNEL=pf_filter_wg_kernel \
  EPIPF_FUSED=1 BENCH_ARGS="--config 1 --chains 6144 --pipelines 4" STEPS=20
has c3 && prof c3x256 pmc_step_cfg3.json PMC_CONFIG=3 PMC_CHAINS=256 BENCH_ARGS="--config 3"
# configs 4 and 5 propose at h = 5 / h = 1: their initial-draw loops run many launches with a handful of pending chains,
# so the busy fraction is also taken over the MH iterations' launches alone (the last (steps + 2) x (T - 1) x 4
# dispatches: warm-up, timed and counters iterations, four chain-group streams; PMC_TIMED_DISPATCHES)
has c4 && prof c4x256 pmc_step_cfg4.json PMC_CONFIG=4 PMC_CHAINS=256 BENCH_ARGS="--config 4" PMC_TIMED_DISPATCHES=$(((3 + 2) * 14 * 4))
has c5 && prof c5x256 pmc_step_cfg5.json PMC_CONFIG=5 PMC_CHAINS=256 BENCH_ARGS="--config 5" STEPS=10 \
  PMC_TIMED_DISPATCHES=$(((10 + 2) * 13 * 4))
has c5x1 && prof c5x1 pmc_group_cfg5_c1.json PMC_CONFIG=5 PMC_CHAINS=1 PMC_LANES=16 PMC_KERNEL=pf_step_group_kernel \
  BENCH_ARGS="--config 5 --chains 1" STEPS=20
if has ceiling; then
  echo "== loop ceiling ($(date +%T))"
  bash scripts/loop_ceiling.sh > gpurun_out/$T/ceiling.log 2>&1 || { tail -5 gpurun_out/$T/ceiling.log; exit 1; }
  cp gpurun_out/ceiling/loop_ceiling.json gpurun_out/$T/ && cp gpurun_out/ceiling/loop_ceiling.json profiles/
fi
if has bench; then
  echo "== bench ($(date +%T))"
  cp gpurun_out/$T/pmc_*.json profiles/ 2>/dev/null
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 --detail gpurun_out/$T/bench_detail.json > gpurun_out/$T/bench.log 2>&1 || { tail -5 gpurun_out/$T/bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/$T/bench_detail.json')); r=d['roofline']
print('headline', f\"{d['value']:.4e}\", 'frac', r['frac'], 'issue', (r.get('valu_issue') or {}).get('issue_frac'), 'single', f\"{d['single_chain_value']:.3e}\", 'pf16', f\"{d['single_chain_prefetch']['value']:.3e}\", 'pfauto', f\"{d['single_chain_prefetch_auto']['value']:.3e}\")
for k, e in d['configs'].items(): print(k, f\"{e['value']:.4e}\", 'frac', e['roofline']['frac'], 'lanes', e['lanes_per_particle'], 'fixed', f\"{e.get('fixed_theta', {}).get('value', 0):.3e}\", 'pf', (e.get('prefetch_auto') or {}).get('value'))"
fi
if has rccl; then
  echo "== rccl rehearsal ($(date +%T))"
  CH=64 bash scripts/rccl_bench_check.sh > gpurun_out/$T/rccl.txt 2>&1 || { tail -5 gpurun_out/$T/rccl.txt; exit 1; }
  cp gpurun_out/rccl_bench.log gpurun_out/$T/rccl_bench.log
fi
if has abc; then
  echo "== abc bench ($(date +%T))"
  timeout -k 10 300 python scripts/abc_bench.py --runs 10 --cpu-seconds 10 > gpurun_out/$T/abc_bench.log 2>&1 || { tail -5 gpurun_out/$T/abc_bench.log; exit 1; }
  tail -1 gpurun_out/$T/abc_bench.log | cut -c1-300
fi
echo "== done"
