#!/bin/bash
# Config 1 (256 chains, N = 100) bench entry at 1 / 2 / 4 host pipelines (--pipelines), headline shortened.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for P in ${PIPES:-1 2 4}; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-chain --configs 1 --pipelines $P \
      --detail gpurun_out/cfg1_p$P.json > gpurun_out/cfg1_p$P.log 2>&1 || { tail -5 gpurun_out/cfg1_p$P.log; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/cfg1_p$P.json')); e=d['configs']['1']
print('pipelines $P', '%.4e' % e['value'], 'ms/step', round(e['ms_per_step'], 3), 'fixed', '%.4e' % e['fixed_theta']['value'], e['kernel'])"
done
