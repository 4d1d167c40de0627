#!/bin/bash
# Lanes sweep over chain counts (W = 4, 8) for configs 2, 3, 5: where the automatic choice should switch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3k; mkdir -p $OUT
timeout -k 10 900 python scripts/lanes_sweep.py --cfg ${CFGS:-2 3 5} --chains ${CHAINS:-1 2 4 8} --lanes ${LANES:-4 8} --reps 3 --out $OUT/sweep.jsonl > $OUT/sweep.log 2>&1 || { echo "STOP sweep"; tail -5 $OUT/sweep.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/sweep.jsonl'):
    d=json.loads(l); print(d['cfg'], d['chains'], d['lanes'], f\"{d['particle_steps_per_s']:.3e}\")"
