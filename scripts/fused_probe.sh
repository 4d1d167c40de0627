#!/bin/bash
# One MH iteration's wall / filter / device time (scripts/mh_iteration_probe.py) for the one-workgroup filter at each SSA
# width in LANES (EPIPF_FUSED_LANES; "off" = EPIPF_FUSED=0, the step launches), per CASES entry "cfg:particles:chains".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-fused_probe}.jsonl
: > $OUT
for case in ${CASES:-1:100:1 1:100:256 2:100:1 2:256:1 2:100:256}; do
  IFS=: read cfg n ch <<< "$case"
  for w in ${LANES:-off 1 4}; do
    if [ "$w" = off ]; then env="EPIPF_FUSED=0"; else env="EPIPF_FUSED_LANES=$w"; fi
    env $env timeout -k 10 120 python scripts/mh_iteration_probe.py --cfg $cfg --particles $n --chains $ch \
        --iters ${ITERS:-100} --tag "lanes=$w" >> $OUT 2>gpurun_out/fused_probe.err || { tail -5 gpurun_out/fused_probe.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT'):
    d = json.loads(l)
    print(f\"cfg {d['cfg']} N {d['N']:5d} chains {d['chains']:3d} {d['tag']:9s} fused {d['fused']} W {d['lanes']:2d}: step {d['step_us_mean']:8.1f} us  device {d['device_filter_us_mean']:8.1f} us  {d['particle_steps_per_s_step']:.3e} /s\")"
