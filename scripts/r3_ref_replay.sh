#!/bin/bash
# Round 3: bench-scale replay of the reference's resampling (scipy weights on the device's states) for configs 2, 3, 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in "--config 2 --chains 256" "--config 5 --chains 64" "--config 3 --chains 32"; do
  echo "== $a ($(date +%T))"
  timeout -k 10 900 python3 scripts/r3_ref_replay.py $a --workers 12 > "gpurun_out/r3_replay_${a// /_}.log" 2>&1 \
    || { echo "STOP rc=$?"; tail -20 "gpurun_out/r3_replay_${a// /_}.log"; exit 1; }
  tail -1 "gpurun_out/r3_replay_${a// /_}.log"
done
echo "== done"
