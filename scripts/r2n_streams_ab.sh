#!/bin/bash
# Chain-group streams with the XCD-aware placement: EPIPF_STREAMS 2 / 4 / 8, config 2, alternated twice.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
rm -f gpurun_out/ab/b_*.log
CFG=2 STEPS=5 ENVS="EPIPF_STREAMS=4 EPIPF_STREAMS=2 EPIPF_STREAMS=8 EPIPF_STREAMS=4 EPIPF_STREAMS=2 EPIPF_STREAMS=8" bash scripts/ab_env.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
