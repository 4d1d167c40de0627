#!/bin/bash
# One-workgroup filter check: its GPU tests (+ PYTEST_EXTRA), then scripts/fused_probe.sh (MH iteration times per SSA
# width and with the step launches) and, with PHASE=1, scripts/fused_phase.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py ${PYTEST_EXTRA:-} -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fused_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/fused_probe.sh || exit 1
if [ -n "${PHASE:-}" ]; then bash scripts/fused_phase.sh; fi
