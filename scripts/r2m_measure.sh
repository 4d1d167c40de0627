#!/bin/bash
# Round-2 closing measurement with the XCD-aware placement: rocprofv3 kernel trace + PMC passes of the default bench
# (scripts/profile.sh, TAG=r2m), then the default bench line (as the driver runs it).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r2m bash scripts/profile.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r2m_bench.log 2>&1 || { tail -5 gpurun_out/r2m_bench.log; exit 1; }
tail -1 gpurun_out/r2m_bench.log | cut -c1-400
echo "== done"
