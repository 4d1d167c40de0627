set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/lanes_tests.log 2>&1; rc=$?
tail -5 gpurun_out/lanes_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/lanes_tests.log | head -20; exit $rc; }
timeout -k 10 600 python -u scripts/lanes_sweep.py --reps 2 --chains 1 2 8 --lanes 1 2:1 4:1 8:1 16:1 > gpurun_out/lanes_sweep.log 2>&1; rc=$?
tail -50 gpurun_out/lanes_sweep.log
exit $rc
