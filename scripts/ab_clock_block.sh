set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fast_ssa or replays or full_size or oracle" --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
L=$GRAFT_REPO_ROOT/stochastic-epidemic-modelling_amd
for cfg in 2 5; do
CFG=$cfg STEPS=6 ENVS="EPIPF_LIBRARY=$L/lib_old/libepipf.so - EPIPF_LIBRARY=$L/lib_k8/libepipf.so EPIPF_LIBRARY=$L/lib_old/libepipf.so - EPIPF_LIBRARY=$L/lib_k8/libepipf.so" bash scripts/ab_env.sh || exit 1
done
