#!/bin/bash
# Lane-group decision pass on wave masks: the lane-group / ABC / fuzz parity tests, then an A/B of the single-chain
# benches against the previous commit's tree (ab_old, built in place), alternating on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3b
mkdir -p $OUT
ROOT=$(pwd)
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_lanes.py tests/test_abc_gpu.py tests/test_gpu_fuzz.py tests/test_gpu_fuzz_abc.py} > $OUT/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
run() {  # tag dir args...
  local tag=$1 d=$2; shift 2
  (cd $ROOT/$d && timeout -k 10 300 python bench.py --no-cpu-baseline --no-single-chain "$@") > $OUT/$tag.log 2>&1 || { echo "STOP $tag"; tail -5 $OUT/$tag.log; exit 1; }
  tail -1 $OUT/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', f\"{d['value']:.4e}\", f\"ms/step={d['ms_per_step']:.2f}\")"
}
for i in ${ROUNDS:-1 2}; do
  for d in ab_old .; do
    n=$(basename $d)
    run c5x1_${n}_$i $d --config 5 --chains 1 --steps 6 --warmup 2
    run c2x1_${n}_$i $d --config 2 --chains 1 --steps 10 --warmup 2
    [ -z "${SKIP_256:-}" ] && run c5x256_${n}_$i $d --config 5 --steps 3 --warmup 1
  done
done
[ -z "${SKIP_ABC:-}" ] && for d in ab_old .; do
  n=$(basename $d)
  (cd $ROOT/$d && timeout -k 10 300 python scripts/abc_bench.py ${ABC_ARGS:-}) > $OUT/abc_$n.log 2>&1 || { echo "STOP abc $n"; tail -5 $OUT/abc_$n.log; exit 1; }
  echo "abc_$n $(tail -1 $OUT/abc_$n.log)"
done
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 400 python scripts/lanes_sweep.py --cfg 2 5 --chains 1 2 8 --lanes ${SWEEP_LANES:-4 8} --reps 3 --out $OUT/lanes_sweep.jsonl > $OUT/sweep.log 2>&1 || { echo "STOP sweep"; tail -5 $OUT/sweep.log; exit 1; }
  cat $OUT/lanes_sweep.jsonl
fi
echo done
