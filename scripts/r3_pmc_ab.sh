#!/bin/bash
# Round 3: per-dispatch SQ counters of pf_step_kernel, the round-2 tree (ab_old/, side A) against this tree (B): one
# rocprofv3 --pmc pass each on a short default bench.  Every step has its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ROOT=$(pwd)
mkdir -p gpurun_out/pmcab
for side in A B; do
  dir=$ROOT; [ $side = A ] && dir=$ROOT/ab_old
  (cd $dir && timeout -s KILL 180 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS} \
      --kernel-include-regex pf_step_kernel -d $ROOT/gpurun_out/pmcab/$side -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-single-chain) > gpurun_out/pmcab/$side.log 2>&1 \
      || { echo "STOP $side rc=$?"; tail -5 gpurun_out/pmcab/$side.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for side in "AB":
    per = collections.defaultdict(list)
    for p in glob.glob(f"gpurun_out/pmcab/{side}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(p)):
            if "pf_step_kernel" in r["Kernel_Name"]:
                agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), v in agg.items():
            per[c].append(v)
    print(side, {c: round(sum(v) / len(v)) for c, v in sorted(per.items())}, "dispatches", len(per.get("SQ_WAVES", [])))
PY
echo "== done"
