#!/bin/bash
# VALU / SALU instruction counts of pf_step_kernel with and without SSA events (scripts/overhead_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ovh; mkdir -p $OUT
for c in noev bench; do
  CASE=$c timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD --kernel-include-regex pf_step_kernel -d $OUT/$c -o run --output-format csv -- python3 scripts/overhead_probe.py > $OUT/$c.log 2>&1 || { echo "STOP $c rc=$?"; tail -5 $OUT/$c.log; exit 1; }
  grep "particle-steps" $OUT/$c.log
done
python3 - <<'PY'
import csv, glob, collections
for c in ("noev", "bench"):
    f = glob.glob(f"gpurun_out/ovh/{c}/**/run_counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(float); disp = set()
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    waves = tot["SQ_WAVES"]
    print(c, "dispatches", len(disp), {k: round(v / waves, 1) for k, v in tot.items()}, "per wave")
PY
