#!/bin/bash
# PMC passes of the ABC trial kernel (scripts/abc_bench.py): instruction mix, VALU busy, LDS bank conflicts.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r2p; mkdir -p $OUT
B="scripts/abc_bench.py --runs 1 --cpu-seconds 0.2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex abc_trials_kernel -d $OUT/sq -o run --output-format csv -- python3 $B > $OUT/sq.log 2>&1 || { echo STOP sq; tail -3 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex abc_trials_kernel -d $OUT/valu -o run --output-format csv -- python3 $B > $OUT/valu.log 2>&1 || { echo STOP valu; tail -3 $OUT/valu.log; exit 1; }
EPIPF_PROFILE=2 timeout -k 10 120 python3 $B > $OUT/bench.jsonl 2>&1 || { echo STOP bench; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ("sq", "valu"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r2p/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(p, {k: "%.4g" % (sum(v) / len(v)) for k, v in acc.items()}, "launches", len(next(iter(acc.values()))) if acc else 0)
PY
tail -1 $OUT/bench.jsonl | cut -c1-600
