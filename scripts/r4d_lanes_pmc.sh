#!/bin/bash
# PMC of the lane-group kernel at one chain (config ${CFG:-5}) after the fixed-point decision pass, per lane shape W:K:
# instructions per wave, VALU-active and wave cycles, waits; and the kernel trace for the launch durations.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r4d}; mkdir -p $OUT
CFG=${CFG:-5}
for S in ${SHAPES:-8:1 8:2 16:1}; do
  n=${S/:/_}
  B="scripts/lanes_sweep.py --cfg $CFG --chains 1 --lanes $S --reps 1 --out $OUT/pmcsweep_$n.jsonl"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex pf_step_group_kernel -d $OUT/sq_$n -o run --output-format csv -- python3 $B > $OUT/sq_$n.log 2>&1 || { echo STOP sq $n; tail -3 $OUT/sq_$n.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-include-regex pf_step_group_kernel -d $OUT/valu_$n -o run --output-format csv -- python3 $B > $OUT/valu_$n.log 2>&1 || { echo STOP valu $n; tail -3 $OUT/valu_$n.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/trace_$n -o run --output-format csv -- python3 $B > $OUT/trace_$n.log 2>&1 || { echo STOP trace $n; exit 1; }
done
OUT=$OUT SHAPES="${SHAPES:-8:1 8:2 16:1}" python3 - <<'PY'
import csv, glob, collections, json, os
out = {}
O = os.environ["OUT"]
for S in os.environ["SHAPES"].split():
    n = S.replace(":", "_")
    acc = collections.defaultdict(list)
    for p in ("sq", "valu"):
        for f in glob.glob(f"{O}/{p}_{n}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    dur = []
    for f in glob.glob(f"{O}/trace_{n}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "pf_step_group_kernel" in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = avg["SQ_WAVES"]
    out[S] = {"avg_launch_us": sum(dur) / len(dur), "launches": len(dur), "pmc_avg_per_launch": avg,
              "valu_per_wave": avg["SQ_INSTS_VALU"] / w, "salu_per_wave": avg["SQ_INSTS_SALU"] / w,
              "wave_cycles_per_wave": avg["SQ_WAVE_CYCLES"] * 4 / w,
              "valu_active_cycles_per_wave": avg["SQ_ACTIVE_INST_VALU"] * 4 / w,
              "any_active_cycles_per_wave": avg["SQ_ACTIVE_INST_ANY"] * 4 / w,
              "wait_inst_any_cycles_per_wave": avg["SQ_WAIT_INST_ANY"] * 4 / w}
    print(S, json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out[S].items() if k != "pmc_avg_per_launch"}))
json.dump(out, open(f"{O}/lanes_pmc.json", "w"), indent=1)
PY
echo done
