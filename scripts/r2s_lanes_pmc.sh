#!/bin/bash
# PMC of the lane-group step kernel at one chain (config 2 and 5): instructions per launch, VALU busy, waves.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r2s; mkdir -p $OUT
for cfg in 2 5; do
  B="scripts/lanes_sweep.py --cfg $cfg --chains 1 --lanes 4 --reps 1 --out $OUT/sweep_$cfg.jsonl"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex pf_step_group_kernel -d $OUT/sq_$cfg -o run --output-format csv -- python3 $B > $OUT/sq_$cfg.log 2>&1 || { echo STOP sq $cfg; tail -3 $OUT/sq_$cfg.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex pf_step_group_kernel -d $OUT/valu_$cfg -o run --output-format csv -- python3 $B > $OUT/valu_$cfg.log 2>&1 || { echo STOP valu $cfg; tail -3 $OUT/valu_$cfg.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/trace_$cfg -o run --output-format csv -- python3 $B > $OUT/trace_$cfg.log 2>&1 || { echo STOP trace $cfg; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json
out = {}
for cfg in (2, 5):
    acc = collections.defaultdict(list)
    for p in ("sq", "valu"):
        for f in glob.glob(f"gpurun_out/r2s/{p}_{cfg}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    dur = []
    for f in glob.glob(f"gpurun_out/r2s/trace_{cfg}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "pf_step_group_kernel" in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    busy = avg["SQ_ACTIVE_INST_VALU"] * 4 / (avg["GRBM_GUI_ACTIVE"] / 8 * 1024)
    out[cfg] = {"avg_launch_us": sum(dur) / len(dur), "launches": len(dur), "pmc_avg_per_launch": avg,
                "valu_busy_frac_chip": busy,
                "valu_per_wave": avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]}
    print(cfg, json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in out[cfg].items() if k != "pmc_avg_per_launch"}))
json.dump(out, open("gpurun_out/r2s/lanes_pmc.json", "w"), indent=1)
PY
