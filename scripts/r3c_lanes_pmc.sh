#!/bin/bash
# One-chain lane-group kernel after the mask-based decision pass: lanes sweep (W = 4, 8, 16; 1, 2, 4 chains;
# configs 2, 3, 5), then PMC of config 5 at one chain for W = 4 and 8 (instructions, VALU busy, waits).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r3c; mkdir -p $OUT
timeout -k 10 500 python scripts/lanes_sweep.py --cfg 2 3 5 --chains 1 2 4 --lanes 4 8 16 --reps 3 --out $OUT/sweep.jsonl > $OUT/sweep.log 2>&1 || { echo "STOP sweep"; tail -5 $OUT/sweep.log; exit 1; }
cat $OUT/sweep.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['cfg'], d['chains'], d['lanes'], f\"{d['particle_steps_per_s']:.3e}\")"
for W in ${PMC_LANES:-4 8}; do
  B="scripts/lanes_sweep.py --cfg 5 --chains 1 --lanes $W --reps 1 --out $OUT/pmcsweep_$W.jsonl"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex pf_step_group_kernel -d $OUT/sq_$W -o run --output-format csv -- python3 $B > $OUT/sq_$W.log 2>&1 || { echo STOP sq $W; tail -3 $OUT/sq_$W.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-include-regex pf_step_group_kernel -d $OUT/valu_$W -o run --output-format csv -- python3 $B > $OUT/valu_$W.log 2>&1 || { echo STOP valu $W; tail -3 $OUT/valu_$W.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $OUT/trace_$W -o run --output-format csv -- python3 $B > $OUT/trace_$W.log 2>&1 || { echo STOP trace $W; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, json, os
out = {}
for W in os.environ.get("PMC_LANES", "4 8").split():
    acc = collections.defaultdict(list)
    for p in ("sq", "valu"):
        for f in glob.glob(f"gpurun_out/r3c/{p}_{W}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    dur = []
    for f in glob.glob(f"gpurun_out/r3c/trace_{W}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "pf_step_group_kernel" in r["Kernel_Name"]:
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = avg["SQ_WAVES"]
    out[W] = {"avg_launch_us": sum(dur) / len(dur), "launches": len(dur), "pmc_avg_per_launch": avg,
              "valu_per_wave": avg["SQ_INSTS_VALU"] / w, "salu_per_wave": avg["SQ_INSTS_SALU"] / w,
              "wave_cycles_per_wave": avg["SQ_WAVE_CYCLES"] * 4 / w,
              "valu_active_cycles_per_wave": avg["SQ_ACTIVE_INST_VALU"] * 4 / w,
              "any_active_cycles_per_wave": avg["SQ_ACTIVE_INST_ANY"] * 4 / w,
              "wait_inst_any_cycles_per_wave": avg["SQ_WAIT_INST_ANY"] * 4 / w}
    print(W, json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in out[W].items() if k != "pmc_avg_per_launch"}))
json.dump(out, open("gpurun_out/r3c/lanes_pmc_cfg5.json", "w"), indent=1)
PY
echo done
