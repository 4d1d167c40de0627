"""Summarise scripts/loop_ceiling.sh's run: per BASELINE config, the SSA event loop's lane-events/s with every lane busy
("uniform") and with one particle per lane ("distinct"), eight waves per SIMD, plus the PMC pass's wave64 VALU instructions per second and VALU busy of the same dispatches.

    python scripts/loop_ceiling_parse.py gpurun_out/ceiling > gpurun_out/ceiling/loop_ceiling.json"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_jsonl(path):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip().startswith("{")]


def pmc_dispatches(d):
    """Per dispatch (in dispatch order): counter totals and duration (s) from the counter-collection CSV."""
    rows = []
    for f in glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    disp = collections.OrderedDict()
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        e = disp.setdefault(int(r["Dispatch_Id"]), {"dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(disp.values())


def build_id():
    sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
    os.environ.setdefault("EPIPF_NO_TORCH_PRELOAD", "1")
    from epipf import _lib
    return _lib.build_id()


def main():
    d = sys.argv[1]
    natural = read_jsonl(os.path.join(d, "natural.jsonl"))
    disp = pmc_dispatches(d)
    # the PMC run repeats the natural run: per (config, variant) one warm-up launch and three timed launches
    assert len(disp) == 4 * len(natural), (len(disp), len(natural))
    out = {"build_id": build_id(), "source": "scripts/loop_ceiling.hip (fast_propagate of csrc/epipf_device.hpp)",
           "unit": "lane-events/s (SSA events, every lane counted)",
           "note": "lane_events_per_s: HIP events around each launch (best of three); valu_instr_per_s, valu_busy, "
                   "clock_ghz: the rocprofv3 PMC run of the same launches", "configs": {}}
    for i, e in enumerate(natural):
        timed = disp[4 * i + 1:4 * i + 4]
        best = max(timed, key=lambda t: t["SQ_INSTS_VALU"] / t["dur"])
        cyc = best["GRBM_GUI_ACTIVE"] / 8.0                          # summed over the 8 XCDs
        e = dict(e)
        e["valu_instr_per_s"] = best["SQ_INSTS_VALU"] / best["dur"]
        e["valu_busy"] = 4.0 * best["SQ_ACTIVE_INST_VALU"] / (1024.0 * cyc)
        e["valu_dual_issue_frac"] = 4.0 * best["SQ_ACTIVE_INST_VALU2"] / (1024.0 * cyc)
        e["clock_ghz"] = cyc / best["dur"] / 1e9
        out["configs"].setdefault(str(e["config"]), {})[e["variant"]] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
