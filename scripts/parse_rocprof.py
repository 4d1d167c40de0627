"""Summarise a scripts/profile.sh session: per-kernel stats of the trace pass and per-launch PMC averages
of the profiled kernel (PMC_KERNEL: pf_step_kernel, or pf_step_group_kernel with PMC_LANES lanes per particle).
Writes <dir>/<PMC_NAME> (default pmc_step_kernel.json; copied to profiles/ when committed: bench.py picks the
profiles/pmc_*.json whose build id, config, chains per GPU and lanes match the run it reports).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
counts 64 B per 128-B request of a wide coalesced stream (read side up to 2x low).  We report the raw
sum and the read-doubled upper estimate; `hbm_bytes_per_launch` is the raw sum (uncorrected, stated)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main(d):
    out = {}
    for p in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        print(f"# kernel stats: {p}")
        for r in rows(p):
            print(f"  {r['Name'][:90]:90s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:10.2f} "
                  f"total_ms={float(r['TotalDurationNs'])/1e6:9.2f} pct={float(r['Percentage']):6.2f}")
            if KERNEL in r["Name"]:
                out["trace_avg_us"] = float(r["AverageNs"]) / 1e3
                out["trace_calls"] = int(r["Calls"])
                out["kernel"] = r["Name"]
    for p in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        ks = sorted((r for r in rows(p) if KERNEL in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
        durs = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in ks)
        if durs:
            n = len(durs)
            print(f"# {KERNEL} durations (us) over {n} launches: min {durs[0]:.1f} p50 {durs[n // 2]:.1f} "
                  f"p90 {durs[int(n * .9)]:.1f} p99 {durs[int(n * .99)]:.1f} max {durs[-1]:.1f} "
                  f"sum {sum(durs) / 1e3:.1f} ms; launches > 5x median: {sum(x > 5 * durs[n // 2] for x in durs)}")
    per = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value
    pass_of = {}                                    # counter -> the pass directory it was collected in
    meta = {}
    for p in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in rows(p):
            if KERNEL not in r["Kernel_Name"]:
                continue
            per[r["Counter_Name"]][(p, r["Dispatch_Id"])] += float(r["Counter_Value"])
            pass_of[r["Counter_Name"]] = os.path.relpath(p, d).split(os.sep)[0]
            meta = {k: r.get(k) for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                          "SGPR_Count", "Scratch_Size")}
    avg = {k: sum(v.values()) / len(v) for k, v in per.items() if v}
    out["pmc_avg_per_launch"] = avg
    out["pmc_launches"] = {k: len(v) for k, v in per.items()}
    out["dispatch"] = meta
    # per counted particle-step (profile.sh): the pass's counter total over all its launches / the particle-steps its
    # bench process ran, count_<pass>.txt -- the bench line's accounting (N x T per chain that runs a filter, degenerate
    # filters included), whatever the grid of each launch
    region = {}
    for k, v in per.items():
        cp_ = os.path.join(d, f"count_{pass_of.get(k)}.txt")
        if os.path.exists(cp_):
            ps = sum(int(line) for line in open(cp_) if line.strip())
            if ps > 0:
                region[k] = sum(v.values()) / ps
    if region:
        out["per_counted_particle_step"] = True
        out["pmc_per_particle_step"] = region
        if "SQ_INSTS_VALU" in region:
            out["valu_per_particle_step"] = region["SQ_INSTS_VALU"]
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        raw = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
        out["hbm_bytes_per_launch"] = raw
        out["hbm_bytes_per_launch_read_doubled"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
        # per particle-step (LANES lanes per particle): launches of chain groups on concurrent streams have
        # different grid sizes than a one-launch-per-step run, so bench.py scales this figure instead
        lanes = float(meta.get("Grid_Size") or 0) / LANES
        if "FETCH_SIZE" in region and "WRITE_SIZE" in region:
            out["hbm_bytes_per_particle_step"] = (region["FETCH_SIZE"] + region["WRITE_SIZE"]) * 1024.0
            out["hbm_bytes_per_particle_step_read_doubled"] = (2 * region["FETCH_SIZE"] + region["WRITE_SIZE"]) * 1024.0
        elif lanes > 0:
            out["hbm_bytes_per_particle_step"] = raw / lanes
            out["hbm_bytes_per_particle_step_read_doubled"] = out["hbm_bytes_per_launch_read_doubled"] / lanes
    # VALU pipe utilisation (the bound of this kernel): SQ_ACTIVE_INST_VALU counts quad-cycles of VALU
    # execution summed over waves, GRBM_GUI_ACTIVE GPU cycles summed over the 8 XCDs (MI355X_MICROARCH.md), both
    # in the same pass, over the 1024 SIMDs; dispatches are serialised under counter collection
    act, gui = per.get("SQ_ACTIVE_INST_VALU", {}), per.get("GRBM_GUI_ACTIVE", {})
    both = [k for k in act if k in gui]
    if both:
        out["valu_busy_frac"] = 4.0 * sum(act[k] for k in both) / (1024.0 * sum(gui[k] for k in both) / 8.0)
        # PMC_TIMED_DISPATCHES = D: the same fraction over the pass's last D dispatches -- the bench run's MH iterations
        # after its initial-draw loop (at h = 1 that loop's launches carry a handful of live chains each)
        if TIMED and len(both) > TIMED:
            last = sorted(both, key=lambda k: int(k[1]))[-TIMED:]
            out["valu_busy_frac_timed"] = 4.0 * sum(act[k] for k in last) / (1024.0 * sum(gui[k] for k in last) / 8.0)
            out["timed_dispatches"] = TIMED
    lanes = float(meta.get("Grid_Size") or 0) / LANES
    if lanes > 0:   # LANES lanes per particle (padding of the last block included: < 0.5% at N = 10^4)
        out["particle_steps_per_launch"] = lanes
    # the library build these counters belong to (bench.py uses them only for the same build id)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "stochastic-epidemic-modelling_amd"))
    from epipf import _lib
    out["build_id"] = _lib.build_id()
    out.update({k: v for k, v in (("config", CONFIG), ("chains_per_gpu", CHAINS)) if v is not None})
    out["lanes"] = LANES
    print(json.dumps(out, indent=1))
    with open(os.path.join(d, NAME), "w") as f:
        json.dump(out, f, indent=1)


CONFIG = int(os.environ["PMC_CONFIG"]) if os.environ.get("PMC_CONFIG") else None        # bench --config profiled
CHAINS = int(os.environ["PMC_CHAINS"]) if os.environ.get("PMC_CHAINS") else None        # bench --chains profiled
KERNEL = os.environ.get("PMC_KERNEL", "pf_step_kernel")                                  # kernel name profiled
LANES = int(os.environ.get("PMC_LANES", "1"))                                            # its lanes per particle
NAME = os.environ.get("PMC_NAME", "pmc_step_kernel.json")
TIMED = int(os.environ.get("PMC_TIMED_DISPATCHES", "0"))                                 # last D dispatches: timed

if __name__ == "__main__":
    main(sys.argv[1])
