"""Time the UNMODIFIED reference particle filter in the build container and calibrate the C port against it.

BASELINE.md §3 / SURVEY.md §8d: the reference's own CPU rate is measured here (it never travels to the GPU box),
with `jobs=1` (one core) and `jobs=-1` (every core of this container), on BASELINE config 2's data at a reduced
particle count (a full N = 10^4 filter is hours on one core; per-particle work is independent, so the rate in
particle-steps/s does not depend on N beyond joblib's per-call overhead, reported by the two N values).  The C
restatement (oracle/, the `cpu_baseline` of bench.py) is timed on the same workload at 1 thread and at every
thread, which gives the port/reference factor that converts the GPU box's port timings into reference units.

Reference draws come from numpy's real global RandomState (np.random.seed), the port's from the keyed Philox
stream, so the two runs are different realisations of the same filter; events per particle-step are counted on
both sides (the reference's by a counting wrapper around its own sir_simulate, in a separate untimed run).

Usage (build container only):  python scripts/time_reference.py [--out profiles/r2_reference_timing.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def time_reference(pm, Y, meta, N, jobs, seed):
    np.random.seed(seed)
    t0 = time.perf_counter()
    z, hid, anc = pm.particle_filter(Y, pm.ModelType.SIR, np.array(meta["theta"], dtype=float), False, meta["probs"], N,
                                     meta["n_population"], meta["mu"], jobs=jobs)
    dt = time.perf_counter() - t0
    assert z is not None
    return dt


def reference_events(pm, ga, Y, meta, N, seed):
    """Events per particle-step of the reference (untimed): count the loop iterations of its sir_simulate by
    wrapping numpy's exponential draw (one per event, gillespie_algo.py:62) for one jobs=1 filter."""
    count = [0, 0]
    real, real_sim = ga.np.random.exponential, pm.sir_simulate

    def counting(*a, **k):
        count[0] += 1
        return real(*a, **k)

    def calls(*a, **k):
        count[1] += 1
        return real_sim(*a, **k)

    ga.np.random.exponential = counting
    pm.sir_simulate = calls
    try:
        np.random.seed(seed)
        pm.particle_filter(Y, pm.ModelType.SIR, np.array(meta["theta"], dtype=float), False, meta["probs"], N, meta["n_population"],
                           meta["mu"], jobs=1)
    finally:
        ga.np.random.exponential = real
        pm.sir_simulate = real_sim
    # the time is drawn before the overshoot test (gillespie_algo.py:62-66): one rejected draw per call that
    # ends by overshooting the step (every call that does not end by extinction)
    return (count[0] - count[1]) / (N * (Y.shape[0] - 1))


def time_port(Y, meta, N, threads, min_seconds=3.0):
    import oracle
    oracle.set_num_threads(threads)
    n = ev = 0
    t0 = time.perf_counter()
    while True:
        o = oracle.particle_filter(Y, "sir", tuple(meta["theta"]), False, meta["probs"], N, meta["n_population"],
                                   meta["mu"], key=7, filter_index=n)
        n += 1
        ev += o["events"]
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    ps = n * N * (Y.shape[0] - 1)
    return dict(threads=threads, filters=n, seconds=dt, particle_steps_per_s=ps / dt, events_per_s=ev / dt,
                events_per_particle_step=ev / ps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--particles", type=int, nargs="+", default=[64, 256])
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r2_reference_timing.json"))
    args = ap.parse_args()
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.path.insert(0, args.reference)
    import gillespie_algo as ga  # noqa: E402  (unmodified reference, read-only)
    import pmcmc as pm  # noqa: E402
    from epipf import datasets

    Y, meta = datasets.benchmark_dataset(args.config)
    T = Y.shape[0]
    cores = os.cpu_count()
    out = dict(config=args.config, T=T, theta=list(meta["theta"]), host_cpu=cpu_model(), host_cpus=cores,
               reference={}, port={})
    # joblib's loky pool starts on the first jobs=-1 call: warm it up outside the timed region
    pm.particle_filter(Y[:3], pm.ModelType.SIR, np.array(meta["theta"], dtype=float), False, meta["probs"], 16,
                       meta["n_population"], meta["mu"], jobs=-1)
    for N in args.particles:
        for jobs in (1, -1):
            dt = time_reference(pm, Y, meta, N, jobs, seed=1000 + N)
            ps = N * (T - 1)
            rec = dict(N=N, jobs=jobs, cores=1 if jobs == 1 else cores, seconds=dt, particle_steps_per_s=ps / dt)
            out["reference"][f"N{N}_jobs{jobs}"] = rec
            print(json.dumps(rec), flush=True)
    Nr = args.particles[-1]
    epps = reference_events(pm, ga, Y, meta, Nr, seed=1000 + Nr)
    out["reference_events_per_particle_step"] = epps
    for rec in out["reference"].values():
        rec["events_per_s"] = rec["particle_steps_per_s"] * epps
    for N in (Nr, 10000):
        for th in (1, cores):
            rec = time_port(Y, meta, N, th)
            out["port"][f"N{N}_threads{th}"] = rec
            print(json.dumps(rec), flush=True)
    ref1 = out["reference"][f"N{Nr}_jobs1"]["particle_steps_per_s"]
    refall = out["reference"][f"N{Nr}_jobs-1"]["particle_steps_per_s"]
    port1 = out["port"]["N10000_threads1"]["particle_steps_per_s"]
    portall = out["port"][f"N10000_threads{cores}"]["particle_steps_per_s"]
    out["factor_port_over_reference_1core"] = port1 / ref1
    out["factor_port_over_reference_allcores"] = portall / refall
    out["note"] = ("reference rates at N in --particles extrapolate linearly to N=10^4 (per-particle work is "
                   "independent); the port is timed at N=10^4 directly")
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("factor_port_over_reference_1core", "factor_port_over_reference_allcores",
                                           "reference_events_per_particle_step")}))


if __name__ == "__main__":
    main()
