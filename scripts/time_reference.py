"""Time the UNMODIFIED reference particle filter in the build container and calibrate the C port against it, per
BASELINE config.

BASELINE.md §3 / SURVEY.md §8d: the reference's own CPU rate is measured here (it never travels to the GPU box), with
`jobs=1` (one core) and `jobs=-1` (every core of this container), on each BASELINE config's data
(epipf.datasets.benchmark_dataset) at a reduced particle count where the config's N would take hours (per-particle work
is independent, so the rate in particle-steps/s does not depend on N beyond joblib's per-call overhead, which the two N
values show).  The C restatement (oracle/, the `cpu_baseline` of bench.py) is timed on the same workload at 1 thread
and at every thread, which gives the port/reference factor that converts the GPU box's port timings into reference
units (bench.py: `reference_calibrated`, one factor per config).

Reference draws come from numpy's real global RandomState (np.random.seed), the port's from the keyed Philox stream, so
the two runs are different realisations of the same filter; events per particle-step are counted on both sides (the
reference's by a counting wrapper around its own simulator, in a separate untimed run).

Usage (build container only, nothing else running):
    python scripts/time_reference.py --config 1 3 4 5   ->  profiles/reference_timing_cfg<c>.json
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

# particle counts timed on the reference, per config (the config's own N where a filter takes seconds)
REF_PARTICLES = {1: [100], 2: [64, 256], 3: [32, 96], 4: [32, 96], 5: [16, 48]}
SIMULATOR = {"sir": "sir_simulate", "seir": "seir_simulate", "sir_subgroups": "sir_subgroups_simulate"}


def cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def ref_args(pm, meta):
    """(ModelType, theta, n_population, mu) in the reference's argument types (pmcmc.py:123-175)."""
    th = np.asarray(meta["theta"], dtype=float)
    if meta["model"] == "sir_subgroups":
        G = int(round(np.sqrt(th.size - 1)))
        return (pm.ModelType.SIR_SUBGROUPS, (th[:G * G].reshape(G, G), th[-1]),
                np.asarray(meta["n_population"], dtype=float), np.asarray(meta["mu"], dtype=float))
    mt = pm.ModelType.SIR if meta["model"] == "sir" else pm.ModelType.SEIR
    return mt, th, meta["n_population"], meta["mu"]


def port_theta(meta):
    th = np.asarray(meta["theta"], dtype=float)
    if meta["model"] == "sir_subgroups":
        G = int(round(np.sqrt(th.size - 1)))
        return (th[:G * G].reshape(G, G), th[-1])
    return tuple(th)


def time_reference(pm, Y, meta, N, jobs, seed):
    mt, th, npop, mu = ref_args(pm, meta)
    np.random.seed(seed)
    t0 = time.perf_counter()
    z, hid, anc = pm.particle_filter(Y, mt, th, meta.get("observations", False), meta["probs"], N, npop, mu,
                                     jobs=jobs)
    dt = time.perf_counter() - t0
    return dt, z is not None


def reference_events(pm, ga, Y, meta, N, seed):
    """Events per particle-step of the reference (untimed): count its simulator's exponential draws (one per loop
    iteration, gillespie_algo.py:62 / 133 / 208) and calls in one jobs=1 filter."""
    count = [0, 0]
    name = SIMULATOR[meta["model"]]
    real, real_sim = ga.np.random.exponential, getattr(pm, name)

    def counting(*a, **k):
        count[0] += 1
        return real(*a, **k)

    def calls(*a, **k):
        count[1] += 1
        return real_sim(*a, **k)

    ga.np.random.exponential = counting
    setattr(pm, name, calls)
    mt, th, npop, mu = ref_args(pm, meta)
    try:
        np.random.seed(seed)
        pm.particle_filter(Y, mt, th, meta.get("observations", False), meta["probs"], N, npop, mu, jobs=1)
    finally:
        ga.np.random.exponential = real
        setattr(pm, name, real_sim)
    # the time is drawn before the overshoot test (:62-66): one rejected draw per call that ends by overshooting the
    # step (every call that does not end by extinction)
    return (count[0] - count[1]) / max(1, count[1])


def time_port(Y, meta, N, threads, min_seconds=3.0):
    import oracle
    oracle.set_num_threads(threads)
    n = ev = 0
    th = port_theta(meta)
    t0 = time.perf_counter()
    while True:
        o = oracle.particle_filter(Y, meta["model"], th, meta.get("observations", False), meta["probs"], N,
                                   meta["n_population"], meta["mu"], key=7, filter_index=n)
        n += 1
        ev += o["events"]
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    ps = n * N * (Y.shape[0] - 1)
    return dict(threads=threads, filters=n, seconds=dt, particle_steps_per_s=ps / dt, events_per_s=ev / dt,
                events_per_particle_step=ev / ps)


def calibrate(pm, ga, cfg, out_path):
    from epipf import datasets
    Y, meta = datasets.benchmark_dataset(cfg)
    T = Y.shape[0]
    cores = os.cpu_count()
    out = dict(config=cfg, model=meta["model"], T=T, N_config=meta["N"], theta=list(np.asarray(meta["theta"], float)),
               host_cpu=cpu_model(), host_cpus=cores, reference={}, port={})
    mt, th, npop, mu = ref_args(pm, meta)
    # joblib's loky pool starts on the first jobs=-1 call: warm it up outside the timed region
    pm.particle_filter(Y[:3], mt, th, meta.get("observations", False), meta["probs"], 16, npop, mu, jobs=-1)
    for N in REF_PARTICLES[cfg]:
        for jobs in (1, -1):
            dt, ok = time_reference(pm, Y, meta, N, jobs, seed=1000 + N)
            # the metric counts N x (T - 1) propagated particle-steps per filter; a degenerate filter (None triple)
            # stops early and is reported, not used
            rec = dict(N=N, jobs=jobs, cores=1 if jobs == 1 else cores, seconds=dt, completed=ok,
                       particle_steps_per_s=N * (T - 1) / dt)
            out["reference"][f"N{N}_jobs{jobs}"] = rec
            print(json.dumps(rec), flush=True)
    Nr = REF_PARTICLES[cfg][-1]
    epps = reference_events(pm, ga, Y, meta, Nr, seed=1000 + Nr)
    out["reference_events_per_particle_step"] = epps
    for rec in out["reference"].values():
        rec["events_per_s"] = rec["particle_steps_per_s"] * epps
    for th_ in (1, cores):
        rec = time_port(Y, meta, meta["N"], th_)
        out["port"][f"N{meta['N']}_threads{th_}"] = rec
        print(json.dumps(rec), flush=True)
    ref1 = out["reference"][f"N{Nr}_jobs1"]["particle_steps_per_s"]
    refall = out["reference"][f"N{Nr}_jobs-1"]["particle_steps_per_s"]
    port1 = out["port"][f"N{meta['N']}_threads1"]["particle_steps_per_s"]
    portall = out["port"][f"N{meta['N']}_threads{cores}"]["particle_steps_per_s"]
    out["factor_port_over_reference_1core"] = port1 / ref1
    out["factor_port_over_reference_allcores"] = portall / refall
    out["note"] = (f"reference timed at N in {REF_PARTICLES[cfg]} (per-particle work is independent, the rate "
                   f"extrapolates linearly to the config's N = {meta['N']}); the port is timed at N = {meta['N']}; "
                   f"both on this build container's {cores} CPUs ({cpu_model()})")
    with open(out_path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: out[k] for k in ("config", "factor_port_over_reference_1core",
                                           "factor_port_over_reference_allcores",
                                           "reference_events_per_particle_step")}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--config", type=int, nargs="+", default=[1, 2, 3, 4, 5])
    args = ap.parse_args()
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.path.insert(0, args.reference)
    import gillespie_algo as ga  # noqa: E402  (unmodified reference, read-only)
    import pmcmc as pm  # noqa: E402
    for cfg in args.config:
        calibrate(pm, ga, cfg, os.path.join(REPO, "profiles", f"reference_timing_cfg{cfg}.json"))


if __name__ == "__main__":
    main()
