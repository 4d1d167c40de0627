"""Benchmark: SIR PMCMC particle-steps/s on MI355X (BASELINE.json metric, config 2).

A "step" is one Metropolis-Hastings iteration of every chain on this rank: host proposals, one batched
GPU particle filter (N=10,000 particles x T=200 observations per chain, SIR, binomial observations,
population 10,000), on-device path sampling, host accept/reject.  value = N x T x (chains that ran a
filter) over all ranks / max-over-ranks wall time of the K timed steps (inputs resident in HBM).

Multi-GPU: one process per GPU (torch.distributed.run); chains are independent, so each rank runs its
own `--chains` chains with no collective on the data path; the posterior draws of the timed steps are
all-gathered over RCCL at the end of the timed region (pmcmc chain gather).

Also reported: roofline of the dominant kernel (pf_step_kernel, HIP-event timed on the engine's stream),
a CPU baseline (the oracle C restatement, OpenMP, on a bounded sample) on rank 0 at N=1, and `configs`: short
timed runs of the other BASELINE workloads -- config 1 at 6,144 chains per GPU, configs 3, 4, 5 at 256 and config 5 at ONE chain per
GPU (BASELINE's "8 independent chains across 8 GPUs" layout, the lane-group kernel) -- each with its own roofline where
a PMC profile of that (config, chains, lanes) on this library build is committed (profiles/pmc_*.json), and its own
CPU baseline with the reference-calibrated rate of that config (profiles/reference_timing_cfg<c>.json).
"""
import argparse
import gc
import glob
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters
VALU_PEAK = 1024 * 2.4e9 / 2   # wave64 VALU instructions/s: 1024 SIMDs, 2.4 GHz, one wave64 instruction per 2 cycles
MODEL_NAMES = {"sir": "SIR", "seir": "SEIR", "sir_subgroups": "multi-subgroup SIR", "sir_subgroups2": "SIR subgroups2"}
# the `configs` workloads: name -> (BASELINE config, chains per GPU)
CONFIG_RUNS = {"1": (1, 6144, 4), "3": (3, 256, 1), "4": (4, 256, 1), "5": (5, 256, 1), "5x1": (5, 1, 1)}


def parse():
    ap = argparse.ArgumentParser()
    # under a launcher (WORLD_SIZE set) --gpus defaults to the world size; without one, to 1
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chains", type=int, default=int(os.environ.get("EPIPF_BENCH_CHAINS", 256)),
                    help="independent MH chains per GPU (batched in one launch per filter step)")
    ap.add_argument("--particles", type=int, default=None, help="default: the config's N (SURVEY.md §8d)")
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--proposal", choices=["config", "fixed_theta"], default="config",
                    help="MH proposal h * sigma: the config's (epipf.datasets.PROPOSALS) or h = 1e-4, sigma = I")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--single-chain", action=argparse.BooleanOptionalAction, default=True,
                    help="also time 1 chain/GPU (N=1 only): one filter per MH iteration, and speculative MH (extra fields)")
    ap.add_argument("--configs", default="1,3,4,5,5x1",
                    help="extra timed workloads for the `configs` object (comma list of " + ", ".join(CONFIG_RUNS) +
                         "; 'none' to skip)")
    ap.add_argument("--configs-steps", type=int, default=4, help="timed MH iterations per `configs` workload")
    ap.add_argument("--configs-cpu-seconds", type=float, default=3.0,
                    help="CPU baseline per `configs` workload: seconds of port filters at 1 thread and at all threads")
    ap.add_argument("--pipelines", type=int, default=int(os.environ.get("EPIPF_BENCH_PIPELINES", 0)),
                    help="chain groups on their own engine + host thread, so each group's MH host work overlaps the "
                         "others' filters (epipf.pmcmc.run_pipelined); 0 = the headline on one lockstep sampler and each "
                         "`configs` entry at its own (CONFIG_RUNS: config 1 in four groups, DESIGN.md §7)")
    ap.add_argument("--prefetch", type=int, default=16, help="filter slots per round of the speculative single chain")
    # ~40 rounds: a speculative round commits ~8 iterations at config 2; 60 iterations (6 rounds) moved the adaptive
    # width's figure by +-20% from run to run (profiles/r4y_prefetch_cfg5.txt), 200 still by ~+-7% (BENCH_r05)
    ap.add_argument("--prefetch-iters", type=int, default=400, help="MH iterations timed for the speculative chain")
    ap.add_argument("--detail", default=None,
                    help="file for the full result (every diagnostic and `configs` entry); the printed line is the "
                         "compact form and names this file.  Default gpurun_out/bench_detail_n<N>.json")
    return ap.parse_args()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def host_threads():
    """CPU threads this process may use: the box's allotment (OMP_NUM_THREADS is set to it on the GPU box; the
    machine's full CPU count, os.cpu_count(), is many times that), else the affinity mask."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(env))) if env and env.isdigit() else avail


def reference_calibration(cfg):
    """The port/reference factors scripts/time_reference.py measured for BASELINE config `cfg` in the build container
    (the unmodified reference's particle_filter at jobs=1 / jobs=-1 next to the port on the same data), or None."""
    path = os.path.join(REPO, "profiles", f"reference_timing_cfg{cfg}.json")
    if not os.path.exists(path):
        return None, None
    return json.load(open(path)), os.path.relpath(path, REPO)


def cpu_baseline(Y, meta, N, seconds, cfg):
    """The oracle (C restatement of the reference filter, OpenMP over particles) on the GPU box's host, at 1 thread
    and at every thread this process is allotted.  Sample: whole filters of N particles x T steps of the config's data
    (the bench config's N; the `configs` entries a capped N, the rate per particle-step not depending on N) repeated
    until `seconds` elapse (at least one) per thread count.  The reference itself never runs on the GPU box:
    scripts/time_reference.py times it in the build container next to the same port, per config, and the
    port/reference factor it measured (profiles/reference_timing_cfg<c>.json) converts the port's rates into the
    reference's (`reference_calibrated`)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    oracle.build()
    th = np.array(meta["theta"], dtype=np.float64)
    if meta["model"].startswith("sir_subgroups"):                     # (beta[G][G], gamma), pmcmc.py:289-296
        G = int(round(np.sqrt(th.size - 1)))
        th = (th[:G * G].reshape(G, G), th[-1])

    def timed(threads, budget):
        oracle.set_num_threads(threads)
        t0 = time.perf_counter()
        n = ev = 0
        while True:
            o = oracle.particle_filter(Y, meta["model"], th, meta.get("observations", False), meta["probs"], N,
                                       meta["n_population"], meta["mu"], key=7, filter_index=n)
            n += 1
            ev += o["events"]
            if time.perf_counter() - t0 >= budget:
                break
        dt = time.perf_counter() - t0
        return n, dt, ev, oracle.num_threads()

    allt = host_threads()
    n, dt, ev, used = timed(allt, seconds)
    n1, dt1, ev1, _ = timed(1, seconds)
    value, value1 = n * N * Y.shape[0] / dt, n1 * N * Y.shape[0] / dt1
    base = dict(value=value, unit="particle-steps/s", cores=used, kind="port",
                sample=f"{n} full filter(s) of config {cfg} (N={N}, T={Y.shape[0]}) on {used} threads in {dt:.1f}s "
                       f"({ev / dt:.3g} events/s); host CPU: {cpu_model()}, {used} threads allotted to this process of "
                       f"{os.cpu_count()} on the machine",
                single_core={"value": value1, "cores": 1, "sample": f"{n1} full filter(s) in {dt1:.1f}s",
                             "events_per_s": ev1 / dt1})
    cal, cal_path = reference_calibration(cfg)
    if cal:
        f1, fall = cal["factor_port_over_reference_1core"], cal["factor_port_over_reference_allcores"]
        base["reference_calibrated"] = {
            # an ESTIMATE: the factor was measured on the build container's CPU, the port's rate here on the GPU box's;
            # dividing one by the other assumes the port/reference ratio does not depend on the host
            "estimate": "cross-host extrapolation (port rate on this host / port-over-reference factor measured on "
                        "the build container)",
            "reference_1core_value": value1 / f1,
            "reference_allcores_value": value / fall,
            "factor_port_over_reference_1core": f1,
            "factor_port_over_reference_allcores": fall,
            "reference_measured": {k: v["particle_steps_per_s"] for k, v in cal["reference"].items()},
            "reference_events_per_particle_step": cal.get("reference_events_per_particle_step"),
            "reference_host": f"{cal['host_cpu']} ({cal['host_cpus']} CPUs), build container",
            "source": f"{cal_path} (scripts/time_reference.py: unmodified reference particle_filter, jobs=1 / "
                      f"jobs=-1, config {cfg} data)"}
    return base


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv, gpus, port):
    """The command `bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) runs as its child: one rank per GPU
    under torch.distributed.run on this node, the same form the driver uses, with this invocation's arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(args, argv):
    """Parent side of a self-launched N-GPU bench.  Runs before anything initialises the GPU (counting devices does
    not on this image), starts the ranks as a child process (never an exec) and returns its exit code; the ranks'
    output (rank 0's JSON line) passes straight through."""
    import subprocess
    backend = os.environ.get("EPIPF_DIST_BACKEND", "nccl")
    if backend == "nccl":
        import torch
        ndev = torch.cuda.device_count()
        if args.gpus > ndev:
            print(f"bench.py: --gpus {args.gpus} but this node has {ndev} GPU(s); the nccl (RCCL) backend needs one "
                  f"GPU per rank", file=sys.stderr, flush=True)
            return 2
    cmd = launcher_command(argv, args.gpus, free_port())
    print(f"bench.py: launching {args.gpus} ranks ({backend}): {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ, EPIPF_BENCH_LAUNCHED="1"))


def resolve_gpus(args, env):
    """--gpus against the launcher's WORLD_SIZE: absent -> the world size (1 without a launcher); an explicit value
    that differs from a launcher's world size is an error (returns a message), as one rank per GPU is the contract."""
    world = int(env["WORLD_SIZE"]) if "WORLD_SIZE" in env else None
    if args.gpus is None:
        args.gpus = world or 1
        return None
    if world is not None and world != args.gpus:
        return f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}"
    return None


class Ctx:
    """Rank context shared by the timed runs."""

    def __init__(self, world, rank, local, dist, force_dist, backend):
        self.world, self.rank, self.local = world, rank, local
        self.dist, self.force_dist, self.backend = dist, force_dist, backend

    def barrier(self):
        import torch
        if self.dist is not None:
            self.dist.barrier()
        torch.cuda.synchronize()

    def max_sum(self, dt, filters):
        """(max over ranks of dt, sum over ranks of filters)."""
        if self.dist is None:
            return dt, filters
        import torch
        tt = torch.tensor([dt, float(filters)], dtype=torch.float64,
                          device=f"cuda:{self.local}" if self.backend == "nccl" else "cpu")
        self.dist.all_reduce(tt[0:1], op=self.dist.ReduceOp.MAX)
        self.dist.all_reduce(tt[1:2], op=self.dist.ReduceOp.SUM)
        return float(tt[0]), int(tt[1])


def proposal(meta, kind):
    """(h, sigma, description) of the MH random walk: the config's own (epipf.datasets.PROPOSALS) or fixed_theta."""
    if kind == "fixed_theta":
        from epipf.datasets import FIXED_THETA
        return FIXED_THETA["h"], FIXED_THETA["sigma"], FIXED_THETA["proposal"]
    return meta["h"], meta["sigma"], meta["proposal"]




def timed_chains(ctx, args, cfg, chains, steps, warmup, kind, pipelines=1, streams_env=4):
    """`chains` independent MH chains per rank of BASELINE config `cfg`: warmup, then `steps` timed MH iterations
    between barriers (+ the end-of-run RCCL all-gather of the draws), then one untimed iteration with the device
    counters on.  Returns a dict of what the bench line reports."""
    from epipf import _lib, datasets
    from epipf.distributed import gather_draws, shard
    from epipf.engine import Engine
    from epipf.pmcmc import ChainSampler, chain_key, run_pipelined
    Y, meta = datasets.benchmark_dataset(cfg)
    N, T = (args.particles if cfg == args.config and args.particles else meta["N"]), Y.shape[0]
    h, sigma, pdesc = proposal(meta, kind)
    gid = shard(chains * ctx.world, ctx.world, ctx.rank)              # global chain ids of this rank
    P = max(1, min(pipelines, chains))
    samplers = []
    for k in range(P):                                               # contiguous chain groups, one engine each
        ids = gid[k * chains // P:(k + 1) * chains // P]
        kw = {}
        if P > 1:
            eng_k = Engine(meta["model"], len(np.atleast_1d(meta["n_population"])), N, T, len(ids), device=ctx.local)
            eng_k.set_streams(max(1, streams_env // P))
            kw["engine"] = eng_k
        samplers.append(ChainSampler(Y, meta["model"], list(meta["theta"]), h, sigma=sigma,
                                     iters=warmup + steps + 2, observations=meta.get("observations", False),
                                     probs=meta["probs"], n_particles=N, n_population=meta["n_population"],
                                     mu=meta["mu"], rngs=[np.random.RandomState(args.seed + g) for g in ids],
                                     keys=[chain_key(args.seed, g) for g in ids], device=ctx.local, mh_ratio="log",
                                     **kw))
    engines = [s.eng for s in samplers]
    streams = P * max(1, streams_env // P) if P > 1 else min(streams_env, chains)   # concurrent step launches
    for s_ in samplers:
        s_.initialise()
    run_pipelined(samplers, warmup) if P > 1 else [samplers[0].step() for _ in range(warmup)]

    def stats_sum():
        tot = {}
        for e in engines:
            for k_, v in e.stats().items():
                tot[k_] = tot.get(k_, 0) + v
        return tot

    def accept_counts():
        return sum(a for s_ in samplers for a in s_.acceptances), sum(f for s_ in samplers for f in s_.filters_run)

    for e in engines:
        e.reset_stats()
        e.set_profiling(_lib.PROFILE_TIMING)     # HIP events only: the timed kernels are the production ones
    a0, f0 = accept_counts()
    ctx.barrier()
    t0 = time.perf_counter()
    if P > 1:
        filters = run_pipelined(samplers, steps)
    else:
        filters = sum(samplers[0].step() for _ in range(steps))
    # end of run: gather every rank's posterior draws over RCCL (xGMI), SURVEY.md §8e
    packed = np.concatenate([s_.packed_draws(upto=samplers[0].i) for s_ in samplers])   # == pack_draws(results())
    gathered = gather_draws(packed, ctx.local, force=ctx.force_dist)
    ctx.barrier()
    dt = time.perf_counter() - t0
    a1, f1 = accept_counts()
    st = stats_sum()
    # one extra, untimed MH iteration with device counters on: SSA events/s and SIMD lane use
    for e in engines:
        e.reset_stats()
        e.set_profiling(_lib.PROFILE_COUNTERS)
    run_pipelined(samplers, 1) if P > 1 else samplers[0].step()
    for e in engines:
        e.set_profiling(_lib.PROFILE_OFF)
    cst = stats_sum()
    dt_max, filters_all = ctx.max_sum(dt, filters)
    lanes = int(engines[0].stats()["last_lanes"]) or 1
    # the path every engine took on its last run: the roofline's launch arithmetic assumes one path for all of them
    paths = sorted({(int(e.stats().get("last_fused", 0)), int(e.stats()["last_lanes"]) or 1) for e in engines})
    fused = paths[0][0]
    if fused:                                      # one launch per filter batch, one stream per engine
        streams = P
    return dict(Y=Y, meta=meta, N=N, T=T, chains=chains, P=P, streams=streams, samplers=samplers, engines=engines,
                fused=fused, paths=paths,
                dt=dt_max, filters=filters, filters_all=filters_all, value=filters_all * N * T / dt_max, st=st, cst=cst,
                lanes=lanes, h=h, sigma=sigma, proposal=pdesc, gathered=gathered,
                acceptance_rate=(a1 - a0) / max(1, f1 - f0), steps=steps, warmup=warmup)


def n_comp(meta):
    return {"sir": 3, "seir": 4}.get(meta["model"], 3 * len(np.atleast_1d(meta["n_population"])))


def pmc_profile(cfg, chains, lanes):
    """The committed PMC pass of this (config, chains per GPU, lanes per particle) on the library timed here
    (profiles/pmc_*.json, written by scripts/parse_rocprof.py; matched on the library's build id -- a hash of every
    kernel source and flag, epipf_build_id -- so after any kernel change it reads as stale and the PMC fields are
    null).  Returns (profile, path) or ({}, None)."""
    from epipf import _lib
    bid = _lib.build_id()
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_*.json"))):
        try:
            p = json.load(open(path))
        except (OSError, ValueError):
            continue
        if (p.get("build_id") == bid and p.get("config", 2) == cfg and p.get("chains_per_gpu", 256) == chains
                and p.get("lanes", 1) == lanes):
            return p, os.path.relpath(path, REPO)
    return {}, None


def loop_ceiling(cfg):
    """The SSA event loop's measured ceiling for this config on the library timed here (profiles/loop_ceiling.json,
    scripts/loop_ceiling.sh: the library's own event loop with every lane busy, eight waves per SIMD; matched on build
    id like the PMC passes).  Returns (entry, path) or ({}, None)."""
    from epipf import _lib
    path = os.path.join(REPO, "profiles", "loop_ceiling.json")
    try:
        p = json.load(open(path))
    except (OSError, ValueError):
        return {}, None
    c = p.get("configs", {}).get(str(cfg)) or {}
    if p.get("build_id") != _lib.build_id() or "uniform" not in c:
        return {}, None
    e = dict(c["uniform"])
    e["lane_events_per_s_distinct"] = (c.get("distinct") or {}).get("lane_events_per_s")
    return e, os.path.relpath(path, REPO)


def roofline(run, value):
    """Roofline of the run's dominant kernel: pf_step_kernel (one lane per particle) or pf_step_group_kernel (W lanes
    per particle).  Both are bound by vector-instruction issue (the SSA event loop), not by HBM: the
    primary roofline is VALU issue, from the committed PMC pass's SQ_INSTS_VALU per particle-step x the live rate;
    the HBM figures the north star asks for are in `hbm` (algorithmic 8C + 40 B per particle-step over the launch
    duration)."""
    st, meta, N = run["st"], run["meta"], run["N"]
    # one GPU's roofline: this rank's share of the whole-job rate (`value` counts every rank's filters; N > 1 ranks)
    if run.get("filters_all"):
        value = value * run["filters"] / run["filters_all"]
    lanes = run["lanes"]
    steps = run["steps"]
    launches = max(1, st["step_kernel_launches"])
    avg_launch_s = st["step_kernel_ms"] / 1e3 / launches
    step_wall_s = st["step_ms"] / 1e3 / max(1, st["step_launches"])
    # particle-steps per kernel launch: one filter step of a chain group, or (the one-workgroup filter) every step of
    # an engine's chains
    units_per_launch = run["filters"] * N / steps / run["streams"] * (run["T"] if run.get("fused") else 1)
    bytes_per_unit = 8 * n_comp(meta) + 40                            # 8C+40 B per particle-step
    live_gbs = units_per_launch * bytes_per_unit / avg_launch_s / 1e9
    # chip level: algorithmic bytes of every particle-step of the timed region over its wall time
    chip_gbs = run["filters"] * N * run["T"] * bytes_per_unit / run["dt"] / 1e9
    pmc, pmc_path = pmc_profile(run["cfg"], run["chains"], lanes)
    traffic = traffic_raw = valu = rocprof_us = None
    if pmc:
        # MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts half the bytes of a coalesced read stream, so
        # `traffic` doubles the read side (FETCH x 2 + WRITE); the raw counter sum is `traffic_raw`
        per_unit = pmc.get("hbm_bytes_per_particle_step_read_doubled")
        traffic = per_unit * units_per_launch if per_unit else None
        raw_unit = pmc.get("hbm_bytes_per_particle_step")
        traffic_raw = raw_unit * units_per_launch if raw_unit else None
        rocprof_us = pmc.get("trace_avg_us")
        ins = pmc.get("pmc_avg_per_launch", {}).get("SQ_INSTS_VALU")
        units = pmc.get("particle_steps_per_launch")
        # timed-region profiles (scripts/profile.sh REGION=1) carry the VALU count per counted particle-step itself;
        # older ones: the launch average over the grid's particle-steps
        per_ps = pmc.get("valu_per_particle_step") or (ins / units if ins and units else None)
        if per_ps:
            # over the MH iterations' dispatches alone where the pass recorded it (PMC_TIMED_DISPATCHES)
            busy = pmc.get("valu_busy_frac_timed") or pmc.get("valu_busy_frac")
            valu = {"achieved": per_ps * value, "instr_per_particle_step": per_ps,
                    # the flat peak prices every wave64 instruction at 2 cycles (VALU_PEAK)
                    "flat_peak": VALU_PEAK, "flat_frac": per_ps * value / VALU_PEAK,
                    # AMD's VALUBusy (SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE) of the PMC pass: per-wave VALU cycles
                    # per SIMD-cycle, ~1.1 at the loop's ceiling (dual issue), and the pass serialises the chain
                    # groups' dispatches, so it reads low against the live run
                    "pmc_valu_busy_frac": busy,
                    "pmc_busy_over": "MH iterations' dispatches" if pmc.get("valu_busy_frac_timed") else "all dispatches"}
    ceil, ceil_path = loop_ceiling(run["cfg"])
    cst = run.get("cst") or {}
    ev_ps = cst["events"] / cst["particle_steps"] if cst.get("particle_steps") else None
    if valu and ceil:
        # the loop's own saturated issue rate (PMC pass of the ceiling run): achieved / ceiling near 1 = the SIMDs
        # issue VALU as fast as the loop can; the events fraction below is what that issue buys (lane use, phases)
        valu["ceiling"] = ceil["valu_instr_per_s"]
        valu["issue_frac"] = valu["achieved"] / ceil["valu_instr_per_s"]
    hbm_us = rocprof_us or avg_launch_s * 1e6
    hbm_gbs = units_per_launch * bytes_per_unit / (hbm_us / 1e6) / 1e9
    hbm = {"achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm_gbs / HBM_PEAK_GBS,
           "duration_source": f"rocprofv3 average kernel duration ({pmc_path})" if rocprof_us
           else "HIP events (launch to completion)",
           "frac_hip_event_span": live_gbs / HBM_PEAK_GBS, "chip_level_frac": chip_gbs / HBM_PEAK_GBS,
           "bytes_per_particle_step": bytes_per_unit, "traffic": traffic, "traffic_raw": traffic_raw}
    # frac: SSA events (the path's algorithmic unit, every particle's events) per second against the measured ceiling
    # of the same event loop on this chip -- every lane busy, no per-step phases, no launch tails, eight waves per SIMD
    # (scripts/loop_ceiling.hip).  Without a ceiling of this build: VALU issue against the flat 2-cycle peak.
    if ceil and ev_ps:
        prim = {"achieved": value * ev_ps, "peak": ceil["lane_events_per_s"], "unit": "lane-events/s",
                "peak_kind": f"measured SSA-loop ceiling, every lane busy ({ceil_path})",
                "frac": value * ev_ps / ceil["lane_events_per_s"],
                "events_per_particle_step": ev_ps,
                "ceiling_one_particle_per_lane": ceil.get("lane_events_per_s_distinct")}
    else:
        prim = {"achieved": valu["achieved"] if valu else None, "peak": VALU_PEAK, "unit": "wave64 VALU instr/s",
                "peak_kind": "flat (2 cycles per wave64 instr)",
                "frac": valu["achieved"] / VALU_PEAK if valu else None}
    out = {"bound": "valu", "kernel": kernel_name(run), **prim,
            "traffic": traffic, "valu_issue": valu, "hbm": hbm,
            "avg_launch_us": avg_launch_s * 1e6, "particle_steps_per_launch": units_per_launch,
            "concurrent_launches_per_step": run["streams"], "step_wall_us": step_wall_s * 1e6,
            # the same kernel's average dispatch duration in the committed rocprofv3 trace of this workload; the
            # HIP-event figure above also counts the time a launch waits for CUs held by concurrent chain-group launches
            "rocprof_avg_launch_us": rocprof_us,
            "pmc_profile": {"path": pmc_path, "build_id": pmc.get("build_id")}}
    paths = run.get("paths", [(run.get("fused", 0), lanes)])
    if len(paths) > 1:
        # engines on different paths (one-workgroup filter vs step launches, or different lanes): the summed launch
        # times over the summed launches mix two kernels, so no per-launch figure is physical
        out["valid"] = False
        out["invalid_reason"] = f"engines took different paths (fused, lanes): {paths}"
        for k in ("achieved", "frac", "traffic"):
            out[k] = None
    else:
        out["valid"] = True
    return out


def kernel_name(run):
    if run.get("fused"):
        return f"pf_filter_wg_kernel (one workgroup per chain, W={run['lanes']})"
    return "pf_step_kernel" if run["lanes"] == 1 else f"pf_step_group_kernel (W={run['lanes']})"


def run_summary(run):
    cst = run["cst"]
    ps = cst["particle_steps"]
    return {"value": run["value"], "unit": "particle-steps/s", "ms_per_step": run["dt"] * 1e3 / run["steps"],
            "steps": run["steps"], "warmup": run["warmup"], "chains_per_gpu": run["chains"],
            "particles": run["N"], "T_obs": run["T"], "lanes_per_particle": run["lanes"],
            "kernel": kernel_name(run),
            "h": run["h"], "proposal": run["proposal"], "acceptance_rate": run["acceptance_rate"],
            "events_per_particle_step": cst["events"] / ps if ps else None,
            "events_per_s": run["value"] * cst["events"] / ps if ps else None}


def prefetch_chain(args, Y, meta, N, T, local, slots, iters, h=1e-4, sigma=None, start=20):
    """One chain with speculative MH (epipf.prefetch): filters of future iterations share one batched launch sequence;
    only filters on the realised path count.  slots = "auto" lets the sampler size its rounds.  The
    timed window starts at MH iteration `start` (or later, once the auto width has measured every candidate): a
    round's yield depends on the accept / reject pattern of the chain segment it covers, so two widths are compared
    on the same segment (the auto leg first, then the fixed width from the auto leg's start)."""
    import torch
    from epipf.pmcmc import chain_key
    from epipf.prefetch import PrefetchSampler
    s2 = PrefetchSampler(Y, meta["model"], list(meta["theta"]), h, sigma=sigma, iters=start + iters + 1000,
                         probs=meta["probs"],
                         observations=meta.get("observations", False), n_particles=N,
                         n_population=meta["n_population"], mu=meta["mu"],
                         rngs=[np.random.RandomState(args.seed)], keys=[chain_key(args.seed, 0)], device=local,
                         mh_ratio="log", slots=slots)
    s2.initialise()
    while s2.i < start or not s2.tuned:              # slots="auto": warm up until every width has been measured
        s2.advance()
    torch.cuda.synchronize()
    i0, f0, r0, sp0, a0 = s2.i, s2.filters_run[0], s2.rounds, s2.speculative_filters, s2.acceptances[0]
    assert i0 + iters <= s2.iters, (i0, iters, s2.iters)   # the auto width's warm-up ends within the sampler's span
    t2 = time.perf_counter()
    while s2.i < i0 + iters:
        s2.advance()
    torch.cuda.synchronize()
    dt2 = time.perf_counter() - t2
    return {"value": (s2.filters_run[0] - f0) * N * T / dt2, "slots": slots, "slots_used": s2.slots,
            "start_iteration": i0, "iterations": s2.i - i0, "rounds": s2.rounds - r0,
            "iterations_per_round": (s2.i - i0) / max(1, s2.rounds - r0),
            "filters_evaluated": s2.speculative_filters - sp0,
            "acceptance_rate": (s2.acceptances[0] - a0) / max(1, s2.filters_run[0] - f0),
            "ms_per_iteration": dt2 * 1e3 / max(1, s2.i - i0)}


def config_runs(ctx, args):
    """The `configs` object: short timed runs of the other BASELINE workloads on every rank (one rank per GPU; the
    config-5 one-chain entry is BASELINE's 8-chain layout at 8 GPUs), at the config's own proposal and at
    fixed_theta where that differs."""
    from epipf.engine import release_engines
    names = [] if args.configs.strip().lower() in ("", "none") else [c.strip() for c in args.configs.split(",")]
    out = {}
    cpu_done = {}
    for name in names:
        if name not in CONFIG_RUNS:
            raise SystemExit(f"bench.py: unknown --configs entry {name!r}")
        cfg, chains, pipes = CONFIG_RUNS[name]
        release_engines()                                              # no idle contexts beside this entry's
        gc.collect()
        steps = args.configs_steps * (5 if chains == 1 else 1)        # one-chain MH iterations are short
        from epipf import datasets
        Yc, mc = datasets.benchmark_dataset(cfg)
        # config 1 (N x T = 5,000 per filter): one-workgroup filters (one per chain, 1,536 to a launch) and the host
        # draws in C, four chain groups on host threads so that each group's host work overlaps the others' filters
        # (run_pipelined; profiles/r5v_cfg1_chains.jsonl: 256 chains 2.0e9, 1024 5.3e9, 6144 in four groups
        # 1.4-1.6e10; more groups than the 4 hardware queues share queues and stall)
        pipelines = (args.pipelines or pipes) if chains > 1 and mc["N"] * Yc.shape[0] <= 20000 else 1
        if cfg == 1:
            steps *= 25                                                # 2-3 ms MH steps: time a few hundred ms
        entry = None
        # N <= 512 (config 1): the engine's first eight runs of a batch size time the one-workgroup filter against the
        # step launches (EPIPF_FUSED=auto, epipf_api.cpp): warm up past them
        warm = 10 if mc["N"] <= 512 else (1 if chains > 1 else 2)
        for kind in ("config", "fixed_theta"):
            run = timed_chains(ctx, args, cfg, chains, steps, warm, kind, pipelines=pipelines)
            run["cfg"] = cfg
            if entry is None:
                entry = run_summary(run)
                entry["workload"] = (f"BASELINE config {cfg}: {run['meta']['model'].upper()} PMCMC, N={run['N']}, "
                                     f"T={run['T']}, {chains} chain(s) per GPU")
                entry["pipelines"] = run["P"]
                entry["roofline"] = roofline(run, run["value"])
                if run["proposal"] == proposal(run["meta"], "fixed_theta")[2]:
                    entry["proposal_kind"] = "fixed_theta (the config has no reference proposal)"
                    break
                entry["proposal_kind"] = "config"
            else:
                entry["fixed_theta"] = run_summary(run)
            # release the leg's engines (their HIP streams) before the next one: idle contexts' streams still hold
            # hardware queues, and the next leg's concurrent engines could be placed on a shared one
            run["samplers"] = run["engines"] = None
            gc.collect()
        run["samplers"] = run["engines"] = None
        gc.collect()
        if chains == 1 and ctx.rank == 0 and ctx.world == 1:
            # at the config's proposal (config 5: h = 1, acceptance often 0 over a segment: each round then commits about
            # as many iterations as it has slots) and at the near-fixed theta (acceptance ~0.6: the speculation tree's
            # other extreme); the acceptance is reported beside each
            entry["prefetch_auto"] = prefetch_chain(args, run["Y"], run["meta"], run["N"], run["T"], ctx.local, "auto",
                                                    160, h=entry["h"], sigma=run["meta"]["sigma"])
            fh, fs, _ = proposal(run["meta"], "fixed_theta")
            if fh != entry["h"]:
                entry["prefetch_auto_fixed_theta"] = prefetch_chain(args, run["Y"], run["meta"], run["N"], run["T"],
                                                                    ctx.local, "auto", 160, h=fh, sigma=fs)
        if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline and args.configs_cpu_seconds > 0 \
                and name not in cpu_done:
            # the same CPU baseline as the headline's, per config, on a capped particle count
            cpu_done[name] = cpu_baseline(run["Y"], run["meta"], min(run["N"], 2048), args.configs_cpu_seconds, cfg)
        if name in cpu_done:
            entry["cpu_baseline"] = cpu_done[name]
            entry["speedup_vs_cpu_baseline"] = entry["value"] / cpu_done[name]["value"]
            rc = cpu_done[name].get("reference_calibrated")
            if rc:
                entry["speedup_vs_reference_1core_estimated"] = entry["value"] / rc["reference_1core_value"]
                entry["speedup_vs_reference_allcores_estimated"] = entry["value"] / rc["reference_allcores_value"]
        out[name] = entry
    return out


# The driver parses the JSON line out of an 8 KB stdout tail (BENCH_r05: a 21.7 KB line was not parsed).  The line
# carries the headline with its full roofline and CPU baseline and one compact row per `configs` entry; everything
# else goes to the detail file the line names.
LINE_LIMIT = 6000
# headline keys dropped, in this order, if the line still exceeds LINE_LIMIT (the detail file keeps them all)
OPTIONAL_KEYS = ("gathered_rhat", "rank_devices", "proposal", "data", "speedup_vs_reference_allcores_estimated",
                 "speedup_vs_reference_1core_estimated", "speedup_vs_cpu_single_core", "events_per_s",
                 "single_chain_value")


def compact_config(e):
    """One `configs` entry as a row of the printed line: rate, timing, layout, roofline fractions, CPU baseline."""
    r = e.get("roofline") or {}
    cb = e.get("cpu_baseline") or {}
    return {"value": e.get("value"), "ms_per_step": e.get("ms_per_step"), "steps": e.get("steps"),
            "chains_per_gpu": e.get("chains_per_gpu"), "lanes": e.get("lanes_per_particle"),
            "roofline_frac": r.get("frac"), "roofline_valid": r.get("valid", True),
            "hbm_frac": (r.get("hbm") or {}).get("frac"),
            "cpu_baseline": cb.get("value"), "cpu_cores": cb.get("cores"),
            "acceptance_rate": e.get("acceptance_rate")}


def compact_cpu_baseline(base):
    if not base:
        return base
    out = {k: base[k] for k in ("value", "unit", "cores", "kind", "sample") if k in base}
    if "single_core" in base:
        out["single_core_value"] = base["single_core"]["value"]
    rc = base.get("reference_calibrated")
    if rc:
        out["reference_estimate"] = {k: rc[k] for k in ("reference_1core_value", "reference_allcores_value",
                                                       "factor_port_over_reference_1core", "estimate") if k in rc}
    return out


def compact_line(full, detail_path):
    """The printed line: `full` without the bulky diagnostics, `configs` as compact rows, `detail` naming the file
    that holds `full`.  Never longer than LINE_LIMIT characters."""
    keep = ("metric", "value", "unit", "n_gpus", "ranks", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "events_per_s",
            "lanes_per_particle", "library_build_id", "single_chain_value", "speedup_vs_cpu_baseline",
            "speedup_vs_cpu_single_core", "speedup_vs_reference_1core_estimated",
            "speedup_vs_reference_allcores_estimated", "proposal", "gathered_draws_shape", "gathered_rhat",
            "rank_devices")
    line = {k: full[k] for k in keep if k in full}
    line["cpu_baseline"] = compact_cpu_baseline(full.get("cpu_baseline"))
    line["configs"] = {k: compact_config(v) for k, v in (full.get("configs") or {}).items()}
    line["detail"] = detail_path
    for k in OPTIONAL_KEYS:
        if len(json.dumps(line)) <= LINE_LIMIT:
            break
        line.pop(k, None)
    if len(json.dumps(line)) > LINE_LIMIT:           # last resort: the rows' secondary fields
        for row in line["configs"].values():
            for k in ("acceptance_rate", "cpu_cores", "lanes", "roofline_valid"):
                row.pop(k, None)
    return line


def write_detail(full, path):
    """Write the full result (every field, every `configs` entry in full) as JSON; returns the path written, or None
    when it cannot be written (the printed line still goes out)."""
    if path is None:
        path = os.path.join(REPO, "gpurun_out", f"bench_detail_n{full.get('n_gpus', 1)}.json")
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
    except OSError as e:
        print(f"bench.py: could not write the detail file {path}: {e}", file=sys.stderr)
        return None
    return os.path.relpath(path, REPO) if os.path.abspath(path).startswith(REPO) else path


def main():
    args = parse()
    msg = resolve_gpus(args, os.environ)
    if msg:
        sys.exit(msg)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("EPIPF_DIST_BACKEND", "nccl")   # nccl = RCCL over xGMI; gloo only for rehearsals
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    dist = None
    # EPIPF_BENCH_DIST=1: the distributed path (process group, max/sum reductions, RCCL all-gather) even at one rank,
    # so that a one-GPU box rehearses the RCCL code of the driver's N-GPU runs (scripts/rccl_bench_check.sh)
    force_dist = os.environ.get("EPIPF_BENCH_DIST") == "1"
    devices = [[platform.node(), local]]
    if world > 1 or force_dist:
        import torch
        import torch.distributed as dist
        ndev = torch.cuda.device_count()
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if backend == "nccl" and local_world > ndev:
            sys.exit(f"bench.py: {local_world} ranks on this node but {ndev} GPU(s); nccl (RCCL) needs one GPU per rank")
        local = local % max(ndev, 1)      # one GPU per rank on a full node; ranks share GPUs in gloo rehearsals
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
        devices = [None] * world
        dist.all_gather_object(devices, [platform.node(), local])
        if backend == "nccl":                                       # one distinct GPU per rank
            assert len({tuple(d) for d in devices}) == world, f"ranks share a GPU under nccl: {devices}"
    import torch

    from epipf import _lib
    from epipf.chains_io import gelman_rubin
    from epipf.distributed import unpack_draws

    ctx = Ctx(world, rank, local, dist, force_dist, backend)
    C = args.chains
    from epipf import datasets
    Y, meta0 = datasets.benchmark_dataset(args.config)
    N0, T0 = (args.particles or meta0["N"]), Y.shape[0]
    pipelines = args.pipelines or 1                  # > 1: chain groups' host work overlapping (run_pipelined)
    streams_env = max(1, min(int(os.environ.get("EPIPF_STREAMS", 4)), 8))
    run = timed_chains(ctx, args, args.config, C, args.steps, args.warmup, args.proposal, pipelines, streams_env)
    run["cfg"] = args.config
    meta, N, T, P, st, cst = run["meta"], run["N"], run["T"], run["P"], run["st"], run["cst"]
    value, dt = run["value"], run["dt"]
    lanes = run["lanes"]
    roof = roofline(run, value)
    # SSA events per second of job time: events per particle-step (counters iteration) x the measured rate
    events_per_s = value * cst["events"] / cst["particle_steps"] if cst["particle_steps"] else None
    lane_use = cst["lane_iterations"] / cst["wave_lane_slots"] if cst["wave_lane_slots"] else None
    gathered = run["gathered"]
    # Gelman-Rubin R-hat (helpers.py:15-43) of the gathered chains' timed draws: a bench run is tens of iterations
    # from a fixed start, far too short for a convergence diagnostic, so it is reported, not judged
    rhat = None
    th_g, _ = unpack_draws(gathered, len(run["samplers"][0].thetas[0, 0]))
    if th_g.shape[0] >= 2 and th_g.shape[1] >= 3:
        with np.errstate(divide="ignore", invalid="ignore"):
            rhat = [None if not np.isfinite(v) else float(v) for v in gelman_rubin(list(th_g))]

    single = prefetch = s1 = None
    if args.single_chain and rank == 0 and world == 1:
        from epipf.pmcmc import ChainSampler, chain_key
        s1 = ChainSampler(Y, meta["model"], list(meta["theta"]), run["h"], sigma=run["sigma"], iters=args.steps + 2,
                          probs=meta["probs"], observations=meta.get("observations", False),
                          n_particles=N, n_population=meta["n_population"], mu=meta["mu"],
                          rngs=[np.random.RandomState(args.seed)], keys=[chain_key(args.seed, 0)], device=local,
                          mh_ratio="log")
        s1.initialise()
        s1.step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        f1 = sum(s1.step() for _ in range(args.steps))
        torch.cuda.synchronize()
        single = f1 * N * T / (time.perf_counter() - t1)
        prefetch_auto = prefetch_chain(args, Y, meta, N, T, local, "auto", args.prefetch_iters, h=run["h"],
                                       sigma=run["sigma"])
        prefetch = prefetch_chain(args, Y, meta, N, T, local, args.prefetch, args.prefetch_iters, h=run["h"],
                                  sigma=run["sigma"], start=prefetch_auto["start_iteration"])

    run["samplers"] = run["engines"] = s1 = None                       # the headline's contexts, released
    configs = config_runs(ctx, args)

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(Y, meta, N, args.cpu_baseline_seconds, args.config)

    if rank == 0:
        # distinct GPUs, not ranks: (host, device) pairs over all ranks (gloo rehearsals put several ranks on one)
        n_gpus = len({tuple(d) for d in devices})
        line = {
            "metric": f"particle-steps/sec (N_particles x T_obs x MH-iters) on {MODEL_NAMES[meta['model']]} PMCMC",
            "value": value,
            "unit": "particle-steps/s",
            "n_gpus": n_gpus,
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic ({meta['describe']}); Philox-keyed filter draws",
            "config": {"workload": f"BASELINE config {args.config}: {meta['model'].upper()} PMCMC, N={N} particles, "
                                   f"pop={meta['n_population']}, {T} obs, {C} independent chains per GPU",
                       "particles": N, "T_obs": T, "chains_per_gpu": C, "population": meta["n_population"],
                       "pipelines": P,
                       "parallelism": f"chains sharded over {n_gpus} GPU(s) ({world} rank(s)), RCCL all-gather of "
                                      f"draws at end"},
            "proposal": {"h": run["h"], "sigma": run["sigma"], "kind": args.proposal, "source": run["proposal"],
                         "acceptance_rate": run["acceptance_rate"]},
            "roofline": roof,
            "events_per_s": events_per_s,
            "ssa_lane_utilisation": lane_use if lanes == 1 else None,
            "lanes_per_particle": lanes,
            "resample_fallbacks": st["resample_fallbacks"],
            # draws of the untimed counters iteration whose uniform lies within scipy's error envelope of a CDF
            # boundary: the only draws where the reference's own weights could pick another ancestor;
            # of that iteration's resampling draws (the test runs with the device counters only)
            "resample_ref_ambiguous": cst["resample_ref_ambiguous"],
            "resample_draws": cst["particle_steps"] * (T - 1) // T,
            "library_build_id": _lib.build_id(),
            "pmc_profile": {"build_id": roof["pmc_profile"]["build_id"], "path": roof["pmc_profile"]["path"],
                            "current": roof["pmc_profile"]["path"] is not None},
            "events_per_particle_step": cst["events"] / cst["particle_steps"] if cst["particle_steps"] else None,
            # particle-steps the certified f32 SSA path handed to the exact loop, and waves that waited on one
            "ssa_exact_particle_frac": cst["ssa_exact_lanes"] / cst["particle_steps"] if cst["particle_steps"] else None,
            "ssa_exact_wave_frac": cst["ssa_exact_waves"] * 64 / cst["particle_steps"] if cst["particle_steps"] else None,
            # every rank's posterior draws after the RCCL all-gather, and their Gelman-Rubin R-hat per parameter
            "gathered_draws_shape": list(gathered.shape),
            "gathered_rhat": rhat,
            "rank_devices": [f"{h}:{d}" for h, d in devices],
            "configs": configs,
            "cpu_baseline": base,
        }
        if single is not None:
            line["single_chain_value"] = single
        if prefetch is not None:
            line["single_chain_prefetch"] = prefetch
            line["single_chain_prefetch_auto"] = prefetch_auto
        if base is not None:
            line["speedup_vs_cpu_baseline"] = value / base["value"]
            line["speedup_vs_cpu_single_core"] = value / base["single_core"]["value"]
            if "reference_calibrated" in base:
                line["speedup_vs_reference_1core_estimated"] = value / base["reference_calibrated"]["reference_1core_value"]
                line["speedup_vs_reference_allcores_estimated"] = \
                    value / base["reference_calibrated"]["reference_allcores_value"]
        detail = write_detail(line, args.detail)
        print(json.dumps(compact_line(line, detail)), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
