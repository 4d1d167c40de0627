"""BASELINE config 1 (N = 100, T = 50) MH throughput by chains per GPU and host pipelines (ChainSamplers with private
engines on host threads, epipf.pmcmc.run_pipelined), at the config's proposal and at the near-fixed theta.  One JSON
line per case: particle-steps/s, ms per MH iteration, the path each engine settled on (1 = one-workgroup filter).
  python scripts/cfg1_chains_probe.py [--chains 1024,2048] [--pipelines 1,2] [--steps 40]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
from epipf import datasets  # noqa: E402
from epipf.engine import Engine  # noqa: E402
from epipf.pmcmc import ChainSampler, chain_key, run_pipelined  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", type=int, default=1)
ap.add_argument("--chains", default="1024,2048")
ap.add_argument("--pipelines", default="1,2")
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--warmup", type=int, default=10)
args = ap.parse_args()

Y, meta = datasets.benchmark_dataset(args.cfg)
N, T = meta["N"], Y.shape[0]
for C in [int(x) for x in args.chains.split(",")]:
    for P in [int(x) for x in args.pipelines.split(",")]:
        for kind, (h, sigma) in (("config", (meta["h"], meta["sigma"])), ("fixed", (1e-4, None))):
            samplers = []
            for k in range(P):
                ids = range(k * C // P, (k + 1) * C // P)
                kw = {}
                if P > 1:
                    kw["engine"] = Engine(meta["model"], 1, N, T, len(ids))
                samplers.append(ChainSampler(Y, meta["model"], list(meta["theta"]), h, sigma=sigma,
                                             iters=args.warmup + args.steps + 2, probs=meta["probs"],
                                             n_particles=N, n_population=meta["n_population"], mu=meta["mu"],
                                             rngs=[np.random.RandomState(2024 + g) for g in ids],
                                             keys=[chain_key(2024, g) for g in ids], mh_ratio="log", **kw))
            for s in samplers:
                s.initialise()
            run_pipelined(samplers, args.warmup) if P > 1 else [samplers[0].step() for _ in range(args.warmup)]
            t0 = time.perf_counter()
            if P > 1:
                f = run_pipelined(samplers, args.steps)
            else:
                f = sum(samplers[0].step() for _ in range(args.steps))
            dt = time.perf_counter() - t0
            print(json.dumps(dict(chains=C, pipelines=P, proposal=kind,
                                  value=f * N * T / dt, ms_per_iter=dt / args.steps * 1e3,
                                  fused=[int(s.eng.stats().get("last_fused", 0)) for s in samplers])), flush=True)
