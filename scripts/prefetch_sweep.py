"""Single-chain speculative MH (epipf.prefetch) on one GPU: particle-steps/s of the realised chain against the
number of filter slots per round, BASELINE config CFG (default 2: N=10^4, T=200) at proposal scale H (default 1e-4; the
config's own h with H=config).  slots=0 is the one-filter-per-iteration loop, "auto" the adaptive width (warmed up until
every width was measured).  One JSON line per slot count."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))

from epipf import datasets  # noqa: E402
from epipf.pmcmc import ChainSampler, chain_key  # noqa: E402
from epipf.prefetch import PrefetchSampler  # noqa: E402


def main():
    cfg = int(os.environ.get("CFG", 2))
    iters = int(os.environ.get("ITERS", 60))
    Y, meta = datasets.benchmark_dataset(cfg)
    hs = os.environ.get("H", "1e-4")
    h = meta["h"] if hs == "config" else float(hs)
    sigma = meta["sigma"] if hs == "config" else None
    N, T = meta["N"], Y.shape[0]
    for slots in [x if x == "auto" else int(x) for x in os.environ.get("SLOTS", "0 8 16 24 32 48 64 96").split()]:
        kw = dict(iters=iters + 200, sigma=sigma, probs=meta["probs"], observations=meta.get("observations", False), n_particles=N,
                  n_population=meta["n_population"], mu=meta["mu"], rngs=[np.random.RandomState(2024)],
                  keys=[chain_key(2024, 0)], mh_ratio="log")
        if slots:
            s = PrefetchSampler(Y, meta["model"], list(meta["theta"]), h, **kw, slots=slots)
            adv = s.advance
        else:
            s = ChainSampler(Y, meta["model"], list(meta["theta"]), h, **kw)
            adv = s.step
        s.initialise()
        while s.i < 20 or not getattr(s, "tuned", True):
            adv()
        i0, f0, r0 = s.i, s.filters_run[0], getattr(s, "rounds", 0)
        t0 = time.perf_counter()
        while s.i < i0 + iters:
            adv()
        dt = time.perf_counter() - t0
        rounds = getattr(s, "rounds", s.i) - r0 if slots else s.i - i0
        print(json.dumps({"config": cfg, "slots": slots, "slots_used": getattr(s, "slots", 0), "h": h, "value": (s.filters_run[0] - f0) * N * T / dt,
                          "ms_per_iteration": dt * 1e3 / (s.i - i0), "iterations": s.i - i0, "rounds": rounds,
                          "iterations_per_round": (s.i - i0) / max(1, rounds),
                          "acceptance": (s.acceptances[0] - 1) / max(1, s.filters_run[0])}), flush=True)


if __name__ == "__main__":
    main()
