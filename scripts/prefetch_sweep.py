"""Single-chain speculative MH (epipf.prefetch) on one GPU: particle-steps/s of the realised chain against the
number of filter slots per round, BASELINE config 2 (N=10^4, T=200).  slots=0 is the one-filter-per-iteration
loop.  One JSON line per slot count."""
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
    h = float(os.environ.get("H", 1e-4))
    Y, meta = datasets.benchmark_dataset(cfg)
    N, T = meta["N"], Y.shape[0]
    for slots in [int(x) for x in os.environ.get("SLOTS", "0 8 16 24 32 48 64 96").split()]:
        kw = dict(iters=iters + 25, probs=meta["probs"], observations=meta.get("observations", False), n_particles=N,
                  n_population=meta["n_population"], mu=meta["mu"], rngs=[np.random.RandomState(2024)],
                  keys=[chain_key(2024, 0)], mh_ratio="log")
        if slots:
            s = PrefetchSampler(Y, meta["model"], list(meta["theta"]), h, **kw, slots=slots)
            adv = s.advance
        else:
            s = ChainSampler(Y, meta["model"], list(meta["theta"]), h, **kw)
            adv = s.step
        s.initialise()
        while s.i < 20:
            adv()
        i0, f0, r0 = s.i, s.filters_run[0], getattr(s, "rounds", 0)
        t0 = time.perf_counter()
        while s.i < i0 + iters:
            adv()
        dt = time.perf_counter() - t0
        rounds = getattr(s, "rounds", s.i) - r0 if slots else s.i - i0
        print(json.dumps({"config": cfg, "slots": slots, "h": h, "value": (s.filters_run[0] - f0) * N * T / dt,
                          "ms_per_iteration": dt * 1e3 / (s.i - i0), "iterations": s.i - i0, "rounds": rounds,
                          "iterations_per_round": (s.i - i0) / max(1, rounds),
                          "acceptance": (s.acceptances[0] - 1) / max(1, s.filters_run[0])}), flush=True)


if __name__ == "__main__":
    main()
