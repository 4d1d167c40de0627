"""One chain, config 2, sequential MH (one filter per iteration): for a rocprofv3 kernel trace of the latency-bound
path (gaps between the 199 dependent step launches of a filter)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
from epipf import datasets  # noqa: E402
from epipf.pmcmc import ChainSampler, chain_key  # noqa: E402

Y, meta = datasets.benchmark_dataset(2)
s = ChainSampler(Y, "sir", list(meta["theta"]), 1e-4, iters=12, probs=0.1, n_particles=meta["N"],
                 n_population=meta["n_population"], mu=meta["mu"], rngs=[np.random.RandomState(5)],
                 keys=[chain_key(5, 0)], mh_ratio="log")
s.initialise()
for _ in range(10):
    s.step()
print("done", flush=True)
