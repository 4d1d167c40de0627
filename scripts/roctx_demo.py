"""A short PMCMC run on the debug library (libepipf_debug.so: roctx ranges per epipf_run and filter step), for a
rocprofv3 --marker-trace capture (scripts/roctx_trace.sh).  Config 2 data, 4 chains, N = 2000, 3 MH iterations."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("EPIPF_LIBRARY", os.path.join(REPO, "stochastic-epidemic-modelling_amd", "lib", "libepipf_debug.so"))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))

from epipf import _lib, datasets  # noqa: E402
from epipf.pmcmc import ChainSampler, chain_key  # noqa: E402

assert _lib.build_id().endswith("-debug"), _lib.build_id()
Y, meta = datasets.benchmark_dataset(2)
s = ChainSampler(Y, meta["model"], list(meta["theta"]), 1e-4, iters=4, probs=meta["probs"], n_particles=2000,
                 n_population=meta["n_population"], mu=meta["mu"], rngs=[np.random.RandomState(g) for g in range(4)],
                 keys=[chain_key(7, g) for g in range(4)], mh_ratio="log")
s.initialise()
for _ in range(3):
    s.step()
print("roctx demo done:", _lib.build_id())
