"""Wall-time breakdown of one lockstep MH iteration at the bench config (256 chains, config 2): host proposals,
the filter call (epipf_run: H2D params, init + T-1 step launches on 4 streams, D2H), on-device path sampling, host
accept/reject -- to locate the gap between a bare filter batch and an MH step."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
from epipf import _lib, datasets  # noqa: E402
from epipf import pmcmc as pm  # noqa: E402

Y, meta = datasets.benchmark_dataset(int(os.environ.get("CFG", 2)))
C = int(os.environ.get("CHAINS", 256))
s = pm.ChainSampler(Y, meta["model"], list(meta["theta"]), 1e-4, iters=int(os.environ.get("K", 6)) + 4, probs=meta["probs"],
                    observations=meta.get("observations", False), n_particles=meta["N"],
                    n_population=meta["n_population"], mu=meta["mu"],
                    rngs=[np.random.RandomState(2024 + g) for g in range(C)],
                    keys=[pm.chain_key(2024, g) for g in range(C)], mh_ratio="log")
tim = {"run": 0.0, "path": 0.0}
run0, path0 = s.eng.run, s._path_sample


def run_t(*args, **kw):
    t = time.perf_counter()
    r = run0(*args, **kw)
    tim["run"] += time.perf_counter() - t
    return r


def path_t(ok):
    t = time.perf_counter()
    r = path0(ok)
    tim["path"] += time.perf_counter() - t
    return r


s.eng.run, s._path_sample = run_t, path_t
s.initialise()
s.step()
s.eng.reset_stats()
s.eng.set_profiling(_lib.PROFILE_TIMING)
tim = {"run": 0.0, "path": 0.0}
K = int(os.environ.get("K", 6))
t0 = time.perf_counter()
for _ in range(K):
    s.step()
dt = (time.perf_counter() - t0) / K
st = s.eng.stats()
print(f"MH step {dt * 1e3:.2f} ms: epipf_run {tim['run'] / K * 1e3:.2f} ms (device init+steps "
      f"{(st['init_ms'] + st['step_ms']) / K:.2f} ms, init {st['init_ms'] / K:.2f}), path sample "
      f"{tim['path'] / K * 1e3:.2f} ms, host rest {(dt - (tim['run'] + tim['path']) / K) * 1e3:.2f} ms", flush=True)
