"""Per-step overhead of pf_step_kernel: the same config-2 batch (256 chains, N = 10^4, T = 200) with the
bench's theta and with rates that give one SSA loop iteration per particle-step (beta = 0, gamma = 1e-12), so the
second time is the resample / gather / weight / scan work alone."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
from epipf import datasets  # noqa: E402
from epipf.engine import Engine  # noqa: E402

Y, meta = datasets.benchmark_dataset(2)
N, T, C = meta["N"], Y.shape[0], int(os.environ.get("CHAINS", 256))
eng = Engine("sir", 1, N, T, C, device=0)
eng.set_observations(Y)
eng.set_population(meta["n_population"], meta["mu"])
Yc = np.tile(np.array([998.0, 2.0, 0.0]), (T, 1))       # observations the frozen initial states can explain
cases = (("bench theta", meta["theta"]), ("no events", (0.0, 1e-12)), ("bench theta", meta["theta"]))
only = os.environ.get("CASE")                                  # "bench" / "noev": one case (PMC passes)
if only:
    cases = [c for c in cases if (c[1][0] == 0.0) == (only == "noev")][:1]
for name, th in cases:
    eng.set_observations(Yc if th[0] == 0.0 else Y)
    thetas = np.tile(np.asarray(th, dtype=np.float64), (C, 1))
    eng.run(thetas, meta["probs"], np.arange(C) + 7, 0)
    ts = []
    for r in range(3):
        t0 = time.perf_counter()
        lz, st = eng.run(thetas, meta["probs"], np.arange(C) + 7, r + 1)
        ts.append(time.perf_counter() - t0)
    dt = min(ts)
    print(f"{name:12s} theta={th}: {dt * 1e3:8.2f} ms per batch, {dt / (T - 1) * 1e6:8.1f} us per step, "
          f"{C * N * T / dt:.3e} particle-steps/s, ok chains {int((st == 0).sum())}/{C}", flush=True)
eng.close()
