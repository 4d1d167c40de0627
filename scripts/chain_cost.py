"""Round 4 diagnostic: how unequal are the chains of one config-5 MH iteration at h = 1?  Draws 256 proposals
theta0 + N(0, I) (the config's h = 1, sigma = I random walk from the true theta), keeps the live ones (no negative
component: pmcmc.py:333-337 runs no filter otherwise), and runs each live proposal as its own one-lane filter with the
device counters on: events, status, the step it died at, and its wall time.  Then one batched run of all live chains
(the bench's layout) for the batched wall time.  Prints the distribution."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))
from epipf import _lib, datasets  # noqa: E402
from epipf.engine import Engine, model_id, theta_vector  # noqa: E402

cfg = int(os.environ.get("CFG", "5"))
Y, meta = datasets.benchmark_dataset(cfg)
G = len(np.atleast_1d(meta["n_population"])) if meta["model"].startswith("sir_sub") else 1
N, T = meta["N"], Y.shape[0]
rng = np.random.RandomState(7)
th0 = np.asarray(meta["theta"], dtype=np.float64)
h = float(os.environ.get("H", meta.get("h") or 1.0))
props = th0 + np.sqrt(h) * rng.standard_normal((256, th0.size))
live = props[(props >= 0).all(axis=1)]
print(f"config {cfg}: {len(live)} of 256 proposals live (h = {h})", flush=True)

def tv(p):
    return theta_vector(model_id(meta["model"]), (p[:G * G].reshape(G, G), p[-1]) if G > 1 else tuple(p))[0]

eng = Engine(meta["model"], G, N, T, len(live))
eng.set_observations(Y)
eng.set_population(meta["n_population"], meta["mu"])
eng.set_lanes(1)
rows = []
for i, p in enumerate(live):
    eng.reset_stats()
    eng.set_profiling(_lib.PROFILE_COUNTERS)
    lz, st = eng.run(tv(p)[None, :], [meta["probs"]], [i + 1], [1])
    ev = eng.stats()["events"]
    eng.set_profiling(_lib.PROFILE_OFF)
    t0 = time.perf_counter()
    eng.run(tv(p)[None, :], [meta["probs"]], [i + 1], [2])
    dt = time.perf_counter() - t0
    dead = int(np.argmax(~np.isfinite(lz[0]))) if not np.isfinite(lz[0]).all() else T
    rows.append(dict(theta=[round(x, 3) for x in p], status=int(st[0]), steps_run=dead, events=int(ev),
                     ms=dt * 1e3))
ev = np.array([r["events"] for r in rows], dtype=float)
ms = np.array([r["ms"] for r in rows])
ok = np.array([r["status"] == 0 for r in rows])
print(f"degenerate: {(~ok).sum()} of {len(rows)}; steps run by degenerate ones: "
      f"{sorted(r['steps_run'] for r in rows if r['status'])}")
q = np.percentile(ev / (N * T), [0, 10, 50, 90, 99, 100])
print("events per particle-step (counted N*T): min/p10/p50/p90/p99/max", np.round(q, 1), "mean", round(ev.mean() / (N * T), 1))
top = np.sort(ev)[::-1]
print("share of all events in the top 1 / 5 / 10 / 25% of chains:",
      [round(top[:max(1, int(len(top) * f))].sum() / top.sum(), 3) for f in (0.01, 0.05, 0.1, 0.25)])
print("one-chain wall ms: p50", round(np.median(ms), 2), "max", round(ms.max(), 2), "sum", round(ms.sum(), 1))
thetas = np.stack([tv(p) for p in live])
for w in (1, 0):
    eng.set_lanes(w)
    eng.run(thetas, [meta["probs"]] * len(live), list(range(1, len(live) + 1)), [3] * len(live))
    t0 = time.perf_counter()
    eng.run(thetas, [meta["probs"]] * len(live), list(range(1, len(live) + 1)), [4] * len(live))
    dt = time.perf_counter() - t0
    print(f"batched run of the {len(live)} live chains, lanes {w or 'auto'}: {dt * 1e3:.2f} ms, "
          f"{len(live) * N * T / dt:.3e} particle-steps/s")
with open(os.path.join(REPO, "gpurun_out", f"chain_cost_cfg{cfg}.jsonl"), "w") as f:
    for r in rows:
        f.write(json.dumps(r) + "\n")
