"""would ordering a chain's particles by predicted step work raise SIMD lane use?

For BASELINE config 2 (oracle filter, keyed stream) take every step's particle-steps with their real event counts
(oracle full-path SSA on the filter's own draws: particle j at step p draws counter (k, j, p, f)), and compute the
lane utilisation of 64-lane waves (loop iterations = events + 1 for the overshooting draw; a wave runs as long as
its longest lane) for three orders of the N particles: the filter's (lane j = particle j, random parents), sorted by
the parent state's total rate (beta S I / N + gamma I: the predicted events of the step), and sorted by the actual
event count (the ceiling of any ordering).  Writes profiles/r2_lane_use_model.json."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "stochastic-epidemic-modelling_amd")]
import oracle  # noqa: E402
from epipf import datasets  # noqa: E402


def lane_use(iters, order):
    it = iters[order]
    n = (len(it) // 64) * 64
    w = it[:n].reshape(-1, 64)
    return float(w.sum() / (64.0 * w.max(axis=1).sum()))


def main():
    Y, meta = datasets.benchmark_dataset(2)
    N = meta["N"]
    beta, gamma = meta["theta"]
    key, f = 4242, 0
    o = oracle.particle_filter(Y, "sir", meta["theta"], False, 0.1, N, meta["n_population"], meta["mu"], key=key,
                               filter_index=f)
    hid, anc = o["hidden"], o["ancestry"]
    tot = {"filter_order": [0.0, 0.0], "sorted_by_rate": [0.0, 0.0], "sorted_by_events": [0.0, 0.0]}
    per_step = []
    for p in range(1, Y.shape[0], 3):
        parents = hid[p - 1][anc[p]]
        _, _, nev, fin = oracle.simulate_path("sir", parents, (beta, gamma), 1.0, key=key, filter_index=f, step=p, cap=0)
        assert np.array_equal(fin, hid[p])
        iters = nev.astype(np.float64) + (parents[:, 1] > 0)          # + the overshooting draw (if any event loop ran)
        S, I = parents[:, 0].astype(float), parents[:, 1].astype(float)
        rate = beta * S * I / N + gamma * I
        orders = {"filter_order": np.arange(N), "sorted_by_rate": np.argsort(-rate, kind="stable"),
                  "sorted_by_events": np.argsort(-iters, kind="stable")}
        row = {"p": p, "mean_events": float(nev.mean())}
        for k, od in orders.items():
            u = lane_use(iters, od)
            row[k] = u
            it = iters[od][: (N // 64) * 64].reshape(-1, 64)
            tot[k][0] += it.sum()
            tot[k][1] += 64.0 * it.max(axis=1).sum()
        per_step.append(row)
    out = {k: v[0] / v[1] for k, v in tot.items()}
    out["steps_sampled"] = len(per_step)
    out["per_step"] = per_step[::6]
    print(json.dumps({k: out[k] for k in tot}))
    with open(os.path.join(REPO, "profiles", "r2_lane_use_model.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
