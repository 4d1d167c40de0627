"""Replayed particle-steps of the lane-group kernel (certified f32 clock) vs the one-lane kernel, one chain."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))


def main():
    from epipf import _lib, datasets
    from epipf.engine import Engine, model_id, theta_vector
    for cfg in (2, 5):
        Y, meta = datasets.benchmark_dataset(cfg)
        mid = model_id(meta["model"])
        base = np.asarray(meta["theta"], dtype=np.float64)
        G = int(round(np.sqrt(base.size - 1))) if mid >= 2 else 1
        th = theta_vector(mid, (base[:G * G].reshape(G, G), base[-1]) if mid >= 2 else tuple(base))[0]
        eng = Engine(meta["model"], G, meta["N"], Y.shape[0], 1)
        eng.set_observations(Y)
        eng.set_population(meta["n_population"], meta["mu"])
        for W in (1, 4, 8):
            eng.set_lanes(W)
            eng.set_profiling(_lib.PROFILE_COUNTERS)
            eng.reset_stats()
            eng.run(th[None], [meta["probs"]], [5], [1], observations=bool(meta.get("observations", False)))
            s = eng.stats()
            ps = meta["N"] * (Y.shape[0] - 1)
            print(json.dumps(dict(cfg=cfg, W=W, events_per_ps=s["events"] / ps, replayed_particle_steps=s["ssa_exact_lanes"],
                                  replay_frac=s["ssa_exact_lanes"] / ps, waves_with_replay=s["ssa_exact_waves"],
                                  step_ms=s["step_ms"])), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
