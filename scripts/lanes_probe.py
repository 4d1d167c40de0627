"""Per-step kernel time of one chain vs SSA lanes per particle, with the bench theta and with no events
(theta = 0: every particle-step ends at its first draw), BASELINE configs 2 and 5.  HIP-event step_ms / launches."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))


def main():
    from epipf import _lib, datasets
    from epipf.engine import Engine, model_id, theta_vector
    shapes = [s for s in (sys.argv[1:] or ["1:1", "4:1", "4:2", "8:1"])]
    for cfg in (2, 5):
        Y, meta = datasets.benchmark_dataset(cfg)
        mid = model_id(meta["model"])
        base = np.asarray(meta["theta"], dtype=np.float64)
        G = int(round(np.sqrt(base.size - 1))) if mid >= 2 else 1
        th = theta_vector(mid, (base[:G * G].reshape(G, G), base[-1]) if mid >= 2 else tuple(base))[0]
        eng = Engine(meta["model"], G, meta["N"], Y.shape[0], 1)
        eng.set_observations(Y)
        eng.set_population(meta["n_population"], meta["mu"])
        obs = bool(meta.get("observations", False))
        for spec in shapes:
            W, K = (int(v) for v in spec.split(":"))
            eng.set_lanes(W, K if W > 1 else 0)
            for label, theta in (("bench", th), ("no_events", np.zeros_like(th))):
                eng.set_profiling(_lib.PROFILE_COUNTERS)
                eng.run(theta[None], [meta["probs"]], [5], [1], observations=obs)
                ev = eng.stats()["events"]
                eng.set_profiling(_lib.PROFILE_TIMING)
                eng.reset_stats()
                for f in range(3):
                    eng.run(theta[None], [meta["probs"]], [5], [1], observations=obs)
                s = eng.stats()
                rec = dict(cfg=cfg, W=W, K=s["last_lane_events"], theta=label,
                           us_per_step=1e3 * s["step_ms"] / max(1, s["step_launches"]),
                           events_per_particle_step=ev / (meta["N"] * (Y.shape[0] - 1)))
                print(json.dumps(rec), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
