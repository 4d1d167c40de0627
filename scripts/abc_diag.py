"""ABC kernel diagnostics: trial order vs length-ordered lanes on the same trials (device counters + timing)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "stochastic-epidemic-modelling_amd"))


def main():
    from epipf import _lib
    from epipf.engine import get_engine
    Y = np.load(os.path.join(REPO, "tests", "golden", "datasets.npz"))["sir_noisy"]
    pr = {"beta": [0.0, 5.0], "gamma": [0.0, 5.0]}
    eng = get_engine("sir", 1, 1, 1, 1)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    ref = None
    for order in ("0", "1"):
        os.environ["EPIPF_ABC_ORDER"] = order
        for level in (_lib.PROFILE_TIMING, _lib.PROFILE_COUNTERS):
            eng.set_profiling(level)
            eng.abc_trials(Y, pr, 3, 0, 0, n, rows=False)   # warm
            eng.reset_stats()
            th, _, dist = eng.abc_trials(Y, pr, 3, 0, 0, n, rows=False)
            s = eng.stats()
            if ref is None:
                ref = dist
            assert np.array_equal(dist, ref)
            print(f"order={order} level={level} ms={s['abc_ms']:.2f} trials/s={n / s['abc_ms'] * 1e3:.4g} "
                  f"events={s['events']} li={s['lane_iterations']} slots={s['wave_lane_slots']} "
                  f"use={s['lane_iterations'] / max(s['wave_lane_slots'], 1):.3f}", flush=True)
    eng.set_profiling(_lib.PROFILE_OFF)


if __name__ == "__main__":
    main()
