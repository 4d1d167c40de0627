"""Where the one-workgroup filter first departs from the oracle (diagnostic): first differing step, ancestors vs states."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "stochastic-epidemic-modelling_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle  # noqa: E402
from epipf.engine import Engine  # noqa: E402

g = np.load(os.path.join(REPO, "tests", "golden", "datasets.npz"))
Y = g["sir_binom"][:30]
for N in (65, 100, 128):
    eng = Engine("sir", 1, N, Y.shape[0], 1)
    eng.set_observations(Y)
    eng.set_population(4820, 20)
    lz, st = eng.run(np.array([[2.0, 1.0]]), [0.1], [71], [3])
    hid, anc = eng.history(1)
    s = eng.stats()
    eng.close()
    o = oracle.particle_filter(Y, "sir", (2.0, 1.0), False, 0.1, N, 4820, 20, key=71, filter_index=3)
    bad_h = [p for p in range(Y.shape[0]) if (hid[0, p] != o["hidden"][p]).any()]
    bad_a = [p for p in range(Y.shape[0]) if (anc[0, p] != o["ancestry"][p]).any()]
    print(f"N={N} lanes={s['last_lanes']} fused={s['last_fused']} st={st[0]} first bad hidden step "
          f"{bad_h[:1]} first bad ancestry step {bad_a[:1]}", flush=True)
    if bad_h:
        p = bad_h[0]
        rows = np.flatnonzero((hid[0, p] != o["hidden"][p]).any(axis=1))
        print("  step", p, "bad particles", rows[:20].tolist(), "anc dev", anc[0, p, rows[:8]].tolist(), "anc ora",
              o["ancestry"][p, rows[:8]].tolist())
        print("  dev", hid[0, p, rows[:4]].tolist(), "ora", o["hidden"][p, rows[:4]].tolist())
        print("  lz dev", lz[0, :p + 2].round(6).tolist())
        print("  lz ora", o["log_zetas"][:p + 2].round(6).tolist())
