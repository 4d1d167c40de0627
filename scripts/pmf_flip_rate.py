"""How often would an ancestor differ if the filter's weights were scipy's binom.pmf (Boost, the reference's) instead
of the lgamma restatement the device and the oracle evaluate (pmcmc.py:178-181)?  DESIGN.md §4 bound.

Runs oracle filters of BASELINE config 2 (N = 10^4, T = 200, keyed stream), recomputes every step's weights both ways
from the filter's own states, resamples both with the step's keyed uniforms (numpy legacy choice: cumsum / normalise /
searchsorted right, pmcmc.py:187-190) and counts ancestors that differ.  Also the weights' relative difference.
Build container only (scipy); writes profiles/r2_pmf_flip_rate.json."""
import json
import os
import sys
import time

import numpy as np
from scipy.stats import binom

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "stochastic-epidemic-modelling_amd")]
import oracle  # noqa: E402
import philox as ph  # noqa: E402
from epipf import datasets  # noqa: E402


def choice(w, u):
    p = w / sum(w.tolist())                     # builtin sum, pmcmc.py:185
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return cdf.searchsorted(u, side="right")


def main(filters=3):
    Y, meta = datasets.benchmark_dataset(2)
    N, T = meta["N"], Y.shape[0]
    pmf_c = np.vectorize(lambda k, n: oracle.lib().oracle_binom_pmf(float(k), float(n), 0.1))
    draws = flips = 0
    maxrel = 0.0
    nrel = 0
    exact_rel = 0
    t0 = time.time()
    for f in range(filters):
        key = 5000 + f
        o = oracle.particle_filter(Y, "sir", meta["theta"], False, 0.1, N, meta["n_population"], meta["mu"], key=key,
                                   filter_index=f)
        hid, anc = o["hidden"], o["ancestry"]
        for p in range(1, T):
            x = hid[p - 1].astype(np.float64)
            y = Y[p - 1]
            ours = np.min(np.stack([pmf_c(y[k], x[:, k]) for k in range(3)]), axis=0)
            ref = np.min(np.stack([binom.pmf(y[k], x[:, k], 0.1) for k in range(3)]), axis=0)
            ok = ref > 0
            rel = np.abs(ours[ok] / ref[ok] - 1.0)
            maxrel = max(maxrel, float(rel.max()) if rel.size else 0.0)
            nrel += int(rel.size)
            exact_rel += int(np.count_nonzero(rel == 0))
            u = ph.resample_uniforms(key, f, p, N)
            a_ours, a_ref = choice(ours, u), choice(ref, u)
            assert np.array_equal(a_ours, anc[p]), "restated weights must reproduce the oracle's ancestors"
            flips += int(np.count_nonzero(a_ours != a_ref))
            draws += N
    out = dict(config=2, filters=filters, draws=draws, ancestor_flips=flips, flip_rate=flips / draws,
               weight_max_rel_diff=maxrel, weights_compared=nrel, weights_bit_equal_frac=exact_rel / nrel,
               seconds=time.time() - t0)
    print(json.dumps(out))
    with open(os.path.join(REPO, "profiles", "r2_pmf_flip_rate.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
