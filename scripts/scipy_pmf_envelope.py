"""How far is scipy.stats.binom.pmf (the reference's weight, pmcmc.py:179; scipy 1.15 -> Boost ibeta_derivative) from
the true binomial pmf, as a function of n?  DESIGN.md §4: the envelope E(n) the device's reference-ambiguity count
(epipf_stats.resample_ref_ambiguous) assumes for scipy's error.  Also measures the oracle's compensated restatement
(oracle/epipf_oracle.c:binom_logpmf, the device's operations) against the same truth.

Truth: mpmath at 200 bits of C(n, k) p^k (1-p)^(n-k) for the double p.  Samples: n log-uniform in [1, 2e5], p = 0.1
(every BASELINE config) or uniform in [0.001, 0.999], k from the bulk (+-4 sd), the tails (+-4..40 sd) and uniform
in [0, n].  Only pmf values >= 1e-300 count (smaller ones underflow alike).  Build container only (scipy, mpmath);
writes profiles/r3_scipy_pmf_envelope.json.
Usage: python scripts/scipy_pmf_envelope.py [samples]"""
import json
import os
import sys
import time

import mpmath
import numpy as np
from scipy.stats import binom

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402

mpmath.mp.prec = 200


def envelope(n):
    """E(n): the bound bench and engine use (keep in sync with epipf_api.cpp: ref_pmf_envelope)."""
    return 4e-12 + 1e-16 * n


def main(M=120000):
    rs = np.random.RandomState(11)
    n = np.floor(np.exp(rs.uniform(0, np.log(2e5), M))).astype(np.int64)
    p = np.where(rs.rand(M) < 0.5, 0.1, rs.uniform(0.001, 0.999, M))
    sd = np.sqrt(n * p * (1 - p))
    kind = rs.randint(0, 3, M)
    off = np.where(kind == 0, rs.randn(M) * 4, np.sign(rs.randn(M)) * rs.uniform(4, 40, M))
    k = np.where(kind == 2, np.floor(rs.rand(M) * (n + 1)), np.round(n * p + off * sd))
    k = np.clip(k, 0, n).astype(np.int64)
    sc = binom.pmf(k, n, p)
    ours = oracle.binom_pmf(k, n, p)
    edges = [1, 10, 100, 1000, 3000, 10000, 30000, 100000, 200001]
    stats = {}
    worst = []
    t0 = time.time()
    for i in range(M):
        N, K = int(n[i]), int(k[i])
        P = mpmath.mpf(float(p[i]))
        tru = mpmath.binomial(N, K) * P ** K * (1 - P) ** (N - K)
        if tru < mpmath.mpf("1e-300"):
            continue
        es = abs(float(mpmath.mpf(float(sc[i])) / tru - 1))
        eo = abs(float(mpmath.mpf(float(ours[i])) / tru - 1))
        b = int(np.searchsorted(edges, N, side="right") - 1)
        s = stats.setdefault(b, {"n_lo": edges[b], "n_hi": edges[b + 1], "count": 0, "scipy_max": 0.0,
                                 "scipy_sum": 0.0, "ours_max": 0.0, "scipy_over_envelope_max": 0.0})
        s["count"] += 1
        s["scipy_max"] = max(s["scipy_max"], es)
        s["scipy_sum"] += es
        s["ours_max"] = max(s["ours_max"], eo)
        s["scipy_over_envelope_max"] = max(s["scipy_over_envelope_max"], es / envelope(N))
        if es > 0.5 * envelope(N):
            worst.append((es / envelope(N), N, K, float(p[i]), es))
    rows = []
    for b in sorted(stats):
        s = stats[b]
        s["scipy_mean"] = s.pop("scipy_sum") / s["count"]
        rows.append(s)
        print(f"n in [{s['n_lo']:6d},{s['n_hi']:6d}) {s['count']:6d} cases: scipy max {s['scipy_max']:.3g} "
              f"mean {s['scipy_mean']:.3g}  max/E(n) {s['scipy_over_envelope_max']:.3f}   ours max {s['ours_max']:.3g}")
    worst.sort(reverse=True)
    out = {"samples": M, "seconds": time.time() - t0, "envelope": "E(n) = 4e-12 + 1e-16 n", "bins": rows,
           "max_scipy_over_envelope": max(r["scipy_over_envelope_max"] for r in rows),
           "max_ours_rel_err": max(r["ours_max"] for r in rows),
           "worst_cases": [dict(ratio=w[0], n=w[1], k=w[2], p=w[3], rel_err=w[4]) for w in worst[:20]]}
    print(json.dumps({k: v for k, v in out.items() if k != "bins"}))
    with open(os.path.join(REPO, "profiles", "r3_scipy_pmf_envelope.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 120000)
