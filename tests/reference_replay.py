"""Replays the reference's own resampling step on the device's particle states (test helper).

For every step p of a filter the device ran, recompute the weights exactly as /root/reference/pmcmc.py:177-181 does --
scipy.stats.binom.pmf / norm.pdf of the observed row against the states of step p-1 (group sums for SIR_SUBGROUPS2,
:172-175), min over the columns -- normalise with the builtin sum (:185) and draw numpy legacy choice (:187-190:
cumsum, divide by the last entry, searchsorted right) on the step's keyed uniforms (the RNG-injection shim's stream,
oracle/philox.py).  The ancestors that come out are the reference's, given the states; the device's must equal them.
This pins the one third-party function the device restates (scipy's pmf) to scipy itself rather than
to the oracle.  Needs scipy (present in this image and on the GPU box)."""
import numpy as np

import philox as ph


def reference_weights(y, x, model, observations, probs):
    """pmcmc.py:177-181 for one step: y = Y[p-1] [K], x = hidden[p-1] [N, C] (int) -> weights [N] f64."""
    from scipy.stats import binom, norm
    x = np.asarray(x, dtype=np.float64)
    if model == "sir_subgroups2":
        G = x.shape[1] // 3
        xs = 0
        for g in range(G):                                   # builtin sum over groups, :173
            xs = xs + x[:, 3 * g:3 * g + 3]
        x = xs
    K = y.shape[0]
    if not observations:
        cols = [binom.pmf(y[i], x[:, i], probs) for i in range(K)]
    else:
        cols = [norm.pdf(y[i], x[:, i], probs * x[:, i] + .0001) for i in range(K)]
    return np.min(np.array(cols), axis=0)


def numpy_choice(w, u):
    """np.random.choice(range(N), N, p=w / sum(w)) given its uniforms; None where numpy raises ValueError."""
    s = sum(w.tolist())                                      # builtin sum, :185
    if not (s > 0) or not np.isfinite(s):
        return None
    p = np.asarray(w) / s
    if np.any(np.isnan(p)) or np.any(p < 0):
        return None
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return cdf.searchsorted(u, side="right")


def replay(Y, hidden, ancestry, model, observations, probs, key, filter_index, steps=None):
    """Compare the device's ancestors with the reference's at each step.  Returns (draws, mismatches)."""
    T, N = hidden.shape[0], hidden.shape[1]
    draws = bad = 0
    for p in (steps if steps is not None else range(1, T)):
        w = reference_weights(Y[p - 1], hidden[p - 1], model, observations, probs)
        a = numpy_choice(w, ph.resample_uniforms(key, filter_index, p, N))
        assert a is not None, f"the reference would raise at step {p} where the device did not"
        draws += N
        bad += int(np.count_nonzero(a != ancestry[p]))
    return draws, bad
