"""Drop-in for the reference's abc_algo.py (ABC rejection sampling for the SIR model), on the GPU.

`abc_algo(observed_data, no_of_samples, threshold, priors)` keeps the reference's signature and return
value (abc_algo.py:17-109): a dict {"beta": [...], "gamma": [...]} of accepted draws and the array of
accepted daily trajectories [no_of_samples, T, 4] with columns (day, S, I, R).  The rejection loop runs
batched in libepipf.so (epipf_abc): one GPU lane per trial, accepted trials taken in trial order, so the
result is the reference's sequential loop driven by the keyed ABC stream -- trial t draws its
prior, initial counts and Gillespie events from Philox counters (·, t, 3..5 << 24, run).

Random numbers: key = the module stream (`epipf.seed_stream`), run index = one per abc_algo call (counted
separately from the particle filter's indices).
"""
import numpy as np

from .engine import get_engine
from .pmcmc import _STREAM


def distance_function(I_1, I_2, R_1, R_2):
    """abc_algo.py:9-13 (host helper, identical arithmetic: numpy means of absolute differences)."""
    return (np.mean(abs(np.asarray(I_1) - np.asarray(I_2))) + np.mean(abs(np.asarray(R_1) - np.asarray(R_2)))) / 2


def _take_run_index():
    r = _STREAM.next_abc_run
    _STREAM.next_abc_run = r + 1
    return r


def abc_run(observed_data, no_of_samples, threshold, priors, key=None, run_index=None, max_trials=2**32, batch=0,
            device=0):
    """Full result of one ABC run: dict(beta, gamma, trajectories, trials, accepted, key, run_index)."""
    key = _STREAM.key if key is None else int(key)
    run_index = _take_run_index() if run_index is None else int(run_index)
    eng = get_engine("sir", 1, 1, 1, 1, device)
    theta, traj, trials, acc = eng.abc(observed_data, no_of_samples, threshold, priors, key, run_index, max_trials,
                                       batch)
    return dict(beta=[float(v) for v in theta[:, 0]], gamma=[float(v) for v in theta[:, 1]], trajectories=traj,
                trials=trials, accepted=acc, key=key, run_index=run_index)


def abc_algo(observed_data, no_of_samples, threshold, priors, key=None, run_index=None, max_trials=2**32, batch=0,
             device=0):
    """abc_algo.py:17-109.  Returns (posterior_distr, trajectories).

    Unlike the reference, which loops forever when the threshold is unreachable, at most `max_trials` trials
    run; fewer than no_of_samples accepted draws then raise RuntimeError."""
    r = abc_run(observed_data, no_of_samples, threshold, priors, key, run_index, max_trials, batch, device)
    if r["accepted"] < int(no_of_samples):
        raise RuntimeError(f"abc_algo: {r['accepted']} of {no_of_samples} samples accepted within "
                           f"{r['trials']} trials (threshold {threshold})")
    return {"beta": r["beta"], "gamma": r["gamma"]}, r["trajectories"]
