"""Gillespie simulators with the reference's signatures (gillespie_algo.py), run on the GPU.

`sir_simulate`, `seir_simulate`, `sir_subgroups_simulate` (gillespie_algo.py:10-75, 78-146, 148-233)
with last_values_only=True propagate one state through the same kernel code the particle filter
uses; the `*_batch` variants propagate many states in one launch (one lane per state).  Draws come
from the keyed Philox stream: state j, event k -> counter (k, j, step, filter_index).
Full-path mode (last_values_only=False, used by the reference's ABC sampler and plots) is not on
the particle-filter path and is not provided by this engine.
"""
import numpy as np

from .engine import get_engine


def _stream(key, filter_index):
    from .pmcmc import _STREAM
    return (_STREAM.key if key is None else key), (0 if filter_index is None else filter_index)


def simulate_batch(type_model, states, theta, max_time=1.0, *, key=None, filter_index=None, step=0, device=0):
    """Propagate int states [n, C] over [0, max_time]; returns (states_out [n, C] int32, events)."""
    from .engine import model_id, theta_vector
    mid = model_id(type_model)
    _, G = theta_vector(mid, theta)
    states = np.asarray(states)
    eng = get_engine(mid, G, 1, 1, 1, device)
    k, f = _stream(key, filter_index)
    return eng.simulate(np.rint(states).astype(np.int32), theta, max_time, k, f, step)


def _full_path_unsupported():
    raise NotImplementedError("last_values_only=False (full event path) is not part of the GPU particle-filter "
                              "path; see DESIGN.md §8 (ABC / full-path SSA is a later row)")


def sir_simulate(population, theta_proposal, max_time, last_values_only, *, key=None, filter_index=None, step=0):
    """gillespie_algo.py:10-75 (last_values_only=True).  Returns (s, i, r) floats."""
    if not last_values_only:
        _full_path_unsupported()
    out, _ = simulate_batch("sir", np.asarray(population, dtype=float).reshape(1, 3), theta_proposal, max_time,
                            key=key, filter_index=filter_index, step=step)
    return tuple(float(v) for v in out[0])


def seir_simulate(population, theta_proposal, max_time, last_values_only, *, key=None, filter_index=None, step=0):
    """gillespie_algo.py:78-146 (last_values_only=True).  Returns (s, e, i, r) floats."""
    if not last_values_only:
        _full_path_unsupported()
    out, _ = simulate_batch("seir", np.asarray(population, dtype=float).reshape(1, 4), theta_proposal, max_time,
                            key=key, filter_index=filter_index, step=step)
    return tuple(float(v) for v in out[0])


def sir_subgroups_simulate(population, betas_proposal, gamma_proposal, max_time, last_values_only, *, key=None,
                           filter_index=None, step=0):
    """gillespie_algo.py:148-233 (last_values_only=True).  Returns [[s, i, r] per group]."""
    if not last_values_only:
        _full_path_unsupported()
    pop = np.asarray(population, dtype=float)
    G = pop.shape[0]
    out, _ = simulate_batch("sir_subgroups", pop.reshape(1, 3 * G), (betas_proposal, gamma_proposal), max_time,
                            key=key, filter_index=filter_index, step=step)
    return [[float(v) for v in out[0, 3 * g:3 * g + 3]] for g in range(G)]
