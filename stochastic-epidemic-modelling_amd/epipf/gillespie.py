"""Gillespie simulators with the reference's signatures (gillespie_algo.py), run on the GPU.

`sir_simulate`, `seir_simulate`, `sir_subgroups_simulate` (gillespie_algo.py:10-75, 78-146, 148-233)
with last_values_only=True propagate one state through the same kernel code the particle filter
uses; with last_values_only=False they return the reference's full path dict (event times and the
compartments after every event, from epipf_simulate_path).  `simulate_batch` / `simulate_path_batch`
propagate many states in one launch (one lane per state).  Draws come from the keyed Philox stream:
state j, event k -> counter (k, j, step, filter_index).
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


def simulate_path_batch(type_model, states, theta, max_time=1.0, *, key=None, filter_index=None, step=0, device=0):
    """Full paths from int states [n, C]: (times [n, cap], states [n, cap, C], n_events [n], final [n, C])."""
    from .engine import model_id, theta_vector
    mid = model_id(type_model)
    _, G = theta_vector(mid, theta)
    eng = get_engine(mid, G, 1, 1, 1, device)
    k, f = _stream(key, filter_index)
    return eng.simulate_path(np.rint(np.asarray(states)).astype(np.int32), theta, max_time, k, f, step)


def _path_dict(names, x0, times, states, n, time_first):
    """The reference's conditions dict: the initial value then one entry per event (gillespie_algo.py:68-70);
    counts keep the type of the caller's population entries, as the reference's `value + stoichiometry` does
    (np.int64 entries give np.int64 counts, Python ints give ints, floats give floats)."""
    conv = [type(v) for v in x0]
    cols = {}
    for c, name in enumerate(names):
        cols[name] = [x0[c]] + [conv[c](v) for v in states[:n, c].tolist()]
    tl = [0.0] + times[:n].tolist()
    return {"time": tl, **cols} if time_first else {**cols, "time": tl}


def _one_path(model, names, population, theta, max_time, time_first, key, filter_index, step):
    pop = population if isinstance(population, np.ndarray) else np.asarray(population, dtype=object)
    flat = list(pop.reshape(-1))          # the caller's elements: numpy scalars stay numpy scalars
    t, x, n, _ = simulate_path_batch(model, np.asarray(flat, dtype=float).reshape(1, -1), theta, max_time, key=key,
                                     filter_index=filter_index, step=step)
    return _path_dict(names, flat, t[0], x[0], int(n[0]), time_first)


def sir_simulate(population, theta_proposal, max_time, last_values_only, *, key=None, filter_index=None, step=0):
    """gillespie_algo.py:10-75.  last_values_only=True: (s, i, r) floats; False: the reference's
    {"s": [...], "i": [...], "r": [...], "time": [...]} path."""
    if not last_values_only:
        return _one_path("sir", ("s", "i", "r"), population, theta_proposal, max_time, False, key, filter_index, step)
    out, _ = simulate_batch("sir", np.asarray(population, dtype=float).reshape(1, 3), theta_proposal, max_time,
                            key=key, filter_index=filter_index, step=step)
    return tuple(float(v) for v in out[0])


def seir_simulate(population, theta_proposal, max_time, last_values_only, *, key=None, filter_index=None, step=0):
    """gillespie_algo.py:78-146.  last_values_only=True: (s, e, i, r) floats; False: the reference's path dict."""
    if not last_values_only:
        return _one_path("seir", ("s", "e", "i", "r"), population, theta_proposal, max_time, False, key,
                         filter_index, step)
    out, _ = simulate_batch("seir", np.asarray(population, dtype=float).reshape(1, 4), theta_proposal, max_time,
                            key=key, filter_index=filter_index, step=step)
    return tuple(float(v) for v in out[0])


def sir_subgroups_simulate(population, betas_proposal, gamma_proposal, max_time, last_values_only, *, key=None,
                           filter_index=None, step=0):
    """gillespie_algo.py:148-233.  last_values_only=True: [[s, i, r] per group]; False: the reference's
    {"time": [...], "s_0": [...], "i_0": [...], "r_0": [...], "s_1": ...} path."""
    pop = np.asarray(population)
    G = pop.shape[0]
    if not last_values_only:
        names = tuple(f"{c}_{g}" for g in range(G) for c in ("s", "i", "r"))
        return _one_path("sir_subgroups", names, pop, (betas_proposal, gamma_proposal), max_time, True, key,
                         filter_index, step)
    out, _ = simulate_batch("sir_subgroups", pop.astype(float).reshape(1, 3 * G), (betas_proposal, gamma_proposal),
                            max_time, key=key, filter_index=filter_index, step=step)
    return [[float(v) for v in out[0, 3 * g:3 * g + 3]] for g in range(G)]
