"""Full-path SSA on the device (epipf_simulate_path; gillespie_algo.py *_simulate with last_values_only=False,
:68-75 / :139-146 / :218-233).  Event times must equal the reference's bit for bit (the device clock is the
reference's: reference-order propensities, IEEE divisions, glibc's log -- DESIGN.md §4) and the compartment rows
exactly.  `-m gpu`."""
import numpy as np
import pytest

import oracle
from conftest import load_golden, path_rows, path_theta

pytestmark = pytest.mark.gpu

CASES = sorted(load_golden("path_golden.npz"))


def _engine(model, G=1):
    from epipf.engine import Engine
    return Engine(model, G, 1, 1, 1)


@pytest.mark.parametrize("name", CASES)
def test_device_path_matches_reference_golden(path_golden, name):
    rec = path_golden[name]
    model, theta = path_theta(rec)
    eng = _engine(model, 2 if model == "sir_subgroups" else 1)
    t, x, nev, fin = eng.simulate_path(rec["states"], theta, float(rec["max_time"]), int(rec["key"]), int(rec["f"]),
                                       int(rec["step"]))
    eng.close()
    np.testing.assert_array_equal(nev, rec["counts"])
    for j, (tj, xj) in enumerate(path_rows(rec)):
        n = len(tj)
        assert np.array_equal(t[j, :n].view(np.int64), tj.view(np.int64)), (name, j)
        np.testing.assert_array_equal(x[j, :n], xj)
        np.testing.assert_array_equal(fin[j], xj[-1] if n else rec["states"][j])


@pytest.mark.parametrize("model,G,theta,tmax", [("sir", 1, (0.25, 0.1), 1.0), ("sir", 1, (2.0, 1.0), 2.5),
                                                ("seir", 1, (0.5, 0.2, 0.1), 3.0),
                                                ("sir_subgroups", 2, (np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5), 1.0),
                                                ("sir_subgroups", 3, (np.full((3, 3), 1.5), 0.7), 0.8)])
def test_device_path_vs_oracle_and_last_values(model, G, theta, tmax):
    """2000 random starts: the path equals the oracle's event for event, and its final state and event count equal
    the last-value kernel's (the certified f32 loop with replays) -- one stream, three code paths."""
    rs = np.random.RandomState(17 + G)
    n = 2000
    if model == "sir":
        st = np.stack([9000 - rs.randint(0, 3000, n), rs.randint(0, 900, n), rs.randint(0, 100, n)], 1)
    elif model == "seir":
        st = np.stack([9000 - rs.randint(0, 3000, n), rs.randint(0, 300, n), rs.randint(0, 300, n),
                       rs.randint(0, 100, n)], 1)
    else:
        st = np.concatenate([np.stack([2000 - rs.randint(0, 500, n), rs.randint(0, 100, n), rs.randint(0, 50, n)], 1)
                             for _ in range(G)], 1)
    eng = _engine(model, G)
    t, x, nev, fin = eng.simulate_path(st, theta, tmax, key=91, filter_index=4, step=7)
    last, ev = eng.simulate(st, theta, tmax, key=91, filter_index=4, step=7)
    eng.close()
    np.testing.assert_array_equal(fin, last)
    assert int(nev.sum()) == ev
    ot, ox, onev, ofin = oracle.simulate_path(model, st, theta, tmax, key=91, filter_index=4, step=7)
    np.testing.assert_array_equal(nev, onev)
    np.testing.assert_array_equal(fin, ofin)
    for j in range(n):
        k = nev[j]
        assert np.array_equal(t[j, :k].view(np.int64), ot[j, :k].view(np.int64)), j
        np.testing.assert_array_equal(x[j, :k], ox[j, :k])


def test_path_buffer_overflow_and_growth(path_golden):
    """A short buffer keeps the first max_events events and reports the full count; Engine.simulate_path without
    max_events grows the buffer to the longest path (same draws)."""
    rec = path_golden["path_sir_1.0"]
    model, theta = path_theta(rec)
    eng = _engine(model)
    t, x, nev, fin = eng.simulate_path(rec["states"], theta, 1.0, 78, 5, 3, max_events=7)
    assert t.shape == (len(rec["states"]), 7)
    np.testing.assert_array_equal(nev, rec["counts"])
    for j, (tj, xj) in enumerate(path_rows(rec)):
        m = min(7, len(tj))
        np.testing.assert_array_equal(t[j, :m], tj[:m])
        np.testing.assert_array_equal(x[j, :m], xj[:m])
    t2, x2, nev2, fin2 = eng.simulate_path(rec["states"], theta, 1.0, 78, 5, 3)
    assert t2.shape[1] == max(1024, int(rec["counts"].max()))
    np.testing.assert_array_equal(fin2, fin)
    t0, x0, nev0, fin0 = eng.simulate_path(rec["states"], theta, 1.0, 78, 5, 3, max_events=0)
    np.testing.assert_array_equal(nev0, rec["counts"])
    np.testing.assert_array_equal(fin0, fin)
    eng.close()


def test_dropin_full_path_dicts(path_golden):
    """gillespie_algo-style calls with last_values_only=False return the reference's dict: keys in its order, the
    initial value then one entry per event, counts keeping the caller's type, times bit-exact (trajectory 0 of each
    golden case: the drop-in's single path draws as trajectory j = 0)."""
    from epipf import gillespie as gl
    for name, keys in (("path_sir_3.5", ["s", "i", "r", "time"]), ("path_seir_2.0", ["s", "e", "i", "r", "time"]),
                       ("path_sub_4.0", ["time", "s_0", "i_0", "r_0", "s_1", "i_1", "r_1"])):
        rec = path_golden[name]
        tj, xj = path_rows(rec)[0]
        x0 = rec["states"][0]
        kw = dict(key=78, filter_index=5, step=3)
        if name.startswith("path_sub"):
            pop = np.array(x0.reshape(2, 3), dtype=np.int64)
            cond = gl.sir_subgroups_simulate(pop, np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5, float(rec["max_time"]), False,
                                             **kw)
            cols = [f"{c}_{g}" for g in range(2) for c in ("s", "i", "r")]
        else:
            fn = gl.sir_simulate if name.startswith("path_sir") else gl.seir_simulate
            cond = fn([float(v) for v in x0], np.array(rec["theta"]), float(rec["max_time"]), False, **kw)
            cols = keys[:-1]
        assert list(cond) == keys
        assert cond["time"][0] == 0.0 and cond["time"][1:] == tj.tolist()
        for c, col in enumerate(cols):
            assert cond[col] == [x0[c]] + xj[:, c].tolist()
            # the reference's counts are population[...] + stoichiometry: np.int64 for an int64 array, float for floats
            want = np.int64 if name.startswith("path_sub") else float
            assert all(type(v) is want for v in cond[col]), (col, {type(v) for v in cond[col]})
        last = gl.sir_simulate([float(v) for v in x0], np.array(rec["theta"]), float(rec["max_time"]), True, **kw) \
            if name.startswith("path_sir") else None
        if last is not None:
            assert list(last) == [cond[k][-1] for k in cols]
