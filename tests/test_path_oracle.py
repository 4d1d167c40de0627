"""Full-path SSA (gillespie_algo.py *_simulate with last_values_only=False, SURVEY.md / VERDICT r1 item 7): the CPU
oracle's path recorder against the unmodified reference run under the keyed stream (tests/golden/path_golden.npz):
event times and compartment rows bit-exact, every trajectory.  CPU only."""
import numpy as np
import pytest

import oracle
from conftest import load_golden, path_rows, path_theta

CASES = sorted(load_golden("path_golden.npz"))


@pytest.mark.parametrize("name", CASES)
def test_oracle_path_matches_reference(path_golden, name):
    rec = path_golden[name]
    model, theta = path_theta(rec)
    t, x, nev, fin = oracle.simulate_path(model, rec["states"], theta, float(rec["max_time"]), key=int(rec["key"]),
                                          filter_index=int(rec["f"]), step=int(rec["step"]))
    np.testing.assert_array_equal(nev, rec["counts"])
    for j, (tj, xj) in enumerate(path_rows(rec)):
        n = len(tj)
        assert np.array_equal(t[j, :n].view(np.int64), tj.view(np.int64)), (name, j)   # times bit for bit
        np.testing.assert_array_equal(x[j, :n], xj)
        np.testing.assert_array_equal(fin[j], xj[-1] if n else rec["states"][j])


def test_oracle_path_final_equals_last_values(path_golden):
    rec = path_golden["path_sir_3.5"]
    model, theta = path_theta(rec)
    _, _, nev, fin = oracle.simulate_path(model, rec["states"], theta, 3.5, key=78, filter_index=5, step=3)
    last, ev = oracle.simulate(model, rec["states"], theta, 3.5, key=78, filter_index=5, step=3)
    np.testing.assert_array_equal(fin, last)
    assert int(nev.sum()) == ev
