"""The XCD-aware placement of the step launches (step_block, csrc/epipf_step.hpp; EPIPF_XCD_MAP) only moves work
between XCDs: filters on the 1-D remapped grid equal the 2-D grid's bit for bit, for grid sizes that are and are not
multiples of 8 (ragged chains x blocks), on the one-lane and the lane-group kernels.  Needs an MI355X: `-m gpu`."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(xcd, N, chains, lanes, Y):
    from epipf.engine import Engine
    old = os.environ.get("EPIPF_XCD_MAP")
    os.environ["EPIPF_XCD_MAP"] = str(xcd)
    try:
        eng = Engine("sir", 1, N, Y.shape[0], chains)
    finally:
        if old is None:
            os.environ.pop("EPIPF_XCD_MAP", None)
        else:
            os.environ["EPIPF_XCD_MAP"] = old
    try:
        eng.set_observations(Y)
        eng.set_population(4820.0, 20.0)
        eng.set_lanes(lanes)
        th = np.array([[2.0 + 0.1 * c, 1.0 + 0.05 * c] for c in range(chains)])
        lz, st = eng.run(th, [0.1] * chains, [77 + c for c in range(chains)], [c for c in range(chains)])
        hid, anc = eng.history(chains)
        return lz, st, hid, anc
    finally:
        eng.close()


@pytest.mark.parametrize("N,chains,lanes", [(320, 3, 1), (1000, 5, 1), (130, 7, 4), (64, 8, 1), (10000, 2, 1)])
def test_xcd_placement_matches_2d_grid(datasets_golden, N, chains, lanes):
    Y = datasets_golden["sir_binom"]
    a = _run(0, N, chains, lanes, Y)
    b = _run(1, N, chains, lanes, Y)
    assert np.all(a[1] == 0) and np.array_equal(a[1], b[1])
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
