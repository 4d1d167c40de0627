"""Randomised parity sweep of the GPU ABC trial kernel (abc_algo.py:17-109 per trial) against the CPU oracle
(oracle/abc_oracle.c): seeded cases over T = 1..40 observed days, initial counts from empty to 10^5 (Y[0] sets the
Poisson means of the initial state, abc_algo.py:38-39), prior boxes from a point to [0, 8]^2, run indices, trial
offsets up to 2^32 - n, with and without the length ordering (EPIPF_ABC_ORDER).  Priors, day tables and distances
must equal the oracle's bit for bit.  Needs an MI355X: `-m gpu`."""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("EPIPF_FUZZ_ABC_CASES", 24))


def _case(seed):
    rs = np.random.RandomState(9100 + seed)
    T = int(rs.choice([1, 2, 7, 8, 15, 23, 40]))
    S0 = float(rs.choice([0, 50, 4800, 20000, 100000]))
    I0 = float(rs.choice([0, 1, 20, 500]))
    R0 = float(rs.choice([0, 5, 100]))
    Y = np.zeros((T, 3))
    Y[0] = (S0, I0, R0)
    for t in range(1, T):                                # observed rows: only the distance reads them
        Y[t] = np.floor(Y[t - 1] * rs.uniform(0.7, 1.1, 3) + rs.randint(0, 30, 3))
    lo = rs.uniform(0, 2, 2)
    hi = lo + rs.choice([0.0, 0.5, 3.0, 6.0], 2)
    pr = {"beta": [float(lo[0]), float(hi[0])], "gamma": [float(lo[1]), float(hi[1])]}
    n = int(rs.choice([1, 63, 300, 1000, 2500]))
    t0 = int(rs.choice([0, 12345, 2**32 - 3000]))
    return dict(Y=Y, pr=pr, key=int(rs.randint(1, 2**31)), run=int(rs.randint(0, 1000)), t0=t0, n=n,
                order=bool(rs.rand() < 0.7))


@pytest.mark.parametrize("seed", range(CASES))
def test_random_abc_trials_match_oracle(seed):
    from epipf.engine import Engine
    a = _case(seed)
    old = os.environ.get("EPIPF_ABC_ORDER")
    os.environ["EPIPF_ABC_ORDER"] = "1" if a["order"] else "0"
    eng = Engine("sir", 1, 1, 1, 1)
    try:
        th, rows, dist = eng.abc_trials(a["Y"], a["pr"], a["key"], a["run"], a["t0"], a["n"])
    finally:
        eng.close()
        if old is None:
            os.environ.pop("EPIPF_ABC_ORDER", None)
        else:
            os.environ["EPIPF_ABC_ORDER"] = old
    oth, orows, odist, _ = oracle.abc_trials(a["Y"], a["pr"], a["key"], a["run"], a["t0"], a["n"])
    np.testing.assert_array_equal(th, oth, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(rows, orows, err_msg=f"seed {seed}")
    np.testing.assert_array_equal(dist, odist, err_msg=f"seed {seed}")


@pytest.mark.parametrize("seed", range(max(CASES // 2, 1)))
def test_random_abc_runs_with_early_rejection_match_oracle(seed, monkeypatch):
    """Whole epipf_abc runs (batched rejection loop) on the random cases, thresholds placed ON oracle distances so that
    ties at the threshold decide acceptance: with early rejection on (default) and off, the accepted draws, their day
    tables and the trial count equal the oracle's first k+1 accepted trials (abc_algo.py:30-33, trial order)."""
    from epipf.engine import Engine
    a = _case(seed)
    rs = np.random.RandomState(7700 + seed)
    M = 3000
    oth, orows, odist, _ = oracle.abc_trials(a["Y"], a["pr"], a["key"], a["run"], 0, M)
    k = int(rs.choice([0, 3, 30, 300]))
    thr = float(np.sort(odist)[k])
    acc_idx = np.nonzero(~(odist > thr))[0][:k + 1]
    batch = int(rs.choice([0, 700, 5000]))
    eng = Engine("sir", 1, 1, 1, 1)
    try:
        for early in ("1", "0"):
            monkeypatch.setenv("EPIPF_ABC_EARLY", early)
            theta, traj, trials, acc = eng.abc(a["Y"], k + 1, thr, a["pr"], a["key"], a["run"], batch=batch)
            msg = f"seed {seed} early {early} k {k} thr {thr}"
            assert acc == k + 1 and trials == int(acc_idx[-1]) + 1, msg
            np.testing.assert_array_equal(theta, oth[acc_idx], err_msg=msg)
            np.testing.assert_array_equal(traj[:, :, 1:], orows[acc_idx].astype(np.float64), err_msg=msg)
    finally:
        eng.close()
