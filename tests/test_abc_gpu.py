"""Parity of the GPU ABC rejection sampler (epipf_abc / epipf_abc_trials through the C ABI) with the reference
golden vectors (abc_algo.abc_algo run unmodified on the keyed ABC stream) and the CPU oracle
(oracle/abc_oracle.c).  Draws, day tables, distances and trial counts are bit-exact.  Needs an MI355X."""
import numpy as np
import pytest

import oracle
from conftest import load_golden

pytestmark = pytest.mark.gpu

ABC_CASES = ["noisy_400", "noisy_150", "extinct_all", "float_obs_15", "float_obs_200"]


@pytest.fixture(scope="module")
def abc_golden():
    return load_golden("abc_golden.npz")


@pytest.fixture(scope="module")
def engine():
    from epipf.engine import get_engine
    return get_engine("sir", 1, 1, 1, 1)


def priors_of(rec):
    p = rec["priors"]
    return {"beta": [float(p[0]), float(p[1])], "gamma": [float(p[2]), float(p[3])]}


@pytest.mark.parametrize("name", ABC_CASES)
def test_abc_matches_reference_golden(abc_golden, name):
    from epipf.abc import abc_run
    rec = abc_golden["abc_" + name]
    r = abc_run(rec["Y"], int(rec["n"]), float(rec["threshold"]), priors_of(rec), key=int(rec["key"]),
                run_index=int(rec["f"]))
    assert r["accepted"] == int(rec["n"])
    np.testing.assert_array_equal(r["beta"], rec["beta"])
    np.testing.assert_array_equal(r["gamma"], rec["gamma"])
    np.testing.assert_array_equal(r["trajectories"], rec["trajectories"])
    assert r["trials"] == int(rec["trials"])


@pytest.mark.parametrize("name", ABC_CASES)
def test_abc_trials_match_oracle(abc_golden, engine, name):
    """Per-trial theta, day table and distance over a few thousand trials of every golden configuration."""
    rec = abc_golden["abc_" + name]
    n = 3000 if rec["Y"].shape[0] < 100 else 600
    th, rows, dist = engine.abc_trials(rec["Y"], priors_of(rec), int(rec["key"]), int(rec["f"]), 0, n)
    oth, orows, odist, _ = oracle.abc_trials(rec["Y"], priors_of(rec), int(rec["key"]), int(rec["f"]), 0, n)
    np.testing.assert_array_equal(th, oth)
    np.testing.assert_array_equal(rows, orows)
    np.testing.assert_array_equal(dist, odist)


def test_abc_trials_high_indices_and_other_run(abc_golden, engine):
    rec = abc_golden["abc_noisy_400"]
    for t0, run in ((4_000_000_000, 0), (123_456, 7)):
        th, rows, dist = engine.abc_trials(rec["Y"], priors_of(rec), 99, run, t0, 512)
        oth, orows, odist, _ = oracle.abc_trials(rec["Y"], priors_of(rec), 99, run, t0, 512)
        np.testing.assert_array_equal(th, oth)
        np.testing.assert_array_equal(rows, orows)
        np.testing.assert_array_equal(dist, odist)


@pytest.mark.parametrize("batch", [0, 1, 7, 40, 100000])
def test_abc_batching_does_not_change_results(abc_golden, engine, batch):
    rec = abc_golden["abc_noisy_400"]
    theta, traj, trials, acc = engine.abc(rec["Y"], int(rec["n"]), float(rec["threshold"]), priors_of(rec),
                                          int(rec["key"]), int(rec["f"]), batch=batch)
    assert acc == int(rec["n"]) and trials == int(rec["trials"])
    np.testing.assert_array_equal(theta[:, 0], rec["beta"])
    np.testing.assert_array_equal(traj, rec["trajectories"])


def edge_inputs(datasets_golden):
    Y = datasets_golden["sir_noisy"].copy()
    one_day = Y[:1].copy()
    no_infected = Y.copy()
    no_infected[0] = (4820, 0, 0)
    zero_pop = np.zeros((5, 3))
    fixed_prior = {"beta": [2.0, 2.0], "gamma": [1.0, 1.0]}
    wide = {"beta": [0.0, 5.0], "gamma": [0.0, 5.0]}
    return [(one_day, wide), (no_infected, wide), (zero_pop, wide), (Y, fixed_prior), (Y[:9], wide)]


def test_abc_edge_cases_match_oracle(datasets_golden, engine):
    """T = 1, I0 = 0 (no events), an empty population, a degenerate prior, T < 8 (numpy's short sum)."""
    for Y, pr in edge_inputs(datasets_golden):
        th, rows, dist = engine.abc_trials(Y, pr, 5, 0, 0, 700)
        oth, orows, odist, _ = oracle.abc_trials(Y, pr, 5, 0, 0, 700)
        np.testing.assert_array_equal(th, oth)
        np.testing.assert_array_equal(rows, orows)
        np.testing.assert_array_equal(dist, odist)


def test_abc_max_trials_bounds_an_unreachable_threshold(abc_golden, engine):
    from epipf.abc import abc_algo
    rec = abc_golden["abc_noisy_400"]
    theta, traj, trials, acc = engine.abc(rec["Y"], 3, -1.0, priors_of(rec), 1, 0, max_trials=5000)
    assert acc == 0 and trials == 5000 and theta.shape == (0, 2)
    with pytest.raises(RuntimeError):
        abc_algo(rec["Y"], 3, -1.0, priors_of(rec), key=1, max_trials=1000)
    theta, traj, trials, acc = engine.abc(rec["Y"], 0, 1e9, priors_of(rec), 1, 0)
    assert acc == 0 and trials == 0


def test_abc_bad_arguments_raise(abc_golden, engine):
    from epipf._lib import EpipfError
    rec = abc_golden["abc_noisy_400"]
    Y = rec["Y"].copy()
    Y[0, 1] = -3.0
    with pytest.raises(EpipfError):
        engine.abc_trials(Y, priors_of(rec), 1, 0, 0, 4)
    with pytest.raises(EpipfError):
        engine.abc_trials(rec["Y"], {"beta": [-1.0, 1.0], "gamma": [0, 1]}, 1, 0, 0, 4)
    with pytest.raises(ValueError):
        engine.abc_trials(np.ones((4, 4)), priors_of(rec), 1, 0, 0, 4)


def test_abc_large_run_properties(abc_golden, engine):
    """A production-size run (hundreds of thousands of trials): every accepted draw satisfies the reference's
    acceptance rule recomputed on the host, lies in the prior box, and its trajectory is a valid SIR path."""
    from epipf.abc import distance_function
    rec = abc_golden["abc_noisy_400"]
    Y = rec["Y"]
    pr = priors_of(rec)
    theta, traj, trials, acc = engine.abc(Y, 2000, 150.0, pr, 2024, 3)
    assert acc == 2000 and trials > 2000
    for s in range(acc):
        d = distance_function(traj[s, :, 2], Y[:, 1], traj[s, :, 3], Y[:, 2])
        assert not (d > 150.0)
    assert np.all((theta >= 0) & (theta <= 5))
    np.testing.assert_array_equal(traj[:, :, 0], np.broadcast_to(np.arange(Y.shape[0]), traj.shape[:2]))
    tot = traj[:, :, 1:].sum(axis=2)
    assert np.all(tot == tot[:, :1])
    assert np.all(np.diff(traj[:, :, 1], axis=1) <= 0) and np.all(np.diff(traj[:, :, 3], axis=1) >= 0)
    # the last accepted trial and a sample of the rest agree with the oracle trial by trial
    th, rows, dist = engine.abc_trials(Y, pr, 2024, 3, trials - 1, 1)
    assert not (dist[0] > 150.0)
    np.testing.assert_array_equal(th[0], theta[-1])
    oth, orows, odist, _ = oracle.abc_trials(Y, pr, 2024, 3, trials - 1, 1)
    np.testing.assert_array_equal(orows[0], traj[-1, :, 1:].astype(np.int32))


@pytest.mark.parametrize("lanes,frac", [(2, 0.25), (4, 0.25), (8, 0.25), (16, 0.25), (4, 1.0), (16, 1.0), (4, 0.003)])
def test_abc_lane_groups_equal_one_lane_and_oracle(abc_golden, engine, monkeypatch, lanes, frac):
    """The longest trials on lane groups (abc_trials_group_kernel, W lanes per trial, concurrent with the one-lane
    kernel): theta, day tables and distances bit-identical to the one-lane kernel and to the oracle, for every
    group width and share of the trials (all of them, a quarter, a handful)."""
    rec = abc_golden["abc_noisy_150"]
    n = 6000
    out = {}
    for w in (1, lanes):
        monkeypatch.setenv("EPIPF_ABC_LANES", str(w))
        monkeypatch.setenv("EPIPF_ABC_GROUP_FRAC", str(frac))
        out[w] = engine.abc_trials(rec["Y"], priors_of(rec), 4242, 3, 1000, n)
    for a, b in zip(out[1], out[lanes]):
        np.testing.assert_array_equal(a, b)
    oth, orows, odist, _ = oracle.abc_trials(rec["Y"], priors_of(rec), 4242, 3, 1000, n)
    np.testing.assert_array_equal(out[lanes][0], oth)
    np.testing.assert_array_equal(out[lanes][1], orows)
    np.testing.assert_array_equal(out[lanes][2], odist)


@pytest.mark.parametrize("name", ABC_CASES)
def test_abc_lane_groups_reference_goldens(abc_golden, monkeypatch, name):
    """The five reference ABC runs end to end with every trial on lane groups (share 1.0)."""
    from epipf.abc import abc_run
    monkeypatch.setenv("EPIPF_ABC_LANES", "4")
    monkeypatch.setenv("EPIPF_ABC_GROUP_FRAC", "1.0")
    rec = abc_golden["abc_" + name]
    r = abc_run(rec["Y"], int(rec["n"]), float(rec["threshold"]), priors_of(rec), key=int(rec["key"]),
                run_index=int(rec["f"]))
    np.testing.assert_array_equal(r["beta"], rec["beta"])
    np.testing.assert_array_equal(r["gamma"], rec["gamma"])
    np.testing.assert_array_equal(r["trajectories"], rec["trajectories"])
    assert r["trials"] == int(rec["trials"])


def _abc_both_ways(monkeypatch, engine, Y, n, thr, pr, key, run, **kw):
    out = {}
    for early in ("0", "1"):
        monkeypatch.setenv("EPIPF_ABC_EARLY", early)
        out[early] = engine.abc(Y, n, thr, pr, key, run, **kw)
    for a, b in zip(out["0"], out["1"]):
        np.testing.assert_array_equal(a, b)
    return out["1"]


@pytest.mark.parametrize("name", ABC_CASES)
def test_abc_early_rejection_changes_nothing(abc_golden, engine, monkeypatch, name):
    """epipf_abc stops a trial once its partial distance sum proves distance > threshold: accepted
    draws, trajectories and the trial count are identical with it off (EPIPF_ABC_EARLY=0) and on, and equal the
    reference's golden run."""
    rec = abc_golden["abc_" + name]
    theta, traj, trials, acc = _abc_both_ways(monkeypatch, engine, rec["Y"], int(rec["n"]), float(rec["threshold"]),
                                              priors_of(rec), int(rec["key"]), int(rec["f"]))
    assert acc == int(rec["n"]) and trials == int(rec["trials"])
    np.testing.assert_array_equal(theta[:, 0], rec["beta"])
    np.testing.assert_array_equal(traj, rec["trajectories"])


def test_abc_early_rejection_at_the_threshold(abc_golden, engine, monkeypatch):
    """Thresholds placed exactly on trial distances (the oracle's): a trial with distance == threshold is accepted
    (abc_algo.py:30-33), so the early bound must never reject it.  Also the production setting (2000 samples at
    150, hundreds of thousands of trials) with lane groups on part of small batches."""
    rec = abc_golden["abc_noisy_150"]
    Y, pr = rec["Y"], priors_of(rec)
    _, _, odist, _ = oracle.abc_trials(Y, pr, 77, 2, 0, 4000)
    srt = np.sort(odist)
    for k in (5, 40, 400):
        thr = float(srt[k])
        theta, traj, trials, acc = _abc_both_ways(monkeypatch, engine, Y, k + 1, thr, pr, 77, 2, batch=1000)
        assert acc == k + 1
        last = np.nonzero(~(odist > thr))[0][k]
        assert trials == last + 1
        np.testing.assert_array_equal(traj[-1, :, 1:], oracle.abc_trials(Y, pr, 77, 2, last, 1)[1][0])
    _abc_both_ways(monkeypatch, engine, Y, 2000, 150.0, pr, 2024, 3)
    monkeypatch.setenv("EPIPF_ABC_LANES", "4")
    monkeypatch.setenv("EPIPF_ABC_GROUP_FRAC", "0.25")
    _abc_both_ways(monkeypatch, engine, Y, 300, 150.0, pr, 2024, 4, batch=20000)
