"""Pin the ABC oracle (oracle/abc_oracle.c) before trusting it: every case of tests/golden/abc_golden.npz,
written by running the unmodified abc_algo.abc_algo (abc_algo.py:17-109) on the keyed ABC stream
(tests/golden/make_golden.py run_abc_cases), plus the two pieces of third-party arithmetic it restates:
numpy's pairwise summation (np.mean, abc_algo.py:12) and the stream's Poisson draw."""
import numpy as np
import pytest

import oracle
import philox as ph
from conftest import load_golden

ABC_CASES = ["noisy_400", "noisy_150", "extinct_all", "float_obs_15", "float_obs_200"]


@pytest.fixture(scope="module")
def abc_golden():
    return load_golden("abc_golden.npz")


def priors_of(rec):
    p = rec["priors"]
    return {"beta": [float(p[0]), float(p[1])], "gamma": [float(p[2]), float(p[3])]}


@pytest.mark.parametrize("name", ABC_CASES)
def test_oracle_abc_matches_reference(abc_golden, name):
    """Posterior draws, daily trajectories and the number of trials the reference ran, all bit-exact."""
    rec = abc_golden["abc_" + name]
    post, trajs, trials = oracle.abc_algo(rec["Y"], int(rec["n"]), float(rec["threshold"]), priors_of(rec),
                                          key=int(rec["key"]), run_index=int(rec["f"]), batch=32)
    np.testing.assert_array_equal(post["beta"], rec["beta"])
    np.testing.assert_array_equal(post["gamma"], rec["gamma"])
    np.testing.assert_array_equal(trajs, rec["trajectories"])
    assert trials == int(rec["trials"])


def test_oracle_abc_trial_distances_reproduce_acceptance(abc_golden):
    """Trials the reference rejected have distance > threshold; the accepted ones do not."""
    rec = abc_golden["abc_noisy_400"]
    th, rows, dist, _ = oracle.abc_trials(rec["Y"], priors_of(rec), int(rec["key"]), int(rec["f"]), 0,
                                          int(rec["trials"]))
    acc = np.nonzero(~(dist > float(rec["threshold"])))[0]
    assert len(acc) == int(rec["n"]) and acc[-1] == int(rec["trials"]) - 1
    np.testing.assert_array_equal(th[acc, 0], rec["beta"])
    np.testing.assert_array_equal(rows[acc], rec["trajectories"][:, :, 1:].astype(np.int32))


def test_pairwise_sum_matches_numpy():
    """np.add.reduce / np.mean order on contiguous float64 (blocks of 128, 8 accumulators, halving above)."""
    rs = np.random.RandomState(0)
    L = oracle.lib()
    for _ in range(600):
        n = int(rs.randint(1, 1200))
        a = np.ascontiguousarray(np.abs(rs.standard_normal(n) * 10.0 ** rs.randint(-3, 9, n)))
        assert L.oracle_pairwise_sum(oracle._p(a), n) == np.add.reduce(a)
        assert np.mean(a) == np.add.reduce(a) / n


@pytest.mark.parametrize("lam", [1.0, 3.0, 20.0, 4815.0, 9980.0, 123456.0])
def test_poisson_mode_inversion_c_matches_python(lam):
    L = oracle.lib()
    pm = ph.poisson_mode_pmf(lam)
    assert L.oracle_poisson_mode_pmf(lam) == pm
    for t in range(300):
        u = ph.abc_init_uniform(7, 1, t, 0)
        assert L.oracle_poisson_mode_inversion(lam, u, pm) == ph.poisson_mode_inversion(lam, u, pm)


def test_poisson_mode_inversion_distribution():
    """The keyed initial-count draw is Poisson: mean, variance and the small-lambda pmf."""
    L = oracle.lib()
    for lam in (3.0, 4800.0):
        pm = L.oracle_poisson_mode_pmf(lam)
        k = np.array([L.oracle_poisson_mode_inversion(lam, ph.abc_init_uniform(11, 0, t, 0), pm)
                      for t in range(20000)])
        se = np.sqrt(lam / len(k))
        assert abs(k.mean() - lam) < 5 * se
        assert abs(k.var() / lam - 1) < 0.05
    from scipy.stats import poisson
    freq = np.bincount(k := np.array([L.oracle_poisson_mode_inversion(3.0, ph.abc_init_uniform(12, 0, t, 1),
                                                                      L.oracle_poisson_mode_pmf(3.0))
                                      for t in range(20000)]), minlength=8)[:8] / 20000
    np.testing.assert_allclose(freq, poisson.pmf(np.arange(8), 3.0), atol=0.01)
    assert L.oracle_poisson_mode_inversion(0.0, 0.5, 0.0) == 0
    assert L.oracle_poisson_mode_inversion(5.0, 1.0 - 2.0 ** -53, L.oracle_poisson_mode_pmf(5.0)) >= 0
