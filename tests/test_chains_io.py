"""Chain CSV layout, warm start and Gelman-Rubin against the reference's own code
paths: tests/experiments/pobs/prob_.05.py:50-61 (savetxt layout), tests/test_pmcmc_noisy.py:32-40 (warm start)
and helpers.py:15-43 (gelman_rubin_test, restated verbatim below because helpers.py cannot be imported
here: it imports arviz, which is absent)."""
import numpy as np

from epipf import chains_io as io


def _reference_gelman_rubin(chains):
    # helpers.py:15-43, statement for statement
    M = len(chains)
    N, no_params = chains[0].shape
    mean_params = np.zeros((M, no_params))
    var_params = np.zeros((M, no_params))
    for m, chain in enumerate(chains):
        for param in range(no_params):
            mean_param = np.mean(chain[:, param])
            var_param = 1.0 / (N - 1) * np.sum((chain[:, param] - mean_param) ** 2)
            mean_params[m, param] = mean_param
            var_params[m, param] = var_param
    theta_hat = np.mean(mean_params, axis=0)
    W = np.mean(var_params, axis=0)
    B = N / (M - 1) * np.sum((mean_params - theta_hat) ** 2, axis=0)
    V = (N - 1) / N * W + (M + 1) / (M * N) * B
    return np.sqrt(V / W)


def test_gelman_rubin_matches_reference():
    rs = np.random.RandomState(4)
    chains = [rs.normal(size=(500, 3)) * [1, 2, 3] + rs.normal(size=3) for _ in range(4)]
    np.testing.assert_array_equal(io.gelman_rubin(chains), _reference_gelman_rubin(chains))
    same = [rs.normal(size=(4000, 2)) for _ in range(3)]
    assert np.all(np.abs(io.gelman_rubin(same) - 1) < 0.01)


def test_save_load_roundtrip(tmp_path):
    rs = np.random.RandomState(1)
    th, lk, tr = rs.rand(30, 2), rs.rand(30), rs.randint(0, 100, (15, 30, 3)).astype(float)
    io.save_run(str(tmp_path), th, lk, tr)
    names = sorted(p.name for p in tmp_path.iterdir())
    assert names == ["likelihoods.csv", "sampled_trajs_infected.csv", "sampled_trajs_recovered.csv",
                     "sampled_trajs_susceptible.csv", "thetas.csv"]
    # the reference writes with np.savetxt(..., delimiter=","): same bytes
    ref = tmp_path / "ref.csv"
    np.savetxt(ref, th, delimiter=",")
    assert ref.read_bytes() == (tmp_path / "thetas.csv").read_bytes()
    th2, lk2, tr2 = io.load_run(str(tmp_path))
    np.testing.assert_array_equal(th2, th)
    np.testing.assert_array_equal(lk2, lk)
    np.testing.assert_array_equal(tr2, tr)


def test_warm_start_matches_reference_recipe():
    rs = np.random.RandomState(2)
    thetas = np.repeat(rs.rand(200, 2), 3, axis=0)
    theta0, sigma = io.warm_start(thetas)
    thetas2 = thetas[100:, :]               # tests/test_pmcmc_noisy.py:35-40
    thetas3 = thetas2[::20]
    thetas_unique = np.unique(thetas3, axis=0)
    assert theta0 == thetas[-1].tolist()
    np.testing.assert_array_equal(sigma, np.cov(thetas_unique.T, ddof=0))


def test_hdi_is_the_narrowest_interval():
    """The HDI is arviz's (absent here): the narrowest interval of floor(0.95 n) + 1 sorted draws -- checked against
    a brute force over every window, on skewed, bimodal, tied and tiny samples; and helpers.py:5-13's
    (mean, low, high) shape for 1-D and 2-D data."""
    rs = np.random.RandomState(8)
    for x in (rs.gamma(2.0, 1.0, 1000), np.concatenate([rs.normal(0, 1, 300), rs.normal(6, 0.5, 700)]),
              np.round(rs.normal(size=200), 1), rs.rand(3), np.array([5.0])):
        s = np.sort(x)
        k = int(np.floor(0.95 * s.size))
        best = min(range(s.size - k), key=lambda i: (s[i + k] - s[i], i))
        np.testing.assert_array_equal(io.hdi(x), [s[best], s[best + k]])
    th = rs.normal(size=(2, 500))
    m, lo, hi = io.mean_credible_interval(th)
    np.testing.assert_array_equal(m, th.mean(axis=1))
    assert lo < 0 < hi and np.mean((th >= lo) & (th <= hi)) >= 0.95
    m1, lo1, hi1 = io.mean_credible_interval(th[0])
    assert m1 == th[0].mean() and lo1 < hi1


def test_running_mean_and_posterior_mse():
    x = np.arange(10.0)
    np.testing.assert_allclose(io.running_mean(x, 3), np.convolve(x, np.ones(3) / 3, mode="valid"))
    chain = np.array([[0.2, 0.1], [0.3, 0.1]])
    assert io.posterior_mse(np.array([0.25, 0.1]), chain) == np.mean((chain - [0.25, 0.1]) ** 2)
