"""Statistical validation on the device, the way the reference validates its own runs (it pins no
numbers; it checks "consistent likelihoods" by repeating the filter at N = 10 / 100 / 1000,
tests/test_particles_noisy.py:35-88, and posterior recovery by trace / KDE plots against the true parameters, the
unique-theta acceptance rate and Gelman-Rubin across chains, tests/test_pmcmc_p.py:107-317, helpers.py:15-43).
Keyed streams make these deterministic: the thresholds below are properties of the estimator, checked on fixed
draws.  Needs an MI355X: `-m gpu`."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_likelihood_estimates_are_consistent(datasets_golden):
    """48 independent filters at the true theta (config-2 data, first 50 days) for N = 100, 1000, 10000: the spread of
    log z-hat shrinks like 1/N and its mean rises towards log z (Jensen: E log z-hat ~ log z - var / 2)."""
    from epipf.engine import Engine
    Y = datasets_golden["cfg2_binom"][:50]
    stats = {}
    for N in (100, 1000, 10000):
        eng = Engine("sir", 1, N, Y.shape[0], 48)
        eng.set_observations(Y)
        eng.set_population(10000.0, 20.0)
        lz, st = eng.run(np.tile([0.25, 0.1], (48, 1)), [0.1] * 48, [1000 + c for c in range(48)], [0] * 48)
        eng.close()
        assert np.all(st == 0)
        ll = lz[:, -1]
        stats[N] = (ll.mean(), ll.var())
    print("log z-hat mean / variance by N:", stats)
    (m1, v1), (m2, v2), (m3, v3) = stats[100], stats[1000], stats[10000]
    assert v1 > v2 > v3, stats
    assert v1 / v3 > 20, stats                   # ~100x in theory (variance ~ 1/N)
    assert m3 >= m2 - 3 * np.sqrt(v2 / 48) and m2 >= m1 - 3 * np.sqrt(v1 / 48), stats
    assert abs(m3 - m2) < 3 * np.sqrt(v2 / 48 + v3 / 48) + 0.5 * v2, stats


def test_posterior_recovers_the_truth_across_chains(datasets_golden):
    """8 chains of SIR PMCMC (N = 1000, all 200 days of the config-2 data simulated from beta = .25, gamma = .1), started
    away from the truth: after burn-in every chain's posterior mean is within 10% of the truth, Gelman-Rubin across
    the chains is below 1.1 and the unique-theta acceptance rate (tests/test_pmcmc_p.py:291-295) is moderate."""
    from epipf.chains_io import gelman_rubin
    from epipf.pmcmc import ModelType, particle_mcmc_chains
    Y = datasets_golden["cfg2_binom"]
    res = particle_mcmc_chains(Y, ModelType.SIR, [0.3, 0.12], 1e-4, n_chains=600, probs=0.1, n_particles=1000,
                               n_population=10000, mu=20, chains=8, seed=77, mh_ratio="log")
    burn = 300
    draws = [np.asarray(r.thetas)[burn:] for r in res]
    truth = np.array([0.25, 0.1])
    for d in draws:
        assert np.all(np.abs(d.mean(axis=0) / truth - 1) < 0.10), d.mean(axis=0)
    rhat = gelman_rubin(draws)
    print("posterior means", [np.round(d.mean(axis=0), 4).tolist() for d in draws], "R-hat", rhat)
    assert np.all(rhat < 1.1), rhat
    for r in res:
        th = np.asarray(r.thetas)
        acc = len(np.unique(th[:, 0])) / len(th)
        assert 0.01 < acc < 0.9, acc
