"""Chain results on disk in the reference's layout, warm-start resume, and the Gelman-Rubin statistic.

  save_run / load_run     tests/experiments/pobs/prob_.05.py:50-61: `thetas.csv [iters, d]`,
                          `likelihoods.csv [iters]`, `sampled_trajs_<compartment>.csv [T, iters]`
                          written with np.savetxt(..., delimiter=",")
  warm_start              tests/test_pmcmc_noisy.py:32-40 (and tests/test_under.py:37-49): start at the
                          last draw, proposal covariance from the unique burned-in, thinned draws (ddof=0)
  gelman_rubin            helpers.py:15-43 gelman_rubin_test (potential scale reduction per parameter)
  hdi / mean_credible_interval, running_mean, posterior_mse
                          helpers.py:5-13, :46-48, :51-54 -- the reference's posterior summaries (its HDI is
                          arviz's, which is not installed: restated as arviz computes it, the narrowest interval
                          holding floor(0.95 n) + 1 sorted draws)
"""
import os

import numpy as np

COMPARTMENTS = {3: ("susceptible", "infected", "recovered"),
                4: ("susceptible", "exposed", "infected", "recovered")}


def compartment_names(C):
    """Reference names for SIR/SEIR; `s{g}`, `i{g}`, `r{g}` per group for the subgroup models."""
    if C in COMPARTMENTS:
        return COMPARTMENTS[C]
    return tuple(f"{k}{g}" for g in range(C // 3) for k in ("susceptible", "infected", "recovered"))


def save_run(directory, thetas, likelihoods, sampled_trajs):
    """np.savetxt the three outputs of particle_mcmc exactly as the reference's experiment scripts do.
    sampled_trajs is [T, iters, C] (particle_mcmc's return layout)."""
    os.makedirs(directory, exist_ok=True)
    np.savetxt(os.path.join(directory, "thetas.csv"), np.asarray(thetas), delimiter=",")
    np.savetxt(os.path.join(directory, "likelihoods.csv"), np.asarray(likelihoods), delimiter=",")
    tr = np.asarray(sampled_trajs)
    for c, name in enumerate(compartment_names(tr.shape[2])):
        np.savetxt(os.path.join(directory, f"sampled_trajs_{name}.csv"), tr[:, :, c], delimiter=",")


def load_run(directory, C=None):
    """Inverse of save_run: (thetas [iters, d], likelihoods [iters], sampled_trajs [T, iters, C] or None)."""
    thetas = np.loadtxt(os.path.join(directory, "thetas.csv"), delimiter=",", ndmin=2)
    likelihoods = np.loadtxt(os.path.join(directory, "likelihoods.csv"), delimiter=",", ndmin=1)
    trajs = None
    names = compartment_names(C) if C else next(
        (v for v in (COMPARTMENTS[4], COMPARTMENTS[3])
         if all(os.path.exists(os.path.join(directory, f"sampled_trajs_{n}.csv")) for n in v)), None)
    if names:
        cols = [np.loadtxt(os.path.join(directory, f"sampled_trajs_{n}.csv"), delimiter=",", ndmin=2) for n in names]
        trajs = np.stack(cols, axis=2)
    return thetas, likelihoods, trajs


def warm_start(thetas, burn_in=100, thin=20):
    """(theta_proposal, sigma) for resuming a run, tests/test_pmcmc_noisy.py:35-40:
    thetas[burn_in:][::thin] -> unique rows -> np.cov(.T, ddof=0); start at thetas[-1]."""
    thetas = np.asarray(thetas, dtype=np.float64)
    kept = np.unique(thetas[burn_in:][::thin], axis=0)
    return thetas[-1].tolist(), np.cov(kept.T, ddof=0)


def gelman_rubin(chains):
    """helpers.py:15-43: R-hat per parameter for M chains of equal length N ([N, d] each)."""
    chains = [np.asarray(c, dtype=np.float64) for c in chains]
    M = len(chains)
    N, d = chains[0].shape
    means = np.zeros((M, d))
    var = np.zeros((M, d))
    for m, c in enumerate(chains):          # per column, same reductions and rounding as the reference
        for k in range(d):
            mk = np.mean(c[:, k])
            var[m, k] = 1.0 / (N - 1) * np.sum((c[:, k] - mk) ** 2)
            means[m, k] = mk
    theta_hat = np.mean(means, axis=0)
    W = np.mean(var, axis=0)
    B = N / (M - 1) * ((means - theta_hat) ** 2).sum(axis=0)
    V = (N - 1) / N * W + (M + 1) / (M * N) * B
    return np.sqrt(V / W)


def hdi(samples, hdi_prob=0.95):
    """arviz.hdi of the flattened draws (a 2-D array is (chain, draw), as arviz reads it): with the draws sorted,
    k = floor(hdi_prob n) and the interval [x_i, x_{i+k}] of least width, the first one on ties."""
    x = np.sort(np.asarray(samples, dtype=np.float64).reshape(-1))
    n = x.size
    k = int(np.floor(hdi_prob * n))
    width = x[k:] - x[:n - k]
    i = int(np.argmin(width))
    return np.array([x[i], x[i + k]])


def mean_credible_interval(data, alpha=0.95):
    """helpers.py:5-13: (mean, hdi_low, hdi_high); the mean per row for 2-D data, the HDI (95%, as the reference:
    it never passes `alpha` on) over all draws."""
    a = np.array(data)
    m = np.mean(a, axis=1) if len(a.shape) == 2 else np.mean(a)
    return (m, *hdi(a, 0.95))


def running_mean(x, N):
    """helpers.py:46-48: the length-N moving average of x."""
    cumsum = np.cumsum(np.insert(x, 0, 0))
    return (cumsum[N:] - cumsum[:-N]) / float(N)


def posterior_mse(true_prm, chain):
    """helpers.py:51-54: mean squared error of the draws against the true parameter."""
    return np.mean((chain - true_prm) ** 2)
