"""Synthetic observation datasets, restating the reference's own recipes.

  differential_sir / _seir / _sir_subgroups     pmcmc.py:16-51   (ODE right-hand sides, same expression order)
  *_simulate_discrete                            pmcmc.py:54-113  (odeint, then the last sample of each ceil-day)
  thin_binomial                                  tests/test_pmcmc_p.py:21-29, tests/test_simulations_subgroups.py:57-64
  noise_normal                                   tests/test_pmcmc_noisy.py:21-29 (Gaussian noise, cast to int)
Returned arrays drop the reference's pandas DataFrame wrapper: discrete series are [days, 1 + C] with the
time column first (the DataFrame's column order for SIR/SEIR).  `benchmark_dataset(cfg)` builds the
BASELINE.json configurations.
"""
import numpy as np


def differential_sir(n_sir, t, beta, gamma):
    N = sum(n_sir)
    dS_dt = -beta * n_sir[0] * n_sir[1] / N
    dI_dt = ((beta * n_sir[0] / N) - gamma) * n_sir[1]
    dR_dt = gamma * n_sir[1]
    return dS_dt, dI_dt, dR_dt


def differential_seir(n_seir, t, beta, alpha, gamma):
    N = sum(n_seir)
    dS_dt = -beta * n_seir[0] * n_seir[2] / N
    dE_dt = beta * n_seir[0] * n_seir[2] / N - alpha * n_seir[1]
    dI_dt = alpha * n_seir[1] - gamma * n_seir[2]
    dR_dt = gamma * n_seir[2]
    return dS_dt, dE_dt, dI_dt, dR_dt


def differential_sir_subgroups(n_sir, t, beta, gamma):
    G = len(beta)
    N = sum(n_sir)
    out = []
    idx = [1 + 3 * j for j in range(G)]
    for i in range(G):
        force = sum(beta[i] * n_sir[idx])
        out += [-n_sir[i * 3] * force / N, n_sir[i * 3] * force / N - gamma * n_sir[i * 3 + 1],
                gamma * n_sir[i * 3 + 1]]
    return tuple(out)


def _last_sample_per_day(t, solution):
    days = np.ceil(t).astype(int)
    rows = [int(np.nonzero(days == i)[0][-1]) for i in range(days[-1] + 1)]
    return rows


def sir_simulate_discrete(y0, t, beta, gamma):
    from scipy.integrate import odeint
    sol = odeint(differential_sir, y0, t, args=(beta, gamma))
    rows = _last_sample_per_day(t, sol)
    return np.column_stack([np.asarray(t)[rows], sol[rows]])


def seir_simulate_discrete(y0, t, beta, alpha, gamma):
    from scipy.integrate import odeint
    sol = odeint(differential_seir, y0, t, args=(beta, alpha, gamma))
    rows = _last_sample_per_day(t, sol)
    return np.column_stack([np.asarray(t)[rows], sol[rows]])


def sir_subgroups_simulate_discrete(y0, t, beta, gamma):
    """Columns: S0, I0, R0, S1, ... then time LAST (pmcmc.py:99-113 DataFrame order)."""
    from scipy.integrate import odeint
    y0 = [i for item in np.asarray(y0).tolist() for i in item]
    sol = odeint(differential_sir_subgroups, y0, t, args=(np.asarray(beta).tolist(), gamma))
    rows = _last_sample_per_day(t, sol)
    return np.column_stack([sol[rows], np.asarray(t)[rows]])


def thin_binomial(values, prob, rs):
    return np.array([[rs.binomial(v, prob) for v in row] for row in values], dtype=np.float64)


def noise_normal(values, ratio, rs):
    return np.array([[rs.normal(v, ratio * v) for v in row] for row in values]).astype(int).astype(np.float64)


def benchmark_dataset(cfg):
    """Observation matrices for the BASELINE.json configs.  Returns (Y, meta)."""
    if cfg == 1:
        ode = sir_simulate_discrete((180, 20, 0), np.linspace(0, 49, num=500), 2, 1)[:, 1:]
        return thin_binomial(ode, 0.1, np.random.RandomState(2)), dict(
            model="sir", n_population=200, mu=20, theta=(2.0, 1.0), probs=0.1, N=100,
            describe="ODE SIR y0=(180,20,0), beta=2, gamma=1, 50 daily rows, binomial thinning p=.1, RandomState(2)")
    if cfg == 2:
        ode = sir_simulate_discrete((9980, 20, 0), np.linspace(0, 199, num=2000), 0.25, 0.1)[:, 1:]
        return thin_binomial(ode, 0.1, np.random.RandomState(1)), dict(
            model="sir", n_population=10000, mu=20, theta=(0.25, 0.1), probs=0.1, N=10000,
            describe="ODE SIR y0=(9980,20,0), beta=.25, gamma=.1, 200 daily rows, binomial thinning p=.1, "
                     "RandomState(1)")
    if cfg == 3:
        ode = seir_simulate_discrete((9980, 0, 20, 0), np.linspace(0, 199, num=2000), 0.5, 0.2, 0.1)[:, 1:]
        return noise_normal(ode, 0.1, np.random.RandomState(3)), dict(
            model="seir", n_population=10000, mu=20, theta=(0.5, 0.2, 0.1), probs=0.1, observations=True, N=10000,
            describe="ODE SEIR y0=(9980,0,20,0), beta=.5, alpha=.2, gamma=.1, 200 daily rows, Gaussian noise "
                     "N(x, .1x) cast to int, RandomState(3); normal observation model")
    if cfg == 4:
        ode = sir_simulate_discrete((4800, 20, 0), np.linspace(0, 14, num=200), 2, 1)[:, 1:]
        return thin_binomial(ode, 0.1, np.random.RandomState(11)), dict(
            model="sir", n_population=4820, mu=20, theta=(2.0, 1.0), probs=0.1, N=50000,
            describe="ODE SIR y0=(4800,20,0), beta=2, gamma=1, 15 daily rows, binomial thinning p=.1 "
                     "(under-reported counts), RandomState(11)")
    if cfg == 5:
        pop = np.array([[2000, 30, 0], [3000, 40, 0]])
        ode = sir_subgroups_simulate_discrete(pop, np.linspace(0, 14, num=200), np.array([[5, 2], [1, 3]]), 0.5)
        return thin_binomial(ode[:, :6], 0.1, np.random.RandomState(14)), dict(
            model="sir_subgroups", n_population=[2030, 3040], mu=[30, 40], theta=[4.0, 1.0, 1.0, 4.0, 1.0],
            probs=0.1, N=10000,
            describe="ODE 2-group SIR pop=[[2000,30,0],[3000,40,0]], beta=[[5,2],[1,3]], gamma=.5, 15 daily rows, "
                     "binomial thinning p=.1, RandomState(14)")
    raise ValueError(f"unknown benchmark config {cfg}")
