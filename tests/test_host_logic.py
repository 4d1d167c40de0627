"""Host-side MH logic (epipf.pmcmc) on CPU: the GPU engine is replaced, inside this test only, by a
stand-in that answers from the oracle, so the accept/reject / RNG-order / probs=None / subgroup /
adaptive logic is checked against the reference's own PMCMC runs (tests/golden/pmcmc_golden.npz)
without a GPU.  The product has no such fallback: epipf.engine.Engine always requires libepipf + a GPU."""
import sys

import numpy as np
import pytest

from epipf import pmcmc as pm
from oracle_engine import fake_get_engine


@pytest.fixture
def oracle_engine(monkeypatch):
    monkeypatch.setattr(pm, "get_engine", fake_get_engine)


@pytest.mark.parametrize("name", ["sir_small", "sir_p", "sub", "cfg1_full", "test_pmcmc_p"])
def test_mh_loop_reproduces_reference_trace(oracle_engine, pmcmc_golden, name):
    rec = pmcmc_golden["pmcmc_" + name]
    model = str(rec["model"])
    sub = model.startswith("SIR_SUB")
    sigma = None if rec["sigma"].size == 0 else rec["sigma"]
    probs = None if float(rec["probs"]) < 0 else float(rec["probs"])
    pm.seed_stream(int(rec["key"]), 0)
    np.random.seed(int(rec["seed"]))
    th, lk, tr = pm.particle_mcmc(rec["Y"], model.lower(), list(rec["params"]), float(rec["h"]),
                                  adaptive=bool(rec["adaptive"]), sigma=sigma, n_chains=int(rec["iters"]),
                                  probs=probs, n_particles=int(rec["N"]),
                                  n_population=rec["npop"] if sub else float(rec["npop"][0]),
                                  mu=rec["mu"] if sub else float(rec["mu"][0]), progress=False, prefetch=0)
    np.testing.assert_array_equal(th, rec["thetas"])
    np.testing.assert_array_equal(tr, rec["trajs"])
    np.testing.assert_allclose(lk, rec["likelihoods"], rtol=1e-9)
    assert pm._STREAM.next_filter == int(rec["n_filters"])


def test_log_ratio_matches_reference_ratio_when_finite():
    from scipy.stats import multivariate_normal  # noqa: F401
    rs = np.random.RandomState(0)
    for _ in range(200):
        lz_new, lz_old = rs.uniform(-60, -10, 2)
        th_new, th_old = rs.uniform(0.5, 2, 2), rs.uniform(0.5, 2, 2)
        ref = pm._reference_ratio(np.exp(lz_new), np.exp(lz_old), th_new, th_old, [2.0, 1.0], 0.01 * np.eye(2))
        assert abs(pm._log_ratio(lz_new, lz_old) - ref) <= 1e-9 * max(1.0, ref)


def test_log_ratio_survives_underflow():
    # zetas underflow at T~200 (pmcmc.py:183): the reference's ratio is 0/0 -> nan -> min(1, nan) = 1
    assert pm._reference_ratio(np.float64(0.0), np.float64(0.0), np.ones(2), np.ones(2), [1.0, 1.0],
                               np.eye(2)) == 1
    assert pm._log_ratio(-900.0, -905.0) == 1.0
    assert abs(pm._log_ratio(-905.0, -900.0) - np.exp(-5.0)) < 1e-15


def test_multichain_lockstep_equals_independent_runs(oracle_engine, datasets_golden):
    Y = datasets_golden["cfg1_binom"][:8]
    kw = dict(Y=Y, type_model="sir", parameters=[2.0, 1.0], h=0.02, n_chains=6, probs=0.1, n_particles=16,
              n_population=200, mu=20, mh_ratio="log")
    multi = pm.particle_mcmc_chains(**kw, chains=3, seed=5)
    for c in range(3):
        single = pm.particle_mcmc_chains(**kw, rngs=[np.random.RandomState(5 + c)], keys=[pm.chain_key(5, c)])[0]
        np.testing.assert_array_equal(single.thetas, multi[c].thetas)
        np.testing.assert_array_equal(single.sampled_trajs, multi[c].sampled_trajs)
        np.testing.assert_allclose(single.log_likelihoods, multi[c].log_likelihoods)


@pytest.mark.parametrize("d", [1, 2, 3, 5])
def test_cached_mvn_factor_equals_legacy_multivariate_normal(d):
    """ChainSampler draws proposals as mvn_apply(standard_normal(d), mvn_factor(cov), mean) with the factor cached
    per chain: the same values, bit for bit, and the same RandomState consumption as numpy's legacy
    multivariate_normal(mean, cov) (pmcmc.py:277, :330), for isotropic, correlated and adaptive-style covariances."""
    rs = np.random.RandomState(11 + d)
    for trial in range(600):
        h = 10.0 ** rs.uniform(-6, 0)
        if trial % 3 == 0:
            cov = h * np.eye(d)
        else:
            a = rs.standard_normal((d + 3, d))
            cov = h * (np.cov(a.T, ddof=0).reshape(d, d) + 1e-4 * np.eye(d))
        mean = rs.uniform(0, 3, d)
        seed = int(rs.randint(0, 2**31))
        ref, mine = np.random.RandomState(seed), np.random.RandomState(seed)
        fac = pm.mvn_factor(cov)
        for _ in range(3):
            a_ = ref.multivariate_normal(mean, cov)
            b_ = pm.mvn_apply(mine.standard_normal(d), fac, mean)
            assert a_.shape == b_.shape == (d,)
            assert np.array_equal(a_, b_), (cov, a_, b_)
        assert ref.uniform() == mine.uniform()          # same stream position afterwards


def test_pipelined_samplers_equal_one_lockstep_sampler(datasets_golden):
    """run_pipelined (one host thread + private engine per chain group, bench.py --pipelines) gives every chain
    exactly the draws, likelihoods and trajectories of one lockstep ChainSampler over all chains."""
    from oracle_engine import OracleEngine
    Y = datasets_golden["cfg1_binom"][:8]
    kw = dict(Y=Y, type_model="sir", parameters=[2.0, 1.0], h=0.02, iters=7, probs=0.1, n_particles=16,
              n_population=200, mu=20, mh_ratio="log")
    ids = list(range(5))
    whole = pm.ChainSampler(**kw, rngs=[np.random.RandomState(30 + g) for g in ids],
                            keys=[pm.chain_key(30, g) for g in ids], engine=OracleEngine(0, 1, 16, 8, 5))
    whole.initialise()
    ran = sum(whole.step() for _ in range(6))
    groups = [[0, 1], [2], [3, 4]]
    parts = [pm.ChainSampler(**kw, rngs=[np.random.RandomState(30 + g) for g in grp],
                             keys=[pm.chain_key(30, g) for g in grp], engine=OracleEngine(0, 1, 16, 8, len(grp)))
             for grp in groups]
    for s in parts:
        s.initialise()
    switch = sys.getswitchinterval()
    assert pm.run_pipelined(parts, 6) == ran
    assert sys.getswitchinterval() == switch          # lowered only while the threads run
    got = [r for s in parts for r in s.results()]
    for a, b in zip(whole.results(), got):
        np.testing.assert_array_equal(a.thetas, b.thetas)
        np.testing.assert_array_equal(a.log_likelihoods, b.log_likelihoods)
        np.testing.assert_array_equal(a.sampled_trajs, b.sampled_trajs)
        assert a.acceptances == b.acceptances and a.filters_run == b.filters_run
    with pytest.raises(ValueError):
        pm.run_pipelined([parts[0], parts[0]], 1)
    from epipf.distributed import pack_draws
    for upto in (None, 3, whole.i):                   # bench.py's vectorised gather rows == pack_draws(results())
        np.testing.assert_array_equal(whole.packed_draws(upto), pack_draws(whole.results(), upto=upto))
        np.testing.assert_array_equal(np.concatenate([s.packed_draws(upto) for s in parts]),
                                      pack_draws(got, upto=upto))


def test_random_sample_is_legacy_uniform():
    """The MH acceptance draw (pmcmc.py:395, np.random.uniform()) is taken as random_sample(): legacy uniform is
    low + (high - low) * random_sample() = 0 + 1 * U, the same double and the same stream consumption."""
    a, b = np.random.RandomState(9), np.random.RandomState(9)
    for _ in range(20000):
        assert a.uniform() == b.random_sample()
        a.standard_normal(2), b.standard_normal(2)
    assert a.randint(0, 1000) == b.randint(0, 1000)
    np.random.seed(4)
    x = np.random.uniform()
    np.random.seed(4)
    assert np.random.random_sample() == x


@pytest.mark.parametrize("probs", [0.1, None])
def test_c_host_draws_equal_the_python_loop(datasets_golden, probs):
    """More than FUSE_PATH_CHAINS chains take the C host draws (epipf_mh_propose / epipf_mh_decide, csrc/host_mh.cpp):
    thetas, likelihoods, trajectories, counters and every chain's final RandomState equal the Python loop's
    (host_draws=False).  probs=None: d = 3, odd, so that run keeps the Python loop -- checked too."""
    from oracle_engine import OracleEngine
    Y = datasets_golden["cfg1_binom"][:6]
    nc = 20
    params = [2.0, 1.0] if probs is not None else [2.0, 1.0, 0.1]
    kw = dict(Y=Y, type_model="sir", parameters=params, h=0.05, iters=12, probs=probs, n_particles=12,
              n_population=200, mu=20, mh_ratio="log")
    runs = []
    for hd in (True, False):
        rngs = [np.random.RandomState(50 + c) for c in range(nc)]
        s = pm.ChainSampler(**kw, rngs=rngs, keys=[pm.chain_key(50, c) for c in range(nc)],
                            engine=OracleEngine(0, 1, 12, 6, nc), host_draws=hd)
        assert (s._host is not None) == (hd and probs is not None)
        res = s.run()
        runs.append((res, [r.get_state() for r in rngs]))
    (ra, sa), (rb, sb) = runs
    for a, b in zip(ra, rb):
        np.testing.assert_array_equal(a.thetas, b.thetas)
        np.testing.assert_array_equal(a.log_likelihoods, b.log_likelihoods)
        np.testing.assert_array_equal(a.sampled_trajs, b.sampled_trajs)
        assert a.acceptances == b.acceptances and a.filters_run == b.filters_run
    for u, v in zip(sa, sb):
        assert np.array_equal(u[1], v[1]) and u[2:] == v[2:]
