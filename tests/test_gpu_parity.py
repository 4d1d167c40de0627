"""Parity of the HIP path (libepipf.so through its C ABI) with the reference golden vectors and the
CPU oracle.  Integer outputs (states, ancestors, trajectories) must be bit-exact; log-likelihoods
within 1e-9 absolute (1e-6 relative is the north-star bound).  Needs an MI355X: `-m gpu`."""
import numpy as np
import pytest

import oracle
import reference_replay
from conftest import case_args

pytestmark = pytest.mark.gpu

FILTER_CASES = ["sir_binom", "sir_normal", "seir_binom", "sub_binom", "sub2_binom", "cfg1_sir", "cfg2_sir",
                "cfg3_seir_normal", "sir_theta_off", "degenerate"]


def engine_for(a, chains=1, lanes=0):
    """The cached engine for a case; lanes: SSA lanes per particle (0 = automatic: the lane-group kernel for runs
    below ~8 chains of 10^4 particles, 1 = the one-lane kernel), set on every call."""
    from epipf.engine import get_engine, model_id, theta_vector
    mid = model_id(a["model"])
    th, G = theta_vector(mid, a["theta"])
    eng = get_engine(mid, G, a["N"], a["Y"].shape[0], chains)
    eng.set_observations(a["Y"])
    eng.set_population(a["npop"], a["mu"])
    eng.set_lanes(lanes)
    return eng, th


@pytest.mark.parametrize("name", FILTER_CASES)
def test_filter_matches_reference_golden(filter_golden, name):
    rec = filter_golden["filter_" + name]
    a = case_args(rec)
    eng, th = engine_for(a)
    lz, st = eng.run(th[None], [a["probs"]], [a["key"]], [a["f"]], observations=a["observations"])
    assert int(st[0]) == int(rec["status"])
    if st[0]:
        return
    hid, anc = eng.history(1)
    np.testing.assert_array_equal(hid[0], rec["hidden"])
    np.testing.assert_array_equal(anc[0], rec["ancestry"])
    z = rec["zetas"]
    ok = z > 1e-290
    np.testing.assert_allclose(lz[0][ok], np.log(z[ok]), rtol=0, atol=1e-9)


@pytest.mark.parametrize("lanes", [0, 1])
@pytest.mark.parametrize("name", FILTER_CASES)
def test_filter_matches_oracle(filter_golden, name, lanes):
    rec = filter_golden["filter_" + name]
    a = case_args(rec)
    eng, th = engine_for(a, lanes=lanes)
    lz, st = eng.run(th[None], [a["probs"]], [a["key"]], [a["f"]], observations=a["observations"])
    o = oracle.particle_filter(a["Y"], a["model"], a["theta"], a["observations"], a["probs"], a["N"], a["npop"],
                               a["mu"], key=a["key"], filter_index=a["f"])
    assert int(st[0]) == o["status"]
    if o["status"]:
        return
    hid, anc = eng.history(1)
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("lanes", [0, 1])
@pytest.mark.parametrize("seed", range(6))
def test_filter_random_configs_vs_oracle(datasets_golden, seed, lanes):
    """Seeded random (theta, N, key) on every model: bit-exact states/ancestors vs the oracle."""
    rs = np.random.RandomState(100 + seed)
    model = ["sir", "seir", "sir_subgroups", "sir_subgroups2", "sir", "seir"][seed]
    obs = bool(seed >= 4)
    N = int(rs.choice([1, 7, 64, 65, 300, 1000]))
    if model == "sir":
        Y, th, npop, mu = datasets_golden["sir_noisy" if obs else "sir_binom"], rs.uniform(1.5, 2.5, 2) * [1, .5], 4820, 20
        probs = 0.5 if obs else 0.1
    elif model == "seir":
        Y, th, npop, mu = datasets_golden["seir_binom"], rs.uniform(0.8, 1.2, 3) * [4, 1, 1], 4820, 20
        probs = 0.3 if obs else 0.1
    else:
        Y = datasets_golden["sub_binom" if model == "sir_subgroups" else "sub2_binom"][:6]
        th = (np.array([[5, 2], [1, 3]]) * rs.uniform(0.8, 1.2, (2, 2)), 0.5)
        npop, mu, probs = np.array([2030., 3040.]), np.array([30., 40.]), 0.1
        N = min(N, 300)
    a = dict(Y=Y, model=model, theta=th, observations=obs, probs=probs, N=N, npop=npop, mu=mu,
             key=int(rs.randint(1, 2**31)), f=int(rs.randint(0, 1000)))
    eng, thv = engine_for(a, lanes=lanes)
    lz, st = eng.run(thv[None], [probs], [a["key"]], [a["f"]], observations=obs)
    o = oracle.particle_filter(Y, model, th, obs, probs, N, npop, mu, key=a["key"], filter_index=a["f"])
    assert int(st[0]) == o["status"]
    if o["status"]:
        return
    hid, anc = eng.history(1)
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("N,chains", [(12800, 1), (12865, 2), (50000, 2), (140000, 1)])
def test_filter_segmented_block_prefix_vs_oracle(datasets_golden, N, chains):
    """N past 200 blocks of 64: the block-sum prefix is segmented (S = 2, 4, 16 blocks per segment; level 2 of the
    resampling search walks a segment in global memory).  Bit-exact states/ancestors vs the oracle; every chain of a
    batch, at the config-4 shape (pop 4820, ~500 events per particle-step)."""
    Y = datasets_golden["sir_binom"][:4]
    a = dict(Y=Y, model="sir", theta=(2.0, 1.0), N=N, npop=4820, mu=20)
    eng, thv = engine_for(a, chains)
    keys = [77 + c for c in range(chains)]
    lz, st = eng.run(np.repeat(thv[None], chains, 0), [0.1] * chains, keys, [3] * chains)
    hid, anc = eng.history(chains)
    for c in range(chains):
        o = oracle.particle_filter(Y, "sir", (2.0, 1.0), False, 0.1, N, 4820, 20, key=keys[c], filter_index=3)
        assert int(st[c]) == o["status"] == 0
        np.testing.assert_array_equal(hid[c], o["hidden"])
        np.testing.assert_array_equal(anc[c], o["ancestry"])
        np.testing.assert_allclose(lz[c], o["log_zetas"], rtol=1e-12, atol=1e-9)


def test_batched_chains_equal_single_runs(datasets_golden):
    """Chain c of a batched launch is bit-identical to running it alone (no cross-chain coupling),
    and inactive chains are skipped."""
    Y = datasets_golden["sir_binom"]
    a = dict(Y=Y, model="sir", theta=(2.0, 1.0), N=200, npop=4820, mu=20)
    eng, _ = engine_for(a, chains=5)
    thetas = np.array([[2.0, 1.0], [2.2, 0.9], [1.8, 1.1], [2.0, 1.0], [2.5, 1.3]])
    keys = np.array([11, 12, 13, 14, 15], dtype=np.uint64)
    fidx = np.array([0, 3, 5, 7, 9])
    act = np.array([1, 1, 0, 1, 1])
    lz, st = eng.run(thetas, 0.1, keys, fidx, active=act)
    assert list(st) == [0, 0, 2, 0, 0]
    hid, anc = eng.history(5)
    for c in (0, 1, 3, 4):
        o = oracle.particle_filter(Y, "sir", thetas[c], False, 0.1, 200, 4820, 20, key=int(keys[c]),
                                   filter_index=int(fidx[c]))
        np.testing.assert_array_equal(hid[c], o["hidden"])
        np.testing.assert_array_equal(anc[c], o["ancestry"])
        np.testing.assert_allclose(lz[c], o["log_zetas"], rtol=1e-12, atol=1e-9)


def test_deterministic_reruns(datasets_golden):
    Y = datasets_golden["cfg2_binom"]
    a = dict(Y=Y, model="sir", theta=(0.25, 0.1), N=2000, npop=10000, mu=20)
    eng, th = engine_for(a)
    r1 = eng.run(th[None], 0.1, 7, 1)
    h1 = eng.history(1)
    r2 = eng.run(th[None], 0.1, 7, 1)
    h2 = eng.history(1)
    np.testing.assert_array_equal(r1[0], r2[0])
    np.testing.assert_array_equal(h1[0], h2[0])
    np.testing.assert_array_equal(h1[1], h2[1])


@pytest.mark.parametrize("name", ["sir_1.0", "sir_2.5", "sir_edge_1.0", "sir_edge_2.5", "seir_1.0", "seir_2.5",
                                  "sub_1.0", "sub_2.5"])
def test_simulate_matches_reference_golden(kernels_golden, name):
    from epipf import simulate_batch
    rec = kernels_golden["ssa_" + name]
    model = str(rec["model"])
    theta = (rec["theta"][:4].reshape(2, 2), float(rec["theta"][4])) if model == "sub" else rec["theta"]
    mname = {"sir": "sir", "seir": "seir", "sub": "sir_subgroups"}[model]
    out, _ = simulate_batch(mname, rec["states"], theta, float(rec["max_time"]), key=int(rec["key"]),
                            filter_index=int(rec["f"]), step=int(rec["step"]))
    np.testing.assert_array_equal(out, rec["out"])


def test_simulate_large_batch_vs_oracle():
    from epipf import simulate_batch
    rs = np.random.RandomState(3)
    n = 20000
    I = rs.randint(0, 500, n)
    R = rs.randint(0, 500, n)
    st = np.stack([10000 - I - R, I, R], 1)
    out, ev = simulate_batch("sir", st, (0.25, 0.1), 3.0, key=123, filter_index=4, step=9)
    o, oev = oracle.simulate("sir", st, (0.25, 0.1), 3.0, 123, 4, 9)
    np.testing.assert_array_equal(out, o)
    assert ev == oev
    np.testing.assert_array_equal(out.sum(1), 10000)  # conservation


@pytest.mark.parametrize("n", [1, 2, 5, 64, 257, 1000])
def test_resample_matches_numpy_choice(kernels_golden, n):
    from epipf.engine import get_engine
    rec = kernels_golden[f"resample_{n}"]
    eng = get_engine("sir", 1, 8, 2, 1)
    out, _ = eng.resample(rec["w"], rec["u"])
    np.testing.assert_array_equal(out, rec["expected"])


@pytest.mark.parametrize("n", [3000, 4097, 20001])
def test_resample_ties_take_the_exact_path(n):
    """Uniforms placed exactly on (and one ulp around) numpy's CDF boundaries: the certified search must
    hand them to the wave-cooperative exact path (many such lanes per wave, ragged last chunk) and still
    equal numpy's answer."""
    from epipf.engine import get_engine
    eng = get_engine("sir", 1, 8, 2, 1)
    rs = np.random.RandomState(5 + n)
    w = rs.random_sample(n) ** 4
    w[rs.random_sample(n) < 0.2] = 0.0
    p = w / sum(w)
    cdf = p.cumsum()
    cdf /= cdf[-1]
    idx = rs.randint(0, n - 1, 300)
    u = np.concatenate([cdf[idx], np.nextafter(cdf[idx], 0), np.nextafter(cdf[idx], 1), rs.random_sample(100)])
    u = np.resize(u[(u >= 0) & (u < 1)], n)
    out, fb = eng.resample(w, u)
    np.testing.assert_array_equal(out, oracle.resample(w, u))
    assert fb > 0


def test_resample_degenerate_weights():
    from epipf.engine import get_engine
    eng = get_engine("sir", 1, 8, 2, 1)
    out, _ = eng.resample(np.zeros(100), np.full(100, 0.5))
    assert out is None


def test_path_sampler_matches_host_version(filter_golden):
    from epipf import particle_path_sampler
    rec = filter_golden["filter_sir_binom"]
    a = case_args(rec)
    eng, th = engine_for(a)
    eng.run(th[None], [a["probs"]], [a["key"]], [a["f"]])
    hid, anc = eng.history(1)
    for chosen in (0, 5, a["N"] - 1):
        dev = eng.path_sample([chosen])[0]
        np.random.seed(0)
        # host reference implementation with the same pick
        traj = np.zeros((hid.shape[1], hid.shape[3]))
        traj[-1] = hid[0, -1, chosen]
        c = chosen
        for p in range(hid.shape[1] - 2, -1, -1):
            c = int(anc[0, p, c])
            traj[p] = hid[0, p, c]
        np.testing.assert_array_equal(dev, traj)
    np.random.seed(3)
    host = particle_path_sampler(hid[0].astype(float), anc[0].astype(float))
    np.random.seed(3)
    dev = eng.path_sample([np.random.randint(0, a["N"])])[0]
    np.testing.assert_array_equal(dev, host)


def test_dropin_particle_filter_signature(filter_golden):
    from epipf import ModelType, particle_filter, seed_stream
    rec = filter_golden["filter_seir_binom"]
    a = case_args(rec)
    seed_stream(a["key"], a["f"])
    z, hid, anc = particle_filter(a["Y"], ModelType.SEIR, np.array(a["theta"]), False, a["probs"], a["N"],
                                  a["npop"], a["mu"], jobs=-1)
    np.testing.assert_array_equal(hid, rec["hidden"].astype(float))
    np.testing.assert_array_equal(anc, rec["ancestry"].astype(float))
    np.testing.assert_allclose(z, rec["zetas"], rtol=1e-9)
    assert hid.dtype == np.float64 and anc.dtype == np.float64
    rec = filter_golden["filter_degenerate"]
    a = case_args(rec)
    assert particle_filter(a["Y"], "sir", a["theta"], n_particles=a["N"], key=a["key"], filter_index=0) == \
        (None, None, None)


@pytest.mark.parametrize("prefetch", [0, 32, "auto"])
@pytest.mark.parametrize("name", ["sir_small", "sir_p", "sub", "sir_adaptive", "cfg1_full", "test_pmcmc_p"])
def test_pmcmc_matches_reference_golden(pmcmc_golden, name, prefetch):
    """particle_mcmc under np.random.seed(s) + seed_stream(key): identical accept/reject trace, thetas,
    sampled trajectories; likelihoods within 1e-9 relative.  cfg1_full is BASELINE config 1 itself (N=100, pop 200,
    T=50, 500 MH iterations) and test_pmcmc_p the reference's tests/test_pmcmc_p.py shape (N=100, pop 4820, T=15,
    probs=None, h=5 and its Sigma), both run through the unmodified reference (tests/golden/make_golden.py)."""
    from epipf import particle_mcmc, seed_stream
    rec = pmcmc_golden["pmcmc_" + name]
    model = str(rec["model"])
    G = len(rec["npop"])
    npop = rec["npop"] if model.startswith("SIR_SUB") else float(rec["npop"][0])
    mu = rec["mu"] if model.startswith("SIR_SUB") else float(rec["mu"][0])
    sigma = None if rec["sigma"].size == 0 else rec["sigma"]
    probs = None if float(rec["probs"]) < 0 else float(rec["probs"])
    seed_stream(int(rec["key"]), 0)
    np.random.seed(int(rec["seed"]))
    th, lk, tr = particle_mcmc(rec["Y"], model.lower(), list(rec["params"]), float(rec["h"]),
                               adaptive=bool(rec["adaptive"]), sigma=sigma, n_chains=int(rec["iters"]),
                               probs=probs, n_particles=int(rec["N"]), n_population=npop, mu=mu, progress=False,
                               prefetch=prefetch)
    assert G >= 1
    np.testing.assert_array_equal(th, rec["thetas"])
    np.testing.assert_array_equal(tr, rec["trajs"])
    np.testing.assert_allclose(lk, rec["likelihoods"], rtol=1e-9)


@pytest.mark.parametrize("slots", [5, 48])
def test_prefetch_equals_lockstep_on_device(datasets_golden, slots):
    """Speculative MH (epipf.prefetch) on the GPU: one config-2-shaped chain (N=2000, T=200) and a 3-chain run,
    every committed value and the final RandomState equal to the one-filter-per-iteration loop."""
    from epipf.pmcmc import ChainSampler, chain_key
    from epipf.prefetch import PrefetchSampler
    Y = datasets_golden["cfg2_binom"]
    for chains, h in ((1, 1e-4), (3, 1e-3)):
        kw = dict(iters=30, probs=0.1, n_particles=2000, n_population=10000.0, mu=20.0, mh_ratio="log")
        out = []
        for cls, extra in ((ChainSampler, {}), (PrefetchSampler, {"slots": slots})):
            rngs = [np.random.RandomState(40 + c) for c in range(chains)]
            s = cls(Y, "sir", [0.25, 0.1], h, **kw, rngs=rngs, keys=[chain_key(40, c) for c in range(chains)],
                    **extra)
            out.append((s.run(), [r.get_state() for r in rngs], s))
        (ra, sa, _), (rb, sb, pre) = out
        for x, y in zip(ra, rb):
            np.testing.assert_array_equal(x.thetas, y.thetas)
            np.testing.assert_array_equal(x.log_likelihoods, y.log_likelihoods)
            np.testing.assert_array_equal(x.sampled_trajs, y.sampled_trajs)
            assert (x.acceptances, x.filters_run) == (y.acceptances, y.filters_run)
        for u, v in zip(sa, sb):
            assert np.array_equal(u[1], v[1]) and u[2:] == v[2:]
        assert pre.rounds < 29


def test_multichain_equals_single_chain(datasets_golden):
    from epipf import particle_mcmc_chains
    Y = datasets_golden["cfg1_binom"][:20]
    kw = dict(Y=Y, type_model="sir", parameters=[2.0, 1.0], h=0.01, n_chains=15, probs=0.1, n_particles=64,
              n_population=200, mu=20, mh_ratio="log")
    multi = particle_mcmc_chains(**kw, chains=4, seed=21)
    for c in range(4):
        single = particle_mcmc_chains(**kw, rngs=[np.random.RandomState(21 + c)],
                                      keys=[multi_key(21, c)])[0]
        np.testing.assert_array_equal(single.thetas, multi[c].thetas)
        np.testing.assert_array_equal(single.sampled_trajs, multi[c].sampled_trajs)


def test_stream_groups_and_pipelines_do_not_change_results(datasets_golden):
    """epipf_set_streams (1, 3, 8 chain groups) leaves every chain bit-identical, and run_pipelined over private
    engines (bench.py --pipelines) equals one lockstep sampler over the same chains."""
    from epipf.engine import Engine
    from epipf.pmcmc import ChainSampler, chain_key, run_pipelined
    Y = datasets_golden["cfg2_binom"][:60]
    eng = Engine("sir", 1, 3000, Y.shape[0], 9)
    eng.set_observations(Y)
    eng.set_population(10000, 20)
    th = np.tile([0.25, 0.1], (9, 1)) + np.linspace(0, 0.02, 9)[:, None]
    ref = None
    for n in (1, 3, 8):
        eng.set_streams(n)
        lz, st = eng.run(th, 0.1, np.arange(9) + 50, 2)
        hid, anc = eng.history(9)
        if ref is None:
            ref = (lz, st, hid, anc)
            continue
        for x, y in zip(ref, (lz, st, hid, anc)):
            np.testing.assert_array_equal(x, y)
    with pytest.raises(Exception):
        eng.set_streams(9)
    eng.close()
    kw = dict(iters=8, probs=0.1, n_particles=2000, n_population=10000.0, mu=20.0, mh_ratio="log")
    whole = ChainSampler(Y, "sir", [0.25, 0.1], 1e-3, **kw, rngs=[np.random.RandomState(60 + g) for g in range(6)],
                         keys=[chain_key(60, g) for g in range(6)])
    whole.initialise()
    ran = sum(whole.step() for _ in range(7))
    parts = []
    for grp in ([0, 1, 2], [3], [4, 5]):
        e = Engine("sir", 1, 2000, Y.shape[0], len(grp))
        e.set_streams(1)
        parts.append(ChainSampler(Y, "sir", [0.25, 0.1], 1e-3, **kw, rngs=[np.random.RandomState(60 + g) for g in grp],
                                  keys=[chain_key(60, g) for g in grp], engine=e))
    for s in parts:
        s.initialise()
    assert run_pipelined(parts, 7) == ran
    for a, b in zip(whole.results(), [r for s in parts for r in s.results()]):
        np.testing.assert_array_equal(a.thetas, b.thetas)
        np.testing.assert_array_equal(a.log_likelihoods, b.log_likelihoods)
        np.testing.assert_array_equal(a.sampled_trajs, b.sampled_trajs)
    for s in parts:
        s.eng.close()


def multi_key(seed, c):
    from epipf import chain_key
    return chain_key(seed, c)


def test_systematic_resampling_vs_oracle(datasets_golden):
    Y = datasets_golden["sir_binom"]
    a = dict(Y=Y, model="sir", theta=(2.0, 1.0), N=500, npop=4820, mu=20)
    eng, th = engine_for(a)
    lz, st = eng.run(th[None], 0.1, 77, 2, resample="systematic")
    o = oracle.particle_filter(Y, "sir", (2.0, 1.0), False, 0.1, 500, 4820, 20, key=77, filter_index=2,
                               resample="systematic")
    hid, anc = eng.history(1)
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_array_equal(hid[0], o["hidden"])


@pytest.mark.parametrize("lanes", [1, 0])
def test_full_size_cfg2_properties(datasets_golden, lanes):
    """BASELINE config 2 at full size (N=10,000, T=200), one-lane and lane-group kernels: conservation, ancestor
    range, states / ancestors / log-likelihoods vs the oracle (threaded C)."""
    Y = datasets_golden["cfg2_binom"]
    a = dict(Y=Y, model="sir", theta=(0.25, 0.1), N=10000, npop=10000, mu=20)
    eng, th = engine_for(a, lanes=lanes)
    lz, st = eng.run(th[None], 0.1, 2024, 0)
    assert st[0] == 0
    hid, anc = eng.history(1)
    assert np.all(hid[0].sum(axis=2) == 10000)
    assert anc.min() >= 0 and anc.max() < 10000
    o = oracle.particle_filter(Y, "sir", (0.25, 0.1), False, 0.1, 10000, 10000, 20, key=2024, filter_index=0)
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-8)


def _engine_with_fast_ssa(enabled, N, T, chains, model="sir", groups=1, slack=None):
    """A fresh context with the certified f32 event loop on or off (EPIPF_SSA_FAST is read at create), and
    optionally its clock band widened `slack` times (EPIPF_CLOCK_SLACK: more replays, same results).  One lane per
    particle: these tests are about the one-lane kernel's f32 loop and its replays (the lane-group kernel has its
    own in tests/test_gpu_lanes.py)."""
    import os
    from epipf.engine import Engine
    env = {"EPIPF_SSA_FAST": "1" if enabled else "0", "EPIPF_CLOCK_SLACK": None if slack is None else str(slack)}
    old = {k: os.environ.get(k) for k in env}
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    try:
        eng = Engine(model, groups, N, T, chains)
        eng.set_lanes(1)
        return eng
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("model,groups,ds,theta,npop,obs", [
    ("sir", 1, "cfg2_binom", [[0.25, 0.1], [0.5, 0.2], [0.3, 0.05]], 10000.0, False),
    ("seir", 1, "cfg3_noisy", [[0.5, 0.2, 0.1], [0.9, 0.3, 0.2], [0.4, 0.2, 0.05]], 10000.0, True),
    ("sir_subgroups", 2, "sub_binom", [[5.0, 2.0, 1.0, 3.0, 0.5], [4.0, 2.0, 1.0, 3.0, 0.5], [5.0, 1.5, 1.0, 2.5, 0.6]],
     [2030.0, 3040.0], False),
])
@pytest.mark.parametrize("slack", [300, 30000])
def test_replays_on_purpose_equal_exact_path(datasets_golden, model, groups, ds, theta, npop, obs, slack):
    """Stress the replay path: the f32 loop's clock band widened 300x / 30000x hands a large share of particle-steps
    to the replay (the wave-cooperative one for SIR / SEIR, the per-lane exact loop for subgroups); states,
    ancestors and likelihoods stay bit-identical to the exact loop's."""
    Y = datasets_golden[ds][:40]
    N, T, C = 3000, Y.shape[0], len(theta)
    th = np.array(theta)
    out = []
    for fast, sl in ((True, slack), (False, None)):
        eng = _engine_with_fast_ssa(fast, N, T, C, model=model, groups=groups, slack=sl)
        eng.set_observations(Y)
        eng.set_population(npop, [30.0, 40.0] if groups > 1 else 20.0)
        eng.set_profiling(2)
        lz, st = eng.run(th, [0.1] * C, [31 + c for c in range(C)], [2] * C, observations=obs)
        hid, anc = eng.history(C)
        out.append((lz, st, hid, anc, eng.stats()))
        eng.close()
    (lz1, st1, h1, a1, s1), (lz0, st0, h0, a0, s0) = out
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(h1, h0)
    np.testing.assert_array_equal(a1, a0)
    np.testing.assert_array_equal(lz1, lz0)
    assert s1["events"] == s0["events"]
    assert s1["ssa_exact_lanes"] > (0.002 if slack == 300 else 0.3) * s1["particle_steps"]


def test_fast_ssa_path_equals_exact_path_at_scale(datasets_golden):
    """Config-2-sized filters (N = 10^4, T = 200, 8 chains, ~1.4e9 events): the certified f32 event loop and
    the f64 loop give bit-identical states, ancestors and likelihoods.  At this size a few thousand particle-
    steps take the replay path and a few thousand events the exact channel fallback."""
    Y = datasets_golden["cfg2_binom"]
    T, N, C = Y.shape[0], 10000, 8
    th = np.array([[0.25, 0.1], [0.3, 0.1], [0.2, 0.12], [0.25, 0.08], [0.5, 0.2], [0.25, 0.1], [0.4, 0.3],
                   [0.1, 0.05]])
    out = []
    for fast in (True, False):
        eng = _engine_with_fast_ssa(fast, N, T, C)
        eng.set_observations(Y)
        eng.set_population(10000.0, 20.0)
        eng.set_profiling(2)
        lz, st = eng.run(th, [0.1] * C, [11 + c for c in range(C)], [3] * C)
        hid, anc = eng.history(C)
        out.append((lz, st, hid, anc, eng.stats()))
        eng.close()
    (lz1, st1, h1, a1, s1), (lz0, st0, h0, a0, s0) = out
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(h1, h0)
    np.testing.assert_array_equal(a1, a0)
    np.testing.assert_array_equal(lz1, lz0)
    assert s1["events"] == s0["events"]
    assert 0 < s1["ssa_exact_lanes"] < 1e-2 * C * N * T      # replays happen, rarely


def test_fast_ssa_simulate_equals_exact_path():
    """epipf_simulate over assorted horizons and parameters, fast path on vs off (same bits)."""
    rs = np.random.RandomState(5)
    n = 20000
    st = np.stack([9000 - rs.randint(0, 3000, n), rs.randint(0, 900, n), rs.randint(0, 100, n)], 1)
    for theta, tmax in (((0.25, 0.1), 1.0), ((2.0, 1.0), 0.37), ((1.5, 0.5), 2.5), ((0.0, 0.3), 1.0),
                        ((3.0, 0.0), 1.0), ((1e-9, 1e-9), 1.0)):
        res = []
        for fast in (True, False):
            eng = _engine_with_fast_ssa(fast, 1, 1, 1)
            res.append(eng.simulate(st, np.array(theta), tmax, key=9, filter_index=1, step=4))
            eng.close()
        np.testing.assert_array_equal(res[0][0], res[1][0])
        assert res[0][1] == res[1][1]


@pytest.mark.parametrize("model,groups,ds,theta,npop,mu,obs", [
    ("seir", 1, "cfg3_noisy", [[0.5, 0.2, 0.1], [0.7, 0.3, 0.15], [0.4, 0.25, 0.05], [0.5, 0.2, 0.1]], 10000.0,
     20.0, True),
    ("sir_subgroups", 2, "sub_binom", [[5, 2, 1, 3, 0.5], [4, 1, 1, 4, 1.0], [6, 2.5, 1.5, 3, 0.6],
                                       [5, 2, 1, 3, 0.5]], [2030.0, 3040.0], [30.0, 40.0], False),
    ("sir_subgroups2", 2, "sub2_binom", [[5, 2, 1, 3, 0.5], [4, 1, 1, 4, 1.0], [6, 2.5, 1.5, 3, 0.6],
                                         [5, 2, 1, 3, 0.5]], [2030.0, 3040.0], [30.0, 40.0], False),
])
def test_fast_ssa_path_equals_exact_path_other_models(datasets_golden, model, groups, ds, theta, npop, mu, obs):
    """SEIR and two-group filters at N = 5000: certified f32 loop and f64 loop give identical bits."""
    Y = datasets_golden[ds]
    T, N, C = Y.shape[0], 5000, len(theta)
    th = np.array(theta, dtype=np.float64)
    out = []
    for fast in (True, False):
        eng = _engine_with_fast_ssa(fast, N, T, C, model, groups)
        eng.set_observations(Y)
        eng.set_population(npop, mu)
        eng.set_profiling(2)
        lz, st = eng.run(th, [0.1] * C, [21 + c for c in range(C)], [5] * C, observations=obs)
        hid, anc = eng.history(C)
        out.append((lz, st, hid, anc, eng.stats()))
        eng.close()
    (lz1, st1, h1, a1, s1), (lz0, st0, h0, a0, s0) = out
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(h1, h0)
    np.testing.assert_array_equal(a1, a0)
    np.testing.assert_array_equal(lz1, lz0)
    assert s1["events"] == s0["events"] and s1["ssa_exact_lanes"] < s0["ssa_exact_lanes"]


@pytest.mark.parametrize("model,T,N,mu", [("sir", 1, 65, 20.0), ("sir", 2, 1, 20.0), ("sir", 3, 500, 20.0),
                                          ("seir", 2, 130, 20.0), ("sir", 6, 300, 0.0), ("sir_subgroups", 2, 64, 20.0),
                                          ("sir_subgroups2", 3, 200, 0.0)])
def test_filter_short_horizons_and_extinct_starts_vs_oracle(datasets_golden, model, T, N, mu):
    """Edge shapes: T = 1 (init only, no step kernel), T = 2 / 3, a single particle, and mu = 0 (every initial
    infected count 0: no SSA event anywhere); bit-exact vs the oracle."""
    if model == "sir":
        Y, th, npop = datasets_golden["sir_binom"][:T], (2.0, 1.0), 4820.0
    elif model == "seir":
        Y, th, npop = datasets_golden["seir_binom"][:T], (4.0, 1.0, 1.0), 4820.0
    else:
        Y = datasets_golden["sub_binom" if model == "sir_subgroups" else "sub2_binom"][:T]
        th, npop = (np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5), np.array([2030.0, 3040.0])
    mus = np.array([mu, mu]) if model.startswith("sir_sub") else mu
    if mu == 0.0:                                   # nobody infected: observations of I and R are 0 (weights > 0)
        Y = Y.copy()
        Y[:, 1:] = 0.0
    a = dict(Y=Y, model=model, theta=th, N=N, npop=npop, mu=mus)
    eng, thv = engine_for(a)
    lz, st = eng.run(thv[None], [0.1], [123], [4])
    o = oracle.particle_filter(Y, model, th, False, 0.1, N, npop, mus, key=123, filter_index=4)
    assert int(st[0]) == o["status"]
    if o["status"]:
        return
    hid, anc = eng.history(1)
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("cfg,chains,lanes,streams,checked", [
    (3, 2, 0, None, None), (3, 2, 1, None, None),
    (4, 2, 0, None, None), (4, 2, 1, None, None),
    (5, 2, 0, None, None), (5, 2, 1, None, None),
    # the bench's own layout: many chains on 4 chain-group streams, one lane per particle (pf_step_kernel, XCD-aware
    # grid), a seeded subset of the chains checked -- the kernel that produces bench.py's config-3 / config-5 numbers
    (3, 16, 1, 4, (0, 5, 10, 15)), (5, 16, 1, 4, (0, 6, 9, 15)),
])
def test_full_size_baseline_configs_vs_oracle(cfg, chains, lanes, streams, checked):
    """BASELINE configs 3 (SEIR, normal observations, N = 10^4, T = 200), 4 (SIR under-reported, N = 5*10^4, all 15
    rows: segmented block prefix) and 5 (2-group SIR, N = 10^4) at their full bench size, on the bench's own
    dataset and starting theta plus perturbed thetas (one batched launch, one chain each), on the automatic kernel
    choice (lanes = 0: the lane-group kernel at 2 chains) and on the one-lane pf_step_kernel (lanes = 1): states and
    ancestors bit-exact vs the oracle (pmcmc.py:123-233 restated), log-likelihoods within 1e-9 absolute."""
    from epipf import datasets
    from epipf.engine import Engine, model_id, theta_vector
    Y, meta = datasets.benchmark_dataset(cfg)
    N = meta["N"]
    mid = model_id(meta["model"])
    base = np.asarray(meta["theta"], dtype=np.float64)
    thetas = np.stack([base * (1.0 + 0.07 * (c % 5) * (-1) ** (np.arange(base.size) + c // 5))
                       for c in range(chains)])
    if mid >= 2:
        G = int(round(np.sqrt(base.size - 1)))
        ref_th = [(t[:G * G].reshape(G, G), t[-1]) for t in thetas]
    else:
        G = 1
        ref_th = [tuple(t) for t in thetas]
    eng = Engine(meta["model"], G, N, Y.shape[0], chains)
    eng.set_observations(Y)
    eng.set_population(meta["n_population"], meta["mu"])
    eng.set_lanes(lanes)
    eng.set_profiling(2)                   # device counters on: reference-ambiguous draws are counted
    if streams:
        eng.set_streams(streams)
    obs = bool(meta.get("observations", False))
    keys = [9000 + 17 * c for c in range(chains)]
    lz, st = eng.run(np.stack([theta_vector(mid, t)[0] for t in ref_th]), [meta["probs"]] * chains, keys,
                     [5 + c for c in range(chains)], observations=obs)
    stats = eng.stats()
    ran_lanes = stats["last_lanes"]
    hid, anc = eng.history(chains)
    eng.close()
    if lanes == 1:
        assert ran_lanes == 1, "the one-lane kernel did not run"
    elif cfg in (3, 5):
        assert ran_lanes > 1, "expected the lane-group kernel at 2 chains"
    draws = bad = 0
    for c in (checked or range(chains)):
        o = oracle.particle_filter(Y, meta["model"], ref_th[c], obs, meta["probs"], N, meta["n_population"],
                                   meta["mu"], key=keys[c], filter_index=5 + c)
        assert int(st[c]) == o["status"] == 0, (c, st[c], o["status"])
        np.testing.assert_array_equal(hid[c], o["hidden"])
        np.testing.assert_array_equal(anc[c], o["ancestry"])
        np.testing.assert_allclose(lz[c], o["log_zetas"], rtol=1e-12, atol=1e-9)
        # and against the reference itself: scipy's weights on these states, numpy's choice on the keyed uniforms
        d, b = reference_replay.replay(Y, hid[c], anc[c], meta["model"], obs, meta["probs"], keys[c], 5 + c)
        draws += d
        bad += b
    # reference-ambiguous draws (uniform within scipy's error envelope of a CDF boundary) are counted for every
    # chain of the launch: expected ~0.67 E N per draw, i.e. well below one here
    print(f"cfg {cfg} lanes {ran_lanes}: {draws} draws replayed against scipy, {bad} differ; "
          f"{stats['resample_ref_ambiguous']} reference-ambiguous draws of {chains * N * (Y.shape[0] - 1)}")
    assert bad == 0
    assert stats["resample_ref_ambiguous"] <= 3


def test_weight_tie_path_equals_oracle(datasets_golden, monkeypatch):
    """particle_weight's all-columns pass (binom_weight_tied, normally ~1e-6 of particle-steps) forced for every
    particle (EPIPF_TIE_SCALE widens the tie band to everything): SIR, SEIR and both subgroup models stay bit-exact to
    the oracle -- the out-of-line pass computes the same compensated minimum."""
    from epipf.engine import Engine, model_id, theta_vector
    monkeypatch.setenv("EPIPF_TIE_SCALE", "1e300")
    cases = [("sir", datasets_golden["sir_binom"], (2.0, 1.0), 4820.0, 20.0),
             ("seir", datasets_golden["seir_binom"], (4.0, 1.0, 1.0), 4820.0, 20.0),
             ("sir_subgroups", datasets_golden["sub_binom"][:6], (np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5),
              np.array([2030.0, 3040.0]), np.array([30.0, 40.0])),
             ("sir_subgroups2", datasets_golden["sub2_binom"][:6], (np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5),
              np.array([2030.0, 3040.0]), np.array([30.0, 40.0]))]
    for model, Y, th, npop, mu in cases:
        mid = model_id(model)
        thv, G = theta_vector(mid, th)
        for lanes in (1, 0):
            eng = Engine(model, G, 700, Y.shape[0], 1)        # created after the env: it reads EPIPF_TIE_SCALE
            eng.set_observations(Y)
            eng.set_population(npop, mu)
            eng.set_lanes(lanes)
            lz, st = eng.run(thv[None], [0.1], [55], [2])
            hid, anc = eng.history(1)
            eng.close()
            o = oracle.particle_filter(Y, model, th, False, 0.1, 700, npop, mu, key=55, filter_index=2)
            assert int(st[0]) == o["status"] == 0, (model, lanes)
            np.testing.assert_array_equal(hid[0], o["hidden"], err_msg=f"{model} lanes {lanes}")
            np.testing.assert_array_equal(anc[0], o["ancestry"], err_msg=f"{model} lanes {lanes}")
            np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


def test_large_population_weights_vs_oracle():
    """A population of 2*10^5: the binary128 log-factorial table is built by several host threads (above 64k entries)
    and the weights' counts reach 10^5; bit-exact states and ancestors vs the oracle (single-threaded table)."""
    from epipf.engine import Engine
    rs = np.random.RandomState(8)
    T, npop = 6, 200000.0
    th = (0.02, 0.01)                                  # a slow epidemic: ~30 events per particle-step
    Y = np.floor(0.1 * np.array([[199400.0, 600.0, 0.0]] * T)) + rs.randint(-20, 20, (T, 3)) * [1, 0, 0]
    eng = Engine("sir", 1, 900, T, 1)
    eng.set_observations(Y)
    eng.set_population(npop, 600.0)
    lz, st = eng.run(np.array([th]), [0.1], [9], [1])
    hid, anc = eng.history(1)
    eng.close()
    o = oracle.particle_filter(Y, "sir", th, False, 0.1, 900, npop, 600.0, key=9, filter_index=1)
    assert int(st[0]) == o["status"] == 0
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)
