"""The one-workgroup filter (epipf_fused.hpp: init and every step of a chain in one launch, N <= 256 with the lanes
automatic) against the CPU oracle and against the multi-launch step kernels (EPIPF_FUSED=0, read at create): states,
ancestors and log-likelihoods bit-exact (likelihoods to 1e-9 absolute against the oracle), for every model, both
observation types, every lane width the size rule picks (N = 1 .. 256: W = 16 .. 2, one to four weight blocks),
skipped and degenerate chains, systematic resampling, and the uncertified-decision and clock-redo paths.  Needs an
MI355X: `-m gpu`."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_on(monkeypatch):
    """The one-workgroup filter wherever it is eligible (EPIPF_FUSED=1; the default measures both paths first)."""
    monkeypatch.setenv("EPIPF_FUSED", "1")


MODELS = ["sir", "sir_normal", "seir", "sir_subgroups", "sir_subgroups2"]


def _case(datasets_golden, model, G=2):
    if model == "sir":
        return dict(Y=datasets_golden["sir_binom"][:30], theta=(2.0, 1.0), obs=False, probs=0.1, npop=4820, mu=20, G=1)
    if model == "sir_normal":
        return dict(Y=datasets_golden["sir_noisy"][:30], theta=(2.1, 0.9), obs=True, probs=0.5, npop=4820, mu=20, G=1,
                    model="sir")
    if model == "seir":
        return dict(Y=datasets_golden["seir_binom"][:30], theta=(4.0, 1.0, 1.0), obs=False, probs=0.1, npop=4820, mu=20,
                    G=1)
    if model in ("sir_subgroups", "sir_subgroups2"):
        Y = datasets_golden["sub_binom" if model == "sir_subgroups" else "sub2_binom"][:8]
        if G == 2:
            return dict(Y=Y, theta=(np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5), obs=False, probs=0.1,
                        npop=np.array([2030.0, 3040.0]), mu=np.array([30.0, 40.0]), G=2)
        # test_gpu_lanes.py's G = 3, 4 case (group-summed observations for the subgroups-2 model)
        beta = np.random.RandomState(G).uniform(0.5, 3.0, (G, G))
        Y3 = datasets_golden["sub_binom"][:6, :3]
        return dict(Y=Y3 if model == "sir_subgroups2" else np.tile(Y3, (1, G)), theta=(beta, 0.7), obs=False,
                    probs=0.1, npop=np.full(G, 1500.0), mu=np.full(G, 15.0), G=G)
    raise ValueError(model)


def _run(model, c, N, chains, keys, fidx, active=None, resample="multinomial", thetas=None, Y=None):
    from epipf.engine import Engine, model_id, theta_vector
    mid = model_id(model)
    th, G = theta_vector(mid, c["theta"])
    Y = c["Y"] if Y is None else Y
    eng = Engine(model, G, N, Y.shape[0], chains)
    eng.set_observations(Y)
    eng.set_population(c["npop"], c["mu"])
    th_all = np.repeat(th[None], chains, 0) if thetas is None else thetas
    lz, st = eng.run(th_all, [c["probs"]] * chains, keys, fidx, observations=c["obs"], active=active,
                     resample=resample)
    s = eng.stats()
    hid, anc = eng.history(chains)
    eng.close()
    return lz, st, hid, anc, s


def _run_both(monkeypatch, *args, **kw):
    """(fused run, multi-launch run) of the same filters."""
    a = _run(*args, **kw)
    monkeypatch.setenv("EPIPF_FUSED", "0")
    try:
        b = _run(*args, **kw)
    finally:
        monkeypatch.setenv("EPIPF_FUSED", "1")
    return a, b


@pytest.mark.parametrize("lanes", [0, 1, 2, 4, 16])
@pytest.mark.parametrize("N", [1, 37, 64, 100, 129, 200, 256, 300, 512])
@pytest.mark.parametrize("model", MODELS)
def test_fused_filter_matches_oracle(datasets_golden, monkeypatch, model, N, lanes):
    """Every SSA width of the one-workgroup filter (EPIPF_FUSED_LANES, read at create; 0: the automatic one)."""
    if N * lanes > 512:
        pytest.skip("N W lanes exceed one workgroup")
    monkeypatch.setenv("EPIPF_FUSED_LANES", str(lanes))
    c = _case(datasets_golden, model)
    name = c.get("model", model)
    keys, fidx = [71, 72], [3, 8]
    lz, st, hid, anc, s = _run(name, c, N, 2, keys, fidx)
    assert s["last_fused"] == 1
    if lanes:
        assert s["last_lanes"] == lanes
    for ch in range(2):
        o = oracle.particle_filter(c["Y"], name, c["theta"], c["obs"], c["probs"], N, c["npop"], c["mu"],
                                   key=keys[ch], filter_index=fidx[ch])
        assert int(st[ch]) == o["status"]
        if o["status"] == 0:
            np.testing.assert_array_equal(hid[ch], o["hidden"])
            np.testing.assert_array_equal(anc[ch], o["ancestry"])
            np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


def test_fused_threshold_and_explicit_lanes(datasets_golden, monkeypatch):
    """N = 513 and explicit lanes (epipf_set_lanes / EPIPF_LANES) take the step launches; EPIPF_FUSED=0 switches the
    one-workgroup filter off."""
    from epipf.engine import Engine
    c = _case(datasets_golden, "sir")
    for N, lanes, env, want in [(512, 0, None, 1), (513, 0, None, 0), (100, 4, None, 0), (100, 0, "0", 0)]:
        if env is not None:
            monkeypatch.setenv("EPIPF_FUSED", env)
        eng = Engine("sir", 1, N, c["Y"].shape[0], 1)
        eng.set_observations(c["Y"])
        eng.set_population(c["npop"], c["mu"])
        if lanes:
            eng.set_lanes(lanes, 0)
        eng.run(np.array([[2.0, 1.0]]), [0.1], [5], [0])
        assert eng.stats()["last_fused"] == want, (N, lanes, env)
        eng.close()
        if env is not None:
            monkeypatch.setenv("EPIPF_FUSED", "1")


@pytest.mark.parametrize("model", MODELS)
def test_fused_equals_step_launches_with_a_skipped_chain(datasets_golden, monkeypatch, model):
    """Five chains of one batch -- different thetas, one skipped (active = 0) -- give the multi-launch path's outputs
    bit for bit."""
    c = _case(datasets_golden, model)
    name = c.get("model", model)
    from epipf.engine import model_id, theta_vector
    th, _ = theta_vector(model_id(name), c["theta"])
    thetas = np.array([th * f for f in (1.0, 0.8, 1.3, 1.0, 0.6)])
    Y = c["Y"].copy()
    N, chains = 150, 5
    keys, fidx = [11, 12, 13, 14, 15], [0, 1, 2, 3, 4]
    act = np.array([1, 1, 0, 1, 1], dtype=np.int32)
    (lz, st, hid, anc, s), (lz2, st2, hid2, anc2, s2) = _run_both(monkeypatch, name, c, N, chains, keys, fidx,
                                                                 active=act, thetas=thetas, Y=Y)
    assert s["last_fused"] == 1 and s2["last_fused"] == 0
    np.testing.assert_array_equal(st, st2)
    assert int(st[2]) == 2                                            # EPIPF_STATUS_SKIPPED
    np.testing.assert_array_equal(lz[st == 0], lz2[st2 == 0])
    for ch in np.flatnonzero(st == 0):
        np.testing.assert_array_equal(hid[ch], hid2[ch])
        np.testing.assert_array_equal(anc[ch], anc2[ch])


def test_fused_degenerate_step(datasets_golden, monkeypatch):
    """Observations above every particle's count from step 4 on: all weights 0 at the resampling of step 4 -> status 1,
    log-likelihood -inf there, as the step launches and the oracle."""
    c = _case(datasets_golden, "sir")
    Y = c["Y"].copy()
    Y[3:] = 1e7
    (lz, st, hid, anc, s), (lz2, st2, *_rest) = _run_both(monkeypatch, "sir", c, 80, 2, [3, 4], [1, 2], Y=Y)
    o = oracle.particle_filter(Y, "sir", c["theta"], False, c["probs"], 80, c["npop"], c["mu"], key=3, filter_index=1)
    assert int(st[0]) == int(st2[0]) == o["status"] == 1
    np.testing.assert_array_equal(lz, lz2)
    assert lz[0, 4] == -np.inf


@pytest.mark.parametrize("model", ["sir", "seir", "sir_subgroups"])
def test_fused_systematic_resampling(datasets_golden, monkeypatch, model):
    c = _case(datasets_golden, model)
    (lz, st, hid, anc, s), (lz2, st2, hid2, anc2, _) = _run_both(monkeypatch, model, c, 120, 3, [5, 6, 7], [0, 0, 1],
                                                                resample="systematic")
    assert s["last_fused"] == 1
    np.testing.assert_array_equal(st, st2)
    np.testing.assert_array_equal(lz, lz2)
    np.testing.assert_array_equal(hid, hid2)
    np.testing.assert_array_equal(anc, anc2)
    o = oracle.particle_filter(c["Y"], model, c["theta"], c["obs"], c["probs"], 120, c["npop"], c["mu"], key=6,
                               filter_index=0, resample="systematic")
    np.testing.assert_array_equal(hid[1], o["hidden"])


@pytest.mark.parametrize("env", [("EPIPF_BAND_SLACK", "3000"), ("EPIPF_CLOCK_SLACK", "1e10")])
@pytest.mark.parametrize("model", ["sir", "sir_normal", "seir", "sir_subgroups", "sir_subgroups2"])
def test_fused_uncertified_paths_equal_oracle(datasets_golden, monkeypatch, model, env):
    """The exact-decision redo (band widened 3000x) and the exact-clock redo (clock bound widened 1e10x) inside the
    one-workgroup filter: the oracle's states, ancestors and likelihoods."""
    monkeypatch.setenv(*env)
    c = _case(datasets_golden, model)
    name = c.get("model", model)
    lz, st, hid, anc, s = _run(name, c, 90, 2, [21, 22], [4, 6])
    assert s["last_fused"] == 1
    for ch in range(2):
        o = oracle.particle_filter(c["Y"], name, c["theta"], c["obs"], c["probs"], 90, c["npop"], c["mu"],
                                   key=[21, 22][ch], filter_index=[4, 6][ch])
        assert int(st[ch]) == o["status"] == 0
        np.testing.assert_array_equal(hid[ch], o["hidden"])
        np.testing.assert_array_equal(anc[ch], o["ancestry"])
        np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("G", [1, 3, 4])
@pytest.mark.parametrize("model", ["sir_subgroups", "sir_subgroups2"])
def test_fused_other_group_counts_equal_step_launches(datasets_golden, monkeypatch, model, G):
    c = _case(datasets_golden, model, G=G)
    (lz, st, hid, anc, s), (lz2, st2, hid2, anc2, _) = _run_both(monkeypatch, model, c, 100, 2, [9, 10], [1, 1])
    assert s["last_fused"] == 1
    np.testing.assert_array_equal(st, st2)
    np.testing.assert_array_equal(lz, lz2)
    for ch in np.flatnonzero(st == 0):              # a degenerate chain's later history rows are never written
        np.testing.assert_array_equal(hid[ch], hid2[ch])
        np.testing.assert_array_equal(anc[ch], anc2[ch])


def test_fused_counts_the_same_events(datasets_golden, monkeypatch):
    """The device event counter (profiling counters) sums the same accepted events as the step launches."""
    from epipf import _lib
    from epipf.engine import Engine
    c = _case(datasets_golden, "sir")
    ev = []
    for env in (None, "0"):
        if env:
            monkeypatch.setenv("EPIPF_FUSED", env)
        eng = Engine("sir", 1, 200, c["Y"].shape[0], 4)
        eng.set_observations(c["Y"])
        eng.set_population(c["npop"], c["mu"])
        eng.set_profiling(_lib.PROFILE_COUNTERS)
        eng.run(np.tile([2.0, 1.0], (4, 1)), [0.1] * 4, [1, 2, 3, 4], [0] * 4)
        ev.append(eng.stats()["events"])
        eng.close()
    monkeypatch.setenv("EPIPF_FUSED", "1")
    assert ev[0] == ev[1] > 0


@pytest.mark.parametrize("N", [100, 700])
def test_run_sampled_equals_run_then_path_sample(datasets_golden, N):
    """epipf_run_sampled (the path sampler on the filter's stream, picks handed over with the filter) against
    epipf_run + epipf_path_sample, on the one-workgroup filter (N = 100) and the step launches (N = 700): the same
    likelihoods and statuses, the same paths, zeros for a skipped chain, a chain with pick -1 and a degenerate one."""
    from epipf.engine import Engine
    c = _case(datasets_golden, "sir")
    Y = c["Y"]
    for degenerate in (False, True):
        if degenerate:
            Y = Y.copy()
            Y[5:] = 1e7
        eng = Engine("sir", 1, N, Y.shape[0], 4)
        eng.set_observations(Y)
        eng.set_population(c["npop"], c["mu"])
        th = np.tile([2.0, 1.0], (4, 1))
        act = np.array([1, 1, 0, 1], dtype=np.int32)
        keys, fidx = [3, 4, 5, 6], [9, 9, 9, 9]
        chosen = np.array([5, -1, 7, N - 1], dtype=np.int32)
        lz, st = eng.run(th, [0.1] * 4, keys, fidx, active=act)
        ref = eng.path_sample(np.maximum(chosen, 0))
        lz2, st2, tr = eng.run(th, [0.1] * 4, keys, fidx, active=act, chosen=chosen)
        eng.close()
        np.testing.assert_array_equal(st, st2)
        np.testing.assert_array_equal(lz, lz2)
        assert int(st[2]) == 2
        for ch in range(4):
            if st[ch] == 0 and chosen[ch] >= 0:
                np.testing.assert_array_equal(tr[ch], ref[ch])
            else:
                assert not tr[ch].any()
        if degenerate:
            assert (st[[0, 1, 3]] == 1).all()


def test_automatic_choice_times_both_paths_with_identical_results(datasets_golden, monkeypatch):
    """EPIPF_FUSED=auto (the default): a batch size's first eight runs alternate the one-workgroup filter and the step
    launches (fused first), then one path stays; every run's outputs are the same."""
    from epipf.engine import Engine
    monkeypatch.setenv("EPIPF_FUSED", "auto")
    c = _case(datasets_golden, "seir")
    eng = Engine("seir", 1, 90, c["Y"].shape[0], 3)
    eng.set_observations(c["Y"])
    eng.set_population(c["npop"], c["mu"])
    th = np.tile([4.0, 1.0, 1.0], (3, 1))
    used, outs = [], []
    for r in range(11):
        lz, st = eng.run(th, [0.1] * 3, [1, 2, 3], [5, 5, 5])
        used.append(eng.stats()["last_fused"])
        outs.append((lz.copy(), st.copy(), *eng.history(3)))
    eng.close()
    assert used[:8] == [1, 0, 1, 0, 1, 0, 1, 0]
    assert len(set(used[8:])) == 1
    for o in outs[1:]:
        for x, y in zip(o, outs[0]):
            np.testing.assert_array_equal(x, y)


def test_automatic_choice_is_shared_by_the_processes_contexts(datasets_golden, monkeypatch):
    """The path choice is per process and per workload (concurrent contexts each timing alone settled on
    different paths): a second context on the same workload takes the first one's decision from its first run, without
    tuning; new observations are a new workload, so that context tunes again (fused first)."""
    from epipf.engine import Engine
    monkeypatch.setenv("EPIPF_FUSED", "auto")
    c = _case(datasets_golden, "seir")
    th = np.tile([4.0, 1.0, 1.0], (2, 1))

    def engine(Y):
        e = Engine("seir", 1, 91, Y.shape[0], 2)
        e.set_observations(Y)
        e.set_population(c["npop"], c["mu"])
        return e

    a, b = engine(c["Y"]), engine(c["Y"])
    used_a = []
    for _ in range(9):
        a.run(th, [0.1] * 2, [1, 2], [5, 5])
        used_a.append(a.stats()["last_fused"])
    assert used_a[:8] == [1, 0, 1, 0, 1, 0, 1, 0]
    choice = used_a[8]
    for _ in range(3):
        b.run(th, [0.1] * 2, [1, 2], [5, 5])
        assert b.stats()["last_fused"] == choice
    # one more row of observations (T - 1 rows: a different T and data): tuning starts again
    b.set_observations(c["Y"][:-1])
    used_b = []
    for _ in range(2):
        b.run(th, [0.1] * 2, [1, 2], [5, 5])
        used_b.append(b.stats()["last_fused"])
    assert used_b == [1, 0]
    a.close()
    b.close()


def test_many_chain_host_draws_on_the_device_engine(datasets_golden, monkeypatch):
    """24 chains of the config-1 shape (N = 100: the one-workgroup filter) through ChainSampler with the C host draws
    (epipf_mh_propose / epipf_mh_decide) and with the Python loop: identical thetas, likelihoods, paths, counters and
    final generator states."""
    from epipf import pmcmc as pm
    monkeypatch.setenv("EPIPF_FUSED", "auto")
    Y = datasets_golden["cfg1_binom"][:20]
    nc = 24
    runs = []
    for hd in (True, False):
        rngs = [np.random.RandomState(300 + c) for c in range(nc)]
        s = pm.ChainSampler(Y, "sir", [2.0, 1.0], 0.02, iters=15, probs=0.1, n_particles=100, n_population=200, mu=20,
                            rngs=rngs, keys=[pm.chain_key(300, c) for c in range(nc)], mh_ratio="log", host_draws=hd,
                            engine_chains=nc)
        assert (s._host is not None) == hd
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
