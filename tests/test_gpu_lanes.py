"""The lane-group step kernel (epipf_group.hip: W = 2, 4, 8, 16 lanes per particle, the latency mode for runs that
do not fill the chip) against the CPU oracle and against the one-lane kernel (W = 1): states and ancestors bit-exact,
log-likelihoods within 1e-9 absolute, for every model, both observation types, extinct starts, the segmented
block prefix, the exact-loop branch (EPIPF_SSA_FAST=0) and the full BASELINE config-2 and config-5 sizes at one
chain.  Needs an MI355X: `-m gpu`."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

LANES = [1, 2, 4, 8, 16]
SHAPES = [(2, 1), (4, 1), (8, 1), (16, 1)]   # (W, K) instantiated


def _case(datasets_golden, model):
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
        return dict(Y=Y, theta=(np.array([[5.0, 2.0], [1.0, 3.0]]), 0.5), obs=False, probs=0.1,
                    npop=np.array([2030.0, 3040.0]), mu=np.array([30.0, 40.0]), G=2)
    raise ValueError(model)


def _run(model, c, N, chains, lanes, keys, fidx, events=0):
    from epipf.engine import Engine, model_id, theta_vector
    mid = model_id(model)
    th, G = theta_vector(mid, c["theta"])
    eng = Engine(model, G, N, c["Y"].shape[0], chains)
    eng.set_observations(c["Y"])
    eng.set_population(c["npop"], c["mu"])
    eng.set_lanes(lanes, events)
    lz, st = eng.run(np.repeat(th[None], chains, 0), [c["probs"]] * chains, keys, fidx, observations=c["obs"])
    used = eng.stats()["last_lanes"]
    hid, anc = eng.history(chains)
    eng.close()
    return lz, st, hid, anc, used


@pytest.mark.parametrize("lanes", LANES)
@pytest.mark.parametrize("model", ["sir", "sir_normal", "seir", "sir_subgroups", "sir_subgroups2"])
def test_lane_groups_match_oracle(datasets_golden, model, lanes):
    c = _case(datasets_golden, model)
    name = c.get("model", model)
    N, chains = 700, 2
    keys, fidx = [31, 32], [4, 9]
    lz, st, hid, anc, used = _run(name, c, N, chains, lanes, keys, fidx)
    assert used == lanes
    for ch in range(chains):
        o = oracle.particle_filter(c["Y"], name, c["theta"], c["obs"], c["probs"], N, c["npop"], c["mu"],
                                   key=keys[ch], filter_index=fidx[ch])
        assert int(st[ch]) == o["status"] == 0
        np.testing.assert_array_equal(hid[ch], o["hidden"])
        np.testing.assert_array_equal(anc[ch], o["ancestry"])
        np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("lanes", [1, 4, 8])
@pytest.mark.parametrize("model", ["sir", "sir_normal", "seir", "sir_subgroups", "sir_subgroups2"])
def test_widened_decision_band_equals_oracle(datasets_golden, monkeypatch, model, lanes):
    """Stress the uncertified-decision paths: the channel decision's band widened 3000x (EPIPF_BAND_SLACK, read at
    create) sends ~1% of decisions to the exact fallback -- the lane groups redo ~8% of their chunks after their
    per-lane certificates fail, the one-lane loop replaces the unsure lanes' mask bits (subgroups) or takes the
    f64 channel (SIR, SEIR) -- and states, ancestors and likelihoods stay the oracle's."""
    monkeypatch.setenv("EPIPF_BAND_SLACK", "3000")
    c = _case(datasets_golden, model)
    name = c.get("model", model)
    N, chains = 700, 2
    keys, fidx = [41, 42], [5, 11]
    lz, st, hid, anc, used = _run(name, c, N, chains, lanes, keys, fidx)
    assert used == lanes
    for ch in range(chains):
        o = oracle.particle_filter(c["Y"], name, c["theta"], c["obs"], c["probs"], N, c["npop"], c["mu"],
                                   key=keys[ch], filter_index=fidx[ch])
        assert int(st[ch]) == o["status"] == 0
        np.testing.assert_array_equal(hid[ch], o["hidden"])
        np.testing.assert_array_equal(anc[ch], o["ancestry"])
        np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("model", ["sir", "seir", "sir_subgroups"])
def test_every_lane_shape_matches_oracle(datasets_golden, model, shape):
    """Every instantiated (lanes, events per lane) shape, one chain, against the oracle."""
    c = _case(datasets_golden, model)
    W, K = shape
    lz, st, hid, anc, used = _run(model, c, 400, 1, W, [8], [6], events=K)
    assert used == W
    o = oracle.particle_filter(c["Y"], model, c["theta"], c["obs"], c["probs"], 400, c["npop"], c["mu"], key=8,
                               filter_index=6)
    assert int(st[0]) == o["status"] == 0
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("shape", [(4, 1), (8, 1), (16, 1)])
@pytest.mark.parametrize("decide", ["seq", "fixed_point"])
@pytest.mark.parametrize("model", ["sir", "seir", "sir_subgroups", "sir_subgroups2"])
def test_decision_passes_equal_oracle_with_widened_band(datasets_golden, monkeypatch, model, decide, shape):
    """Both lane-group decision passes -- the fixed-point one (round 4: every event of a chunk decided at once, iterated
    to the sequential pass's result) and the sequential one it replaced (EPIPF_GROUP_DECIDE=seq) -- with the band
    widened 3000x so that chunks are also redone on the exact fallback: states, ancestors and likelihoods are the
    oracle's (K = 2 was checked the same way while instantiated, profiles/r4c_lane_tests.txt)."""
    monkeypatch.setenv("EPIPF_BAND_SLACK", "3000")
    if decide == "seq":
        monkeypatch.setenv("EPIPF_GROUP_DECIDE", "seq")
    c = _case(datasets_golden, model)
    W, K = shape
    lz, st, hid, anc, used = _run(model, c, 500, 2, W, [51, 52], [3, 8], events=K)
    assert used == W
    for ch in range(2):
        o = oracle.particle_filter(c["Y"], model, c["theta"], c["obs"], c["probs"], 500, c["npop"], c["mu"],
                                   key=[51, 52][ch], filter_index=[3, 8][ch])
        assert int(st[ch]) == o["status"] == 0
        np.testing.assert_array_equal(hid[ch], o["hidden"])
        np.testing.assert_array_equal(anc[ch], o["ancestry"])
        np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("G", [3, 4])
def test_lane_groups_larger_subgroup_models_equal_one_lane(datasets_golden, G):
    """G = 3, 4 (12 and 20 channels, the widest unrolled decision passes): every W equals W = 1."""
    rs = np.random.RandomState(G)
    beta = rs.uniform(0.5, 3.0, (G, G))
    c = dict(Y=np.tile(datasets_golden["sub_binom"][:6, :3], (1, G)), theta=(beta, 0.7), obs=False, probs=0.1,
             npop=np.full(G, 1500.0), mu=np.full(G, 15.0), G=G)
    ref = _run("sir_subgroups", c, 300, 1, 1, [5], [2])
    for lanes in LANES[1:]:
        got = _run("sir_subgroups", c, 300, 1, lanes, [5], [2])
        assert got[4] == lanes
        assert int(got[1][0]) == int(ref[1][0])
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(got[3], ref[3])
        # bit for bit: the 16-particle layout sums the step totals in the 64-particle layout's order
        np.testing.assert_array_equal(got[0], ref[0])


@pytest.mark.parametrize("lone", ["0", "1"])
@pytest.mark.parametrize("G", [2, 3, 4])
def test_subgroup_lane_groups_with_and_without_the_waves_bound(datasets_golden, monkeypatch, G, lone):
    """The subgroup models' W >= 8 lane-group kernels exist with the 4-waves register bound (spilling at G >= 2) and
    without it (epipf_group.hpp group_lone_instance; the host takes the unbounded one for launches whose waves all stay
    resident, EPIPF_GROUP_LONE forces either): both are the oracle's, bit for bit."""
    monkeypatch.setenv("EPIPF_GROUP_LONE", lone)
    if G == 2:
        c = _case(datasets_golden, "sir_subgroups")
    else:
        rs = np.random.RandomState(G)
        c = dict(Y=np.tile(datasets_golden["sub_binom"][:6, :3], (1, G)), theta=(rs.uniform(0.5, 3.0, (G, G)), 0.7),
                 obs=False, probs=0.1, npop=np.full(G, 1500.0), mu=np.full(G, 15.0), G=G)
    for lanes in (8, 16):
        lz, st, hid, anc, used = _run("sir_subgroups", c, 450, 2, lanes, [71, 72], [1, 6])
        assert used == lanes
        for ch in range(2):
            o = oracle.particle_filter(c["Y"], "sir_subgroups", c["theta"], False, 0.1, 450, c["npop"], c["mu"],
                                       key=[71, 72][ch], filter_index=[1, 6][ch])
            assert int(st[ch]) == o["status"] == 0
            np.testing.assert_array_equal(hid[ch], o["hidden"])
            np.testing.assert_array_equal(anc[ch], o["ancestry"])
            np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("lanes", [2, 16])
def test_lane_groups_extinct_starts_and_short_horizons(datasets_golden, lanes):
    """Populations that die out inside a chunk of W events (mu = 1: many particles start with one infected) and
    T = 2: the group's extinction and step-boundary exits."""
    Y = datasets_golden["sir_binom"][:2]
    c = dict(Y=Y, theta=(1.2, 1.0), obs=False, probs=0.1, npop=4820, mu=1.0, G=1)
    lz, st, hid, anc, _ = _run("sir", c, 333, 1, lanes, [17], [0])
    o = oracle.particle_filter(Y, "sir", (1.2, 1.0), False, 0.1, 333, 4820, 1.0, key=17, filter_index=0)
    assert int(st[0]) == o["status"]
    if o["status"] == 0:
        np.testing.assert_array_equal(hid[0], o["hidden"])
        np.testing.assert_array_equal(anc[0], o["ancestry"])


def test_lane_groups_exact_loop_branch(datasets_golden, monkeypatch):
    """EPIPF_SSA_FAST=0: no particle may take the f32 channel test, so every group runs the exact loop branch."""
    monkeypatch.setenv("EPIPF_SSA_FAST", "0")
    c = _case(datasets_golden, "seir")
    lz, st, hid, anc, used = _run("seir", c, 500, 1, 8, [3], [1])
    assert used == 8
    o = oracle.particle_filter(c["Y"], "seir", c["theta"], False, 0.1, 500, 4820, 20, key=3, filter_index=1)
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])


def test_lane_groups_segmented_prefix(datasets_golden):
    """N = 12865 (202 blocks: a segmented block-sum prefix) through W = 8 and 16."""
    Y = datasets_golden["sir_binom"][:4]
    c = dict(Y=Y, theta=(2.0, 1.0), obs=False, probs=0.1, npop=4820, mu=20, G=1)
    o = oracle.particle_filter(Y, "sir", (2.0, 1.0), False, 0.1, 12865, 4820, 20, key=77, filter_index=3)
    for lanes in (8, 16):
        lz, st, hid, anc, _ = _run("sir", c, 12865, 1, lanes, [77], [3])
        np.testing.assert_array_equal(hid[0], o["hidden"])
        np.testing.assert_array_equal(anc[0], o["ancestry"])
        np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("lanes", [0, 4])
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_lane_groups_full_size_single_chain_vs_oracle(cfg, lanes):
    """Every BASELINE config at full size with one chain (the north star's layout for config 5), on the automatic
    lane choice (W = 16 up to 320 particle blocks, 8 up to 640, 4 above) and on W = 4: config 2 (SIR, N = 10^4, T = 200), 3
    (SEIR, normal observations), 4 (N = 5*10^4: 782 particle blocks, a segmented block-sum prefix), 5 (2-group SIR)
    -- bit-exact vs the oracle."""
    from epipf import datasets
    from epipf.engine import Engine, model_id, theta_vector
    Y, meta = datasets.benchmark_dataset(cfg)
    mid = model_id(meta["model"])
    base = np.asarray(meta["theta"], dtype=np.float64)
    if mid >= 2:
        G = int(round(np.sqrt(base.size - 1)))
        ref_th = (base[:G * G].reshape(G, G), base[-1])
    else:
        G, ref_th = 1, tuple(base)
    eng = Engine(meta["model"], G, meta["N"], Y.shape[0], 1)
    eng.set_observations(Y)
    eng.set_population(meta["n_population"], meta["mu"])
    if lanes:
        eng.set_lanes(lanes)
    obs = bool(meta.get("observations", False))
    lz, st = eng.run(theta_vector(mid, ref_th)[0][None], [meta["probs"]], [4242], [7], observations=obs)
    blocks = (meta["N"] + 63) // 64
    if mid < 2:                                          # SIR / SEIR
        auto = 16 if blocks <= 320 else 8 if blocks <= 960 else 4
    else:
        auto = 16 if blocks <= 960 else 4
    assert eng.stats()["last_lanes"] == (lanes or auto)
    hid, anc = eng.history(1)
    eng.close()
    o = oracle.particle_filter(Y, meta["model"], ref_th, obs, meta["probs"], meta["N"], meta["n_population"],
                               meta["mu"], key=4242, filter_index=7)
    assert int(st[0]) == o["status"] == 0
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


def test_automatic_lane_choice():
    """SIR / SEIR: up to two chains of 10^4 particles get 16 lanes, up to 6 chains 8, up to 8 chains 4; subgroup models:
    16 lanes up to 6 chains, then 4 up to 8; a batch that fills the chip keeps one lane per particle."""
    from epipf.engine import Engine
    Y = np.zeros((3, 3))
    eng = Engine("sir", 1, 10000, 3, 256)
    eng.set_observations(Y)
    eng.set_population(10000, 20)
    for chains, want in [(1, 16), (2, 16), (3, 8), (4, 8), (6, 8), (7, 4), (8, 4), (9, 1), (256, 1)]:
        eng.run(np.tile([0.25, 0.1], (chains, 1)), [0.1] * chains, list(range(1, chains + 1)), [0] * chains)
        assert eng.stats()["last_lanes"] == want, (chains, eng.stats()["last_lanes"])
    eng.close()
    eng = Engine("sir_subgroups", 2, 10000, 3, 16)
    eng.set_observations(np.zeros((3, 6)))
    eng.set_population([2000, 3000], [20, 30])
    th = np.array([4.0, 1.0, 1.0, 4.0, 1.0])
    for chains, want in [(1, 16), (4, 16), (6, 16), (7, 4), (8, 4), (9, 1)]:
        eng.run(np.tile(th, (chains, 1)), [0.1] * chains, list(range(1, chains + 1)), [0] * chains)
        assert eng.stats()["last_lanes"] == want, (chains, eng.stats()["last_lanes"])
    eng.close()


@pytest.mark.parametrize("lanes", [1, 4])
def test_populations_past_the_f32_range_take_the_exact_loop(lanes):
    """A population of 2*10^7 (> 2^24: counts no longer exact in f32) makes every particle ineligible for the certified
    f32 loop, so both kernels run the exact f64 event loop (the one-lane kernel per lane, the lane-group kernel per
    group): bit-exact vs the oracle, and the f32 loop is not used (no replays counted)."""
    from epipf import _lib
    npop, T, N = 2.0e7, 6, 256
    Y = np.stack([np.full(T, 0.1 * (npop - 40.0)), 0.1 * np.array([20., 40., 80., 150., 300., 600.]),
                  np.floor(0.1 * np.array([0., 10., 30., 70., 150., 300.]))], axis=1).astype(np.float64)
    Y = np.floor(Y)
    c = dict(Y=Y, theta=(1.6, 0.9), obs=False, probs=0.1, npop=npop, mu=20.0, G=1)
    from epipf.engine import Engine
    eng = Engine("sir", 1, N, T, 1)
    eng.set_observations(Y)
    eng.set_population(npop, 20.0)
    eng.set_lanes(lanes)
    eng.set_profiling(_lib.PROFILE_COUNTERS)
    lz, st = eng.run(np.array([[1.6, 0.9]]), [0.1], [12], [3])
    stats = eng.stats()
    hid, anc = eng.history(1)
    eng.close()
    o = oracle.particle_filter(Y, "sir", (1.6, 0.9), False, 0.1, N, npop, 20.0, key=12, filter_index=3)
    assert int(st[0]) == o["status"] == 0
    assert stats["last_lanes"] == lanes and stats["events"] > 0
    np.testing.assert_array_equal(hid[0], o["hidden"])
    np.testing.assert_array_equal(anc[0], o["ancestry"])
    np.testing.assert_allclose(lz[0], o["log_zetas"], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("lanes", [8, 16])
@pytest.mark.parametrize("model", ["sir", "seir", "sir_subgroups"])
def test_certified_clock_redo_equals_oracle(datasets_golden, monkeypatch, model, lanes):
    """The lane-group filter's certified clock (round 4: tau from multiplications by fl(1/N), every clock decision
    certified against the bound on its distance from the exact loop's t) redoes a particle-step on the exact clock when
    a decision falls inside the bound.  EPIPF_CLOCK_SLACK widens the bound 1e10x, so that most step-ending chunks redo:
    states, ancestors and likelihoods stay the oracle's."""
    monkeypatch.setenv("EPIPF_CLOCK_SLACK", "1e10")
    c = _case(datasets_golden, model)
    lz, st, hid, anc, used = _run(model, c, 600, 2, lanes, [61, 62], [2, 7])
    assert used == lanes
    for ch in range(2):
        o = oracle.particle_filter(c["Y"], model, c["theta"], c["obs"], c["probs"], 600, c["npop"], c["mu"],
                                   key=[61, 62][ch], filter_index=[2, 7][ch])
        assert int(st[ch]) == o["status"] == 0
        np.testing.assert_array_equal(hid[ch], o["hidden"])
        np.testing.assert_array_equal(anc[ch], o["ancestry"])
        np.testing.assert_allclose(lz[ch], o["log_zetas"], rtol=1e-12, atol=1e-9)


def _run_layout(monkeypatch, model, c, N, chains, lanes, block, keys, fidx):
    """_run on a context created with EPIPF_GROUP_BLOCK=block (read at create: 16- or 64-particle weight blocks)."""
    monkeypatch.setenv("EPIPF_GROUP_BLOCK", str(block))
    try:
        return _run(model, c, N, chains, lanes, keys, fidx)
    finally:
        monkeypatch.delenv("EPIPF_GROUP_BLOCK")


@pytest.mark.parametrize("N", [10000, 12865, 25000])
def test_step_totals_do_not_depend_on_the_weight_layout(datasets_golden, monkeypatch, N):
    """the weight layout (16- or 64-particle blocks) follows the number of chains sharing a launch, so a
    filter's log-likelihood must not depend on it.  The 16-particle layout sums each step's total in the 64-particle
    layout's order (scan_block_sums16): one lane per particle, W = 8 and 16 on either layout, one and eight chains --
    log-likelihoods bit-identical, states and ancestors the oracle's.  N = 10^4 (157 / 625 blocks, flat prefix),
    12865 (202 64-blocks: a segmented 64-layout prefix, S = 2), 25000 (1563 16-blocks: the segmented 16-layout)."""
    c = dict(_case(datasets_golden, "sir"))
    c["Y"] = datasets_golden["sir_binom"][:6]
    ref = _run("sir", c, N, 1, 1, [91], [4])
    runs = [_run_layout(monkeypatch, "sir", c, N, 1, W, blk, [91], [4]) for W in (8, 16) for blk in (16, 64)]
    eight = _run_layout(monkeypatch, "sir", c, N, 8, 16, 16, [91] + list(range(92, 99)), [4] * 8)
    for got in runs + [eight]:
        assert int(got[1][0]) == int(ref[1][0]) == 0
        np.testing.assert_array_equal(got[0][0], ref[0][0])
        np.testing.assert_array_equal(got[2][0], ref[2][0])
        np.testing.assert_array_equal(got[3][0], ref[3][0])
    o = oracle.particle_filter(c["Y"], "sir", c["theta"], False, 0.1, N, c["npop"], c["mu"], key=91, filter_index=4)
    np.testing.assert_array_equal(ref[2][0], o["hidden"])
    np.testing.assert_array_equal(ref[3][0], o["ancestry"])
    np.testing.assert_allclose(ref[0][0], o["log_zetas"], rtol=1e-12, atol=1e-9)


def test_subgroup_totals_do_not_depend_on_the_weight_layout(datasets_golden, monkeypatch):
    """The same for the 2-group model at N = 10^4 (W = 16 on 16-particle blocks, its automatic one-chain layout)."""
    c = _case(datasets_golden, "sir_subgroups")
    c["Y"] = c["Y"][:5]
    ref = _run("sir_subgroups", c, 10000, 1, 1, [93], [1])
    for blk in (16, 64):
        got = _run_layout(monkeypatch, "sir_subgroups", c, 10000, 1, 16, blk, [93], [1])
        np.testing.assert_array_equal(got[0], ref[0])
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(got[3], ref[3])


def test_prefetch_widths_and_chain_counts_agree_at_ten_thousand_particles(datasets_golden):
    """ADVICE r4's case: at N = 10^4 speculative rounds of 2 and 16 slots (W = 16 on 16-particle blocks vs W = 8 / 4 on
    64-particle blocks) and a lone chain vs the same chain among eight give bit-identical log-likelihoods, thetas and
    trajectories."""
    from epipf.pmcmc import ChainSampler, chain_key
    from epipf.prefetch import PrefetchSampler
    Y = datasets_golden["cfg2_binom"][:40]
    kw = dict(iters=12, probs=0.1, n_particles=10000, n_population=10000.0, mu=20.0, mh_ratio="log")
    res = []
    for cls, chains, extra in ((PrefetchSampler, 1, {"slots": 2}), (PrefetchSampler, 1, {"slots": 16}),
                               (ChainSampler, 1, {}), (ChainSampler, 8, {})):
        rngs = [np.random.RandomState(70 + c) for c in range(chains)]
        s = cls(Y, "sir", [0.25, 0.1], 2e-4, **kw, rngs=rngs, keys=[chain_key(70, c) for c in range(chains)], **extra)
        res.append(s.run()[0])
    for r in res[1:]:
        np.testing.assert_array_equal(r.log_likelihoods, res[0].log_likelihoods)
        np.testing.assert_array_equal(r.thetas, res[0].thetas)
        np.testing.assert_array_equal(r.sampled_trajs, res[0].sampled_trajs)
