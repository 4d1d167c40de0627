"""Speculative (prefetching) MH, epipf.prefetch, on CPU: the GPU engine is replaced, inside these tests only,
by the oracle-backed stand-in (tests/oracle_engine.py).  Prefetching must not change a single committed value:
thetas, likelihoods, trajectories, acceptance and filter counts, the filter-index counter and the final state of
the host RandomState all equal the sequential MH loop's (pmcmc.py:325-406) -- for every slot count, with
negative proposals, degenerate filters, probs=None, subgroup models, the adaptive covariance and several chains."""
import numpy as np
import pytest

from epipf import pmcmc as pm
from epipf import prefetch as pf
from oracle_engine import fake_get_engine


@pytest.fixture(autouse=True)
def oracle_engine(monkeypatch):
    monkeypatch.setattr(pm, "get_engine", fake_get_engine)


def _golden_kwargs(rec):
    model = str(rec["model"])
    sub = model.startswith("SIR_SUB")
    return dict(Y=rec["Y"], type_model=model.lower(), parameters=list(rec["params"]), h=float(rec["h"]),
                adaptive=bool(rec["adaptive"]), sigma=None if rec["sigma"].size == 0 else rec["sigma"],
                n_chains=int(rec["iters"]), probs=None if float(rec["probs"]) < 0 else float(rec["probs"]),
                n_particles=int(rec["N"]), n_population=rec["npop"] if sub else float(rec["npop"][0]),
                mu=rec["mu"] if sub else float(rec["mu"][0]))


@pytest.mark.parametrize("slots", [1, 3, 12])
@pytest.mark.parametrize("name", ["sir_small", "sir_p", "sub", "sir_adaptive"])
def test_prefetch_reproduces_reference_trace(pmcmc_golden, name, slots):
    """particle_mcmc (global RandomState + module Philox stream) with prefetching equals the unmodified
    reference's run under the keyed stream (tests/golden/make_golden.py)."""
    rec = pmcmc_golden["pmcmc_" + name]
    if name == "sir_adaptive" and slots == 1:
        pytest.skip("1030 single-slot rounds: covered by slots 3 and 12")
    pm.seed_stream(int(rec["key"]), 0)
    np.random.seed(int(rec["seed"]))
    kw = _golden_kwargs(rec)
    th, lk, tr = pm.particle_mcmc(kw.pop("Y"), kw.pop("type_model"), kw.pop("parameters"), kw.pop("h"), **kw,
                                  progress=False, prefetch=slots)
    np.testing.assert_array_equal(th, rec["thetas"])
    np.testing.assert_array_equal(tr, rec["trajs"])
    np.testing.assert_allclose(lk, rec["likelihoods"], rtol=1e-9)
    assert pm._STREAM.next_filter == int(rec["n_filters"])


def _run(sampler_cls, rngs_seed, chains, **kw):
    rngs = [np.random.RandomState(rngs_seed + c) for c in range(chains)]
    keys = [pm.chain_key(rngs_seed, c) for c in range(chains)]
    args = (kw.pop("Y"), kw.pop("type_model"), kw.pop("parameters"), kw.pop("h"))
    kw["iters"] = kw.pop("n_chains")
    s = sampler_cls(*args, **kw, rngs=rngs, keys=keys)
    res = s.run()
    return s, res, [r.get_state() for r in rngs]


def _assert_same(a, b):
    (sa, ra, sta), (sb, rb, stb) = a, b
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(x.thetas, y.thetas)
        np.testing.assert_array_equal(x.likelihoods, y.likelihoods)
        np.testing.assert_array_equal(x.log_likelihoods, y.log_likelihoods)
        np.testing.assert_array_equal(x.sampled_trajs, y.sampled_trajs)
        assert x.acceptances == y.acceptances
        assert x.filters_run == y.filters_run
    assert list(sa.fnext) == list(sb.fnext)
    for u, v in zip(sta, stb):                     # the host RandomState ends in the same state
        assert u[0] == v[0] and np.array_equal(u[1], v[1]) and u[2:] == v[2:]


CASES = {
    # negative proposals (theta near 0, wide steps) and the log ratio
    "negative_proposals": dict(parameters=[2.0, 1.0], h=0.8, probs=0.1, n_particles=16, mh_ratio="log"),
    # tiny particle counts: steps with all weights zero (degenerate filters -> no pick, no uniform)
    "degenerate_filters": dict(parameters=[2.0, 1.0], h=0.5, probs=0.1, n_particles=2, mh_ratio="reference"),
    # probs=None: the observation probability is a fourth... third parameter, clipped to [0, 1]
    "probs_none": dict(parameters=[2.0, 1.0, 0.1], h=0.01, probs=None, n_particles=6, mh_ratio="reference"),
}


@pytest.mark.parametrize("slots", [2, 7, 16])
@pytest.mark.parametrize("case", sorted(CASES))
def test_prefetch_equals_sequential(datasets_golden, case, slots):
    Y = datasets_golden["sir_binom"]
    kw = dict(Y=Y, type_model="sir", n_chains=40, n_population=4820, mu=20, **CASES[case])
    seq = _run(pm.ChainSampler, 11, 1, **dict(kw))
    pre = _run(pf.PrefetchSampler, 11, 1, **dict(kw), slots=slots)
    _assert_same(seq, pre)
    s = pre[0]
    assert s.rounds <= 40
    if case == "degenerate_filters":
        assert s.degenerate > 0                    # the realised path went through (None, None, None) filters
    if case == "negative_proposals":
        assert seq[1][0].filters_run < 39          # iterations without a filter on the realised path


@pytest.mark.parametrize("slots", [1, 5, 16])
def test_prefetch_multichain_equals_lockstep(datasets_golden, slots):
    Y = datasets_golden["cfg1_binom"][:10]
    kw = dict(Y=Y, type_model="sir", parameters=[2.0, 1.0], h=0.02, n_chains=25, probs=0.1, n_particles=12,
              n_population=200, mu=20, mh_ratio="log")
    _assert_same(_run(pm.ChainSampler, 5, 3, **dict(kw)), _run(pf.PrefetchSampler, 5, 3, **dict(kw), slots=slots))


def test_prefetch_subgroups2(datasets_golden):
    kw = dict(Y=datasets_golden["sub2_binom"], type_model="sir_subgroups2", parameters=[4.0, 1.0, 1.0, 4.0, 1.0], h=0.05, n_chains=15,
              probs=0.1, n_particles=6, n_population=[2000.0, 3000.0], mu=[30.0, 40.0], mh_ratio="log")
    _assert_same(_run(pm.ChainSampler, 9, 1, **dict(kw)), _run(pf.PrefetchSampler, 9, 1, **dict(kw), slots=9))


def test_prefetch_advances_several_iterations_per_round(datasets_golden):
    """A round of K slots commits more than one iteration on average (the point of prefetching)."""
    Y = datasets_golden["cfg1_binom"][:10]
    kw = dict(Y=Y, type_model="sir", parameters=[2.0, 1.0], h=0.02, n_chains=60, probs=0.1, n_particles=12,
              n_population=200, mu=20, mh_ratio="log")
    s, res, _ = _run(pf.PrefetchSampler, 7, 1, **kw, slots=16)
    assert s.rounds * 2 < 60, s.rounds
    assert s.speculative_filters >= res[0].filters_run


@pytest.mark.parametrize("case", sorted(CASES))
def test_prefetch_auto_equals_sequential(datasets_golden, case):
    """slots="auto" (SlotTuner: the width changes from round to round while it explores and re-measures) commits
    exactly the sequential loop's values."""
    Y = datasets_golden["sir_binom"]
    kw = dict(Y=Y, type_model="sir", n_chains=60, n_population=4820, mu=20, **CASES[case])
    seq = _run(pm.ChainSampler, 13, 1, **dict(kw))
    pre = _run(pf.PrefetchSampler, 13, 1, **dict(kw), slots="auto")
    _assert_same(seq, pre)
    assert len({k for k, n in pre[0].tuner.count.items() if n}) > 1      # several widths were used


def test_particle_mcmc_auto_prefetch_reproduces_reference_trace(pmcmc_golden):
    """The drop-in's default (prefetch="auto") against the unmodified reference's trace."""
    rec = pmcmc_golden["pmcmc_sir_p"]
    pm.seed_stream(int(rec["key"]), 0)
    np.random.seed(int(rec["seed"]))
    kw = _golden_kwargs(rec)
    th, lk, tr = pm.particle_mcmc(kw.pop("Y"), kw.pop("type_model"), kw.pop("parameters"), kw.pop("h"), **kw,
                                  progress=False)
    np.testing.assert_array_equal(th, rec["thetas"])
    np.testing.assert_array_equal(tr, rec["trajs"])
    np.testing.assert_allclose(lk, rec["likelihoods"], rtol=1e-9)


def test_expected_iterations_model():
    """E(K) of best-first scheduling: one slot commits one iteration; with acceptance a the second-best node is the
    likelier child; with certain rejection K slots commit K iterations; several chains share the slots."""
    assert pf.expected_iterations(1, [0.3]) == pytest.approx(1.0)
    assert pf.expected_iterations(2, [0.3]) == pytest.approx(1.7)
    assert pf.expected_iterations(2, [0.6]) == pytest.approx(1.6)
    assert pf.expected_iterations(5, [0.0]) == pytest.approx(5.0)
    assert pf.expected_iterations(3, [0.5, 0.5]) == pytest.approx(2.5)
    # a third branch for degenerate filters (probability d): the root, then its degenerate child (0.5), then 0.25
    assert pf.expected_iterations(3, [0.5], [0.5]) == pytest.approx(1.75)
    assert pf.expected_iterations(4, [0.3], [0.0]) == pytest.approx(pf.expected_iterations(4, [0.3]))
    assert pf.expected_iterations_upto(6, [0.3, 0.7], [0.1, 0.0]) == pytest.approx(
        [pf.expected_iterations(k, [0.3, 0.7], [0.1, 0.0]) for k in range(1, 7)])


def test_slot_tuner_picks_the_best_measured_rate():
    """After exploring every candidate three times, the tuner takes the width with the most expected iterations per second:
    with round times flat up to 4 slots and linear beyond, 4 wins at acceptance 0.5."""
    t = pf.SlotTuner(1, 16)
    cost = {1: 1.0, 2: 1.0, 4: 1.0, 8: 2.0, 16: 4.0}
    first = set()
    for _ in range(40):
        k = t.pick([0.5])
        t.record(k, cost[k] * (50.0 if k not in first else 1.0))     # a slow first round per width: not timed
        first.add(k)
    assert t.best == 4


@pytest.mark.parametrize("chains,h", [(1, 0.01), (1, 0.1), (2, 0.03)])
def test_round_cuts_equal_narrower_rounds(datasets_golden, chains, h):
    """The tuner's observed yields (SlotTuner, PrefetchSampler._resolve): the filters a K-slot round commits when its
    realised path is cut at the first node of schedule rank >= K' equal what a K'-slot round commits from the same
    state (best-first scheduling: the K' most probable nodes are the same), for every K' < K."""
    Y = datasets_golden["cfg1_binom"][:12]
    kw = dict(iters=40, probs=0.1, n_particles=24, n_population=200.0, mu=20.0, mh_ratio="log")

    def sampler(slots):
        s = pf.PrefetchSampler(Y, "sir", [2.0, 1.0], h, **kw, rngs=[np.random.RandomState(5 + c) for c in range(chains)],
                               keys=[pm.chain_key(5, c) for c in range(chains)], slots=slots)
        s.initialise()
        return s

    for rounds in range(3):                      # the first rounds from the same state (earlier rounds at width 12)
        wide = sampler(12)
        for _ in range(rounds):
            wide.advance()
        f0 = sum(wide.filters_run)
        nodes = wide._schedule()
        wide._evaluate(nodes)
        _, cut = wide._resolve([1, 2, 4, 8, 12])
        assert cut[12] == sum(wide.filters_run) - f0
        for k in (1, 2, 4, 8):
            narrow = sampler(12)
            for _ in range(rounds):
                narrow.advance()
            narrow.slots = k
            g0 = sum(narrow.filters_run)
            narrow.advance()
            assert cut[k] == sum(narrow.filters_run) - g0, (rounds, k)


def test_slot_tuner_uses_observed_yields():
    """With observed yields fed per width, the tuner follows them rather than the tree model: the model at acceptance
    0.5 favours 8 slots at these round times, the observed cuts saturate at 4."""
    t = pf.SlotTuner(1, 8, prior=2)
    cost = {1: 1.0, 2: 1.0, 4: 1.0, 8: 1.3}
    seen = {1: 1.0, 2: 2.0, 4: 3.0, 8: 3.1}
    first = set()
    for _ in range(60):
        k = t.pick([0.5])
        t.record(k, cost[k] * (50.0 if k not in first else 1.0), {kk: v for kk, v in seen.items() if kk <= k})
        first.add(k)
    assert t.best == 4
