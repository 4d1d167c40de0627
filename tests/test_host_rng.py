"""Host RNG shortcuts of the MH loop against numpy itself (CPU): legacy_randint draws what RandomState.randint(0, n)
draws and leaves the stream where it leaves it; _MTPeek reads that value off the MT19937 state without consuming it;
the per-chain proposal arithmetic equals mvn_apply's."""
import numpy as np
import pytest

from epipf.pmcmc import _MTPeek, _raw_words, legacy_randint, mvn_apply, mvn_factor


def test_legacy_randint_equals_randint_and_its_consumption():
    rs = np.random.RandomState(5)
    for t in range(3000):
        n = int(rs.randint(1, 2**31)) if t % 3 else int(rs.randint(1, 3000))
        a, b = np.random.RandomState(t), np.random.RandomState(t)
        for _ in range(3):
            assert a.randint(0, n) == legacy_randint(b, n)
        assert a.random_sample() == b.random_sample()


def test_legacy_randint_on_the_global_generator_and_fallback():
    np.random.seed(11)
    want = [np.random.randint(0, 977) for _ in range(50)]
    np.random.seed(11)
    assert [legacy_randint(np.random, 977) for _ in range(50)] == want
    g = np.random.default_rng(3)                       # not a legacy RandomState: falls back to its own randint-alike

    class R:
        def randint(self, lo, hi):
            return int(g.integers(lo, hi))
    assert _raw_words(R()) is None
    assert 0 <= legacy_randint(R(), 10) < 10


def test_peek_equals_the_next_draw_without_consuming():
    rs = np.random.RandomState(3)
    unpeekable = 0
    for t in range(4000):
        r = np.random.RandomState(t)
        r.random_sample(int(rs.randint(0, 700)))      # every position in the 624-word state, regenerations included
        n = int(rs.randint(1, 2**31)) if t % 2 else int(rs.randint(1, 20000))
        pk = _MTPeek(_raw_words(r))
        v = pk.randint(n)
        again = pk.randint(n)                          # nothing consumed
        w = legacy_randint(r, n)
        if v is None:
            unpeekable += 1
            assert again is None
        else:
            assert v == again == w
    assert unpeekable < 100                            # only draws that would regenerate the state first


@pytest.mark.parametrize("d", [2, 3, 5])
def test_proposal_into_a_buffer_equals_mvn_apply(d):
    """ChainSampler.step's np.dot(z, factor, out=row) followed by + theta for all chains == mvn_apply per chain."""
    rs = np.random.RandomState(d)
    A = rs.standard_normal((d, d))
    fac = mvn_factor(0.3 * (A @ A.T))
    Z = rs.standard_normal((64, d))
    M = rs.standard_normal((64, d))
    D = np.empty((64, d))
    for c in range(64):
        np.dot(Z[c].reshape(1, d), fac, out=D[c:c + 1])
    P = D + M
    for c in range(64):
        np.testing.assert_array_equal(P[c], mvn_apply(Z[c].copy(), fac, M[c]))


def _states(rngs):
    import ctypes
    return (ctypes.c_void_p * len(rngs))(*[r._bit_generator.ctypes.state_address for r in rngs])


@pytest.mark.parametrize("d", [2, 4, 6])
def test_c_proposals_equal_numpys_multivariate_normal(d):
    """epipf_mh_propose (csrc/host_mh.cpp) against RandomState.standard_normal + mvn_apply on copies of the same
    states: the proposals and the generators' positions afterwards (the next draws) are identical."""
    from epipf import _lib
    from epipf.pmcmc import _NumpyDgemv
    dg = _NumpyDgemv.pointer()
    if not dg:
        pytest.skip("numpy's cblas_dgemv not found / not reproducing np.dot")
    L = _lib.load()
    nc = 40
    rs = np.random.RandomState(d)
    facs = np.stack([mvn_factor(0.01 * (lambda A: A @ A.T)(rs.standard_normal((d, d)))) for _ in range(nc)])
    means = rs.standard_normal((nc, d))
    a = [np.random.RandomState(100 + c) for c in range(nc)]
    b = [np.random.RandomState(100 + c) for c in range(nc)]
    for x, y in zip(a, b):                               # states at different positions, regenerations included
        k = int(rs.randint(0, 700)) * 2
        x.random_sample(k)
        y.random_sample(k)
    for it in range(30):
        P = np.empty((nc, d))
        _lib.check(L.epipf_mh_propose(nc, d, _states(a), _lib.ptr(facs), _lib.ptr(means), _lib.ptr(P), dg), "propose")
        for c in range(nc):
            np.testing.assert_array_equal(P[c], mvn_apply(b[c].standard_normal(d), facs[c], means[c]))
    for x, y in zip(a, b):
        assert x.random_sample() == y.random_sample()


def test_c_picks_and_acceptance_equal_the_python_loop():
    """epipf_mh_decide against legacy randint + random_sample + _log_ratio, for a subset of chains in order (NaN and
    +-inf log-likelihoods included)."""
    from epipf import _lib
    from epipf.pmcmc import _log_ratio
    L = _lib.load()
    nc, N = 50, 977
    rs = np.random.RandomState(9)
    a = [np.random.RandomState(7 * c + 1) for c in range(nc)]
    b = [np.random.RandomState(7 * c + 1) for c in range(nc)]
    for it in range(40):
        ok = np.sort(rs.choice(nc, int(rs.randint(1, nc)), replace=False)).astype(np.int32)
        new = rs.normal(-50, 3, nc)
        old = rs.normal(-50, 3, nc)
        new[rs.randint(0, nc)] = np.nan
        old[rs.randint(0, nc)] = -np.inf
        chosen = np.zeros(nc, dtype=np.int32)
        acc = np.zeros(nc, dtype=np.int32)
        _lib.check(L.epipf_mh_decide(ok.size, _lib.ptr(ok), _states(a), N, _lib.ptr(new), _lib.ptr(old),
                                     _lib.ptr(chosen), _lib.ptr(acc)), "decide")
        for c in ok.tolist():
            assert chosen[c] == legacy_randint(b[c], N)
            assert acc[c] == int(b[c].random_sample() < _log_ratio(new[c], old[c]))


def test_c_peek_equals_the_next_decide_without_consuming():
    """epipf_mh_peek gives the pick the next epipf_mh_decide draws and leaves the states untouched (positions at the
    end of the 624-word state included, where the draw regenerates it)."""
    from epipf import _lib
    L = _lib.load()
    nc, N = 30, 313
    rs = np.random.RandomState(4)
    a = [np.random.RandomState(11 * c + 2) for c in range(nc)]
    for c, r in enumerate(a):
        r.random_sample(311 + c)                         # words 622 + 2c: the next draw regenerates for the first few
    for it in range(20):
        ok = np.sort(rs.choice(nc, int(rs.randint(1, nc)), replace=False)).astype(np.int32)
        before = [r.get_state()[1].copy() for r in a]
        peek = np.full(nc, -1, dtype=np.int32)
        _lib.check(L.epipf_mh_peek(ok.size, _lib.ptr(ok), _states(a), N, _lib.ptr(peek)), "peek")
        assert all(np.array_equal(b, r.get_state()[1]) for b, r in zip(before, a))
        chosen = np.zeros(nc, dtype=np.int32)
        acc = np.zeros(nc, dtype=np.int32)
        z = np.zeros(nc)
        _lib.check(L.epipf_mh_decide(ok.size, _lib.ptr(ok), _states(a), N, _lib.ptr(z), _lib.ptr(z),
                                     _lib.ptr(chosen), _lib.ptr(acc)), "decide")
        np.testing.assert_array_equal(chosen[ok], peek[ok])
