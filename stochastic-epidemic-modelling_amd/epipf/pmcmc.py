"""Drop-in particle filter / PMCMC with the reference's call surface, running on MI355X.

Mirrors /root/reference/pmcmc.py:
  ModelType               pmcmc.py:116-120
  particle_filter         pmcmc.py:123-233   -> libepipf epipf_run (one GPU lane per particle)
  particle_path_sampler   pmcmc.py:236-248   (host version for arrays; particle_mcmc uses the device one)
  particle_mcmc           pmcmc.py:251-408   (host MH loop; filter + path sampling on the GPU)
plus `particle_mcmc_chains`, the same sampler run for several independent chains in lockstep, each
chain one GPU-batched filter per MH iteration.

Random numbers.  The reference draws everything from numpy's global MT19937.  Here:
  * MH proposals (multivariate_normal), acceptance uniforms and the path sampler's randint stay on
    the host RandomState (the global one by default), called in the reference's order;
  * the filter's own draws (initial Poisson states, resampling, Gillespie events) come from the keyed
    Philox stream: key = `key` (default: the module stream, see `seed_stream`), filter
    index = one per particle-filter call.
Under np.random.seed(s) + seed_stream(k) the results equal the reference's driven by the same
keyed stream (tests/golden/make_golden.py), which is how parity is tested.
"""
import ctypes
import math
from enum import Enum

import numpy as np

from . import _lib
from .engine import get_engine, model_id, n_compartments, theta_vector


class ModelType(Enum):
    SIR = "sir"
    SEIR = "seir"
    SIR_SUBGROUPS = "sir_subgroups"
    SIR_SUBGROUPS2 = "sir_subgroups2"


class _Stream:
    key = 0
    next_filter = 0
    next_abc_run = 0   # ABC runs (epipf.abc) count separately: their Philox domains are disjoint


_STREAM = _Stream()


def seed_stream(key, filter_index=0):
    """Set the module's Philox key and reset its filter counter (the analogue of np.random.seed for
    the filter's own draws)."""
    _STREAM.key = int(key) & (2**64 - 1)
    _STREAM.next_filter = int(filter_index)
    _STREAM.next_abc_run = 0


def _take_filter_index():
    f = _STREAM.next_filter
    _STREAM.next_filter += 1
    return f


def chain_key(key, chain):
    """Philox key of chain `chain` of a multi-chain run (chain 0 keeps `key`)."""
    return (int(key) + (int(chain) << 32)) & (2**64 - 1)


def _population(mid, G, n_population, mu):
    if mid >= _lib.SIR_SUBGROUPS:
        npop = np.atleast_1d(np.asarray(n_population, dtype=np.float64))
        mus = np.atleast_1d(np.asarray(mu, dtype=np.float64))
        if npop.size != G or mus.size != G:
            raise ValueError("subgroup models need n_population and mu with one entry per group")
        return npop, mus
    return np.array([float(n_population)]), np.array([float(mu)])


def _check_Y(mid, G, Y):
    Y = np.asarray(Y, dtype=np.float64)
    if Y.ndim != 2:
        raise ValueError("Y must be a 2-D array [T, K]")
    K = 3 if mid == _lib.SIR_SUBGROUPS2 else n_compartments(mid, G)
    if Y.shape[1] != K:
        raise ValueError(f"Y has {Y.shape[1]} columns, model observes {K}")
    return Y


def particle_filter(Y, type_model, theta_proposal, observations=False, probs=.1, n_particles=1000,
                    n_population=4820, mu=20, jobs=4, *, key=None, filter_index=None, resample="multinomial",
                    device=0, return_history=True):
    """pmcmc.py:123-233.  Returns (zetas[T], hidden_process[T,N,C], ancestry_matrix[T,N]) as float64,
    or (None, None, None) when every weight of some step is 0/NaN (the reference's ValueError path).
    `jobs` is accepted for compatibility and ignored (one GPU lane per particle)."""
    mid = model_id(type_model)
    th, G = theta_vector(mid, theta_proposal)
    Y = _check_Y(mid, G, Y)
    npop, mus = _population(mid, G, n_population, mu)
    eng = get_engine(mid, G, n_particles, Y.shape[0], 1, device)
    eng.set_observations(Y)
    eng.set_population(npop, mus)
    k = _STREAM.key if key is None else key
    f = _take_filter_index() if filter_index is None else filter_index
    lz, st = eng.run(th[None, :], [probs], [k], [f], observations=observations, resample=resample)
    if st[0] != _lib.STATUS_OK:
        return None, None, None
    zetas = np.exp(lz[0])
    if not return_history:
        return zetas, None, None
    hid, anc = eng.history(1)
    return zetas, hid[0].astype(np.float64), anc[0].astype(np.float64)


def particle_path_sampler(hidden_process, ancestry_matrix):
    """pmcmc.py:236-248, unchanged semantics (uniform final pick; ancestry[p] indexing)."""
    n_particles = hidden_process.shape[1]
    time_steps = hidden_process.shape[0]
    trajectory = np.zeros((time_steps, hidden_process.shape[2]))
    chosen_path = np.random.randint(0, n_particles)
    trajectory[-1, :] = hidden_process[-1, chosen_path, :]
    for p in range(time_steps - 2, -1, -1):
        chosen_path = int(ancestry_matrix[p, chosen_path])
        trajectory[p, :] = hidden_process[p, chosen_path, :]
    return trajectory


# ---------------------------------------------------------------------------------------- MH
def _reference_ratio(z_new, z_old, theta_new, theta_old, parameters, cov):
    """The reference's acceptance probability, pmcmc.py:376-393, evaluated verbatim (np.float64)."""
    from scipy.stats import multivariate_normal
    if "e" in str(z_new):
        constant = int(str(z_new).split("e-")[-1]) // 2
    else:
        constant = 1
    prob = (
        1e1 ** constant
        * multivariate_normal.pdf(theta_new, np.array(parameters), cov)
        * multivariate_normal.pdf(theta_old, theta_new, cov)
        * z_new
    )
    prob /= (
        1e1 ** constant
        * multivariate_normal.pdf(np.array(parameters), theta_new, cov)
        * multivariate_normal.pdf(theta_new, theta_old, cov)
        * z_old
    )
    return min(1, prob)


def mvn_factor(cov):
    """numpy's legacy RandomState.multivariate_normal(mean, cov) draws z = standard_normal(d) and returns
    z @ (sqrt(s)[:, None] * vh) + mean with (u, s, vh) = svd(cov).  The factor depends on cov only, so a cached
    factor gives bit-identical proposals with the same RNG consumption, without an SVD per draw (67 us -> 3 us)."""
    _, sv, vh = np.linalg.svd(np.asarray(cov, dtype=np.float64))
    return np.sqrt(sv)[:, None] * vh


def mvn_apply(z, fac, mean):
    """The rest of the legacy multivariate_normal arithmetic: np.dot(z, fac), then += mean."""
    x = np.dot(z.reshape(-1, fac.shape[0]), fac)
    x += mean
    return x.reshape(fac.shape[0])


def _raw_words(rng):
    """The MT19937 bit generator behind a legacy RandomState (or the np.random module's global one), else None."""
    if rng is np.random:
        rng = np.random.mtrand._rand
    if type(rng) is np.random.RandomState:
        bg = rng._bit_generator
        if type(bg) is np.random.MT19937:
            return bg
    return None


def legacy_randint(rng, n, bg=None):
    """rng.randint(0, n) for 1 <= n <= 2^32 with the same value and the same stream consumption: numpy's legacy
    bounded draw is masked rejection on 32-bit MT19937 words (v = next32 & mask until v <= n - 1), which is what the
    bit generator's random_raw() returns one at a time -- without randint's argument handling (~2.9 -> ~1.1 us).
    bg: _raw_words(rng), when the caller has it; other generators fall back to rng.randint."""
    if bg is None:
        bg = _raw_words(rng)
        if bg is None:
            return int(rng.randint(0, n))
    r = int(n) - 1
    if r <= 0:
        return 0
    mask = (1 << r.bit_length()) - 1
    while True:
        v = bg.random_raw() & mask
        if v <= r:
            return int(v)


class _MTPeek:
    """The value the next legacy_randint(rng, n) will return, read off the MT19937 state without consuming it (numpy's
    mt19937_state: uint32 key[624], int pos; a draw tempers key[pos++]), or None when the draw would have to regenerate
    the state first.  Lets the path sampler's final particle (pmcmc.py:241), drawn by the reference after the filter,
    be handed to the device with the filter itself (epipf_run_sampled); the real draw still happens in its place and
    is checked against the peeked one."""

    __slots__ = ("_bg", "_key", "_pos")

    def __init__(self, bg):
        addr = bg.ctypes.state_address
        self._bg = bg                                          # keeps the state alive
        self._key = (ctypes.c_uint32 * 624).from_address(addr)
        self._pos = ctypes.c_int.from_address(addr + 624 * 4)

    def randint(self, n):
        r = int(n) - 1
        if r <= 0:
            return 0
        mask = (1 << r.bit_length()) - 1
        pos, key = self._pos.value, self._key
        while pos < 624:
            y = key[pos]
            pos += 1
            y ^= y >> 11
            y ^= (y << 7) & 0x9D2C5680
            y ^= (y << 15) & 0xEFC60000
            y ^= y >> 18
            if y & mask <= r:
                return y & mask
        return None


class _NumpyDgemv:
    """numpy's own cblas_dgemv (its bundled OpenBLAS), the routine behind np.dot of a (1, d) row and a (d, d) matrix:
    passed to epipf_mh_propose so that the C proposals round exactly as multivariate_normal's np.dot.  Found once per
    process and accepted only if it reproduces np.dot bit for bit on random factors; else None (the Python path)."""
    _ptr = 0

    @classmethod
    def pointer(cls):
        if cls._ptr == 0:
            cls._ptr = None
            try:
                import glob
                import os
                libdir = os.path.join(os.path.dirname(os.path.dirname(np.__file__)), "numpy.libs")
                for path in sorted(glob.glob(os.path.join(libdir, "libscipy_openblas64_*.so"))):
                    f = ctypes.CDLL(path).scipy_cblas_dgemv64_
                    i64, P = ctypes.c_int64, ctypes.c_void_p
                    f.argtypes = [ctypes.c_int, ctypes.c_int, i64, i64, ctypes.c_double, P, i64, P, i64,
                                  ctypes.c_double, P, i64]
                    rs = np.random.RandomState(12345)
                    ok = True
                    for d in (2, 4, 6, 8):
                        for _ in range(25):
                            A = rs.standard_normal((d, d))
                            fac = np.ascontiguousarray(mvn_factor(A @ A.T))
                            z = rs.standard_normal(d)
                            y = np.empty(d)
                            f(101, 112, d, d, 1.0, fac.ctypes.data, d, z.ctypes.data, 1, 0.0, y.ctypes.data, 1)
                            ok = ok and bool((y == np.dot(z.reshape(1, d), fac).reshape(d)).all())
                    if ok:
                        cls._ptr = ctypes.cast(f, ctypes.c_void_p).value
                        break
            except (OSError, AttributeError):
                cls._ptr = None
        return cls._ptr


def _log_ratio(lz_new, lz_old):
    """Underflow-free MH acceptance probability min(1, z'/z) from log-likelihoods (the symmetric
    Gaussian proposal terms of pmcmc.py:380-391 cancel)."""
    lr = lz_new - lz_old
    if math.isnan(lr):
        return 0.0
    return min(1.0, math.exp(min(lr, 0.0)))


class ChainResult:
    """Per-chain outputs in the reference's layout plus run counters."""

    def __init__(self, thetas, likelihoods, log_likelihoods, sampled_trajs, acceptances, filters_run):
        self.thetas = thetas
        self.likelihoods = likelihoods
        self.log_likelihoods = log_likelihoods
        self.sampled_trajs = sampled_trajs
        self.acceptances = acceptances
        self.filters_run = filters_run


class ChainSampler:
    """Lockstep random-walk PMCMC over `chains` independent chains (pmcmc.py:251-408 each), one batched
    GPU filter per MH iteration.  `iters` keeps the reference's `n_chains` meaning (MH iterations per
    chain).  Use `initialise()` then `step()` iters-1 times (or `run()`); results via `results()`.

    parameters: the starting theta (pmcmc.py:277), or one per chain as a [chains, d] array; sigma likewise [d, d]
    or [chains, d, d].
    rngs: per-chain RandomState-like objects (proposals, path picks, acceptance uniforms).
    keys: per-chain Philox keys for the filters; filter indices count from `filter_index_start`."""

    FUSE_PATH_CHAINS = 16

    def __init__(self, Y, type_model, parameters, h, adaptive=False, sigma=None, iters=1000, observations=False,
                 probs=.1, n_particles=1000, n_population=4820, mu=20, *, rngs, keys, device=0,
                 mh_ratio="reference", resample="multinomial", filter_index_start=0, engine_chains=0, engine=None,
                 host_draws=True):
        self.rngs = list(rngs)
        self.keys = np.asarray(keys, dtype=np.uint64)
        nc = self.nc = len(self.rngs)
        mid = self.mid = model_id(type_model)
        P = np.asarray(parameters, dtype=np.float64)
        d = self.d = P.shape[-1]
        # per-chain starting points (a [chains, d] array, e.g. warm starts, chains_io.warm_start) or one for all
        if P.ndim == 2 and P.shape[0] != nc:
            raise ValueError(f"parameters has {P.shape[0]} per-chain rows for {nc} chains")
        if P.ndim not in (1, 2):
            raise ValueError("parameters must be [d] or [chains, d]")
        self.params = [(P[c] if P.ndim == 2 else P).tolist() for c in range(nc)]
        self.parameters = self.params[0] if nc else P.tolist()
        self.probs = probs
        self.h = h
        self.adaptive = adaptive
        self.observations = observations
        self.mh_ratio = mh_ratio
        self.resample = resample
        self.N = int(n_particles)
        G = int(round(math.sqrt(d - (2 if probs is None else 1)))) if mid >= _lib.SIR_SUBGROUPS else 1
        Y = _check_Y(mid, G, Y)
        T = self.T = Y.shape[0]
        Cc = n_compartments(mid, G)
        npop, mus = _population(mid, G, n_population, mu)
        self.iters = int(iters)
        if engine is None:
            eng = get_engine(mid, G, n_particles, T, max(nc, int(engine_chains)), device)
        else:                                                     # a private context (run_pipelined)
            eng = engine
            if (eng.model, eng.G, eng.N) != (mid, G, self.N) or eng.t_max < T or eng.max_chains < max(nc, engine_chains):
                raise ValueError("engine does not match the model / particles / T / chains of this sampler")
        self.eng = eng
        self._Y, self._npop, self._mus = Y, npop, mus
        self._bind()
        self.thetas = np.zeros((nc, self.iters, d))
        self.likelihoods = np.zeros((nc, self.iters))
        self.loglik = np.zeros((nc, self.iters))
        # sampled trajectories, iteration-major per chain (one contiguous [T, C] block per MH iteration, so an
        # iteration's bookkeeping is a block copy); `trajs` is the [chains, T, iters, C] view of the reference layout
        self._tr = np.zeros((nc, self.iters, T, Cc))
        self.trajs = self._tr.transpose(0, 2, 1, 3)
        S = None if sigma is None else np.asarray(sigma, dtype=np.float64)
        if S is not None and S.ndim == 3 and S.shape[0] != nc:
            raise ValueError(f"sigma has {S.shape[0]} per-chain matrices for {nc} chains")
        if S is not None and (S.ndim not in (2, 3) or S.shape[-2:] != (d, d)):
            raise ValueError(f"sigma must be [{d}, {d}] or [chains, {d}, {d}]")
        self.std = [np.eye(d) if S is None else (S[c] if S.ndim == 3 else S).copy() for c in range(nc)]
        self._fac = [None] * nc                                  # multivariate_normal factor of h * std[c]
        # per-chain counters as int64 arrays (updated for all chains at once in step())
        self.fnext = np.full(nc, int(filter_index_start), dtype=np.int64)
        self.filters_run = np.zeros(nc, dtype=np.int64)
        # per-chain host RNG entry points, looked up once (a step makes 3 calls per chain)
        self._normal = [r.standard_normal for r in self.rngs]
        self._uniform = [r.random_sample for r in self.rngs]
        self._raw = [_raw_words(r) for r in self.rngs]
        self._dbuf = np.empty((nc, d))
        # up to FUSE_PATH_CHAINS chains the path sampler rides on the filter's launch (epipf_run_sampled): its
        # randint is peeked before the filter (_MTPeek); more chains amortise the separate call better than the peeks
        self._peek = None
        if nc <= self.FUSE_PATH_CHAINS and all(b is not None for b in self._raw):
            self._peek = [_MTPeek(b) for b in self._raw]
        # more chains: the host draws of an iteration in C (epipf_mh_propose / epipf_mh_decide, csrc/host_mh.cpp) --
        # legacy RandomStates the sampler drives alone, an even d (whole gaussian pairs), an empty gaussian cache,
        # the log-space acceptance, and numpy's own dgemv at hand
        self._host = None
        if (host_draws and nc > self.FUSE_PATH_CHAINS and d % 2 == 0 and mh_ratio == "log"
                and all(b is not None for b in self._raw) and len({id(b) for b in self._raw}) == nc
                and all(int(r.get_state()[3]) == 0 for r in (np.random.mtrand._rand if r is np.random else r
                                                            for r in self.rngs))
                and _NumpyDgemv.pointer()):
            self._host = (ctypes.c_void_p * nc)(*[b.ctypes.state_address for b in self._raw])
            self._host_peek = True
            self._facs = np.zeros((nc, d, d))
            self._facs_ok = False
        self.acceptances = np.ones(nc, dtype=np.int64)
        self.dth = d - (1 if probs is None else 0)
        self.i = 0
        self.last_active = 0

    def _bind(self):
        """(Re)load this sampler's observations and population into its engine before a run: a cached engine is
        shared with every other sampler / particle_filter call of the same model, N and device (no-op when
        unchanged, engine.set_observations / set_population compare first)."""
        # the engine holds this sampler's token, not the sampler: no sampler -> engine -> sampler cycle keeping a
        # finished sampler's arrays and the engine's HIP context alive until a GC cycle
        tok = self.__dict__.setdefault("_bind_token", object())
        if getattr(self.eng, "bound_to", None) is tok:    # nothing re-uploaded the engine's data since this sampler's
            return
        self.eng.set_observations(self._Y)
        self.eng.set_population(self._npop, self._mus)
        self.eng.bound_to = tok

    def _propose(self, c, mean):
        """rngs[c].multivariate_normal(mean, h * std[c]) (pmcmc.py:277, :330) with the SVD factor cached per chain."""
        if self._fac[c] is None:
            self._fac[c] = mvn_factor(self.h * self.std[c])
        return mvn_apply(self.rngs[c].standard_normal(self.d), self._fac[c], mean)

    def _split(self, prop):
        """probs / subgroup reshaping, pmcmc.py:283-296 and :339-352 (the subgroup beta matrix is the
        row-major flattening of theta[:G*G], i.e. theta itself)."""
        if self.probs is None:
            probs2 = min(prop[-1], 1)
            probs2 = max(probs2, 0)
            return prop[:-1], probs2
        return prop, self.probs

    def _run_batch(self, props):
        nc = self.nc
        th_all = np.zeros((nc, self.dth))
        pr_all = np.zeros(nc)
        act = np.zeros(nc, dtype=np.int32)
        fidx = np.zeros(nc, dtype=np.uint64)
        stripped = {}
        for c, prop in props.items():
            th, p2 = self._split(prop)
            stripped[c] = (th, p2)
            th_all[c] = th
            pr_all[c] = p2
            act[c] = 1
            fidx[c] = self.fnext[c]
            self.fnext[c] += 1
            self.filters_run[c] += 1
        self._bind()
        lz, st = self.eng.run(th_all, pr_all, self.keys, fidx, observations=self.observations, active=act,
                              resample=self.resample)
        self.last_active = len(props)
        return lz, st, stripped

    def _path_sample(self, ok):
        chosen = np.zeros(self.nc, dtype=np.int32)
        N, rngs, raw = self.N, self.rngs, self._raw
        for c in ok:
            chosen[c] = legacy_randint(rngs[c], N, raw[c])          # pmcmc.py:241, host RNG order kept
        return self.eng.path_sample(chosen)

    def _copy_prev(self, c, i):
        self.thetas[c, i] = self.thetas[c, i - 1]
        self.likelihoods[c, i] = self.likelihoods[c, i - 1]
        self.loglik[c, i] = self.loglik[c, i - 1]
        self._tr[c, i] = self._tr[c, i - 1]

    def initialise(self):
        """The initial draw loop, pmcmc.py:276-318 (repeat until theta >= 0 and the filter succeeded)."""
        pending = list(range(self.nc))
        while pending:
            props = {}
            for c in pending:
                prop = self._propose(c, np.array(self.params[c]))
                if sum(prop < 0) > 0:
                    continue
                props[c] = prop
            if not props:
                continue
            lz, st, stripped = self._run_batch(props)
            ok = [c for c in props if st[c] == _lib.STATUS_OK]
            if ok:
                tr = self._path_sample(ok)
                for c in ok:
                    th, p2 = stripped[c]
                    if self.probs is None:
                        th = np.append(th, p2)
                    self.thetas[c, 0] = th
                    self.loglik[c, 0] = lz[c, -1]
                    self.likelihoods[c, 0] = np.exp(lz[c, -1])
                    self.trajs[c, :, 0, :] = tr[c]
            pending = [c for c in pending if c not in ok]
        self.i = 1

    def _step_one(self):
        """step() for a single chain (particle_mcmc; BASELINE config 5's one chain per GPU) on plain Python scalars:
        the batched step's ~30 small numpy calls cost ~50-90 us an iteration, ~7% of a config-5 one-chain MH
        iteration, between two filters.  Same RNG calls in the same order, same arithmetic (the proposal's np.dot and
        + theta; the log- or reference-ratio acceptance), same bookkeeping."""
        i, d = self.i, self.d
        if self.adaptive and i > 1e3:
            self.std[0] = np.cov(self.thetas[0, :i].T, ddof=0) + 1e-4 * np.eye(self.d)
            self._fac[0] = None
        f = self._fac[0]
        if f is None:
            f = self._fac[0] = mvn_factor(self.h * self.std[0])
        D = self._dbuf
        np.dot(self._normal[0](d).reshape(1, d), f, out=D)
        prop = D[0] + self.thetas[0, i - 1]
        pl = prop.tolist()
        ran = 0
        take = False
        if not any(v < 0 for v in pl):                            # sum(prop < 0) > 0: no filter, :333-337
            ran = 1
            if self.probs is None:                                # :339-346: the last entry is probs
                p2 = min(max(pl[-1], 0.0), 1.0)
                th = prop[:-1]
                new = pl[:-1] + [p2]
            else:
                p2 = float(self.probs)
                th = prop
                new = pl
            fidx = int(self.fnext[0])
            self.fnext[0] += 1
            self.filters_run[0] += 1
            self._bind()
            pre = None
            if self._peek is not None:                            # the path pick, peeked (see _MTPeek)
                v = self._peek[0].randint(self.N)
                if v is not None:
                    pre = [v]
            out = self.eng.run(th[None, :], [p2], self.keys, [fidx], observations=self.observations,
                               resample=self.resample, chosen=pre)
            self.last_active = 1
            if int(out[1][0]) == _lib.STATUS_OK:                  # degenerate filters: rejected, :365-369
                real = legacy_randint(self.rngs[0], self.N, self._raw[0])
                if pre is None:
                    chosen = np.array([real], dtype=np.int32)
                    tr = self.eng.path_sample(chosen)[0]
                elif real == pre[0]:
                    tr = out[2][0]
                else:                                             # (never seen) walk the drawn pick instead
                    self._peek = None
                    tr = self.eng.path_sample(np.array([real], dtype=np.int32))[0]
                lzT = float(out[0][0, -1])
                if self.mh_ratio == "reference":
                    prob = _reference_ratio(np.exp(out[0][0, -1]), self.likelihoods[0, i - 1], np.array(new),
                                            self.thetas[0, i - 1], self.params[0], self.h * self.std[0])
                else:
                    prob = _log_ratio(lzT, float(self.loglik[0, i - 1]))
                if self._uniform[0]() < prob:
                    take = True
                    self.acceptances[0] += 1
                    self.thetas[0, i] = new
                    self.loglik[0, i] = lzT
                    self.likelihoods[0, i] = np.exp(out[0][0, -1])
                    self._tr[0, i] = tr
        if not take:                                              # rejected, negative or degenerate: previous row
            self.thetas[0, i] = self.thetas[0, i - 1]
            self.likelihoods[0, i] = self.likelihoods[0, i - 1]
            self.loglik[0, i] = self.loglik[0, i - 1]
            self._tr[0, i] = self._tr[0, i - 1]
        self.i += 1
        return ran

    def step(self):
        """One MH iteration for every chain, pmcmc.py:325-406.  Returns the number of chains that ran a filter.
        Per chain the RNG calls keep the reference's order (proposal normals, path-pick randint, acceptance
        uniform); everything else -- the negative-proposal test, the batch arrays, the accepted rows and the copies
        of the previous row -- is one array operation over the chains."""
        if self.nc == 1:
            return self._step_one()
        i = self.i
        nc, d = self.nc, self.d
        if self.adaptive and i > 1e3:
            for c in range(nc):
                self.std[c] = np.cov(self.thetas[c, :i].T, ddof=0) + 1e-4 * np.eye(self.d)
                self._fac[c] = None
            self._facs_ok = False
        # multivariate_normal(theta, h std) per chain (mvn_apply's arithmetic: np.dot(z, factor) per chain -- a
        # batched product would take another BLAS kernel and round differently -- then + theta for all chains)
        D, fac, normal = self._dbuf, self._fac, self._normal
        if self._host is not None:
            if not self._facs_ok:                                 # factors (re)computed: start, adaptive update
                for c in range(nc):
                    if fac[c] is None:
                        fac[c] = mvn_factor(self.h * self.std[c])
                self._facs[:] = np.stack(fac)
                self._facs_ok = True
            mean = np.ascontiguousarray(self.thetas[:, i - 1])
            P = np.empty((nc, d))
            _lib.check(_lib.load().epipf_mh_propose(nc, d, self._host, _lib.ptr(self._facs), _lib.ptr(mean),
                                                    _lib.ptr(P), _NumpyDgemv.pointer()), "epipf_mh_propose")
        else:
            for c in range(nc):
                f = fac[c]
                if f is None:
                    f = fac[c] = mvn_factor(self.h * self.std[c])
                np.dot(normal[c](d).reshape(1, d), f, out=D[c:c + 1])
            P = D + self.thetas[:, i - 1]
        live = ~(P < 0).any(axis=1)                               # sum(prop < 0) > 0: no filter, :333-337
        lv = np.flatnonzero(live)
        acc = np.zeros(0, dtype=np.intp)
        if lv.size:
            if self.probs is None:                                # pmcmc.py:339-346: the last entry is probs
                th_all, pr_all = P[:, :-1], np.clip(P[:, -1], 0.0, 1.0)
                new_all = np.concatenate([th_all, pr_all[:, None]], axis=1)
            else:
                th_all, pr_all, new_all = P, np.full(nc, float(self.probs)), P
            fidx = np.zeros(nc, dtype=np.uint64)
            fidx[lv] = self.fnext[lv]
            self.fnext[lv] += 1
            self.filters_run[lv] += 1
            self._bind()
            pre = None
            if self._peek is not None:                            # the path pick, peeked (see _MTPeek)
                pre = np.full(nc, -1, dtype=np.int32)
                for c in lv.tolist():
                    v = self._peek[c].randint(self.N)
                    if v is None:
                        pre = None
                        break
                    pre[c] = v
            elif self._host is not None and self._host_peek:     # many chains: peeked in C (epipf_mh_peek)
                pre = np.full(nc, -1, dtype=np.int32)
                lvc = lv.astype(np.int32)
                _lib.check(_lib.load().epipf_mh_peek(lv.size, _lib.ptr(lvc), self._host, self.N, _lib.ptr(pre)),
                           "epipf_mh_peek")
            out = self.eng.run(np.ascontiguousarray(th_all), pr_all, self.keys, fidx, observations=self.observations,
                               active=live.astype(np.int32), resample=self.resample, chosen=pre)
            lz, st = out[0], out[1]
            self.last_active = int(lv.size)
            ok = np.flatnonzero(live & (st == _lib.STATUS_OK))    # degenerate filters: rejected, :365-369
            if ok.size and self._host is not None:            # picks and acceptance uniforms in C, in order
                chosen = np.zeros(nc, dtype=np.int32)
                acc_f = np.zeros(nc, dtype=np.int32)
                lzT = np.ascontiguousarray(lz[:, -1])
                old = np.ascontiguousarray(self.loglik[:, i - 1])
                _lib.check(_lib.load().epipf_mh_decide(ok.size, _lib.ptr(ok.astype(np.int32)), self._host, self.N,
                                                       _lib.ptr(lzT), _lib.ptr(old), _lib.ptr(chosen),
                                                       _lib.ptr(acc_f)), "epipf_mh_decide")
                if pre is not None and np.array_equal(chosen[ok], pre[ok]):
                    tr = out[2]                                   # walked on the filter's stream
                else:
                    if pre is not None:                           # (never seen) walk the drawn picks instead
                        self._host_peek = False
                    tr = self.eng.path_sample(chosen)
                acc = ok[acc_f[ok] == 1]
                self.acceptances[acc] += 1
                if acc.size:
                    self.thetas[acc, i] = new_all[acc]
                    self.loglik[acc, i] = lzT[acc]
                    self.likelihoods[acc, i] = np.exp(lzT[acc])
                    self._tr[acc, i] = tr[acc]
            elif ok.size:
                okl = ok.tolist()
                if pre is None:
                    tr = self._path_sample(okl)
                else:                                             # the reference's randint, drawn in its place
                    tr = out[2]
                    real = [legacy_randint(self.rngs[c], self.N, self._raw[c]) for c in okl]
                    if real != pre[ok].tolist():                  # (never seen) walk the drawn picks instead
                        self._peek = None
                        chosen = np.zeros(nc, dtype=np.int32)
                        chosen[ok] = real
                        tr = self.eng.path_sample(chosen)
                lzT = lz[:, -1]
                take = []
                uniform = self._uniform
                if self.mh_ratio == "reference":
                    for c in okl:
                        prob = _reference_ratio(np.exp(lzT[c]), self.likelihoods[c, i - 1], new_all[c],
                                                self.thetas[c, i - 1], self.params[c], self.h * self.std[c])
                        if uniform[c]() < prob:                    # == uniform(): 0 + 1*U, 7x cheaper
                            take.append(c)
                else:                                              # _log_ratio, the differences for all chains at once
                    exp, isnan = math.exp, math.isnan
                    for c, lr in zip(okl, (lzT[ok] - self.loglik[ok, i - 1]).tolist()):
                        prob = 0.0 if isnan(lr) else min(1.0, exp(min(lr, 0.0)))
                        if uniform[c]() < prob:
                            take.append(c)
                for c in take:
                    self.acceptances[c] += 1
                if take:
                    acc = np.asarray(take, dtype=np.intp)
                    self.thetas[acc, i] = new_all[acc]
                    self.loglik[acc, i] = lzT[acc]
                    self.likelihoods[acc, i] = np.exp(lzT[acc])
                    self._tr[acc, i] = tr[acc]
        rej = np.ones(nc, dtype=bool)
        rej[acc] = False
        if rej.any():                                             # rejected, negative or degenerate: previous row
            r = np.flatnonzero(rej)
            self.thetas[r, i] = self.thetas[r, i - 1]
            self.likelihoods[r, i] = self.likelihoods[r, i - 1]
            self.loglik[r, i] = self.loglik[r, i - 1]
            self._tr[r, i] = self._tr[r, i - 1]
        self.i += 1
        return int(lv.size)

    def run(self, progress=False, on_iteration=None):
        if self.i == 0:
            self.initialise()
        bar = None
        if progress:
            from tqdm import tqdm
            bar = tqdm(total=self.iters - 1, desc="Chains", position=1)
        while self.i < self.iters:
            n = self.step()
            if bar is not None:
                i = self.i - 1
                bar.update(1)
                bar.set_postfix_str(f"accepted_theta: {self.thetas[0, i]}, "
                                    f"acceptance_ratio: {100 * self.acceptances[0] / (i + 1)}%")
            if on_iteration is not None:
                on_iteration(self.i - 1, n)
        if bar is not None:
            bar.close()
        return self.results()

    def results(self):
        return [ChainResult(self.thetas[c], self.likelihoods[c], self.loglik[c], self.trajs[c],
                            int(self.acceptances[c]), int(self.filters_run[c])) for c in range(self.nc)]

    def packed_draws(self, upto=None):
        """epipf.distributed.pack_draws(self.results(), upto) for all chains at once: [chains, n d + n] rows of
        (thetas flattened, log-likelihoods), n = upto or every iteration."""
        n = self.iters if upto is None else min(int(upto), self.iters)
        return np.concatenate([self.thetas[:, :n].reshape(self.nc, -1), self.loglik[:, :n]], axis=1)


PIPELINE_SWITCH_S = 1e-4


def run_pipelined(samplers, steps):
    """Advance independent ChainSamplers `steps` MH iterations each, one host thread per sampler, and return the
    number of filters run.  Each sampler must own its engine (ChainSampler(..., engine=Engine(...))): a filter call
    releases the GIL for its whole device run (ctypes), so one sampler's host work (proposals, path picks,
    accept/reject) overlaps the other samplers' filters on the device instead of leaving it idle between MH
    iterations.  Every sampler's chains, draws and results are exactly those of calling its step() `steps` times.

    While it runs, the interpreter's thread switch interval is at most PIPELINE_SWITCH_S: a thread back from a filter
    call otherwise can wait out the default 5 ms for the GIL whenever the holder releases and retakes it within short
    C calls -- whole-millisecond stalls in sub-millisecond MH iterations (profiles/r5v_cfg1_chains.jsonl)."""
    import sys
    import threading
    engines = [id(s.eng) for s in samplers]
    if len(set(engines)) != len(engines):
        raise ValueError("run_pipelined needs one engine per sampler")
    counts = [0] * len(samplers)
    errors = []

    def work(k):
        try:
            for _ in range(steps):
                counts[k] += samplers[k].step()
        except BaseException as e:  # noqa: BLE001 -- re-raised in the caller's thread
            errors.append(e)

    threads = [threading.Thread(target=work, args=(k,), daemon=True) for k in range(len(samplers))]
    switch = sys.getswitchinterval()
    sys.setswitchinterval(min(switch, PIPELINE_SWITCH_S))
    try:
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    finally:
        sys.setswitchinterval(switch)
    if errors:
        raise errors[0]
    return sum(counts)


def prefetch_slots(n_particles):
    """Default speculative slots for one chain: about 2.5 resident waves per SIMD of filters in flight
    (2560 waves of 64 particles; a round's latency barely grows until then), within [8, 64].  Config 2
    (N = 10^4, 157 waves per filter) -> 16, the best of scripts/prefetch_sweep.py's sweep there."""
    waves = -(-int(n_particles) // 64)
    return int(min(64, max(8, 2560 // waves)))


def particle_mcmc_chains(Y, type_model, parameters, h, adaptive=False, sigma=None, n_chains=1000,
                         observations=False, probs=.1, n_particles=1000, n_population=4820, mu=20, *,
                         rngs=None, keys=None, chains=1, seed=0, device=0, mh_ratio="reference",
                         resample="multinomial", progress=False, filter_index_start=0, on_iteration=None,
                         prefetch=0):
    """Run `chains` independent PMCMC chains (pmcmc.py:251-408 each).  `n_chains` keeps the reference's
    meaning: MH iterations per chain.  Default rngs: np.random.RandomState(seed + c); default keys:
    chain_key(seed, c).  prefetch=0: lockstep, one batched filter per MH iteration (ChainSampler);
    prefetch=K: speculative MH with max(K, chains) filter slots per batch (epipf.prefetch.PrefetchSampler,
    same results).  Returns a list of ChainResult."""
    if rngs is None:
        rngs = [np.random.RandomState(seed + c) for c in range(chains)]
    if keys is None:
        keys = [chain_key(seed, c) for c in range(len(rngs))]
    args = (Y, type_model, parameters, h, adaptive, sigma, n_chains, observations, probs, n_particles, n_population, mu)
    kw = dict(rngs=rngs, keys=keys, device=device, mh_ratio=mh_ratio, resample=resample,
              filter_index_start=filter_index_start)
    if prefetch:
        from .prefetch import PrefetchSampler
        sampler = PrefetchSampler(*args, slots="auto" if prefetch == "auto" else max(int(prefetch), len(rngs)), **kw)
    else:
        sampler = ChainSampler(*args, **kw)
    return sampler.run(progress=progress, on_iteration=on_iteration)


def particle_mcmc(Y, type_model, parameters, h, adaptive=False, sigma=None, n_chains=1000, observations=False,
                  probs=.1, n_particles=1000, n_population=4820, mu=20, jobs=4, *, key=None, device=0,
                  mh_ratio="reference", resample="multinomial", progress=True, prefetch="auto"):
    """pmcmc.py:251-408 with the same signature and return value (thetas, likelihoods, sampled_trajs).

    Uses numpy's GLOBAL RandomState for proposals / acceptance / path picks, as the reference, and the
    module Philox stream (seed_stream) for the filters.  mh_ratio="reference" evaluates the reference's
    acceptance expression verbatim (linear likelihoods, MVN factors); "log" uses log-likelihoods and
    stays correct when the likelihood underflows (T ≳ 150 observations).  prefetch=K evaluates up to K
    speculative MH iterations per batched GPU launch (epipf.prefetch; identical results, and the global
    RandomState ends where the sequential loop leaves it); "auto" sizes each round from the chain's acceptance
    rate and the measured round time (epipf.prefetch.SlotTuner); prefetch=0 runs one filter per iteration."""
    k = _STREAM.key if key is None else key
    # "auto": speculative MH whose round width follows the chain's acceptance rate and the measured round time
    # (epipf.prefetch.SlotTuner), within [1, 2 prefetch_slots(n_particles)]
    res = particle_mcmc_chains(Y, type_model, parameters, h, adaptive, sigma, n_chains, observations, probs,
                               n_particles, n_population, mu, rngs=[np.random], keys=[k], device=device,
                               mh_ratio=mh_ratio, resample=resample, progress=progress,
                               filter_index_start=_STREAM.next_filter, prefetch=prefetch)[0]
    if key is None:
        _STREAM.next_filter += res.filters_run
    return res.thetas, res.likelihoods, res.sampled_trajs.astype(np.float64)
