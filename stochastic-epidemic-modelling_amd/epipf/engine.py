"""Engine: one libepipf context (device buffers for a model / particle-count / horizon / chain batch).

This is the layer the drop-in `particle_filter` / `particle_mcmc` call.  An engine keeps the
observations, the log-factorial table and the whole particle history resident in HBM; a batched
`run()` moves only per-chain parameters in and log-likelihoods + status out.
"""
import atexit
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check, ptr

# Particle-steps of every epipf_run in this process, counted as bench.py's `value` counts them (N x T per chain that
# runs a filter; chains passed as inactive count nothing).  With EPIPF_PMC_COUNT=<file> the total is appended to <file>
# at exit: scripts/profile.sh divides each rocprofv3 pass's counter totals by it (scripts/parse_rocprof.py).
_PARTICLE_STEPS = [0]


def _write_pmc_count():
    with open(os.environ["EPIPF_PMC_COUNT"], "a") as f:
        f.write(f"{_PARTICLE_STEPS[0]}\n")


if os.environ.get("EPIPF_PMC_COUNT"):
    atexit.register(_write_pmc_count)

MODEL_IDS = {"sir": _lib.SIR, "seir": _lib.SEIR, "sir_subgroups": _lib.SIR_SUBGROUPS,
             "sir_subgroups2": _lib.SIR_SUBGROUPS2}


def model_id(type_model):
    """Accept this package's ModelType, the reference's ModelType (same .value strings) or a string."""
    name = getattr(type_model, "value", type_model)
    if isinstance(name, (int, np.integer)) and 0 <= int(name) <= 3:
        return int(name)
    if isinstance(name, str) and name.lower() in MODEL_IDS:
        return MODEL_IDS[name.lower()]
    raise ValueError(f"unknown model type {type_model!r}")


def n_compartments(mid, G):
    return 3 if mid == _lib.SIR else 4 if mid == _lib.SEIR else 3 * G


def theta_vector(mid, theta):
    """Flatten a reference theta: SIR/SEIR arrays, or (beta[G][G], gamma) for the subgroup models
    (pmcmc.py:211-218 passes theta_proposal[0], theta_proposal[1])."""
    if mid in (_lib.SIR_SUBGROUPS, _lib.SIR_SUBGROUPS2):
        beta, gamma = theta
        beta = np.asarray(beta, dtype=np.float64)
        if beta.ndim != 2 or beta.shape[0] != beta.shape[1]:
            raise ValueError("subgroup theta must be (beta[G][G], gamma)")
        return np.append(beta.reshape(-1), float(gamma)), beta.shape[0]
    th = np.asarray(theta, dtype=np.float64).reshape(-1)
    need = 2 if mid == _lib.SIR else 3
    if th.size != need:
        raise ValueError(f"theta must have {need} entries for this model, got {th.size}")
    return th, 1


class Engine:
    def __init__(self, type_model, groups=1, n_particles=1000, t_max=1, max_chains=1, device=0):
        L = _lib.load()
        self.model = model_id(type_model)
        self.G = int(groups) if self.model >= _lib.SIR_SUBGROUPS else 1
        self.C = n_compartments(self.model, self.G)
        self.K = 3 if self.model == _lib.SIR_SUBGROUPS2 else self.C
        self.N = int(n_particles)
        self.t_max = int(t_max)
        self.max_chains = int(max_chains)
        self.device = int(device)
        h = ctypes.c_void_p()
        check(L.epipf_create(ctypes.byref(h), self.device, self.model, self.G, self.N, self.t_max, self.max_chains),
              "epipf_create")
        self._h = h
        self._L = L
        self._Y = None
        self._pop = None
        self.bound_to = None                             # token of the ChainSampler whose data is loaded (_bind)
        self.T = 0

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.epipf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ inputs
    def set_observations(self, Y):
        Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
        if Y.ndim != 2:
            raise ValueError("Y must be 2-D [T, K]")
        if self._Y is not None and self._Y.shape == Y.shape and np.array_equal(self._Y, Y, equal_nan=True):
            return
        check(self._L.epipf_set_observations(self._h, ptr(Y), Y.shape[0], Y.shape[1]), "epipf_set_observations")
        self._Y = Y.copy()
        self.bound_to = None                             # ChainSampler._bind: the data it bound is gone
        self.T = Y.shape[0]

    def set_population(self, n_population, mu):
        npop = np.ascontiguousarray(np.atleast_1d(np.asarray(n_population, dtype=np.float64)))
        mus = np.ascontiguousarray(np.atleast_1d(np.asarray(mu, dtype=np.float64)))
        if npop.size != self.G or mus.size != self.G:
            raise ValueError(f"n_population and mu need {self.G} entries")
        key = (tuple(npop), tuple(mus))
        if key == self._pop:
            return
        check(self._L.epipf_set_population(self._h, ptr(npop), ptr(mus)), "epipf_set_population")
        self._pop = key
        self.bound_to = None

    # ------------------------------------------------------------------ the filter
    def run(self, thetas, probs, keys, filter_indices, observations=False, active=None, resample="multinomial",
            chosen=None):
        """Run len(thetas) independent filters.  Returns (log_zetas [n, T], status [n]); with chosen [n] (the path
        sampler's final particles, -1 for none) also the sampled trajectories [n, T, C] int32 (epipf_run_sampled)."""
        thetas = np.ascontiguousarray(np.asarray(thetas, dtype=np.float64))
        n = thetas.shape[0]
        probs = np.ascontiguousarray(np.broadcast_to(np.asarray(probs, dtype=np.float64), (n,)))
        keys = np.ascontiguousarray(np.broadcast_to(np.asarray(keys, dtype=np.uint64), (n,)))
        fidx = np.ascontiguousarray(np.broadcast_to(np.asarray(filter_indices, dtype=np.uint64), (n,))
                                    .astype(np.uint32))
        act = None if active is None else np.ascontiguousarray(np.asarray(active, dtype=np.int32))
        lz = np.empty((n, self.T), dtype=np.float64)
        st = np.empty(n, dtype=np.int32)
        mode = _lib.RESAMPLE_MULTINOMIAL if resample == "multinomial" else _lib.RESAMPLE_SYSTEMATIC
        obs = _lib.OBS_NORMAL if observations else _lib.OBS_BINOMIAL
        if chosen is None:
            check(self._L.epipf_run(self._h, n, ptr(thetas), thetas.shape[1], obs, ptr(probs), ptr(keys), ptr(fidx),
                                    ptr(act), mode, ptr(lz), ptr(st)), "epipf_run")
        else:
            ch = np.ascontiguousarray(np.asarray(chosen, dtype=np.int32).reshape(-1))
            if ch.size != n:
                raise ValueError(f"chosen has {ch.size} entries for {n} filters")
            tr = np.empty((n, self.T, self.C), dtype=np.int32)
            check(self._L.epipf_run_sampled(self._h, n, ptr(thetas), thetas.shape[1], obs, ptr(probs), ptr(keys),
                                            ptr(fidx), ptr(act), mode, ptr(ch), ptr(lz), ptr(st), ptr(tr)),
                  "epipf_run_sampled")
        self._last_n = n
        _PARTICLE_STEPS[0] += (n if act is None else int(np.count_nonzero(act))) * self.N * self.T
        return (lz, st) if chosen is None else (lz, st, tr)

    def history(self, n_chains=None):
        """(hidden [n, T, N, C] int32, ancestry [n, T, N] int32) of the last run."""
        n = self._last_n if n_chains is None else int(n_chains)
        hid = np.empty((n, self.T, self.N, self.C), dtype=np.int32)
        anc = np.empty((n, self.T, self.N), dtype=np.int32)
        check(self._L.epipf_copy_history(self._h, n, ptr(hid), ptr(anc)), "epipf_copy_history")
        return hid, anc

    def path_sample(self, chosen):
        chosen = np.ascontiguousarray(np.asarray(chosen, dtype=np.int32).reshape(-1))
        out = np.empty((chosen.size, self.T, self.C), dtype=np.int32)
        check(self._L.epipf_path_sample(self._h, chosen.size, ptr(chosen), ptr(out)), "epipf_path_sample")
        return out

    # ------------------------------------------------------------------ aux entry points
    def simulate(self, states, theta, max_time=1.0, key=0, filter_index=0, step=0):
        states = np.ascontiguousarray(np.asarray(states, dtype=np.int32).reshape(-1, self.C))
        th, _ = theta_vector(self.model, theta)
        th = np.ascontiguousarray(th)
        out = np.empty_like(states)
        ev = np.zeros(1, dtype=np.int64)
        check(self._L.epipf_simulate(self._h, states.shape[0], ptr(states), ptr(th), th.size, float(max_time),
                                     int(key) & (2**64 - 1), int(filter_index) & 0xFFFFFFFF, int(step), ptr(out),
                                     ptr(ev)), "epipf_simulate")
        return out, int(ev[0])

    def simulate_path(self, states, theta, max_time=1.0, key=0, filter_index=0, step=0, max_events=None):
        """Full event paths from int states [n, C]: (times [n, cap], states [n, cap, C] int32, n_events [n],
        final [n, C] int32); row j holds trajectory j's first n_events[j] events.  With max_events=None the buffer
        grows to the longest path (a second call with the same draws when the first guess was short)."""
        states = np.ascontiguousarray(np.asarray(states, dtype=np.int32).reshape(-1, self.C))
        th, _ = theta_vector(self.model, theta)
        th = np.ascontiguousarray(th)
        n = states.shape[0]
        cap = 1024 if max_events is None else int(max_events)
        while True:
            t = np.empty((n, max(cap, 1)))
            x = np.empty((n, max(cap, 1), self.C), dtype=np.int32)
            nev = np.zeros(n, dtype=np.int32)
            fin = np.empty((n, self.C), dtype=np.int32)
            check(self._L.epipf_simulate_path(self._h, n, ptr(states), ptr(th), th.size, float(max_time),
                                              int(key) & (2**64 - 1), int(filter_index) & 0xFFFFFFFF, int(step), cap,
                                              ptr(t), ptr(x), ptr(nev), ptr(fin)), "epipf_simulate_path")
            longest = int(nev.max()) if n else 0
            if max_events is not None or longest <= cap:
                return t[:, :cap], x[:, :cap], nev, fin
            cap = longest

    def resample(self, w, u):
        w = np.ascontiguousarray(np.asarray(w, dtype=np.float64))
        u = np.ascontiguousarray(np.asarray(u, dtype=np.float64))
        out = np.empty(w.size, dtype=np.int32)
        fb = np.zeros(1, dtype=np.int64)
        rc = check(self._L.epipf_resample(self._h, w.size, ptr(w), ptr(u), ptr(out), ptr(fb)), "epipf_resample")
        return (None if rc == _lib.STATUS_DEGENERATE else out), int(fb[0])

    # ------------------------------------------------------------------ ABC rejection (abc_algo.py:17-109)
    @staticmethod
    def _abc_inputs(observed_data, priors):
        Y = np.ascontiguousarray(np.asarray(observed_data, dtype=np.float64))
        if Y.ndim != 2 or Y.shape[1] != 3:
            raise ValueError("observed_data must be [T, 3] (S, I, R), as abc_algo.py:38-45 unpacks it")
        pr = np.ascontiguousarray(np.array([priors["beta"][0], priors["beta"][1], priors["gamma"][0],
                                            priors["gamma"][1]], dtype=np.float64))
        return Y, pr

    def abc_trials(self, observed_data, priors, key=0, run_index=0, t0=0, n=1, rows=True):
        """Trials [t0, t0+n): theta [n,2], rows [n,T,3] int32 (S, I, R per day) or None, distance [n]."""
        Y, pr = self._abc_inputs(observed_data, priors)
        theta = np.empty((n, 2))
        rw = np.empty((n, Y.shape[0], 3), dtype=np.int32) if rows else None
        dist = np.empty(n)
        ev = np.zeros(1, dtype=np.int64)
        check(self._L.epipf_abc_trials(self._h, ptr(Y), Y.shape[0], ptr(pr), int(key) & (2**64 - 1),
                                       int(run_index) & 0xFFFFFFFF, int(t0), int(n), ptr(theta), ptr(rw), ptr(dist),
                                       ptr(ev)), "epipf_abc_trials")
        return theta, rw, dist

    def abc(self, observed_data, no_of_samples, threshold, priors, key=0, run_index=0, max_trials=2**32, batch=0):
        """(theta [n,2], trajectories [n,T,4], trials, accepted) of epipf_abc."""
        Y, pr = self._abc_inputs(observed_data, priors)
        n = int(no_of_samples)
        theta = np.empty((max(n, 1), 2))
        traj = np.empty((max(n, 1), Y.shape[0], 4))
        trials = np.zeros(1, dtype=np.int64)
        acc = np.zeros(1, dtype=np.int32)
        check(self._L.epipf_abc(self._h, ptr(Y), Y.shape[0], n, float(threshold), ptr(pr), int(key) & (2**64 - 1),
                                int(run_index) & 0xFFFFFFFF, int(max_trials), int(batch), ptr(theta), ptr(traj),
                                ptr(trials), ptr(acc)), "epipf_abc")
        a = int(acc[0])
        return theta[:a], traj[:a], int(trials[0]), a

    # ------------------------------------------------------------------ stats
    def set_profiling(self, level=_lib.PROFILE_COUNTERS):
        """level: PROFILE_OFF / PROFILE_TIMING (HIP events only, kernels unchanged) / PROFILE_COUNTERS
        (also device counters of SSA events and lane use).  True/False map to COUNTERS/OFF."""
        if level is True:
            level = _lib.PROFILE_COUNTERS
        elif level is False or level is None:
            level = _lib.PROFILE_OFF
        check(self._L.epipf_set_profiling(self._h, int(level)), "epipf_set_profiling")

    def set_streams(self, n):
        """Concurrent chain-group streams used by run() (1..8)."""
        check(self._L.epipf_set_streams(self._h, int(n)), "epipf_set_streams")

    def set_lanes(self, w, events_per_lane=0):
        """SSA lanes per particle used by run(): 0 = automatic, 1 (one-lane kernel), 2, 4, 8, 16 (lane groups), and
        the events each lane of a group draws per chunk (0 = automatic)."""
        check(self._L.epipf_set_lanes(self._h, int(w), int(events_per_lane)), "epipf_set_lanes")

    def stats(self):
        s = _lib.Stats()
        check(self._L.epipf_get_stats(self._h, ctypes.byref(s)), "epipf_get_stats")
        return s.as_dict()

    def reset_stats(self):
        check(self._L.epipf_reset_stats(self._h), "epipf_reset_stats")


_CACHE = {}


def release_engines():
    """Drop the cached engines: each context closes (its device buffers and HIP streams freed) with its last
    reference.  Idle contexts' streams still hold hardware queues (GPU_MAX_HW_QUEUES, 4 by default), on which the next
    concurrently running engines may otherwise be placed together."""
    _CACHE.clear()


def get_engine(type_model, groups, n_particles, T, chains=1, device=0):
    """Cached engine large enough for (T, chains).  When a bigger one is needed a new context replaces the cached
    one; the old context is not closed here -- a sampler may still hold it -- but released with its last reference
    (Engine.__del__).  Callers that share a cached engine re-bind their observations / population before each run
    (set_observations / set_population are no-ops when nothing changed)."""
    mid = model_id(type_model)
    key = (mid, groups if mid >= _lib.SIR_SUBGROUPS else 1, int(n_particles), int(device))
    eng = _CACHE.get(key)
    if eng is None or eng.t_max < T or eng.max_chains < chains:
        eng = Engine(type_model, groups, n_particles, max(T, eng.t_max if eng else 0),
                     max(chains, eng.max_chains if eng else 0), device)
        _CACHE[key] = eng
    return eng
