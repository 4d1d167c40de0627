"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE -- see epipf_oracle.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
The functions mirror the reference's call surface (pmcmc.py:123-233, gillespie_algo.py)
but take the keyed-stream arguments (key, filter_index) explicitly.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

MODEL_IDS = {"sir": 0, "seir": 1, "sir_subgroups": 2, "sir_subgroups2": 3}


def build(force=False):
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(os.path.join(_HERE, f))
                                          for f in ("epipf_oracle.c", "abc_oracle.c", "Makefile"))
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        i32, u32, u64, f64 = ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double
        L.oracle_particle_filter.argtypes = [i32, i32, i32, i32, i32, P, P, i32, i32, f64, P, P, u64, u32,
                                             i32, P, P, P, P, P]
        L.oracle_particle_filter.restype = i32
        L.oracle_simulate.argtypes = [i32, i32, i32, P, P, i32, f64, u64, u32, u32, P, P]
        L.oracle_simulate.restype = i32
        L.oracle_simulate_path.argtypes = [i32, i32, i32, P, P, i32, f64, u64, u32, u32, ctypes.c_long, P, P, P, P]
        L.oracle_simulate_path.restype = i32
        L.oracle_resample.argtypes = [i32, P, P, P]
        L.oracle_resample.restype = i32
        L.oracle_philox.argtypes = [u32, u32, u32, u32, u64, P]
        L.oracle_num_threads.restype = i32
        L.oracle_set_num_threads.argtypes = [i32]
        L.oracle_log_batch.argtypes = [ctypes.c_long, P, P]
        L.oracle_binom_pmf.argtypes = [f64, f64, f64]
        L.oracle_binom_pmf.restype = f64
        L.oracle_norm_pdf.argtypes = [f64, f64, f64]
        L.oracle_norm_pdf.restype = f64
        L.oracle_abc_trials.argtypes = [P, i32, P, P, P, u64, u32, u32, i32, P, P, P, P]
        L.oracle_abc_trials.restype = i32
        L.oracle_pairwise_sum.argtypes = [P, ctypes.c_long]
        L.oracle_pairwise_sum.restype = f64
        L.oracle_poisson_mode_pmf.argtypes = [f64]
        L.oracle_poisson_mode_pmf.restype = f64
        L.oracle_poisson_mode_inversion.argtypes = [f64, f64, f64]
        L.oracle_poisson_mode_inversion.restype = ctypes.c_long
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def model_id(type_model):
    name = getattr(type_model, "value", type_model)
    return MODEL_IDS[name]


def _theta_vector(mid, theta):
    if mid >= 2:
        beta, gamma = theta
        beta = np.asarray(beta, dtype=np.float64)
        return np.ascontiguousarray(np.append(beta.reshape(-1), float(gamma)), dtype=np.float64), beta.shape[0]
    return np.ascontiguousarray(np.asarray(theta, dtype=np.float64).reshape(-1)), 1


def particle_filter(Y, type_model, theta, observations=False, probs=0.1, n_particles=1000, n_population=4820,
                    mu=20, key=0, filter_index=0, resample="multinomial"):
    """Oracle particle filter.  Returns dict(status, log_zetas, zetas, hidden[T,N,C] int32, ancestry[T,N] int32, events)."""
    mid = model_id(type_model)
    Y = np.ascontiguousarray(np.asarray(Y, dtype=np.float64))
    T, K = Y.shape
    th, G = _theta_vector(mid, theta)
    npop = np.ascontiguousarray(np.atleast_1d(np.asarray(n_population, dtype=np.float64)))
    mus = np.ascontiguousarray(np.atleast_1d(np.asarray(mu, dtype=np.float64)))
    C = 3 if mid == 0 else 4 if mid == 1 else 3 * G
    N = int(n_particles)
    lz = np.zeros(T)
    z = np.zeros(T)
    hidden = np.zeros((T, N, C), dtype=np.int32)
    anc = np.zeros((T, N), dtype=np.int32)
    ev = np.zeros(1, dtype=np.int64)
    st = lib().oracle_particle_filter(mid, G, N, T, K, _p(Y), _p(th), len(th), int(bool(observations)),
                                      float(probs), _p(npop), _p(mus), int(key) & (2**64 - 1),
                                      int(filter_index) & 0xFFFFFFFF,
                                      0 if resample == "multinomial" else 1, _p(lz), _p(z), _p(hidden),
                                      _p(anc), _p(ev))
    if st < 0:
        raise ValueError("oracle_particle_filter: bad arguments")
    return dict(status=st, log_zetas=lz, zetas=z, hidden=hidden, ancestry=anc, events=int(ev[0]))


def simulate(type_model, states, theta, max_time=1.0, key=0, filter_index=0, step=0):
    """Batched last-value SSA (gillespie_algo.*_simulate(..., last_values_only=True)) from int states [n, C]."""
    mid = model_id(type_model)
    th, G = _theta_vector(mid, theta)
    states = np.ascontiguousarray(np.asarray(states, dtype=np.int32))
    out = np.zeros_like(states)
    ev = np.zeros(1, dtype=np.int64)
    st = lib().oracle_simulate(mid, G, states.shape[0], _p(states), _p(th), len(th), float(max_time),
                               int(key) & (2**64 - 1), int(filter_index) & 0xFFFFFFFF, int(step), _p(out), _p(ev))
    if st < 0:
        raise ValueError("oracle_simulate: bad arguments")
    return out, int(ev[0])


def simulate_path(type_model, states, theta, max_time=1.0, key=0, filter_index=0, step=0, cap=None):
    """Batched full-path SSA (gillespie_algo.*_simulate(..., last_values_only=False)) from int states [n, C].
    Returns (times [n, cap], states [n, cap, C], n_events [n], final [n, C]); cap defaults to the longest path."""
    mid = model_id(type_model)
    th, G = _theta_vector(mid, theta)
    states = np.ascontiguousarray(np.asarray(states, dtype=np.int32))
    n, C = states.shape
    if cap is None:
        _, nev, _ = _path_once(mid, G, states, th, max_time, key, filter_index, step, 0)
        cap = int(nev.max()) if n else 0
    return _path_once(mid, G, states, th, max_time, key, filter_index, step, cap, full=True)


def _path_once(mid, G, states, th, max_time, key, f, step, cap, full=False):
    n, C = states.shape
    t = np.zeros((n, max(cap, 1)))
    x = np.zeros((n, max(cap, 1), C), dtype=np.int32)
    nev = np.zeros(n, dtype=np.int32)
    fin = np.zeros((n, C), dtype=np.int32)
    st = lib().oracle_simulate_path(mid, G, n, _p(states), _p(th), len(th), float(max_time), int(key) & (2**64 - 1),
                                    int(f) & 0xFFFFFFFF, int(step), int(cap), _p(t), _p(x), _p(nev), _p(fin))
    if st < 0:
        raise ValueError("oracle_simulate_path: bad arguments")
    if full:
        return t[:, :cap], x[:, :cap], nev, fin
    return t, nev, fin


def resample(w, u):
    """numpy legacy choice(range(N), N, p=w/sum(w)) with the given uniforms; None where numpy raises."""
    w = np.ascontiguousarray(np.asarray(w, dtype=np.float64))
    u = np.ascontiguousarray(np.asarray(u, dtype=np.float64))
    out = np.zeros(len(w), dtype=np.int32)
    if lib().oracle_resample(len(w), _p(w), _p(u), _p(out)):
        return None
    return out


def philox(c0, c1, c2, c3, key):
    out = np.zeros(4, dtype=np.uint32)
    lib().oracle_philox(c0, c1, c2, c3, key, _p(out))
    return out


def binom_pmf(k, n, p):
    L = lib()
    return np.array([L.oracle_binom_pmf(float(a), float(b), float(c)) for a, b, c in zip(k, n, p)])


def norm_pdf(y, x, probs):
    L = lib()
    return np.array([L.oracle_norm_pdf(float(a), float(b), float(c)) for a, b, c in zip(y, x, probs)])


def num_threads():
    return lib().oracle_num_threads()


def log_batch(x):
    """glibc log (libm, the reference's math.log) of every element."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    lib().oracle_log_batch(x.size, _p(x), _p(out))
    return out


def set_num_threads(n):
    """OpenMP threads of the filter / SSA loops for the rest of the process."""
    lib().oracle_set_num_threads(int(n))


# ----------------------------------------------------------------------------------- ABC (abc_algo.py:17-109)
def abc_start(observed_data):
    """Initial-count means (abc_algo.py:38 Y[0].astype(int)) and their mode probabilities."""
    Y = np.asarray(observed_data, dtype=np.float64)
    lams = Y[0, :3].astype(int).astype(np.float64)
    if (lams < 0).any():
        raise ValueError("lam < 0")
    pms = np.array([lib().oracle_poisson_mode_pmf(v) if v > 0 else 0.0 for v in lams])
    return lams, pms


def abc_trials(observed_data, priors, key=0, run_index=0, t0=0, n=1, rows=True):
    """Trials [t0, t0+n): theta [n,2], rows [n,T,3] int32 (S, I, R per day) or None, distance [n], events."""
    Y = np.ascontiguousarray(np.asarray(observed_data, dtype=np.float64)[:, :3])
    T = Y.shape[0]
    pr = np.ascontiguousarray(np.array(list(priors["beta"]) + list(priors["gamma"]), dtype=np.float64))
    lams, pms = abc_start(Y)
    theta = np.zeros((n, 2))
    rw = np.zeros((n, T, 3), dtype=np.int32) if rows else None
    dist = np.zeros(n)
    ev = np.zeros(1, dtype=np.int64)
    st = lib().oracle_abc_trials(_p(Y), T, _p(pr), _p(lams), _p(pms), int(key) & (2**64 - 1),
                                 int(run_index) & 0xFFFFFFFF, int(t0), int(n), _p(theta),
                                 _p(rw) if rows else None, _p(dist), _p(ev))
    if st < 0:
        raise ValueError("oracle_abc_trials: bad arguments")
    return theta, rw, dist, int(ev[0])


def abc_algo(observed_data, no_of_samples, threshold, priors, key=0, run_index=0, batch=4096, max_trials=10**9):
    """abc_algo.abc_algo on the keyed stream: (posterior dict, trajectories [n,T,4] float64, trials)."""
    T = np.asarray(observed_data).shape[0]
    betas, gammas, trajs = [], [], []
    t = 0
    while len(betas) < no_of_samples and t < max_trials:
        n = min(batch, max_trials - t)
        theta, rw, dist, _ = abc_trials(observed_data, priors, key, run_index, t, n)
        for i in np.nonzero(~(dist > threshold))[0]:
            if len(betas) == no_of_samples:
                break
            betas.append(float(theta[i, 0]))
            gammas.append(float(theta[i, 1]))
            trajs.append(np.concatenate([np.arange(T, dtype=np.float64)[:, None], rw[i].astype(np.float64)], 1))
            last = t + int(i)
        t += n
    trials = last + 1 if betas else t
    return {"beta": betas, "gamma": gammas}, np.array(trajs).reshape(-1, T, 4), trials
