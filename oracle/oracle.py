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
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "epipf_oracle.c"))
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
        L.oracle_resample.argtypes = [i32, P, P, P]
        L.oracle_resample.restype = i32
        L.oracle_philox.argtypes = [u32, u32, u32, u32, u64, P]
        L.oracle_num_threads.restype = i32
        L.oracle_binom_pmf.argtypes = [f64, f64, f64]
        L.oracle_binom_pmf.restype = f64
        L.oracle_norm_pdf.argtypes = [f64, f64, f64]
        L.oracle_norm_pdf.restype = f64
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
