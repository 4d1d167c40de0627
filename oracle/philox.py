"""Keyed Philox4x32-10 stream used by every parity check (TEST INFRASTRUCTURE).

This module is part of the oracle: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it.  The product (HIP kernels in
``stochastic-epidemic-modelling_amd/csrc``) carries its own device implementation.

Why a keyed stream: the reference draws every random number from numpy's global
MT19937 ``RandomState`` in a data-dependent serial order (two uniforms per Gillespie
event, ``gillespie_algo.py:62-63``; N uniforms per resample, ``pmcmc.py:188-190``;
Poisson initial states, ``pmcmc.py:157-167``).  A one-lane-per-particle GPU design
cannot reproduce that serial stream, so parity is defined against the reference
*driven by this keyed stream* (SURVEY.md §8c).  The stream definition:

    block  = Philox4x32-10(counter=(c0, c1, c2, c3), key=(lo32(key), hi32(key)))
    U(a,b) = ((b << 32 | a) >> 11) * 2**-53                     (53-bit double in [0,1))

    SSA event k of particle j at filter step p : counter (k, j, p | 0<<24, f)
                                                  tau uniform = U(r0,r1), choice uniform = U(r2,r3)
    multinomial resample draw j at step p      : counter (0, j, p | 1<<24, f), U(r0,r1)
    systematic resample offset at step p       : counter (0, 0, p | 1<<24, f), U(r0,r1)
    initial Poisson draw, group g, particle j  : counter (g, j, 0 | 2<<24, f), U(r0,r1)
    ABC trial t (f = run index)                : prior (0, t, 3<<24, f); initial count c (c, t, 4<<24, f);
                                                  SSA event k (k, t, 5<<24, f)   (see the ABC section below)

``f`` is the filter index (one per particle-filter call), ``key`` a 64-bit seed.
Philox constants follow Salmon et al., "Parallel random numbers: as easy as 1, 2, 3"
(SC'11), and are pinned by the Random123 known-answer vectors in tests/test_oracle.py.
"""
import math
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)

DOMAIN_SSA = 0
DOMAIN_RESAMPLE = 1
DOMAIN_INIT = 2


def philox4x32_10(c0, c1, c2, c3, key):
    """Vectorised Philox4x32-10.  Counters are broadcastable integer arrays (32-bit values),
    ``key`` is ``(k0, k1)`` 32-bit ints.  Returns four uint64 arrays holding 32-bit words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & MASK for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def u01(lo, hi):
    """53-bit uniform double in [0, 1) from two 32-bit words (numpy's Philox convention)."""
    x = (np.asarray(hi, dtype=np.uint64) << np.uint64(32)) | np.asarray(lo, dtype=np.uint64)
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def split_key(key):
    key = int(key) & 0xFFFFFFFFFFFFFFFF
    return key & 0xFFFFFFFF, key >> 32


def ssa_uniforms(key, f, p, j, k):
    """(tau-uniform, choice-uniform) for SSA event ``k`` of particle ``j`` at step ``p``."""
    r = philox4x32_10(k, j, (p & 0xFFFFFF) | (DOMAIN_SSA << 24), f, split_key(key))
    return u01(r[0], r[1]), u01(r[2], r[3])


def resample_uniforms(key, f, p, n):
    r = philox4x32_10(0, np.arange(n), (p & 0xFFFFFF) | (DOMAIN_RESAMPLE << 24), f, split_key(key))
    return u01(r[0], r[1])


def init_uniforms(key, f, g, n):
    r = philox4x32_10(g, np.arange(n), DOMAIN_INIT << 24, f, split_key(key))
    return u01(r[0], r[1])


def poisson_kmax(mu):
    """Iteration cap of the inversion sampler (host-computed, shared with the device)."""
    return int(np.ceil(mu + 40.0 * np.sqrt(mu) + 60.0))


def poisson_inversion(u, mu):
    """Poisson(mu) by sequential CDF inversion, one uniform per draw.

    Shared definition (device, C oracle and golden shim compute it identically):
        pk = exp(-mu); F = pk; k = 0
        while U >= F and k < kmax: k += 1; pk = pk * mu / k; F = F + pk
    """
    import math
    emu = math.exp(-mu)
    kmax = poisson_kmax(mu)
    out = np.empty(len(u), dtype=np.int64)
    for i, ui in enumerate(np.asarray(u, dtype=float)):
        pk = emu
        F = pk
        k = 0
        while ui >= F and k < kmax:
            k += 1
            pk = pk * mu / k
            F = F + pk
        out[i] = k
    return out


# ----------------------------------------------------------------------------------- ABC rejection stream
# abc_algo.py:17-109 draws, per trial t of run f: two prior uniforms (np.random.uniform, :35-36), three Poisson
# initial counts (np.random.poisson(observed_data[0].astype(int)), :38-39), then a full-path SSA
# (sir_simulate(..., False), :40-45).  Keyed definition (trial index t < 2**32, run index f):
#     prior           : counter (0, t, 3<<24, f)   beta = lo + (hi-lo)*U(r0,r1), gamma from U(r2,r3)
#     initial count c : counter (c, t, 4<<24, f)   one uniform U(r0,r1), consumed by poisson_mode_inversion
#     SSA event k     : counter (k, t, 5<<24, f)   tau-uniform U(r0,r1), channel-uniform U(r2,r3)
# numpy's PTRS sampler decides acceptance by comparing sums of log/loggam values; a device cannot reproduce
# glibc's last bits there, so the stream's Poisson draw is exact inversion walking out from the mode with
# IEEE mul/div/add only -- bit-identical on CPU and GPU.  The mode probability is the one transcendental,
# computed once per lambda on the host from glibc's exp/log/lgamma (poisson_mode_pmf).
DOMAIN_ABC_PRIOR = 3
DOMAIN_ABC_INIT = 4
DOMAIN_ABC_SSA = 5


def abc_prior_uniforms(key, f, t):
    r = philox4x32_10(0, t, DOMAIN_ABC_PRIOR << 24, f, split_key(key))
    return float(u01(r[0], r[1])), float(u01(r[2], r[3]))


def abc_init_uniform(key, f, t, c):
    r = philox4x32_10(c, t, DOMAIN_ABC_INIT << 24, f, split_key(key))
    return float(u01(r[0], r[1]))


def abc_ssa_uniforms(key, f, t, k):
    r = philox4x32_10(k, t, DOMAIN_ABC_SSA << 24, f, split_key(key))
    return float(u01(r[0], r[1])), float(u01(r[2], r[3]))


def _libm():
    import ctypes
    import ctypes.util
    lib = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
    lib.lgamma.restype = ctypes.c_double
    lib.lgamma.argtypes = [ctypes.c_double]
    return lib


def poisson_mode_pmf(lam):
    """P(K = floor(lam)) as exp(-lam + m*log(lam) - lgamma(m+1)), glibc's exp/log/lgamma in this order (the
    C host library evaluates the same expression with the same libm)."""
    m = float(math.floor(lam))
    return math.exp(-lam + m * math.log(lam) - _libm().lgamma(m + 1.0))


def poisson_mode_inversion(lam, u, pm):
    """Poisson(lam) by inversion over the support ordered m, m+1, m-1, m+2, m-2, ... (m = floor(lam)):
    return the first k whose running probability sum exceeds u.  Neighbours come from the ratio recurrences
    p(k+1) = p(k)*lam/(k+1), p(k-1) = p(k)*k/lam.  If a full up/down round leaves the sum unchanged (u above
    the floating-point mass) the draw is m.  lam = 0 gives 0."""
    if lam == 0:
        return 0
    m = int(math.floor(lam))
    acc = pm
    if u < acc:
        return m
    khi = klo = m
    phi = plo = pm
    while True:
        prev = acc
        phi = phi * lam / (khi + 1)
        khi += 1
        acc = acc + phi
        if u < acc:
            return khi
        if klo > 0:
            plo = plo * klo / lam
            klo -= 1
            acc = acc + plo
            if u < acc:
                return klo
        if acc == prev:
            return m


def abc_initial_counts(key, f, t, lams, pms):
    return [poisson_mode_inversion(lam, abc_init_uniform(key, f, t, c), pm) for c, (lam, pm) in
            enumerate(zip(lams, pms))]
