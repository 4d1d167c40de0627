// epipf_device.hpp -- device building blocks of the particle filter (gfx950 / CDNA4, wave64).
//
// Everything here is compiled with -ffp-contract=off: each IEEE multiply, add and divide must
// round exactly as CPython/numpy round the reference's expressions, so that Gillespie channel
// choices, state trajectories and resampled ancestors are bit-identical to the reference driven
// by the same keyed Philox stream.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace epipf {

constexpr int kMaxG = 4;                    // largest subgroup count instantiated
constexpr int kMaxC = 3 * kMaxG;            // compartments per particle
constexpr int kMaxTheta = kMaxG * kMaxG + 1;
constexpr uint32_t kDomainSSA = 0u << 24;
constexpr uint32_t kDomainResample = 1u << 24;
constexpr uint32_t kDomainInit = 2u << 24;

enum Model : int { kSIR = 0, kSEIR = 1, kSubgroups = 2, kSubgroups2 = 3 };
enum Obs : int { kBinomial = 0, kNormal = 1 };

// ------------------------------------------------------------------------------- Philox4x32-10
// Salmon et al. SC'11; constants and key schedule of Random123.  Counter words: (c0, c1, c2, c3).
struct Block { uint32_t x, y, z, w; };

// INVX: return ~x (the last round's three-way XOR with truth table 0x69 instead of 0x96, no extra instruction);
// the f32 event loop needs 1 - U, whose low word is ~x.
template <bool INVX = false>
__device__ __forceinline__ Block philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                        uint32_t k1) {
    // Rounds 0-2 keep plain XORs: with a wave-uniform counter word and key, the compiler runs most of them on
    // the scalar unit.  From round 3 on every word is lane-varying and each three-way XOR is one gfx950
    // v_bitop3_b32 (truth table 0x96) instead of two v_xor_b32: 14 fewer VALU instructions per block.
#pragma unroll
    for (int r = 0; r < 9; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;   // one 32x32->64 multiply each
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        uint32_t n0, n2;
        if (r < 3) {
            n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
            n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        } else {
            n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);
            n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        }
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    constexpr unsigned kLastX = INVX ? 0x69u : 0x96u;               // round 9
    const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    return Block{(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, kLastX), (uint32_t)p1,
                 (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96), (uint32_t)p0};
}

// 53-bit uniform in [0, 1): ((hi << 32 | lo) >> 11) * 2^-53  (numpy's Philox double convention).
// With m = (hi:lo) >> 11 split as mh = hi >> 11 (21 bits) and ml = low 32 bits of m, U = mh 2^-21 + ml 2^-53:
// both conversions and the scaling are exact and the fused add of two exact terms whose sum is representable
// is exact, so this equals the 64-bit shift + convert form bit for bit (two 32-bit converts, no 64-bit ops).
__device__ __forceinline__ double u01(uint32_t lo, uint32_t hi) {
    const uint32_t mh = hi >> 11, ml = __builtin_amdgcn_alignbit(hi, lo, 11);
    return fma((double)mh, 0x1.0p-21, (double)ml * 0x1.0p-53);
}

// 1 - U for the same U, exactly: 1 - mh 2^-21 is a multiple of 2^-21 in (0, 1] and the final fused add
// subtracts an exact term from it with a representable result (1 - U = (2^53 - m) 2^-53).
__device__ __forceinline__ double one_minus_u01(uint32_t lo, uint32_t hi) {
    const uint32_t mh = hi >> 11, ml = __builtin_amdgcn_alignbit(hi, lo, 11);
    return fma((double)ml, -0x1.0p-53, fma((double)mh, -0x1.0p-21, 1.0));
}

// ------------------------------------------------------------------------------- index checks
// An ancestor / path index outside [0, n) would mean a search or indexing bug.  The release build clamps it (a
// wrong answer the parity tests catch, never an out-of-bounds access); the debug build (make debug,
// libepipf_debug.so) traps on it instead, so the fault is reported at the kernel that produced it.
__device__ __forceinline__ int checked_index(int i, int n) {
#ifdef EPIPF_DEBUG
    if ((unsigned)i >= (unsigned)n) __builtin_trap();
    return i;
#else
    return min(max(i, 0), n - 1);
#endif
}

// ------------------------------------------------------------------------------- per-chain parameters
struct ChainParam {
    double theta[kMaxTheta];   // SIR: beta,gamma  SEIR: beta,alpha,gamma  groups: beta[G][G], gamma
    double probs;              // binomial p, or normal noise ratio
    double logp, log1mp;       // log(p), log1p(-p): hi parts of their binary128 values (logfact.cpp)
    double logp_lo, log1mp_lo; //   and the lo parts (binom_logpmf)
    double tie_tol;            // particle_weight: bound on the plain column logs' error (host, epipf_run)
    uint32_t k0, k1;           // Philox key
    uint32_t f;                // filter index
    uint32_t flags;            // kChainFastSsa: the certified f32 event loop may run (EPIPF_SSA_FAST=0 clears it)
    int32_t skip;              // 1: this chain runs no filter in this batch (epipf_run's active[] = 0)
    int32_t chosen;            // epipf_run_sampled: the path sampler's final particle (pmcmc.py:241), -1: none
    float thetaf[kMaxTheta];   // theta rounded to f32 on the host (scalar loads: the fast path's rates stay in SGPRs)
    float clock_slack;         // >= 1: widens the f32 loop's clock band (more replays, same results); tests only
    float band_slack;          // >= 1: widens the channel decision's band (more exact decisions and redone chunks,
                               // same results); tests only
};
// chain status codes (include/epipf.h's EPIPF_STATUS_*; epipf_api.cpp checks they agree)
constexpr int32_t kStatusOk = 0, kStatusDegenerate = 1, kStatusSkipped = 2;
constexpr uint32_t kChainFastSsa = 1u;   // (all models)
constexpr uint32_t kChainSeqDecide = 2u; // lane groups: sequential decision pass (EPIPF_GROUP_DECIDE=seq; A/B, tests)

// ------------------------------------------------------------------------------- reference-exact log
// glibc 2.35 log(x), the function behind the reference's draws (numpy legacy exponential = scale * -log(1 - U),
// gillespie_algo.py:62; the keyed-stream shim's math.log): sysdeps/ieee754/dbl-64/e_log.c as the x86_64 libm
// runs it on an FMA CPU (__log_fma, e_log.c compiled with -mfma -mavx2).  Same table (__log_data, copied from
// this machine's libm at build time by gen_glibc_log.py), same operations, same fused multiply-adds -- read off
// that function's machine code -- so every result is the library's bit for bit (tests/test_glibc_log.py compares
// >= 10^8 inputs with math.log).  Defined for normal x > 0 (the SSA calls it on 1 - U >= 2^-53).
// Host-callable too: epipf_glibc_log (epipf_api.cpp) runs this code on the CPU for that test.
#include "glibc_log_data.inc"

struct LogTab { double invc, logc; };
constexpr int kLogTabEntries = 128;

__host__ __device__ inline double glibc_log_impl(double x, const LogTab* __restrict__ tab) {
    const uint64_t ix = __builtin_bit_cast(uint64_t, x);
    constexpr uint64_t LO = 0x3FEE000000000000ull;                    // asuint64(1 - 0x1p-4)
    constexpr uint64_t HI = 0x3FF1090000000000ull;                    // asuint64(1 + 0x1.09p-4)
    if (ix - LO < HI - LO) {                                          // inputs close to 1: poly1 (B), no table
        if (ix == 0x3FF0000000000000ull) return 0.0;
        const double r = x - 1.0;
        const double r2 = r * r, r3 = r * r2;
        double q1 = fma(r, kGlibcLogB[2], kGlibcLogB[1]);
        double q4 = fma(r, kGlibcLogB[5], kGlibcLogB[4]);
        double q7 = fma(r, kGlibcLogB[8], kGlibcLogB[7]);
        q1 = fma(r2, kGlibcLogB[3], q1);
        q4 = fma(r2, kGlibcLogB[6], q4);
        q7 = fma(r2, kGlibcLogB[9], q7);
        q7 = fma(r3, kGlibcLogB[10], q7);
        q4 = fma(q7, r3, q4);
        const double poly = fma(q4, r3, q1);                          // y = r3 (B1 + r B2 + r2 B3 + r3 (...))
        const double rhi = fma(-0x1.0p27, r, fma(r, 0x1.0p27, r));    // w = r 2^27; rhi = r + w - w
        const double rlo = r - rhi;
        const double rr = rhi * rhi;
        const double hi = fma(rr, kGlibcLogB[0], r);                  // w = rhi rhi B0; hi = r + w
        double lo = fma(rr, kGlibcLogB[0], r - hi);                   // lo = r - hi + w
        lo = fma(kGlibcLogB[0] * rlo, r + rhi, lo);                   // lo += B0 rlo (rhi + r)
        return hi + fma(poly, r3, lo);                                // y += lo; y += hi
    }
    const uint64_t tmp = ix - 0x3FE6000000000000ull;                  // OFF
    const int i = (int)((tmp >> 45) & 127);
    const int k = (int)((int64_t)tmp >> 52);
    const double z = __builtin_bit_cast(double, ix - (tmp & 0xFFF0000000000000ull));
    const LogTab e = tab[i];
    const double kd = (double)k;
    const double r = fma(z, e.invc, -1.0);                            // r ~= z/c - 1
    const double w = fma(kd, kGlibcLn2Hi, e.logc);
    const double hi = r + w;
    const double lo = fma(kd, kGlibcLn2Lo, (w - hi) + r);
    const double r2 = r * r;
    const double P = fma(fma(r, kGlibcLogA[4], kGlibcLogA[3]), r2, fma(r, kGlibcLogA[2], kGlibcLogA[1]));
    return fma(r * r2, P, fma(r2, kGlibcLogA[0], lo)) + hi;           // lo + r2 A0 + r r2 (A1 + ...) + hi
}

// The step kernels call it out of line: it runs only on their exact path (replays, ~1% of waves), and inlined, its
// constants and branches raised the whole kernel's SGPR spills from 15 to 44 (reloads every step: -2% at config 2).
// The ABC trial loop, where every event takes it, inlines it (glibc_log_inl).
__device__ __noinline__ double glibc_log(double x, const LogTab* __restrict__ tab) { return glibc_log_impl(x, tab); }
__device__ __forceinline__ double glibc_log_inl(double x, const LogTab* __restrict__ tab) { return glibc_log_impl(x, tab); }

// -log(x) for the lane-group filter's certified clock (epipf_group.hpp, group_propagate<FASTCLK>), where the time only
// has to lie within a certified bound of the reference's, not equal it: glibc's table path for every x (no branch
// for x near 1, no compensated hi/lo sums), ~12 f64 operations instead of both of glibc's paths (a wave's 64 lanes
// almost always hold an x on each side of its branch).  Error against the 64-bit-mantissa log over 1.2e8 inputs
// x = 1 - U (U uniform, U small: x near 1, U near 1: x tiny; tests/test_glibc_log.py::test_clock_log_error_bound):
//   |L' - L| <= kClockLogRel |L'|  where L' >= 2^-10  (largest seen 2.9 ulps: 8 allowed), and
//   |L' - L| <= kClockLogAbs       where L' <  2^-10  (largest seen 2^-60.3: 2^-58 allowed; near x = 1 the table
//                                                      entries' log c cancel against log1p(r))
// The clock bound takes the relative part into kClockEps and the absolute part, times each such event's 1/sum(a), into
// its own term (group_propagate).
constexpr double kClockLogRel = 0x1.0p-50, kClockLogAbs = 0x1.0p-58;
__host__ __device__ inline double clock_log_impl(double x, const LogTab* __restrict__ tab) {
    const uint64_t ix = __builtin_bit_cast(uint64_t, x);
    const uint64_t tmp = ix - 0x3FE6000000000000ull;                  // OFF
    const int i = (int)((tmp >> 45) & 127);
    const int k = (int)((int64_t)tmp >> 52);
    const double z = __builtin_bit_cast(double, ix - (tmp & 0xFFF0000000000000ull));
    const LogTab e = tab[i];
    const double r = fma(z, e.invc, -1.0);                            // z/c - 1, |r| < 2^-8
    const double w = fma((double)k, 0x1.62e42fefa39efp-1, e.logc);    // k ln2 + log c
    const double r2 = r * r;
    const double P = fma(fma(r, kGlibcLogA[4], kGlibcLogA[3]), r2, fma(r, kGlibcLogA[2], kGlibcLogA[1]));
    return w + fma(r * r2, P, fma(r2, kGlibcLogA[0], r));            // log c + k ln2 + log1p(r)
}

// -log(1 - U) for the certified clock (clock_log_impl), 1 - U exact
__device__ __forceinline__ double clock_neg_log_one_minus_u01(uint32_t lo, uint32_t hi, const LogTab* __restrict__ tab) {
    return -clock_log_impl(one_minus_u01(lo, hi), tab);
}

// glibc's {invc, logc} table as the device keeps it (copied into each context, then into LDS by the waves that
// run the exact loop)
inline void glibc_log_table(LogTab* out) {
    for (int i = 0; i < kLogTabEntries; ++i) out[i] = LogTab{kGlibcLogTab[2 * i], kGlibcLogTab[2 * i + 1]};
}

// -log(1 - U), U = u01(lo, hi): the reference's np.random.exponential(1) (gillespie_algo.py:62), 1 - U exact.
// INL: inline the log (the ABC trial loop) instead of calling it.
template <bool INL = false>
__device__ __forceinline__ double neg_log_one_minus_u01(uint32_t lo, uint32_t hi, const LogTab* __restrict__ tab) {
    const double x = one_minus_u01(lo, hi);
    return -(INL ? glibc_log_inl(x, tab) : glibc_log(x, tab));
}

// ------------------------------------------------------------------------------- Gillespie SSA
// Direct method over [0, tmax] from state x (integers held in doubles, as the reference holds them),
// gillespie_algo.py.  Event k of this lane draws Philox block (k, j, ptag, f): tau from (x,y), the
// channel from (z,w).  Both uniforms are consumed before the overshoot test, as in the reference.
// Every lane still in the loop is at the same event index k (all start at 0 and step together), so k is
// read wave-uniform: Philox's first round (and half of its second) then runs on the scalar unit.
//
// The clock is the reference's bit for bit: propensities in its expression order (((beta*S)*I)/N, IEEE
// division), their builtin-sum order, scale = 1/sum (IEEE), tau = scale * -log(1 - U) with glibc's log
// (gillespie_algo.py:37-40, :62), t + tau accumulated as :68.  So every step-boundary decision t + tau > tmax
// (:65) is the reference's -- no tolerance.  The channel decision of the reference is
//   count_i [ fl(c_i / c_last) <= u ],  c = cumsum(fl(a_l / sum(a)))            (numpy choice, :63)
// whose ratios agree with q_i = (a_0 + ... + a_i) * scale to a few ulps.  When every q_i is farther than
// kBand from u the decision is the reference's; otherwise the reference expression is evaluated exactly
// (IEEE divisions in the reference's order).
constexpr double kBand = 0x1.0p-44;

__device__ __noinline__ bool sir_channel_exact(double beta, double gamma, double S, double I, double N, double u) {
    const double a0 = ((beta * S) * I) / N, a1 = gamma * I;         // gillespie_algo.py:38-39
    const double as = a0 + a1;
    const double p0 = a0 / as, p1 = a1 / as;                       // :63
    return (p0 / (p0 + p1)) <= u;
}

__device__ __noinline__ int seir_channel_exact(double beta, double alpha, double gamma, double S, double E, double I,
                                               double N, double u) {
    const double a0 = ((beta * S) * I) / N, a1 = alpha * E, a2 = gamma * I;   // :107-109
    const double as = (a0 + a1) + a2;
    const double p0 = a0 / as, p1 = a1 / as, p2 = a2 / as;
    const double c1 = p0 + p1, c2 = c1 + p2;
    return ((p0 / c2) <= u ? 1 : 0) + ((c1 / c2) <= u ? 1 : 0);       // :134
}

template <int G>
__device__ __forceinline__ int subgroups_channel_exact(const double* th, const double* S, const double* I, double sumN,
                                                       double u) {
    constexpr int NCH = G * G + G;
    const double gamma = th[G * G];
    double a[NCH];
    for (int g = 0; g < G; ++g) {                                      // :180-185
        for (int g2 = 0; g2 < G; ++g2) a[g * (G + 1) + g2] = ((th[g * G + g2] * S[g2]) * I[g]) / sumN;
        a[g * (G + 1) + G] = gamma * I[g];
    }
    double as = 0.0;
    for (int i = 0; i < NCH; ++i) as = as + a[i];                      // :208
    double cdf[NCH];
    double run = 0.0;
    for (int i = 0; i < NCH; ++i) { run = run + a[i] / as; cdf[i] = run; }
    int ch = 0;
    for (int i = 0; i < NCH - 1; ++i) ch += ((cdf[i] / cdf[NCH - 1]) <= u) ? 1 : 0;   // :209-212
    return ch;
}

// Per-model event state: load() from the compartment counts, active() = the reference's loop condition,
// event(r) = one pass of the reference's loop body with Philox block r (returns false, state untouched, when
// the event overshoots tmax: the reference's break), save() back to counts.
//
// Propensities, their sums and tau follow the reference's expressions exactly (see above); rates() is shared by
// event() and tau_of() (the wave-cooperative replay evaluates events' times in parallel with it).
template <int MODEL, int G>
struct SsaState;

template <>
struct SsaState<kSIR, 1> {                                             // gillespie_algo.py:10-75
    double S, I, R, N;
    int nrec;
    __device__ __forceinline__ void load(const double* x, const ChainParam&) {
        S = x[0]; I = x[1]; R = x[2];
        N = (S + I) + R;                                               // :35
        nrec = 0;
    }
    __device__ __forceinline__ bool active() const { return I > 0.0; }   // :48
    // a0 and scale = 1/sum(a) in the reference's order (:38-39, :62)
    __device__ __forceinline__ double rates(const ChainParam& cp, double& a0) const {
        a0 = ((cp.theta[0] * S) * I) / N;                              // beta * s * i / N
        const double a1 = cp.theta[1] * I;                             // gamma * i
        return 1.0 / (a0 + a1);                                        // 1/sum(evaluated_reactions)
    }
    template <bool INL = false>
    __device__ __forceinline__ bool event(const Block& r, double& t, double tmax, const ChainParam& cp,
                                          const LogTab* __restrict__ tab) {
        double a0;
        const double scale = rates(cp, a0);
        const double tau = scale * neg_log_one_minus_u01<INL>(r.x, r.y, tab);   // np.random.exponential(scale), :62
        const double u = u01(r.z, r.w);
        const double q = a0 * scale;
        bool second = q <= u;                                          // choice(2, p=a/sum(a)), :63
        if (fabs(q - u) <= kBand) second = sir_channel_exact(cp.theta[0], cp.theta[1], S, I, N, u);
        const double tn = t + tau;
        if (tn > tmax) return false;                                   // :65-66
        t = tn;                                                        // :68-70; R is not needed in the loop
        S = S + (second ? 0.0 : -1.0);
        I = I + (second ? -1.0 : 1.0);
        nrec += second ? 1 : 0;
        return true;
    }
    __device__ __forceinline__ void save(double* x) const { x[0] = S; x[1] = I; x[2] = R + (double)nrec; }
    // event()'s tau, same expressions
    __device__ __forceinline__ double tau_of(const Block& r, const ChainParam& cp, const LogTab* __restrict__ tab) const {
        double a0;
        return rates(cp, a0) * neg_log_one_minus_u01(r.x, r.y, tab);
    }
};

template <>
struct SsaState<kSEIR, 1> {                                            // gillespie_algo.py:78-146
    double S, E, I, R, N;
    __device__ __forceinline__ void load(const double* x, const ChainParam&) {
        S = x[0]; E = x[1]; I = x[2]; R = x[3];
        N = ((S + E) + I) + R;                                         // :104
    }
    __device__ __forceinline__ bool active() const { return E > 0.0 || I > 0.0; }   // :119
    // cumulative a0, a0 + a1 and scale = 1/sum(a), theta = (beta, alpha, gamma) (:92, :107-109, :133)
    __device__ __forceinline__ double rates(const ChainParam& cp, double& a0, double& a01) const {
        a0 = ((cp.theta[0] * S) * I) / N;
        a01 = a0 + cp.theta[1] * E;
        return 1.0 / (a01 + cp.theta[2] * I);
    }
    __device__ __forceinline__ bool event(const Block& r, double& t, double tmax, const ChainParam& cp,
                                          const LogTab* __restrict__ tab) {
        double a0, a01;
        const double scale = rates(cp, a0, a01);
        const double tau = scale * neg_log_one_minus_u01(r.x, r.y, tab);  // :133
        const double u = u01(r.z, r.w);
        const double q0 = a0 * scale, q1 = a01 * scale;
        int ch = (q0 <= u ? 1 : 0) + (q1 <= u ? 1 : 0);                // :134
        if (fabs(q0 - u) <= kBand || fabs(q1 - u) <= kBand)
            ch = seir_channel_exact(cp.theta[0], cp.theta[1], cp.theta[2], S, E, I, N, u);
        const double tn = t + tau;
        if (tn > tmax) return false;                                   // :136-137
        t = tn;
        S = (ch == 0) ? S - 1.0 : S;
        E = (ch == 0) ? E + 1.0 : (ch == 1) ? E - 1.0 : E;
        I = (ch == 1) ? I + 1.0 : (ch == 2) ? I - 1.0 : I;
        R = (ch == 2) ? R + 1.0 : R;
        return true;
    }
    __device__ __forceinline__ void save(double* x) const { x[0] = S; x[1] = E; x[2] = I; x[3] = R; }
    __device__ __forceinline__ double tau_of(const Block& r, const ChainParam& cp, const LogTab* __restrict__ tab) const {
        double a0, a01;
        return rates(cp, a0, a01) * neg_log_one_minus_u01(r.x, r.y, tab);
    }
};

template <int G>
struct SubgroupsState {                                                // gillespie_algo.py:148-233
    static constexpr int NCH = G * G + G;
    double S[G], I[G], R[G], sumN;
    __device__ __forceinline__ void load(const double* x, const ChainParam&) {
        sumN = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            S[g] = x[3 * g]; I[g] = x[3 * g + 1]; R[g] = x[3 * g + 2];
            sumN = sumN + ((S[g] + I[g]) + R[g]);                      // sum(N), :176,:182
        }
    }
    // cumulative propensities in dict insertion order (s_{g}_{g2} then i_{g}, :180-185) summed as
    // sum(list(evaluated_reactions.values())) (:208); returns 1/sum
    __device__ __forceinline__ double rates(const ChainParam& cp, double* cum) const {
        const double gamma = cp.theta[G * G];
        double run = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int g2 = 0; g2 < G; ++g2) {
                run = run + ((cp.theta[g * G + g2] * S[g2]) * I[g]) / sumN;   // beta[g,g2] s_g2 i_g / sum(N)
                cum[g * (G + 1) + g2] = run;
            }
            run = run + gamma * I[g];                                  // gamma i_g
            cum[g * (G + 1) + G] = run;
        }
        return 1.0 / run;
    }
    __device__ __forceinline__ bool active() const {                   // :192-193, :222
        double infected = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) infected = infected + I[g];
        return infected > 0.0;
    }
    __device__ __forceinline__ bool event(const Block& r, double& t, double tmax, const ChainParam& cp,
                                          const LogTab* __restrict__ tab) {
        double cum[NCH];
        const double ri = rates(cp, cum);
        const double tau = ri * neg_log_one_minus_u01(r.x, r.y, tab);  // :207
        const double u = u01(r.z, r.w);
        int ch = 0;
        bool close = false;
#pragma unroll
        for (int i = 0; i < NCH - 1; ++i) {
            const double q = cum[i] * ri;
            ch += (q <= u) ? 1 : 0;
            close |= fabs(q - u) <= kBand;
        }
        if (close) ch = subgroups_channel_exact<G>(cp.theta, S, I, sumN, u);
        const double tn = t + tau;
        if (tn > tmax) return false;                                   // :215-216
        t = tn;
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int g2 = 0; g2 < G; ++g2)
                if (ch == g * (G + 1) + g2) { S[g2] -= 1.0; I[g2] += 1.0; }   // s_{g}_{g2}: :183
            if (ch == g * (G + 1) + G) { I[g] -= 1.0; R[g] += 1.0; }         // i_{g}: :185
        }
        return true;
    }
    __device__ __forceinline__ void save(double* x) const {
#pragma unroll
        for (int g = 0; g < G; ++g) { x[3 * g] = S[g]; x[3 * g + 1] = I[g]; x[3 * g + 2] = R[g]; }
    }
    __device__ __forceinline__ double tau_of(const Block& r, const ChainParam& cp, const LogTab* __restrict__ tab) const {
        double cum[NCH];
        return rates(cp, cum) * neg_log_one_minus_u01(r.x, r.y, tab);
    }
};
template <int G> struct SsaState<kSubgroups, G> : SubgroupsState<G> {};
template <int G> struct SsaState<kSubgroups2, G> : SubgroupsState<G> {};

// ------------------------------------------------------------------------------- certified f32 fast path
// The exact loop above spends ~45 f64 operations per event (the table log alone ~20, v_rcp_f64 16 cycles).
// The fast path takes every decision in f32 and certifies it (derivation: DESIGN.md §4):
//   channel  the cumulative propensities c_i and their total are f32 sums of positive terms with relative
//            error <= e_as ulp (per model below); q_i = c_i * rcp(total) is then within e_q = 2 e_as + 5 ulp of
//            the reference's ratio (v_rcp_f32 <= 1.53 ulp).  U lies in [uf, uf + 2^-23) for uf its top 23 bits;
//            with uc = uf + 2^-24, every decision q_ref <= U is certain when all |q_i - uc| > kBand >= (e_q + 2)
//            ulp, else the model's *_channel_exact evaluates the reference expression in f64.  Models with more
//            than 3 channels compare c_i against T = uc * total with the band scaled by total (the reciprocal's
//            error drops out: 2 e_as + 2 ulp, inside the same band).
//   clock    time is kept in units of 1/ln 2 and counted down: rem = tmax/ln2 + sum(log2(x_f) * rcp(total)),
//            the event is inside the step iff rem >= 0 (the exact path's t + tau <= tmax, scaled).  x_f = 1 - U
//            from its top word for x >= 2^-8 (one convert, scaled exactly: the convert's rounding plus the dropped
//            low word, <= 2 ulp), from two converts below (<= 3 ulp for x >= 2^-20); v_log_f32 is within 2 ulp of |log2 x|
//            on every float in [2^-20, 1) (exhaustive, scripts/f32_accuracy.hip); below 2^-20 (2^-20 of events)
//            log2 is taken in f64 of the exact x and rounded (tiny_log2, <= 0.5 ulp + 2^-29).  Per event
//            |tau2_f - tau2| <= (e_as + 5.5) ulp |tau2_f| + 4.4 ulp rcp(total), so with R = sum rcp(total) the
//            remaining time is within B = kClockT tmax/ln2 + 5 ulp R of the exact path's, scaled
//            (kClockT = e_as + 7 ulp covers the float evaluation of B and rem and at most 2^26 events).
//            rem > B: the event is the exact path's; rem < -B: the step ends there, as in the exact path;
//            otherwise the lane hands its whole step to the exact loop, from the untouched parent state.
// Eligible lanes: population < 2^24 (counts exact in f32; < 2^26 events per step) and every rate parameter
// zero or in [2^-60, 2^40] (every f32 intermediate stays normal).
constexpr float kUlpF = 0x1.0p-24f;
constexpr float kClockRF = 5.0f * kUlpF;
constexpr double kInvLn2 = 0x1.71547652b82fep0;

__device__ __forceinline__ bool rate_ok(float v) { return v == 0.f || (v >= 0x1.0p-60f && v <= 0x1.0p40f); }

// log2(1 - U) for 1 - U < 2^-20, where the two-convert f32 form of 1 - U loses its relative accuracy: the exact
// 53-bit 1 - U in f64 and the library log2 (<= 1 ulp f64), rounded to f32 (<= 0.5 ulp + 2^-29), inside the 2-ulp
// log budget of the clock bound.  Out of line: it runs for 2^-20 of events.
__device__ __noinline__ float tiny_log2(uint32_t lo, uint32_t hi) { return (float)log2(one_minus_u01(lo, hi)); }

template <int MODEL, int G>
struct FastSsa;

template <>
struct FastSsa<kSIR, 1> {                                              // gillespie_algo.py:10-75
    static constexpr int NCH = 2;
    static constexpr float kBand = 0x1.0p-19f;                         // e_as = 4, e_q = 13
    static constexpr float kClockT = 11.0f * kUlpF;
    double N;
    float S, I, bN, g, S0, SI0;
    __device__ __forceinline__ bool load(const double* x, const ChainParam& cp) {
        N = (x[0] + x[1]) + x[2];                                      // :35
        bN = (float)(cp.theta[0] / N);
        g = cp.thetaf[1];
        S = S0 = (float)x[0];
        I = (float)x[1];
        SI0 = S + I;
        return N < 16777216.0 && rate_ok(bN) && rate_ok(g);
    }
    __device__ __forceinline__ bool active() const { return I > 0.f; }   // :48
    __device__ __forceinline__ float cum(float* c) const {             // :38-39
        c[0] = bN * (S * I);
        return fmaf(g, I, c[0]);
    }
    __device__ __forceinline__ int exact_channel(const ChainParam& cp, double u) const {
        return sir_channel_exact(cp.theta[0], cp.theta[1], (double)S, (double)I, N, u) ? 1 : 0;
    }
    __device__ __forceinline__ void apply(int ch, float s) {           // s = +1 apply, -1 undo; :43-46
        S = S - (ch == 0 ? s : 0.f);
        I = I + (ch == 0 ? s : -s);
    }
    // the counts of s where c holds (the lane-group pass keeps each lane's state before its event with selects, one
    // basic block for the whole pass; the other fields are the particle-step's constants)
    __device__ __forceinline__ void keep_if(bool c, const FastSsa& s) {
        S = c ? s.S : S;
        I = c ? s.I : I;
    }
    // the event from the wave masks below[i] of the certified sides c_i < U total (the lane-group pass,
    // epipf_group.hpp: decide_lo); the selects take the masks as their SGPR conditions
    __device__ __forceinline__ void apply_below(const uint64_t* below) {
        const bool rec = __builtin_amdgcn_inverse_ballot_w64(below[0]);
        S = S - (rec ? 0.f : 1.f);
        I = I + (rec ? -1.f : 1.f);
    }
    // The lane-group fixed-point pass (epipf_group.hpp: decide_fixed_point): this lane's event decided on its own, on
    // decide_lo's Tlo side, as an event count in a byte field (byte 0 infections, byte 1 recoveries), and a state
    // rebuilt from the chunk start b and the counts n of the events before it (small integers: exact in f32)
    static constexpr bool kFixedPoint = true;
    // cc / tot (optional): the cumulative rates and total it decided on, kept for the certificate (event_certified_on)
    __device__ __forceinline__ uint32_t outcome(float ulo, float* cc = nullptr, float* tot = nullptr) const {
        float c[1];
        const float total = cum(c);
        const float Tlo = ulo * total;
        if (cc) { cc[0] = c[0]; *tot = total; }
        return c[0] < Tlo ? 0x100u : 0x1u;
    }
    __device__ __forceinline__ void advance(const FastSsa& b, uint32_t n) {
        const float ni = (float)(n & 0xFFu), nr = (float)((n >> 8) & 0xFFu);
        S = b.S - ni;
        I = (b.I + ni) - nr;
    }
    __device__ __forceinline__ int save(double* x) const {
        const float inf = S0 - S, rec = SI0 - (S + I);
        x[0] = (double)S; x[1] = (double)I; x[2] = x[2] + (double)rec;
        return (int)(inf + rec);
    }
};

template <>
struct FastSsa<kSEIR, 1> {                                             // gillespie_algo.py:78-146
    static constexpr int NCH = 3;
    static constexpr float kBand = 0x1.0p-19f;                         // e_as = 5, e_q = 15
    static constexpr float kClockT = 12.0f * kUlpF;
    double N;
    float S, E, I, bN, al, g, S0, I0, SEI0;
    __device__ __forceinline__ bool load(const double* x, const ChainParam& cp) {
        N = ((x[0] + x[1]) + x[2]) + x[3];                             // :104
        bN = (float)(cp.theta[0] / N);
        al = cp.thetaf[1];
        g = cp.thetaf[2];
        S = S0 = (float)x[0];
        E = (float)x[1];
        I = I0 = (float)x[2];
        SEI0 = (S + E) + I;
        return N < 16777216.0 && rate_ok(bN) && rate_ok(al) && rate_ok(g);
    }
    __device__ __forceinline__ bool active() const { return E > 0.f || I > 0.f; }   // :119
    __device__ __forceinline__ float cum(float* c) const {             // :107-109
        c[0] = bN * (S * I);
        c[1] = fmaf(al, E, c[0]);
        return fmaf(g, I, c[1]);
    }
    __device__ __forceinline__ int exact_channel(const ChainParam& cp, double u) const {
        return seir_channel_exact(cp.theta[0], cp.theta[1], cp.theta[2], (double)S, (double)E, (double)I, N, u);
    }
    __device__ __forceinline__ void apply(int ch, float s) {           // :113-117
        S = S - (ch == 0 ? s : 0.f);
        E = E + (ch == 0 ? s : (ch == 1 ? -s : 0.f));
        I = I + (ch == 1 ? s : (ch == 2 ? -s : 0.f));
    }
    __device__ __forceinline__ void keep_if(bool c, const FastSsa& s) {
        S = c ? s.S : S;
        E = c ? s.E : E;
        I = c ? s.I : I;
    }
    __device__ __forceinline__ void apply_below(const uint64_t* below) {   // below[1] implies below[0]
        const bool b0 = __builtin_amdgcn_inverse_ballot_w64(below[0]), b1 = __builtin_amdgcn_inverse_ballot_w64(below[1]);
        S = S - (b0 ? 0.f : 1.f);
        E = E + (b0 ? (b1 ? 0.f : -1.f) : 1.f);
        I = I + (b1 ? -1.f : (b0 ? 1.f : 0.f));
    }
    // fixed-point pass (see FastSsa<kSIR>): byte 0 S->E, byte 1 E->I, byte 2 I->R
    static constexpr bool kFixedPoint = true;
    __device__ __forceinline__ uint32_t outcome(float ulo, float* cc = nullptr, float* tot = nullptr) const {
        float c[2];
        const float total = cum(c);
        const float Tlo = ulo * total;
        if (cc) { cc[0] = c[0]; cc[1] = c[1]; *tot = total; }
        return c[1] < Tlo ? 0x10000u : c[0] < Tlo ? 0x100u : 0x1u;
    }
    __device__ __forceinline__ void advance(const FastSsa& b, uint32_t n) {
        const float n0 = (float)(n & 0xFFu), n1 = (float)((n >> 8) & 0xFFu), n2 = (float)((n >> 16) & 0xFFu);
        S = b.S - n0;
        E = (b.E + n0) - n1;
        I = (b.I + n1) - n2;
    }
    __device__ __forceinline__ int save(double* x) const {
        const float n0 = S0 - S, n2 = SEI0 - ((S + E) + I), n1 = (I - I0) + n2;
        x[0] = (double)S; x[1] = (double)E; x[2] = (double)I; x[3] = x[3] + (double)n2;
        return (int)((n0 + n1) + n2);
    }
};

template <int G>
struct FastSubgroups {                                                 // gillespie_algo.py:148-233
    static constexpr int NCH = G * G + G;
    static constexpr float kBand = (2 * (4 + NCH) + 7 <= 32) ? 0x1.0p-19f : 0x1.0p-18f;   // (e_q + 2) ulp
    static constexpr float kClockT = (float)(NCH + 11) * kUlpF;        // e_as = 4 + NCH
    double sumN;
    float S[G], I[G], Ng[G], invN, S0sum, R0sum;
    const float* b;                                                    // beta[G][G] then gamma, f32 (SGPRs)
    __device__ __forceinline__ bool load(const double* x, const ChainParam& cp) {
        sumN = 0.0;
        bool ok = true;
        S0sum = 0.f;
        R0sum = 0.f;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            sumN = sumN + ((x[3 * q] + x[3 * q + 1]) + x[3 * q + 2]);  // sum(N), :176,:182
            S[q] = (float)x[3 * q];
            I[q] = (float)x[3 * q + 1];
            Ng[q] = (S[q] + I[q]) + (float)x[3 * q + 2];
            S0sum += S[q];
            R0sum += (float)x[3 * q + 2];
        }
        b = cp.thetaf;
#pragma unroll
        for (int q = 0; q <= G * G; ++q) ok = ok && rate_ok(b[q]);
        invN = (float)(1.0 / sumN);
        return ok && sumN >= 1.0 && sumN < 16777216.0;
    }
    __device__ __forceinline__ bool active() const {                   // :192-193, :222
        float inf = 0.f;
#pragma unroll
        for (int q = 0; q < G; ++q) inf += I[q];
        return inf > 0.f;
    }
    __device__ __forceinline__ float cum(float* c) const {             // channel order, :180-185
        float run = 0.f;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const float cI = I[q] * invN;
#pragma unroll
            for (int q2 = 0; q2 < G; ++q2) {
                run = fmaf(b[q * G + q2] * S[q2], cI, run);
                if (q * (G + 1) + q2 < NCH - 1) c[q * (G + 1) + q2] = run;
            }
            run = fmaf(b[G * G], I[q], run);
            if (q * (G + 1) + G < NCH - 1) c[q * (G + 1) + G] = run;
        }
        return run;
    }
    __device__ __forceinline__ int exact_channel(const ChainParam& cp, double u) const {
        double Sd[G], Id[G];
#pragma unroll
        for (int q = 0; q < G; ++q) { Sd[q] = (double)S[q]; Id[q] = (double)I[q]; }
        return subgroups_channel_exact<G>(cp.theta, Sd, Id, sumN, u);
    }
    // Channel ch = g*(G+1) + c: c < G is infection s_{g}_{c} (S[c] -> I[c], :183), c = G recovery i_{g} (I[g] -> R,
    // :185).  Only one group moves, q = c or g: a per-group select instead of a branch per channel (the compiler
    // turns the channel-by-channel form into a divergent switch).  Whether ch is an infection and the group q it
    // moves are bit fields of compile-time masks (one bit-field extract each, no division by G + 1).
    static constexpr uint32_t chan_mask(int what) {      // what = -1: infection bits; 0/1: bit `what` of q
        uint32_t m = 0;
        for (int ch = 0; ch < NCH; ++ch) {
            const int g = ch / (G + 1), c = ch % (G + 1), q = c < G ? c : g;
            const bool bit = what < 0 ? c < G : ((q >> what) & 1) != 0;
            m |= bit ? (1u << ch) : 0u;
        }
        return m;
    }
    static constexpr uint32_t kInfMask = chan_mask(-1), kQ0 = chan_mask(0), kQ1 = chan_mask(1);
    __device__ __forceinline__ void apply(int ch, float s) {
        static_assert(NCH <= 32 && G <= 4, "channel masks");
        const bool inf = ((kInfMask >> ch) & 1u) != 0u;
        const int q = (int)((kQ0 >> ch) & 1u) | (G > 2 ? (int)(((kQ1 >> ch) & 1u) << 1) : 0);
        const float dS = inf ? s : 0.f, dI = inf ? s : -s;
#pragma unroll
        for (int r = 0; r < G; ++r) {
            const bool hit = q == r;
            S[r] -= hit ? dS : 0.f;
            I[r] += hit ? dI : 0.f;
        }
    }
    // the event from the wave masks below[i] of the certified sides c_i < U total (channel ch fired iff below[ch - 1]
    // and not below[ch]; FastSubgroupsPacked::apply_below), keeping the per-group changes for an undo
    __device__ __forceinline__ void apply_below(const uint64_t* below, float* dS, float* dI) {
        auto hit = [&](int ch) __attribute__((always_inline)) -> uint64_t {
            return (ch == 0 ? ~0ull : below[ch - 1]) & (ch == NCH - 1 ? ~0ull : ~below[ch]);
        };
#pragma unroll
        for (int r = 0; r < G; ++r) {
            uint64_t inf = 0;
#pragma unroll
            for (int g = 0; g < G; ++g) inf |= hit(g * (G + 1) + r);
            const bool fi = __builtin_amdgcn_inverse_ballot_w64(inf);
            const bool fr = __builtin_amdgcn_inverse_ballot_w64(hit(r * (G + 1) + G));
            dS[r] = fi ? 1.f : 0.f;
            dI[r] = fi ? 1.f : (fr ? -1.f : 0.f);
            S[r] = S[r] - dS[r];
            I[r] = I[r] + dI[r];
        }
    }
    __device__ __forceinline__ void undo(const float* dS, const float* dI) {
#pragma unroll
        for (int r = 0; r < G; ++r) {
            S[r] = S[r] + dS[r];
            I[r] = I[r] - dI[r];
        }
    }
    __device__ __forceinline__ int save(double* x) const {
        float inf = S0sum, rec = -R0sum;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const float R = (Ng[q] - S[q]) - I[q];
            inf -= S[q];
            rec += R;
            x[3 * q] = (double)S[q]; x[3 * q + 1] = (double)I[q]; x[3 * q + 2] = (double)R;
        }
        return (int)(inf + rec);
    }
};
// The subgroup model's f32 state in the lane-group pass (epipf_group.hpp), FastSubgroups' arithmetic with the
// counts in pairs of groups (S[q] = S2[q / 2][q % 2]; an odd G's pad slot stays 0): the propensity products and the
// state updates are packed f32 (v_pk_mul_f32 / v_pk_add_f32), one instruction per pair, and the event is applied
// from the decision's wave masks (apply_below).  Same roundings per term as FastSubgroups (the same e_as and band).
template <int G>
struct FastSubgroupsPacked {                                           // gillespie_algo.py:148-233
    static constexpr int NCH = G * G + G;
    static constexpr float kBand = (2 * (4 + NCH) + 7 <= 32) ? 0x1.0p-19f : 0x1.0p-18f;   // (e_q + 2) ulp
    static constexpr float kClockT = (float)(NCH + 11) * kUlpF;        // e_as = 4 + NCH
    using f2 = float __attribute__((ext_vector_type(2)));
    static constexpr int P = (G + 1) / 2;
    double sumN;
    f2 S2[P], I2[P];
    f2 bN2[G][P];                                                      // beta[q][q2] / sum(N)
    float Ng[G], S0sum, R0sum;
    float gam;                                                         // gamma, f32 (a value: a pointer into cp would
                                                                       // pin the whole ChainParam to scratch)
    // packed multiply (the selector scalarises a <2 x float> product whose halves are used apart); rounds each half
    // as v_mul_f32
    static __device__ __forceinline__ f2 pk_mul(f2 a, f2 b) {
        f2 r;
        asm("v_pk_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
        return r;
    }
    __device__ __forceinline__ void keep_if(bool c, const FastSubgroupsPacked& s) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            S2[p] = c ? s.S2[p] : S2[p];
            I2[p] = c ? s.I2[p] : I2[p];
        }
    }
    __device__ __forceinline__ float S(int q) const { return S2[q >> 1][q & 1]; }
    __device__ __forceinline__ float I(int q) const { return I2[q >> 1][q & 1]; }
    __device__ __forceinline__ bool load(const double* x, const ChainParam& cp) {
        sumN = 0.0;
        bool ok = true;
        S0sum = 0.f;
        R0sum = 0.f;
#pragma unroll
        for (int p = 0; p < P; ++p) S2[p] = I2[p] = f2{0.f, 0.f};
#pragma unroll
        for (int q = 0; q < G; ++q) {
            sumN = sumN + ((x[3 * q] + x[3 * q + 1]) + x[3 * q + 2]);  // sum(N), :176,:182
            S2[q >> 1][q & 1] = (float)x[3 * q];
            I2[q >> 1][q & 1] = (float)x[3 * q + 1];
            Ng[q] = (S(q) + I(q)) + (float)x[3 * q + 2];
            S0sum += S(q);
            R0sum += (float)x[3 * q + 2];
        }
        const float* b = cp.thetaf;                                    // beta[G][G] then gamma, f32
#pragma unroll
        for (int q = 0; q <= G * G; ++q) ok = ok && rate_ok(b[q]);
        gam = b[G * G];
        // beta / sum(N) once per step (VGPR pairs, for the packed products).  Each term's error is that of
        // (beta S)(I / sum(N)): four roundings before the accumulating fma (e_as unchanged).
        const float invN = (float)(1.0 / sumN);
#pragma unroll
        for (int q = 0; q < G; ++q)
#pragma unroll
            for (int q2 = 0; q2 < 2 * P; ++q2) bN2[q][q2 >> 1][q2 & 1] = q2 < G ? b[q * G + q2] * invN : 0.f;
        return ok && sumN >= 1.0 && sumN < 16777216.0;
    }
    __device__ __forceinline__ bool active() const {                   // :192-193, :222 (counts are >= 0)
        float inf = I(0);
#pragma unroll
        for (int q = 1; q < G; ++q) inf = inf + I(q);
        return inf > 0.f;
    }
    __device__ __forceinline__ float cum(float* c) const {             // channel order, :180-185
        float run = 0.f;
#pragma unroll
        for (int q = 0; q < G; ++q) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const f2 bs = pk_mul(bN2[q][p], S2[p]);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int q2 = 2 * p + h;
                    if (q2 < G) {
                        run = fmaf(bs[h], I(q), run);
                        if (q * (G + 1) + q2 < NCH - 1) c[q * (G + 1) + q2] = run;
                    }
                }
            }
            run = fmaf(gam, I(q), run);
            if (q * (G + 1) + G < NCH - 1) c[q * (G + 1) + G] = run;
        }
        return run;
    }
    __device__ __forceinline__ int exact_channel(const ChainParam& cp, double u) const {
        double Sd[G], Id[G];
#pragma unroll
        for (int q = 0; q < G; ++q) { Sd[q] = (double)S(q); Id[q] = (double)I(q); }
        return subgroups_channel_exact<G>(cp.theta, Sd, Id, sumN, u);
    }
    // Channel ch = g*(G+1) + c: c < G is infection s_{g}_{c} (S[c] -> I[c], :183), c = G recovery i_{g} (I[g] -> R,
    // :185).  Only one group moves, q = c or g: a per-group select instead of a branch per channel (the compiler
    // turns the channel-by-channel form into a divergent switch).  Whether ch is an infection and the group q it
    // moves are bit fields of compile-time masks (one bit-field extract each, no division by G + 1).
    static constexpr uint32_t chan_mask(int what) {      // what = -1: infection bits; 0/1: bit `what` of q
        uint32_t m = 0;
        for (int ch = 0; ch < NCH; ++ch) {
            const int g = ch / (G + 1), c = ch % (G + 1), q = c < G ? c : g;
            const bool bit = what < 0 ? c < G : ((q >> what) & 1) != 0;
            m |= bit ? (1u << ch) : 0u;
        }
        return m;
    }
    static constexpr uint32_t kInfMask = chan_mask(-1), kQ0 = chan_mask(0), kQ1 = chan_mask(1);
    __device__ __forceinline__ void apply(int ch, float s) {
        static_assert(NCH <= 32 && G <= 4, "channel masks");
        const bool inf = ((kInfMask >> ch) & 1u) != 0u;
        const int q = (int)((kQ0 >> ch) & 1u) | (G > 2 ? (int)(((kQ1 >> ch) & 1u) << 1) : 0);
        const float dS = inf ? s : 0.f, dI = inf ? s : -s;
#pragma unroll
        for (int p = 0; p < P; ++p) {
            f2 ds, di;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const bool hit = q == 2 * p + h;
                ds[h] = hit ? dS : 0.f;
                di[h] = hit ? dI : 0.f;
            }
            S2[p] = S2[p] - ds;
            I2[p] = I2[p] + di;
        }
    }
    // the event from the wave masks below[i] of the certified sides c_i < U total: channel ch happened iff below[ch - 1]
    // and not below[ch] (the c_i are nondecreasing); group r gains an infection from channels g (G + 1) + r and loses
    // one to recovery from channel r (G + 1) + G.  The mask logic is SALU; selects on the masks, one packed add per
    // pair of counts.
    __device__ __forceinline__ void apply_below(const uint64_t* below) {
        auto hit = [&](int ch) __attribute__((always_inline)) -> uint64_t {
            return (ch == 0 ? ~0ull : below[ch - 1]) & (ch == NCH - 1 ? ~0ull : ~below[ch]);
        };
#pragma unroll
        for (int p = 0; p < P; ++p) {
            f2 ds{0.f, 0.f}, di{0.f, 0.f};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = 2 * p + h;
                if (r < G) {
                    uint64_t inf = 0;
#pragma unroll
                    for (int g = 0; g < G; ++g) inf |= hit(g * (G + 1) + r);
                    const bool fi = __builtin_amdgcn_inverse_ballot_w64(inf);
                    const bool fr = __builtin_amdgcn_inverse_ballot_w64(hit(r * (G + 1) + G));
                    ds[h] = fi ? 1.f : 0.f;
                    di[h] = fi ? 1.f : (fr ? -1.f : 0.f);
                }
            }
            S2[p] = S2[p] - ds;
            I2[p] = I2[p] + di;
        }
    }
    // fixed-point pass (see FastSsa<kSIR>): byte r infections of group r, byte G + r recoveries of group r; four byte
    // fields, so G <= 2 (larger G keeps the sequential pass)
    static constexpr bool kFixedPoint = 2 * G <= 4;
    static constexpr uint32_t code(int ch) {             // the event count of channel ch, in its field
        return 1u << (8 * (ch % (G + 1) < G ? ch % (G + 1) : G + ch / (G + 1)));
    }
    __device__ __forceinline__ uint32_t outcome(float ulo, float* cc = nullptr, float* tot = nullptr) const {
        float c[NCH - 1];
        const float total = cum(c);
        const float Tlo = ulo * total;
        if (cc) {
#pragma unroll
            for (int i = 0; i < NCH - 1; ++i) cc[i] = c[i];
            *tot = total;
        }
        uint32_t d = code(0);                            // channel = #{i : c_i < Tlo} (the c_i are nondecreasing)
#pragma unroll
        for (int i = 0; i < NCH - 1; ++i) d = c[i] < Tlo ? code(i + 1) : d;
        return d;
    }
    __device__ __forceinline__ void advance(const FastSubgroupsPacked& b, uint32_t n) {
#pragma unroll
        for (int p = 0; p < P; ++p) {
            f2 ni{0.f, 0.f}, nr{0.f, 0.f};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int r = 2 * p + h;
                if (r < G) {
                    ni[h] = (float)((n >> (8 * r)) & 0xFFu);
                    nr[h] = (float)((n >> (8 * (G + r))) & 0xFFu);
                }
            }
            S2[p] = b.S2[p] - ni;
            I2[p] = (b.I2[p] + ni) - nr;
        }
    }
    __device__ __forceinline__ int save(double* x) const {
        float inf = S0sum, rec = -R0sum;
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const float R = (Ng[q] - S(q)) - I(q);
            inf -= S(q);
            rec += R;
            x[3 * q] = (double)S(q); x[3 * q + 1] = (double)I(q); x[3 * q + 2] = (double)R;
        }
        return (int)(inf + rec);
    }
};
template <int G> struct FastSsa<kSubgroups, G> : FastSubgroups<G> {};
template <int G> struct FastSsa<kSubgroups2, G> : FastSubgroups<G> {};
// the f32 state of the lane-group pass
template <int MODEL, int G> struct GroupSsa { using type = FastSsa<MODEL, G>; };
template <int G> struct GroupSsa<kSubgroups, G> { using type = FastSubgroupsPacked<G>; };
template <int G> struct GroupSsa<kSubgroups2, G> { using type = FastSubgroupsPacked<G>; };

template <int MODEL, int G>
__device__ __forceinline__ bool fast_propagate(double* x, const ChainParam& cp, uint32_t j, uint32_t ptag,
                                               double tmax, int& nev_out, int& iters, bool& eligible) {
    using F = FastSsa<MODEL, G>;
    constexpr int NCH = F::NCH;
    iters = 0;
    nev_out = 0;
    eligible = false;
    if (!(cp.flags & kChainFastSsa)) return false;
    F st;
    if (!st.load(x, cp)) return false;
    eligible = true;
    const float kB = F::kBand * cp.band_slack;                         // the decision band (slack 1: kBand)
    double rem = tmax * kInvLn2;                                       // remaining time, units of 1/ln 2
    const float Bt = (float)rem * F::kClockT * cp.clock_slack;
    float R = 0.f, df = 0.f, B = 0.f;
    uint32_t ks = 0;                                                   // event index, wave-uniform (SGPR)
    bool alive = st.active(), ok = true;
    int ch = 0;
    constexpr int GD = NCH > 3 ? G : 1;
    float dS[GD], dI[GD];                                              // the last event's changes (subgroups)
    Block rn{0u, 0u, 0u, 0u};
    if (alive) rn = philox<true>(0u, j, ptag, cp.f, cp.k0, cp.k1);    // x word inverted: ~x
    while (alive) {
        const Block r = rn;
        ks = __builtin_amdgcn_readfirstlane(ks) + 1u;
        rn = philox<true>(ks, j, ptag, cp.f, cp.k0, cp.k1);
        float c[NCH - 1];
        const float total = st.cum(c);
        const float ri = __builtin_amdgcn_rcpf(total);
        const float uc = __uint_as_float(0x3F800000u | (r.w >> 9)) - (1.0f - kUlpF);   // uf + 2^-24
        uint64_t below[NCH - 1];
        if constexpr (NCH <= 3) {                                      // ratios q_i = c_i / total
            bool close = false;
            ch = 0;
#pragma unroll
            for (int i = 0; i < NCH - 1; ++i) {                        // numpy choice, searchsorted right
                const float q = c[i] * ri;
                ch += (q < uc) ? 1 : 0;
                close |= fabsf(q - uc) <= kB;
            }
            if (close) ch = st.exact_channel(cp, u01(r.z, r.w));
        } else {
            // c_i against U total as wave masks, the lane-group pass's certified bracket (decide_lo,
            // epipf_group.hpp: Tlo = fl((uc - kBand) total), Thi = fl(Tlo + 2 kBand total)); a lane with some c_i in
            // between takes the reference expression in f64 and its bits of the masks are replaced
            const float Tlo = (uc - kB) * total, Thi = fmaf(2.0f * kB, total, Tlo);
            uint64_t unsure = 0;
#pragma unroll
            for (int i = 0; i < NCH - 1; ++i) {
                below[i] = __ballot(c[i] < Tlo);
                unsure |= below[i] ^ __ballot(c[i] < Thi);
            }
            if (unsure) {                                              // wave-uniform, rare
                const bool mine = __builtin_amdgcn_inverse_ballot_w64(unsure);
                int che = 0;
                if (mine) che = st.exact_channel(cp, u01(r.z, r.w));
#pragma unroll
                for (int i = 0; i < NCH - 1; ++i) below[i] = (below[i] & ~unsure) | __ballot(mine && che > i);
            }
        }
        const uint32_t nh = ~r.y;
        float lg = __builtin_amdgcn_logf((float)nh * 0x1.0p-32f);     // 1 - U from its top word: <= 2 ulp for x >= 2^-8
        if (nh < 0x1000000u) {                                         // 1 - U < 2^-8: 0.4% of events
            if (nh < 4096u) lg = tiny_log2(~r.x, r.y);                // 1 - U < 2^-20
            else lg = __builtin_amdgcn_logf(fmaf((float)nh, 0x1.0p-32f, (float)r.x * 0x1.0p-64f));  // r.x is ~x
        }
        rem = rem + (double)(lg * ri);                                 // np.random.exponential
        R += ri;
        df = (float)rem;
        B = fmaf(R, kClockRF, Bt);
        ok = df > B;                                                   // certainly inside the step
        if constexpr (NCH <= 3) st.apply(ch, 1.f);                     // undone below if the lane overshoots
        else st.apply_below(below, dS, dI);
        alive = ok && st.active();
    }
    if (!ok) {
        if (!(df < -B)) return false;                                 // boundary too close to call: exact loop
        if constexpr (NCH <= 3) st.apply(ch, -1.f);                    // the overshooting event is not applied
        else st.undo(dS, dI);
    }
    nev_out = st.save(x);
    iters = nev_out + (ok ? 0 : 1);
    return true;
}

// The exact loop over [0, tmax] from the parent state x (every lane that enters starts at event 0 together, so
// the event index k is wave-uniform).  Software pipelining: event k+1's Philox block (counter-based, so
// independent of event k's outcome) is computed while event k's f64 work runs, which gives each wave two
// independent dependency chains.  The block drawn after the last event is discarded (one per particle-step).
template <int MODEL, int G>
__device__ __forceinline__ int exact_propagate(double* x, const ChainParam& cp, uint32_t j, uint32_t ptag,
                                               double tmax, const LogTab* __restrict__ tab, int& iters) {
    SsaState<MODEL, G> st;
    st.load(x, cp);
    double t = 0.0;
    uint32_t k = 0;
    int nev = 0;
    bool alive = st.active();
    Block rn{0u, 0u, 0u, 0u};
    if (alive) rn = philox(0u, j, ptag, cp.f, cp.k0, cp.k1);
    while (alive) {
        const Block r = rn;                                            // this event's block
        ++k;
        rn = philox(__builtin_amdgcn_readfirstlane(k), j, ptag, cp.f, cp.k0, cp.k1);   // next event's
        const bool ev = st.event(r, t, tmax, cp, tab);
        nev += ev ? 1 : 0;
        alive = ev && st.active();
    }
    st.save(x);
    iters = (int)k;
    return nev;
}

// ------------------------------------------------------------------------------- wave-cooperative replay
// A lane whose f32 loop ended too close to the step boundary to certify (|rem| <= B) needs the exact loop's answer,
// and one lane running ~100 f64 events leaves 63 lanes idle.  The whole wave instead replays that particle in
// chunks of 64 events:
//   1. lane i computes event (base + i)'s Philox block (counter-based: independent of the state);
//   2. one uniform pass applies the chunk's channel decisions in order -- the f32 loop's certified test with the
//      exact fallback, which is the exact loop's decision -- and lane i keeps the state before event base + i;
//   3. lane i evaluates that event's time with the exact loop's expressions (SsaState::tau_of);
//   4. one uniform pass adds the times in event order (t + tau > tmax ends the step, as the exact loop's test).
// The result is the exact loop's, bit for bit (tests/test_gpu_parity.py: EPIPF_SSA_FAST=0 vs 1), at ~20 wave
// instructions per event instead of ~130.  Requires every lane of the wave (call it with full exec).
template <typename F>
__device__ __forceinline__ int fast_channel(const F& st, const ChainParam& cp, uint32_t rz, uint32_t rw) {
    constexpr int NCH = F::NCH;
    float c[NCH - 1];
    const float total = st.cum(c);
    const float ri = __builtin_amdgcn_rcpf(total);
    const float uc = __uint_as_float(0x3F800000u | (rw >> 9)) - (1.0f - kUlpF);
    bool close = false;
    int ch = 0;
    if constexpr (NCH <= 3) {
#pragma unroll
        for (int i = 0; i < NCH - 1; ++i) {
            const float q = c[i] * ri;
            ch += (q < uc) ? 1 : 0;
            close |= fabsf(q - uc) <= F::kBand * cp.band_slack;
        }
    } else {
        const float T = uc * total, band = F::kBand * cp.band_slack * total;
#pragma unroll
        for (int i = 0; i < NCH - 1; ++i) {
            ch += (c[i] < T) ? 1 : 0;
            close |= fabsf(c[i] - T) <= band;
        }
    }
    if (close) ch = st.exact_channel(cp, u01(rz, rw));
    return ch;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const uint64_t b = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, lane), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), lane);
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// row: the particle's output row, holding its parent state on entry and its new state on return (every lane reads
// it; the state is not kept in registers across the replay).  WAVE: the caller's workgroup has other waves (the
// one-workgroup filter), so the row is ordered by a wave-level LDS sync instead of a workgroup barrier.
template <bool WAVE>
__device__ __forceinline__ void replay_sync() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        __syncthreads();
    }
}

template <int MODEL, int G, bool WAVE = false>
__device__ __forceinline__ int coop_replay(int32_t* row, const ChainParam& cp, uint32_t j, uint32_t ptag, double tmax,
                                           const LogTab* __restrict__ tab) {
    using F = FastSsa<MODEL, G>;
    constexpr int C = (MODEL == kSIR) ? 3 : (MODEL == kSEIR) ? 4 : 3 * G;
    const int lane = (int)(threadIdx.x & 63);
    F st;
    {
        double x0[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x0[c] = (double)row[c];
        st.load(x0, cp);                                 // eligible: the f32 loop ran on this particle
    }
    double t = 0.0;
    uint32_t base = 0;
    int nev = 0;
    bool more = st.active();
    F mine = st;                                         // state before event base + lane
    while (more) {
        const Block r = philox(base + (uint32_t)lane, j, ptag, cp.f, cp.k0, cp.k1);
        mine = st;
        int nk = 64;                                     // events of this chunk up to extinction
        for (int i = 0; i < 64; ++i) {
            if (lane == i) mine = st;
            const uint32_t rz = __builtin_amdgcn_readlane(r.z, i), rw = __builtin_amdgcn_readlane(r.w, i);
            st.apply(fast_channel(st, cp, rz, rw), 1.f);
            if (!st.active()) { nk = i + 1; break; }
        }
        double tau = 0.0;
        if (lane < nk) {
            double xk[C];
#pragma unroll
            for (int c = 0; c < C; ++c) xk[c] = (double)row[c];
            mine.save(xk);
            SsaState<MODEL, G> ex;
            ex.load(xk, cp);
            tau = ex.tau_of(r, cp, tab);
        }
        int stop = -1;                                   // first event of the chunk past tmax
        for (int i = 0; i < nk; ++i) {
            const double tn = t + readlane_f64(tau, i);
            if (tn > tmax) { stop = i; break; }
            t = tn;
        }
        if (stop >= 0) {                                 // the step ends before event base + stop
            nev += stop;
            double xs[C];
#pragma unroll
            for (int c = 0; c < C; ++c) xs[c] = (double)row[c];
            mine.save(xs);
            int32_t v[C];
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = (int32_t)readlane_f64(xs[c], stop);
            replay_sync<WAVE>();                         // every lane has read the parent row
            if (lane == 0) {
#pragma unroll
                for (int c = 0; c < C; ++c) row[c] = v[c];
            }
            return nev;
        }
        nev += nk;
        base += 64u;
        more = nk == 64;                                 // else the population died out after the last event
    }
    double xf[C];
#pragma unroll
    for (int c = 0; c < C; ++c) xf[c] = (double)row[c];
    st.save(xf);
    replay_sync<WAVE>();
    if (lane == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c) row[c] = (int32_t)xf[c];
    }
    return nev;
}

// One particle over [0, tmax]: the certified f32 path first; lanes it cannot certify run the exact loop from the
// untouched parent state.
template <int MODEL, int G>
__device__ __forceinline__ int ssa_propagate(double* x, const ChainParam& cp, uint32_t j, uint32_t ptag,
                                             double tmax, const LogTab* __restrict__ tab, int& iters, int& exact) {
    int fast_iters = 0, fast_nev = 0;
    bool eligible = false;
    exact = 1;
    if (fast_propagate<MODEL, G>(x, cp, j, ptag, tmax, fast_nev, fast_iters, eligible)) {
        iters = fast_iters;
        exact = 0;
        return fast_nev;
    }
    int ex_iters = 0;
    const int nev = exact_propagate<MODEL, G>(x, cp, j, ptag, tmax, tab, ex_iters);
    iters = ex_iters + fast_iters;
    return nev;
}

template <int MODEL, int G>
struct Shape {
    static constexpr int C = (MODEL == kSIR) ? 3 : (MODEL == kSEIR) ? 4 : 3 * G;
    static constexpr int K = (MODEL == kSubgroups2) ? 3 : C;
};

// ------------------------------------------------------------------------------- observation weights
// scipy binom.pmf(k, n, p), pmcmc.py:179, evaluated as the log of its closed form
//   L = (log n! - log k! - log (n-k)!) + (k log p + (n-k) log1p(-p))
// carried as an unevaluated sum hi + lo: the log-factorials (lf: hi, lo pairs) and log p / log1p(-p) come from
// binary128 on the host (logfact.cpp), the roundings of the hi parts are recovered exactly (two_sum, fma) and the
// tiny lo terms summed in plain double.  |L - (hi + lo)| stays below ~1e-25 |L|-scale, so the weight
// exp(hi) (1 + lo) is the true pmf to within exp's own rounding and one multiply-add -- scipy's Boost evaluation
// is itself only good to ~1e-12 relative at these n, the restatement is not the limiting error.
// Same operations as oracle/epipf_oracle.c:binom_logpmf.
struct LogW {
    double hi, lo;   // hi = -inf: pmf 0; NaN: bad p (scipy returns nan)
};

__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}

// Dekker's fast two-sum: s + e = a + b exactly when |a| >= |b|
__device__ __forceinline__ void fast_two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    e = b - (s - a);
}

// The log-factorial table: lf[n] = hi and lf[lf_max + 1 + n] = lo of log n!, n = 0..lf_max (binary128 split on the
// host, logfact.cpp).  Hi and lo apart: the ranking pass reads only the hi parts (the table footprint in L1/L2 of
// the old plain weight); the minimum's three entries are read again, hi and lo, once it is known (L1 hits).
struct LfIdx { int n, k, m; };

__device__ __forceinline__ LfIdx lf_index(double k, double n, int lf_max) {
    const int ni = min(max((int)n, 0), lf_max), ki = min(max((int)k, 0), lf_max);
    return LfIdx{ni, ki, min(max(ni - ki, 0), lf_max)};
}

// Plain-double log pmf from the hi parts: the candidate ranking of particle_weight (-inf / NaN as LogW.hi).
__device__ __forceinline__ double binom_logpmf_plain(double k, double n, const ChainParam& cp, const double* lf,
                                                     int lf_max) {
    const double p = cp.probs;
    if (!(p >= 0.0 && p <= 1.0)) return __builtin_nan("");
    if (k < 0.0 || k > n || k != floor(k)) return -__builtin_inf();
    if (p == 0.0) return (k == 0.0) ? 0.0 : -__builtin_inf();
    if (p == 1.0) return (k == n) ? 0.0 : -__builtin_inf();
    const LfIdx ix = lf_index(k, n, lf_max);
    return ((lf[ix.n] - lf[ix.k]) - lf[ix.m]) + (k * cp.logp + (n - k) * cp.log1mp);
}

// The compensated log pmf of a regular case (0 < p < 1, k integral in [0, n]): the plain value's two factorial
// differences as exact fast two-sums (log n! >= log k!, and log(n!/k!) >= log (n-k)!: n!/k! is a product of n-k
// factors each >= its counterpart in (n-k)!), the table's lo parts, the products' exact errors (fma), an exact
// two-sum of the products and one of the total, the lo terms summed in double.
__device__ __forceinline__ LogW binom_logpmf_core(double k, double n, const double* lf, int lf_max, double logp,
                                                  double log1mp, double logp_lo, double log1mp_lo) {
    const LfIdx ix = lf_index(k, n, lf_max);
    const double* lo_tab = lf + lf_max + 1;
    double s1, e1, s2, e2;
    fast_two_sum(lf[ix.n], -lf[ix.k], s1, e1);
    fast_two_sum(s1, -lf[ix.m], s2, e2);
    const double lt = ((lo_tab[ix.n] - lo_tab[ix.k]) - lo_tab[ix.m]) + (e1 + e2);
    const double m = n - k;
    double s3, e3, s4, e4;
    const double p1 = k * logp, f1 = fma(k, logp, -p1);               // exact products: p + f = k * logp
    const double p2 = m * log1mp, f2 = fma(m, log1mp, -p2);
    two_sum(p1, p2, s3, e3);
    two_sum(s2, s3, s4, e4);
    double lo = lt + (e3 + e4);
    lo = lo + (f1 + f2);
    lo = lo + (k * logp_lo + m * log1mp_lo);
    return LogW{s4, lo};
}

// the compensated log pmf with scipy's special cases (lo = 0 there)
__device__ __forceinline__ LogW binom_logpmf(double k, double n, const ChainParam& cp, const double* lf, int lf_max) {
    const double h = binom_logpmf_plain(k, n, cp, lf, lf_max);
    const double p = cp.probs;
    if (!(h > -__builtin_inf()) || p == 0.0 || p == 1.0) return LogW{h, 0.0};   // NaN, pmf 0, or pmf 0 / 1 cases
    return binom_logpmf_core(k, n, lf, lf_max, cp.logp, cp.log1mp, cp.logp_lo, cp.log1mp_lo);
}

// a < b for compensated logs of nearby size (hi - hi is exact within a factor 2, Sterbenz); -inf and NaN by hi
__device__ __forceinline__ bool logw_less(const LogW& a, const LogW& b) {
    if (a.hi != b.hi) {
        const double d = a.hi - b.hi;
        if (!(fabs(d) < 1.0)) return a.hi < b.hi;          // far apart (or infinite): the hi parts decide
        return d + (a.lo - b.lo) < 0.0;
    }
    return a.lo < b.lo;
}

// scipy norm.pdf(y, loc=x, scale=probs*x+1e-4), pmcmc.py:181
__device__ __forceinline__ double normal_pdf(double y, double x, double probs) {
    const double scale = probs * x + 0.0001;
    if (!(scale > 0.0)) return __builtin_nan("");
    const double z = (y - x) / scale;
    return (exp(-(z * z) / 2.0) / 2.5066282746310002) / scale;
}

template <int MODEL, int G>
__device__ __forceinline__ double observed(const double* x, int i) {
    if constexpr (MODEL == kSubgroups2) {
        double xo = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) xo = xo + x[3 * g + i];          // group sum, pmcmc.py:173,229
        return xo;
    } else {
        return x[i];
    }
}

// The binomial weight when two columns' plain logs tie within their error: every column compensated, the smallest
// by the compensated logs.  Out of line (rare, ~1e-6 of particle-steps at config 2): the state comes back from its
// just-written row (`row`, int32 [C]) and the chain's parameters from global memory, so the call passes no arrays
// and the step kernel keeps its registers for the event loop.
template <int MODEL, int G>
__device__ __attribute__((noinline)) double binom_weight_tied(const int32_t* row, const double* yrow,
                                                              const ChainParam* cpp, const double* lf, int lf_max) {
    // a rolled loop reading the state from memory: this function's registers count towards the calling kernel's
    // allocation (an unrolled 6- or 12-column version cost the subgroup step kernels two waves per SIMD)
    constexpr int K = Shape<MODEL, G>::K;
    const ChainParam& cp = *cpp;
    LogW L{0.0, 0.0};
#pragma unroll 1
    for (int i = 0; i < K; ++i) {
        double xo;
        if constexpr (MODEL == kSubgroups2) {
            xo = 0.0;
            for (int g = 0; g < G; ++g) xo = xo + (double)row[3 * g + i];     // group sum, pmcmc.py:173,229
        } else {
            xo = (double)row[i];
        }
        const LogW li = binom_logpmf(yrow[i], xo, cp, lf, lf_max);
        if (i == 0 || logw_less(li, L)) L = li;
    }
    const double e = exp(L.hi);
    return fma(e, L.lo, e);
}

// min over the K observed columns (np.min propagates NaN), pmcmc.py:178-181.  Binomial: exp is monotone, so the
// minimum is taken on the logs and exponentiated once.  The columns are ranked on their plain-double logs (one
// round of table loads, which also yields the table parts of the compensated value); only the smallest is then
// compensated -- unless another column lies within the plain logs' error of it (a near tie: binom_weight_tied,
// every column compensated).  The plain log's error is a few ulps of the sum of its terms' magnitudes, which the
// host bounds per chain (cp.tie_tol, 8x that bound), so outside a near tie the ranking is exact.
// cp: the chain's parameters as the kernel holds them (probs, log p, log1p(-p)); the lo parts and tie_tol are read
// from cpp here, behind a compiler barrier (their loads overlap the table loads): carried from the kernel's start,
// live across the event loop, they cost the step kernels ~40 SGPR spills.  row: this particle's state as stored in
// the history (int32 [C]), read only on the tie path.
template <int MODEL, int G, int OBS>
__device__ __forceinline__ double particle_weight(const double* x, const double* yrow, const ChainParam& cp,
                                                  const ChainParam* cpp, const double* lf, int lf_max,
                                                  const int32_t* row) {
    constexpr int K = Shape<MODEL, G>::K;
    if constexpr (OBS == kNormal) {
        double w = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const double wi = normal_pdf(yrow[i], observed<MODEL, G>(x, i), cp.probs);
            if (i == 0 || isnan(wi)) w = wi;
            else if (!isnan(w) && wi < w) w = wi;
        }
        return w;
    } else {
        asm volatile("" ::: "memory");
        const double logp_lo = cpp->logp_lo, log1mp_lo = cpp->log1mp_lo, tie_tol = cpp->tie_tol;
        // the running minimum m with its operands, and the runner-up m2 (a near tie: m2 - m <= tie_tol); NaN sticks.
        // Only these four doubles live across the columns: keeping each column's table parts for a later select
        // raised the subgroup kernels' registers by a third (75 -> 111 VGPRs at G = 2, two waves per SIMD fewer).
        double m = 0.0, m2 = __builtin_inf(), ys = 0.0, xs = 0.0;
        bool nan = false;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const double xo = observed<MODEL, G>(x, i);
            const double h = binom_logpmf_plain(yrow[i], xo, cp, lf, lf_max);
            nan = nan || isnan(h);
            const bool take = (i == 0) || h < m;
            m2 = (i == 0) ? m2 : (take ? m : fmin(m2, h));
            m = take ? h : m;
            ys = take ? yrow[i] : ys;
            xs = take ? xo : xs;
        }
        if (nan) return __builtin_nan("");                             // np.min propagates NaN
        if (!(m > -__builtin_inf())) return 0.0;                       // a column outside its support: pmf 0
        if (cp.probs == 0.0 || cp.probs == 1.0) return 1.0;            // m finite: every column's pmf is 1
        const int below = (m2 - m <= tie_tol) ? 2 : 1;                 // another column within tie_tol of m
        if (below > 1) return binom_weight_tied<MODEL, G>(row, yrow, cpp, lf, lf_max);
        const LogW L = binom_logpmf_core(ys, xs, lf, lf_max, cp.logp, cp.log1mp, logp_lo, log1mp_lo);
        const double e = exp(L.hi);
        return fma(e, L.lo, e);                                        // exp(hi + lo) = exp(hi) (1 + lo)
    }
}

// ------------------------------------------------------------------------------- block scan (doubles)
// Inclusive scan of one value per thread across a WG-thread block.  The last thread's result is the
// block total.  lds must hold WG/64 doubles.  Order of additions is fixed (deterministic).
template <int WG>
__device__ __forceinline__ double block_inclusive_scan(double x, double* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(x, o, 64);
        if (lane >= o) x = x + y;
    }
    if constexpr (WG > 64) {
        if (lane == 63) lds[wave] = x;
        __syncthreads();
        double off = 0.0;
        for (int q = 0; q < wave; ++q) off = off + lds[q];
        x = off + x;
        __syncthreads();
    }
    return x;
}

// ------------------------------------------------------------------------------- resampling
// numpy legacy choice(range(N), N, p=w/sum(w)) for uniform U (pmcmc.py:185-190) is
//   S = sum(w) (Python builtin: sequential), q = w/S, c = cumsum(q) (sequential), cdf = c / c[N-1],
//   a = searchsorted(cdf, U, 'right') = first i with cdf_i > U.
// The device searches a parallel CDF v_i = (block prefix + in-block prefix) / total instead and certifies
// the answer against the reference's: with r_i = W_i / W the exact ratio of prefix sums,
//   |cdf_i / r_i - 1| <= (i + N + 2) u      (sequential sum, quotients, cumsum, final division)
//   |v_i / r_i - 1|   <= (2D + 1) u         (D = depth of the parallel reduction tree)
// so |cdf_i - v_i| <= delta_i = (i + K) u v_i (1 + 2^-20), K = N + 2D + 8, u = 2^-53.
// v_{a-1} + delta_{a-1} < U < v_a - delta_a proves cdf_{a-1} <= U < cdf_a, i.e. a is numpy's answer.
// Draws that fail the test are resolved exactly by resample_exact_wave.
__device__ __forceinline__ double cert_halfwidth(int i, double v, double cert_k) {
    return ((double)i + cert_k) * 0x1.00001p-53 * v;
}

// The reference's own CDF is numpy's over scipy's weights, which differ from the device's by at most E relative
// each (E: scipy's error envelope plus the device's).  Then |cdf_ref_i - cdf_i| <= 2E v (1 - v)
// (1 + tiny), and ref_k = 2E (1 + 2^-10).  A draw whose U lies within delta_i + that of a boundary of its answer
// may differ from the reference's: counted (resample_ref_ambiguous), never changed.  Every uncertified draw (U
// within delta of a boundary) is counted too, without a finer test against the exact CDF: carrying that test
// into resample_exact_wave cost the step kernels 16 SGPR spills (a v_readlane per use on every step).
__device__ __forceinline__ double ref_halfwidth(double v, double ref_k) {
    return ref_k * (v * (1.0 - v));
}

// Two-level search of v (bpex: exclusive prefix of the block sums and bsum: block sums, both in LDS;
// wloc: in-block inclusive prefix, in HBM/L2).  Returns the candidate index; `certified` says whether the
// bracket test above proved it.
// The search itself compares prefixes against U * total (one multiply instead of an IEEE division per level);
// only the final bracket is evaluated on v = prefix / total.  Where the two orders disagree (a prefix within an
// ulp of U * total) the candidate is off by one, its bracket test fails and the exact fallback decides, so the
// result is still numpy's.
// In-block level: the first m in [0, WG - 1) with base + L[m] > Ut, else WG - 1 (L: the block's in-block inclusive
// prefix, non-decreasing, so base + L[m] is too).  Binary search: log2(WG) dependent loads.  FLAT (WG = 64, the
// latency-bound lane-group kernel): the same index from two rounds of 7 independent loads -- the sub-block maxima
// L[8i + 7], i < 7, give the sub-block s (the count of those <= Ut), then L[8s + j], j < 7, the offset (the count of
// those <= Ut); counting a monotone predicate is the binary search's answer.
template <int WG, bool FLAT = false>
__device__ __forceinline__ int inblock_search(double base, const double* __restrict__ L, double Ut) {
    if constexpr (FLAT && WG == 16) {                   // 16-particle blocks: one round of 15 independent loads
        double c[15];
#pragma unroll
        for (int i = 0; i < 15; ++i) c[i] = L[i];
        int o = 0;
#pragma unroll
        for (int i = 0; i < 15; ++i) o += (base + c[i] > Ut) ? 0 : 1;
        return o;
    } else if constexpr (FLAT) {
        static_assert(WG == 64, "8 x 8 sub-blocks");
        double c[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) c[i] = L[8 * i + 7];
        int s = 0;
#pragma unroll
        for (int i = 0; i < 7; ++i) s += (base + c[i] > Ut) ? 0 : 1;
        const double* Ls = L + 8 * s;
        double f[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) f[j] = Ls[j];
        int o = 0;
#pragma unroll
        for (int j = 0; j < 7; ++j) o += (base + f[j] > Ut) ? 0 : 1;
        return 8 * s + o;
    } else {
        int l = 0, h = WG - 1;
        while (l < h) {
            const int m = (l + h) >> 1;
            if (base + L[m] > Ut) h = m; else l = m + 1;
        }
        return l;
    }
}

template <int WG, bool FLAT = false>
__device__ __forceinline__ int resample_search(double U, const double* bpex, const double* bsum, int B,
                                               double total, const double* wloc, int N, double cert_k,
                                               bool& certified, double ref_k, bool& ambiguous) {
    const double Ut = U * total;
    int lo = 0, hi = B - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (bpex[mid] + bsum[mid] > Ut) hi = mid; else lo = mid + 1;
    }
    const int b = lo;
    const double base = bpex[b];
    const double* L = wloc + (size_t)b * WG;
    const int l = inblock_search<WG, FLAT>(base, L, Ut);
    const int a = b * WG + l;
    const double va = (base + L[l]) / total;
    const double vp = (l > 0) ? (base + L[l - 1]) / total
                              : (b > 0 ? (bpex[b - 1] + bsum[b - 1]) / total : -1.0);
    certified = (va - cert_halfwidth(a, va, cert_k) > U) &&
                (a == 0 || vp + cert_halfwidth(a - 1, vp, cert_k) < U) && a < N;
    if (ref_k > 0.0)                          // counting on (ref_k = 0 otherwise: the test costs ~10 VALU per draw)
        ambiguous = !((va - (cert_halfwidth(a, va, cert_k) + ref_halfwidth(va, ref_k)) > U) &&
                      (a == 0 || vp + (cert_halfwidth(a - 1, vp, cert_k) + ref_halfwidth(vp, ref_k)) < U));
    return a;
}

// The same search over a segmented block-sum prefix (scan_segments in epipf_kernels.hip): level 1 over the LDS
// segment ends seg_end[k] (S blocks per segment), level 2 walks the <= S block sums of the segment from global
// memory with the scan's own additions (so every value equals the scan's), level 3 the block's in-block prefix.
// With S = 1 this is resample_search above, value for value (seg_start = bpex, seg_end = bpex + bsum).
template <bool FLAT = false>
__device__ __forceinline__ int resample_search_seg(double U, const double* seg_start, const double* seg_end, int nseg,
                                                   int S, const double* __restrict__ bsum_g, int B, double total,
                                                   const double* __restrict__ wloc, int WGB, int N, double cert_k,
                                                   bool& certified, double ref_k, bool& ambiguous) {
    const double Ut = U * total;                                        // search on U * total (resample_search)
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (seg_end[mid] > Ut) hi = mid; else lo = mid + 1;
    }
    const int k = lo;
    int b = k * S;
    double base = seg_start[k];                                         // prefix before block b
    if (S > 1) {
        const int ie = min(b + S, B);
        double e = base;
        for (int i = b; i < ie; ++i) {
            const double en = e + bsum_g[i];
            if (en > Ut || i == ie - 1) { b = i; base = e; break; }
            e = en;
        }
    }
    const double* L = wloc + (size_t)b * WGB;
    int l;
    if (FLAT && WGB == 64) {
        l = inblock_search<64, true>(base, L, Ut);
    } else if (FLAT && WGB == 16) {
        l = inblock_search<16, true>(base, L, Ut);
    } else {
        l = 0;
        int h = WGB - 1;
        while (l < h) {
            const int m = (l + h) >> 1;
            if (base + L[m] > Ut) h = m; else l = m + 1;
        }
    }
    const int a = b * WGB + l;
    const double va = (base + L[l]) / total;
    // inclusive prefix through block b-1: the segment's running sum, or the previous segment's end
    const double pb = (b == k * S) ? (k > 0 ? seg_end[k - 1] : 0.0) : base;
    const double vp = (l > 0) ? (base + L[l - 1]) / total : (b > 0 ? pb / total : -1.0);
    certified = (va - cert_halfwidth(a, va, cert_k) > U) &&
                (a == 0 || vp + cert_halfwidth(a - 1, vp, cert_k) < U) && a < N;
    if (ref_k > 0.0)                          // counting on (ref_k = 0 otherwise: the test costs ~10 VALU per draw)
        ambiguous = !((va - (cert_halfwidth(a, va, cert_k) + ref_halfwidth(va, ref_k)) > U) &&
                      (a == 0 || vp + (cert_halfwidth(a - 1, vp, cert_k) + ref_halfwidth(vp, ref_k)) < U));
    return a;
}

// The exact reference draw for every lane of the wave with need == true, all 64 lanes cooperating (call
// from wave-uniform control flow; every lane must be active).  The weights stream through the wave in
// coalesced chunks of 64, kExactDepth chunks in flight (a single chunk ahead leaves each pass bound by one
// L2/HBM round trip per chunk); the sequential sums run on values broadcast with v_readlane, in the
// reference's order:
//   pass 1  S = (((w_0 + w_1) + w_2) + ...)
//   pass 2  last = c_{N-1},  c_i = c_{i-1} + w_i / S
//   pass 3  the needing lanes are served in increasing U: for the current target U*, the first i with
//           fl(c_i / last) > U* (a certified product c_i * (1/last) decides, the IEEE division only within a
//           few ulps of U*); the next target continues from the same i, since cdf is non-decreasing.  Every
//           test in the loop is wave-uniform, and the pass stops at the last target.
// Cost ~3 N dependent f64 adds for the wave.
constexpr int kExactDepth = 4;

struct ExactTarget {          // wave-uniform: smallest U among the lanes still waiting, or done
    double U, lo, hi;
    bool done;
};

__device__ __forceinline__ ExactTarget exact_next_target(bool waiting, double U) {
    double m = waiting ? U : __builtin_inf();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmin(m, __shfl_xor(m, o, 64));
    ExactTarget t;
    t.U = m;
    t.lo = m * (1.0 - 0x1.0p-49);     // |c * (1/last) - c / last| <= 2 ulp of c / last
    t.hi = m * (1.0 + 0x1.0p-49);
    t.done = !(m < __builtin_inf());
    return t;
}

// rotating 4-deep prefetch of 64-element chunks (no indexed arrays, so nothing spills)
struct ChunkStream {
    const double* w;
    int N, lane;
    double x0, x1, x2, x3;
    __device__ __forceinline__ double ld(int i) const { return (i < N) ? w[i] : 0.0; }
    __device__ __forceinline__ void start(const double* w_, int N_) {
        w = w_; N = N_; lane = threadIdx.x & 63;
        x0 = ld(lane); x1 = ld(64 + lane); x2 = ld(128 + lane); x3 = ld(192 + lane);
    }
    __device__ __forceinline__ double next(int cb) {   // chunk at cb; issues the load of chunk cb + 256
        const double x = x0;
        x0 = x1; x1 = x2; x2 = x3;
        x3 = ld(cb + 64 * kExactDepth + lane);
        return x;
    }
};

__device__ __forceinline__ int resample_exact_wave(bool need, double U, const double* __restrict__ w, int N) {
    ChunkStream cs;
    // pass 1: S
    double S = 0.0;
    cs.start(w, N);
#pragma unroll 1
    for (int cb = 0; cb < N; cb += 64) {
        const double x = cs.next(cb);
        if (cb + 64 <= N) {
#pragma unroll 16
            for (int l = 0; l < 64; ++l) S = S + readlane_f64(x, l);
        } else {
            for (int l = 0; l < N - cb; ++l) S = S + readlane_f64(x, l);
        }
    }
    // pass 2: last = c_{N-1}
    double c = 0.0;
    cs.start(w, N);
#pragma unroll 1
    for (int cb = 0; cb < N; cb += 64) {
        const double q = cs.next(cb) / S;
        if (cb + 64 <= N) {
#pragma unroll 16
            for (int l = 0; l < 64; ++l) c = c + readlane_f64(q, l);
        } else {
            for (int l = 0; l < N - cb; ++l) c = c + readlane_f64(q, l);
        }
    }
    const double last = c;
    const double rl = 1.0 / last;

    // pass 3: serve the needing lanes in increasing U
    int ans = N - 1;
    bool waiting = need;
    ExactTarget tg = exact_next_target(waiting, U);
    c = 0.0;
    cs.start(w, N);
#pragma unroll 1
    for (int cb = 0; cb < N && !tg.done; cb += 64) {
        const double q = cs.next(cb) / S;
        const int n = min(64, N - cb);
        for (int l = 0; l < n; ++l) {
            c = c + readlane_f64(q, l);
            const double r = c * rl;
            while (!tg.done && r > tg.lo && (r > tg.hi || c / last > tg.U)) {   // cdf_i > U*: lanes at U* done
                if (waiting && U == tg.U) { ans = cb + l; waiting = false; }
                tg = exact_next_target(waiting, U);
            }
            if (tg.done) break;
        }
    }
    return ans;
}

}  // namespace epipf
