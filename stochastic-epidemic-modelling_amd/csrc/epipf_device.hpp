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

// ------------------------------------------------------------------------------- per-chain parameters
struct ChainParam {
    double theta[kMaxTheta];   // SIR: beta,gamma  SEIR: beta,alpha,gamma  groups: beta[G][G], gamma
    double probs;              // binomial p, or normal noise ratio
    double logp, log1mp;       // log(p), log1p(-p)  (host glibc, identical to the oracle's)
    uint32_t k0, k1;           // Philox key
    uint32_t f;                // filter index
    uint32_t flags;            // kChainFastSsa: the certified f32 event loop may run (EPIPF_SSA_FAST=0 clears it)
    float thetaf[kMaxTheta];   // theta rounded to f32 on the host (scalar loads: the fast path's rates stay in SGPRs)
    float clock_slack;         // >= 1: widens the f32 loop's clock band (more replays, same results); tests only
};
constexpr uint32_t kChainFastSsa = 1u;   // (all models)

// ------------------------------------------------------------------------------- f64 log, table driven
// log(x) for normal x > 0, within 1 ulp of glibc's correctly rounded log (exact near x = 1).  x = 2^k z with
// z in [0.6875, 1.375) (glibc's OFF reduction); z is centred on one of 128 table points c_i
// (LogTab: {1/c_i, log c_i}), r = z/c_i - 1 (|r| < 2^-8) and log1p(r) is a degree-7 polynomial.  Inputs within
// 2^-8 of 1 bypass the table (r = x - 1 exactly).  ~20 instructions against ~45 for the library log.
struct LogTab { double invc, logc; };
constexpr int kLogTabEntries = 128;
constexpr uint64_t kLogOff = 0x3FE6000000000000ull;   // 0.6875

// one entry per thread (i < 128); the bin holding 1.0 gets exactly {1, 0}
__device__ __forceinline__ void log_table_entry(LogTab* tab, int i) {
    if (i < kLogTabEntries) {
        const double c = __longlong_as_double((long long)(kLogOff + ((uint64_t)(2 * i + 1) << 44)));
        const double ic = 1.0 / c;
        const bool one = i == (int)(((0x3FF0000000000000ull - kLogOff) >> 45) & 127);
        tab[i].invc = one ? 1.0 : ic;
        tab[i].logc = one ? 0.0 : -log(ic);
    }
}

// Index, exponent and reduced argument are formed on the high 32-bit word (kLogOff's low word is zero, so
// ix - kLogOff never borrows); inputs within 2^-8 of 1 select the exact {1, 0} bin with k = 0, z = x, so
// r = x - 1 exactly -- no branch.
// P(r) = 1/7 r^5 - 1/6 r^4 + 1/5 r^3 - 1/4 r^2 + 1/3 r - 1/2 by Horner, as five dependent three-operand
// v_fma_f64 with the constants in SGPR pairs, in one asm block: hipcc otherwise copies each constant into
// the destination of a two-address v_fmac_f64 (one 64-bit move per step), and separate asm statements get
// an s_nop between them.  VALU-to-VALU dependencies need no wait states.
__device__ __forceinline__ double log1p_horner(double r) {
    double p;
    asm("v_fma_f64 %0, %1, %2, %3\n\t"
        "v_fma_f64 %0, %1, %0, %4\n\t"
        "v_fma_f64 %0, %1, %0, %5\n\t"
        "v_fma_f64 %0, %1, %0, %6\n\t"
        "v_fma_f64 %0, %1, %0, %7"
        : "=&v"(p)
        : "v"(r), "v"(1.0 / 7.0), "s"(-1.0 / 6.0), "s"(1.0 / 5.0), "s"(-0.25), "s"(1.0 / 3.0), "s"(-0.5));
    return p;
}

constexpr int kLogOneBin = (int)(((0x3FF00000u - 0x3FE60000u) >> 13) & 127);   // bin holding 1.0

__device__ __forceinline__ double fast_log_sel(double x, bool near1, const LogTab* __restrict__ tab) {
    const long long ix = __double_as_longlong(x);
    const uint32_t hi = (uint32_t)(ix >> 32);
    const int lo = (int)ix;
    const uint32_t th = hi - (uint32_t)(kLogOff >> 32);
    const int i = near1 ? kLogOneBin : (int)((th >> 13) & 127);
    const int k = near1 ? 0 : ((int)th >> 20);
    const uint32_t zh = near1 ? hi : hi - (th & 0xFFF00000u);
    const double z = __hiloint2double((int)zh, lo);
    const LogTab e = tab[i];
    const double r = fma(z, e.invc, -1.0);
    const double kd = (double)k;
    const double w = fma(kd, 0x1.62e42fefa3800p-1, e.logc);       // k*ln2_hi + log c (exact product)
    const double hs = w + r;
    double ls = (w - hs) + r;
    ls = fma(kd, 0x1.ef35793c76730p-45, ls);                      // k*ln2_lo
    const double p = log1p_horner(r);
    return hs + fma(r * r, p, ls);                                // log1p(r) = r + r^2 P(r)
}

__device__ __forceinline__ double fast_log(double x, const LogTab* __restrict__ tab) {
    return fast_log_sel(x, fabs(x - 1.0) < 0x1.0p-8, tab);
}

// -log(1 - U), U = u01(lo, hi): the reference's np.random.exponential(1) (gillespie_algo.py:62).
// |(1 - U) - 1| = U < 2^-8  <=>  m < 2^45  <=>  hi >> 11 < 2^13, so the near-1 test is one integer compare.
__device__ __forceinline__ double neg_log_one_minus_u01(uint32_t lo, uint32_t hi, const LogTab* __restrict__ tab) {
    return -fast_log_sel(one_minus_u01(lo, hi), (hi >> 11) < 8192u, tab);
}

// 1/a to ~1 ulp: hardware reciprocal + two Newton steps
__device__ __forceinline__ double recip(double a) {
    double r = __builtin_amdgcn_rcp(a);
    r = fma(fma(-a, r, 1.0), r, r);
    return fma(fma(-a, r, 1.0), r, r);
}

// ------------------------------------------------------------------------------- Gillespie SSA
// Direct method over [0, tmax] from state x (integers held in doubles, as the reference holds them),
// gillespie_algo.py.  Event k of this lane draws Philox block (k, j, ptag, f): tau from (x,y), the
// channel from (z,w).  Both uniforms are consumed before the overshoot test, as in the reference.
// Every lane still in the loop is at the same event index k (all start at 0 and step together), so k is
// read wave-uniform: Philox's first round (and half of its second) then runs on the scalar unit.
//
// Fast path + certified fallback: the channel decision of the reference is
//   count_i [ fl(c_i / c_last) <= u ],  c = cumsum(fl(a_l / sum(a)))            (numpy choice, :63)
// whose ratios agree with q_i = (a_0 + ... + a_i) * (1/sum a) to a few ulps.  When every q_i is farther than
// kBand from u the decision is the reference's; otherwise the reference expression is evaluated exactly
// (IEEE divisions in the reference's order).  The event time uses 1/sum(a) and log to ~1 ulp, so the
// clock t can differ from the reference's by ulps; a step-boundary decision can then differ only when
// t + tau lands within a few ulps of the step end (p ~ 1e-13 per particle-step).
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
// Propensities are formed as (beta/N) * (S*I) and with fused sums: within a few ulps of the reference's
// ((beta*S)*I)/N and a0 + gamma*I, which the 2^-44 channel band and the ulp-level tau tolerance absorb
// (DESIGN.md §4).
template <int MODEL, int G>
struct SsaState;

template <>
struct SsaState<kSIR, 1> {                                             // gillespie_algo.py:10-75
    double S, I, R, N, bN;
    int nrec;
    __device__ __forceinline__ void load(const double* x, const ChainParam& cp) {
        S = x[0]; I = x[1]; R = x[2];
        N = (S + I) + R;                                               // :35
        bN = cp.theta[0] / N;
        nrec = 0;
    }
    __device__ __forceinline__ bool active() const { return I > 0.0; }   // :48
    __device__ __forceinline__ bool event(const Block& r, double& t, double tmax, const ChainParam& cp,
                                          const LogTab* __restrict__ tab) {
        const double gamma = cp.theta[1];
        const double a0 = bN * (S * I);                                // :38
        const double as = fma(gamma, I, a0);                           // :39
        const double ri = recip(as);
        const double tau = ri * neg_log_one_minus_u01(r.x, r.y, tab);  // np.random.exponential, :62
        const double u = u01(r.z, r.w);
        const double q = a0 * ri;
        bool second = q <= u;                                          // choice(2, p=a/sum(a)), :63
        if (fabs(q - u) <= kBand) second = sir_channel_exact(cp.theta[0], gamma, S, I, N, u);
        const double tn = t + tau;
        if (tn > tmax) return false;                                   // :65-66
        t = tn;                                                        // :68-70; R is not needed in the loop
        S = S + (second ? 0.0 : -1.0);
        I = I + (second ? -1.0 : 1.0);
        nrec += second ? 1 : 0;
        return true;
    }
    __device__ __forceinline__ void save(double* x) const { x[0] = S; x[1] = I; x[2] = R + (double)nrec; }
    // event()'s tau, same expressions (the wave-cooperative replay evaluates events' times in parallel)
    __device__ __forceinline__ double tau_of(const Block& r, const ChainParam& cp, const LogTab* __restrict__ tab) const {
        const double a0 = bN * (S * I);
        const double as = fma(cp.theta[1], I, a0);
        return recip(as) * neg_log_one_minus_u01(r.x, r.y, tab);
    }
};

template <>
struct SsaState<kSEIR, 1> {                                            // gillespie_algo.py:78-146
    double S, E, I, R, N, bN;
    __device__ __forceinline__ void load(const double* x, const ChainParam& cp) {
        S = x[0]; E = x[1]; I = x[2]; R = x[3];
        N = ((S + E) + I) + R;                                         // :104
        bN = cp.theta[0] / N;                                          // theta = (beta, alpha, gamma), :92
    }
    __device__ __forceinline__ bool active() const { return E > 0.0 || I > 0.0; }   // :119
    __device__ __forceinline__ bool event(const Block& r, double& t, double tmax, const ChainParam& cp,
                                          const LogTab* __restrict__ tab) {
        const double alpha = cp.theta[1], gamma = cp.theta[2];
        const double a0 = bN * (S * I), a01 = fma(alpha, E, a0);       // :107-109
        const double as = fma(gamma, I, a01);
        const double ri = recip(as);
        const double tau = ri * neg_log_one_minus_u01(r.x, r.y, tab);  // :133
        const double u = u01(r.z, r.w);
        const double q0 = a0 * ri, q1 = a01 * ri;
        int ch = (q0 <= u ? 1 : 0) + (q1 <= u ? 1 : 0);                // :134
        if (fabs(q0 - u) <= kBand || fabs(q1 - u) <= kBand)
            ch = seir_channel_exact(cp.theta[0], alpha, gamma, S, E, I, N, u);
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
        const double a0 = bN * (S * I), a01 = fma(cp.theta[1], E, a0);
        const double as = fma(cp.theta[2], I, a01);
        return recip(as) * neg_log_one_minus_u01(r.x, r.y, tab);
    }
};

template <int G>
struct SubgroupsState {                                                // gillespie_algo.py:148-233
    static constexpr int NCH = G * G + G;
    double S[G], I[G], R[G], sumN, invSumN;
    __device__ __forceinline__ void load(const double* x, const ChainParam&) {
        sumN = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            S[g] = x[3 * g]; I[g] = x[3 * g + 1]; R[g] = x[3 * g + 2];
            sumN = sumN + ((S[g] + I[g]) + R[g]);                      // sum(N), :176,:182
        }
        invSumN = 1.0 / sumN;
    }
    __device__ __forceinline__ bool active() const {                   // :192-193, :222
        double infected = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) infected = infected + I[g];
        return infected > 0.0;
    }
    __device__ __forceinline__ bool event(const Block& r, double& t, double tmax, const ChainParam& cp,
                                          const LogTab* __restrict__ tab) {
        const double gamma = cp.theta[G * G];
        double cum[NCH];
        double run = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) {                                  // channel order, :180-185
            const double cI = I[g] * invSumN;
#pragma unroll
            for (int g2 = 0; g2 < G; ++g2) {
                run = fma(cp.theta[g * G + g2] * S[g2], cI, run);
                cum[g * (G + 1) + g2] = run;
            }
            run = fma(gamma, I[g], run);
            cum[g * (G + 1) + G] = run;
        }
        const double ri = recip(run);
        const double tau = ri * neg_log_one_minus_u01(r.x, r.y, tab);
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
        const double gamma = cp.theta[G * G];
        double run = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const double cI = I[g] * invSumN;
#pragma unroll
            for (int g2 = 0; g2 < G; ++g2) run = fma(cp.theta[g * G + g2] * S[g2], cI, run);
            run = fma(gamma, I[g], run);
        }
        return recip(run) * neg_log_one_minus_u01(r.x, r.y, tab);
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
    // turns the channel-by-channel form into a divergent switch).
    __device__ __forceinline__ void apply(int ch, float s) {
        const int g = ch / (G + 1), c = ch - g * (G + 1);
        const bool inf = c < G;
        const int q = inf ? c : g;
        const float dS = inf ? s : 0.f, dI = inf ? s : -s;
#pragma unroll
        for (int r = 0; r < G; ++r) {
            const bool hit = q == r;
            S[r] -= hit ? dS : 0.f;
            I[r] += hit ? dI : 0.f;
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
template <int G> struct FastSsa<kSubgroups, G> : FastSubgroups<G> {};
template <int G> struct FastSsa<kSubgroups2, G> : FastSubgroups<G> {};

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
    double rem = tmax * kInvLn2;                                       // remaining time, units of 1/ln 2
    const float Bt = (float)rem * F::kClockT * cp.clock_slack;
    float R = 0.f, df = 0.f, B = 0.f;
    uint32_t ks = 0;                                                   // event index, wave-uniform (SGPR)
    bool alive = st.active(), ok = true;
    int ch = 0;
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
        bool close = false;
        ch = 0;
        if constexpr (NCH <= 3) {                                      // ratios q_i = c_i / total
#pragma unroll
            for (int i = 0; i < NCH - 1; ++i) {                        // numpy choice, searchsorted right
                const float q = c[i] * ri;
                ch += (q < uc) ? 1 : 0;
                close |= fabsf(q - uc) <= F::kBand;
            }
        } else {                                                       // c_i against uc * total: one multiply
            const float T = uc * total, band = F::kBand * total;       // per draw instead of one per channel
#pragma unroll
            for (int i = 0; i < NCH - 1; ++i) {
                ch += (c[i] < T) ? 1 : 0;
                close |= fabsf(c[i] - T) <= band;
            }
        }
        if (close) ch = st.exact_channel(cp, u01(r.z, r.w));
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
        st.apply(ch, 1.f);                                             // undone below if the lane overshoots
        alive = ok && st.active();
    }
    if (!ok) {
        if (!(df < -B)) return false;                                 // boundary too close to call: exact loop
        st.apply(ch, -1.f);                                            // the overshooting event is not applied
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
            close |= fabsf(q - uc) <= F::kBand;
        }
    } else {
        const float T = uc * total, band = F::kBand * total;
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
// it; the state is not kept in registers across the replay).
template <int MODEL, int G>
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
            __syncthreads();                             // every lane has read the parent row
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
    __syncthreads();
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
// scipy binom.pmf(k, n, p) restated with a host-built log-factorial table lf[n] = lgamma(n + 1),
// pmcmc.py:179.  Identical expression order to oracle/epipf_oracle.c:binom_pmf.
__device__ __forceinline__ double binom_pmf(double k, double n, const ChainParam& cp, const double* lf,
                                            int lf_max) {
    const double p = cp.probs;
    if (!(p >= 0.0 && p <= 1.0)) return __builtin_nan("");
    if (k < 0.0 || k > n || k != floor(k)) return 0.0;
    if (p == 0.0) return (k == 0.0) ? 1.0 : 0.0;
    if (p == 1.0) return (k == n) ? 1.0 : 0.0;
    const int ni = min(max((int)n, 0), lf_max), ki = min(max((int)k, 0), lf_max);
    double a = lf[ni] - lf[ki];
    a = a - lf[min(max(ni - ki, 0), lf_max)];
    const double b = k * cp.logp;
    const double c = (n - k) * cp.log1mp;
    return exp(a + (b + c));
}

// scipy norm.pdf(y, loc=x, scale=probs*x+1e-4), pmcmc.py:181
__device__ __forceinline__ double normal_pdf(double y, double x, double probs) {
    const double scale = probs * x + 0.0001;
    if (!(scale > 0.0)) return __builtin_nan("");
    const double z = (y - x) / scale;
    return (exp(-(z * z) / 2.0) / 2.5066282746310002) / scale;
}

// log of binom_pmf with the same expression order: -inf for pmf 0, 0 for pmf 1, NaN for bad p
__device__ __forceinline__ double binom_logpmf(double k, double n, const ChainParam& cp, const double* lf, int lf_max) {
    const double p = cp.probs;
    if (!(p >= 0.0 && p <= 1.0)) return __builtin_nan("");
    if (k < 0.0 || k > n || k != floor(k)) return -__builtin_inf();
    if (p == 0.0) return (k == 0.0) ? 0.0 : -__builtin_inf();
    if (p == 1.0) return (k == n) ? 0.0 : -__builtin_inf();
    const int ni = min(max((int)n, 0), lf_max), ki = min(max((int)k, 0), lf_max);
    double a = lf[ni] - lf[ki];
    a = a - lf[min(max(ni - ki, 0), lf_max)];
    const double b = k * cp.logp;
    const double c = (n - k) * cp.log1mp;
    return a + (b + c);
}

// min over the K observed columns (np.min propagates NaN), pmcmc.py:178-181.  Binomial: exp is monotone, so
// min_i exp(L_i) = exp(min_i L_i) -- one exp per particle instead of K, same value.
template <int MODEL, int G, int OBS>
__device__ __forceinline__ double particle_weight(const double* x, const double* yrow, const ChainParam& cp,
                                                  const double* lf, int lf_max) {
    constexpr int K = Shape<MODEL, G>::K;
    double w = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double xo;
        if constexpr (MODEL == kSubgroups2) {
            xo = 0.0;
#pragma unroll
            for (int g = 0; g < G; ++g) xo = xo + x[3 * g + i];       // group sum, pmcmc.py:173,229
        } else {
            xo = x[i];
        }
        const double wi = (OBS == kBinomial) ? binom_logpmf(yrow[i], xo, cp, lf, lf_max) : normal_pdf(yrow[i], xo, cp.probs);
        if (i == 0 || isnan(wi)) w = wi;
        else if (!isnan(w) && wi < w) w = wi;
    }
    return (OBS == kBinomial) ? exp(w) : w;
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

// Two-level search of v (bpex: exclusive prefix of the block sums and bsum: block sums, both in LDS;
// wloc: in-block inclusive prefix, in HBM/L2).  Returns the candidate index; `certified` says whether the
// bracket test above proved it.
// The search itself compares prefixes against U * total (one multiply instead of an IEEE division per level);
// only the final bracket is evaluated on v = prefix / total.  Where the two orders disagree (a prefix within an
// ulp of U * total) the candidate is off by one, its bracket test fails and the exact fallback decides, so the
// result is still numpy's.
template <int WG>
__device__ __forceinline__ int resample_search(double U, const double* bpex, const double* bsum, int B,
                                               double total, const double* wloc, int N, double cert_k,
                                               bool& certified) {
    const double Ut = U * total;
    int lo = 0, hi = B - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (bpex[mid] + bsum[mid] > Ut) hi = mid; else lo = mid + 1;
    }
    const int b = lo;
    const double base = bpex[b];
    const double* L = wloc + (size_t)b * WG;
    int l = 0, h = WG - 1;
    while (l < h) {
        const int m = (l + h) >> 1;
        if (base + L[m] > Ut) h = m; else l = m + 1;
    }
    const int a = b * WG + l;
    const double va = (base + L[l]) / total;
    const double vp = (l > 0) ? (base + L[l - 1]) / total
                              : (b > 0 ? (bpex[b - 1] + bsum[b - 1]) / total : -1.0);
    certified = (va - cert_halfwidth(a, va, cert_k) > U) &&
                (a == 0 || vp + cert_halfwidth(a - 1, vp, cert_k) < U) && a < N;
    return a;
}

// The same search over a segmented block-sum prefix (scan_segments in epipf_kernels.hip): level 1 over the LDS
// segment ends seg_end[k] (S blocks per segment), level 2 walks the <= S block sums of the segment from global
// memory with the scan's own additions (so every value equals the scan's), level 3 the block's in-block prefix.
// With S = 1 this is resample_search above, value for value (seg_start = bpex, seg_end = bpex + bsum).
__device__ __forceinline__ int resample_search_seg(double U, const double* seg_start, const double* seg_end, int nseg,
                                                   int S, const double* __restrict__ bsum_g, int B, double total,
                                                   const double* __restrict__ wloc, int WGB, int N, double cert_k,
                                                   bool& certified) {
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
    int l = 0, h = WGB - 1;
    while (l < h) {
        const int m = (l + h) >> 1;
        if (base + L[m] > Ut) h = m; else l = m + 1;
    }
    const int a = b * WGB + l;
    const double va = (base + L[l]) / total;
    // inclusive prefix through block b-1: the segment's running sum, or the previous segment's end
    const double pb = (b == k * S) ? (k > 0 ? seg_end[k - 1] : 0.0) : base;
    const double vp = (l > 0) ? (base + L[l - 1]) / total : (b > 0 ? pb / total : -1.0);
    certified = (va - cert_halfwidth(a, va, cert_k) > U) &&
                (a == 0 || vp + cert_halfwidth(a - 1, vp, cert_k) < U) && a < N;
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
