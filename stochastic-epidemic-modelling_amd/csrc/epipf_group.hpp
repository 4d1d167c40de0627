// epipf_group.hpp -- the lane-group step kernel: W lanes per particle, for runs too small to fill the chip.
//
// One chain of N = 10^4 particles is 157 waves on 1024 SIMDs, so the one-lane-per-particle step kernel
// (epipf_kernels.hip) is latency-bound there: each SIMD runs one lone wave whose particles step through their
// events one dependent instruction at a time.  Philox being counter-based, a particle's events do
// not have to be drawn one after the other: a group of W lanes (W = 2, 4, 8, 16) draws W consecutive events'
// blocks at once, and only what really is sequential runs event by event --
//   1. lane i of the group draws the Philox block of event base + i;
//   2. a pass over the W events in order applies the channel decisions (the certified f32 test with its exact
//      fallback: the exact loop's decisions) on registers every lane of the group holds; lane i
//      keeps the state before event base + i;
//   3. lane i evaluates its event's time with the exact loop's own expressions (SsaState::tau_of: reference-order
//      propensities, IEEE divisions, glibc's log);
//   4. a pass adds the times in event order and stops at the first t + tau > tmax, as the exact loop does.
// This is the wave-cooperative replay (coop_replay, epipf_device.hpp) with groups of W lanes instead of the whole
// wave: the result is the exact loop's bit for bit, with no f32 clock to certify and therefore no replays.  The
// in-group broadcasts of steps 2 and 4 are DPP moves (quad_perm for W <= 4, gfx950's row_newbcast for 8 and 16),
// not LDS traffic.  Per event a group spends ~1/W of a Philox block plus the two short sequential passes, so a
// particle advances 3-6x faster than on one lane, at W times the lanes: the right trade exactly when the chip has
// idle SIMDs (the host picks W from chains x particles, epipf_api.cpp).
//
// Block = W waves, 64 particles (the same particle blocks, block sums and in-block prefixes as the one-lane
// kernel, so resampling, weights and scans are the same code on the same values):
//   wave 0   scan of the block sums, resampling draw + certified search (+ exact fallback), ancestor, parent
//            rows into LDS                                                        (pmcmc.py:183-199)
//   all      group SSA of the 64 particles (wave w, group g: particle w * 64/W + g) (gillespie_algo.py)
//   wave 0   store the new states, weights against Y[p], in-block scan, block sum  (pmcmc.py:178-181, 222-231)
// (A variant with one-wave workgroups of 64/W particles, spreading a chain's groups over every CU with the in-block
// scan in a second launch, measured 5-20% slower: the step is bound by each wave's own instruction stream, not by
// waves sharing a SIMD; profiles/r2e_lanes_sweep_onewave.jsonl.)
#pragma once
#include "epipf_step.hpp"

#include <type_traits>

#include "epipf_internal.hpp"


namespace epipf {

// Minimum waves per SIMD asked of the lane-group kernel's register allocation: 4 for the subgroup models (139 VGPRs,
// 3 waves per SIMD, without it: two to four chains of 10^4 particles need 4.9-9.8 waves per SIMD; with the bound 128 VGPRs
// and a few spills, +7% / +14% at two / four chains of config 5, unchanged at one), none for SIR / SEIR (-5-7% at four
// chains with it; profiles/r5i_group_waves_ab.txt).
// EPIPF_GROUP_MIN_WAVES (a build flag, `make spill`) forces one bound on every instance: a register budget low enough
// to spill on purpose, for the spill-robustness test (tests/test_gpu_spill.py).
#ifndef EPIPF_GROUP_MIN_WAVES_SUB
#define EPIPF_GROUP_MIN_WAVES_SUB 4
#endif
template <int MODEL>
constexpr int group_min_waves() {
#ifdef EPIPF_GROUP_MIN_WAVES
    return EPIPF_GROUP_MIN_WAVES;
#else
    return MODEL >= kSubgroups ? EPIPF_GROUP_MIN_WAVES_SUB : 1;
#endif
}

// Value of lane I of this lane's group of W consecutive lanes: DPP moves (groups of W <= 16 lie inside one DPP row),
// a swizzle for W = 8.
template <int W, int I>
__device__ __forceinline__ uint32_t group_lane_dpp(uint32_t v) {
    static_assert(I >= 0 && I < W, "lane inside the group");
    if constexpr (W == 16) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + I, 0xF, 0xF, false);       // row_newbcast:I
    } else if constexpr (W == 8) {
        // two groups per DPP row would take two bank-masked row_newbcast moves and a zeroing move; one ds_swizzle in
        // bitmask mode (source lane (lane & 0x18) | I within each half-wave) goes through the LDS crossbar instead
        return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (I << 5));
    } else if constexpr (W == 4) {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, I | (I << 2) | (I << 4) | (I << 6), 0xF, 0xF, false);
    } else {
        static_assert(W == 2, "W in {2, 4, 8, 16}");
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, I | (I << 2) | ((2 + I) << 4) | ((2 + I) << 6), 0xF,
                                                     0xF, false);
    }
}

// for (I = 0; I < W && f(I); ++I) with I a constant expression in f (the DPP control is an immediate), unrolled
// in the source: the compiler declines to unroll the larger models' passes itself.
template <int I, int W>
struct StaticFor {
    template <class Fn>
    __device__ __forceinline__ static void run(Fn& f) {
        if (f(std::integral_constant<int, I>{})) StaticFor<I + 1, W>::run(f);
    }
};
template <int W>
struct StaticFor<W, W> {
    template <class Fn>
    __device__ __forceinline__ static void run(Fn&) {}
};

template <int W, int I>
__device__ __forceinline__ double group_lane_f64(double v) {
    const uint64_t b = __double_as_longlong(v);
    const uint32_t lo = group_lane_dpp<W, I>((uint32_t)b), hi = group_lane_dpp<W, I>((uint32_t)(b >> 32));
    return __longlong_as_double(((uint64_t)hi << 32) | lo);
}

// Channel decision of one event on the f32 state without the exact fallback, applied to st.  The certified test
// brackets U total: with ulo = uc - kBand (exact: uc is an odd multiple of 2^-24 below 1 and kBand a power of two
// >= 2^-19), Tlo = fl(ulo total) and Thi = fl(Tlo + 2 kBand total), c_i < Tlo puts channel i's cumulative rate
// certainly below U total and c_i >= Thi certainly above: the product form's band (FastSsa) less one
// ulp of total for the two roundings, inside kBand's margin over 2 e_as + 2 ulp.  The pass decides on the Tlo side
// alone (decide_lo: the comparisons as wave masks, the channel as SALU logic on them, the state update as selects on
// the masks, FastSsa::apply_below); whether every c_i also lies on the same side of Thi is checked after the pass,
// by the lane that drew the event, on the state before it (event_certified: the same arithmetic on the same values,
// in the parallel phase instead of on the pass's dependent chain).  A live particle's uncertified event makes the
// caller redo the chunk on the exact fallback.  (A test's band_slack > 1 scales kBand: a wider bracket only moves more
// events to the exact fallback.)
template <typename F>
__device__ __forceinline__ void decide_lo(F& st, float ulo) {
    constexpr int NCH = F::NCH;
    float c[NCH - 1];
    const float Tlo = ulo * st.cum(c);
    uint64_t below[NCH - 1];
#pragma unroll
    for (int i = 0; i < NCH - 1; ++i) below[i] = __ballot(c[i] < Tlo);
    st.apply_below(below);
}

// The chunk's decisions in event order (rounds 2-3): event e's uniform broadcast to the group, decide_lo applied to
// the group's state; lane e % W keeps the state before event e.
template <int W, int K, class F>
__device__ __forceinline__ void decide_sequential(F& st, F* mine, const float* ulo, int gl) {
    auto decide = [&](auto I) __attribute__((always_inline)) -> bool {
        constexpr int e = decltype(I)::value;
        mine[e / W].keep_if(gl == e % W, st);
        decide_lo(st, __uint_as_float(group_lane_dpp<W, e % W>(__float_as_uint(ulo[e / W]))));
        return true;
    };
    StaticFor<0, W * K>::run(decide);
}

// the certificate on cumulative rates c and total already evaluated on the state (the fixed-point pass keeps its last
// evaluation's: the same arithmetic on the same values as a recomputation)
template <int NCH>
__device__ __forceinline__ bool event_certified_on(const float* c, float total, float ulo, float kB) {
    const float Tlo = ulo * total, Thi = fmaf(2.0f * kB, total, Tlo);
    bool sure = true;
#pragma unroll
    for (int i = 0; i < NCH - 1; ++i) sure = sure && ((c[i] < Tlo) == (c[i] < Thi));
    return sure;
}

template <typename F>
__device__ __forceinline__ bool event_certified(const F& s, float ulo, float kB) {
    constexpr int NCH = F::NCH;
    float c[NCH - 1];
    const float total = s.cum(c);
    return event_certified_on<NCH>(c, total, ulo, kB) || !s.active();
}

// Inclusive prefix sum over this lane's group of W consecutive lanes (Hillis-Steele on DPP row shifts; a group of
// W <= 16 lies inside one DPP row, whose edge reads 0; for W < 16 a lane whose source lies in the group before it adds
// nothing: a select on a constant lane mask).
constexpr uint64_t group_tail_mask(int W, int k) {     // lanes with (lane % W) >= k
    uint64_t m = 0;
    for (int l = 0; l < 64; ++l) m |= (uint64_t)((l % W) >= k) << l;
    return m;
}

template <int W>
__device__ __forceinline__ uint32_t group_inclusive_scan(uint32_t v) {
    auto level = [&](auto KK) __attribute__((always_inline)) {
        constexpr int k = decltype(KK)::value;
        if constexpr (k < W) {
            uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + k, 0xF, 0xF, true);   // row_shr:k
            if constexpr (W < 16) t = __builtin_amdgcn_inverse_ballot_w64(group_tail_mask(W, k)) ? t : 0u;
            v += t;
        }
    };
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    level(std::integral_constant<int, 4>{});
    level(std::integral_constant<int, 8>{});
    return v;
}

// The same inclusive prefix for doubles (the certified clock's event times, group_propagate<FASTCLK>): per level two DPP
// moves of the halves and one v_add_f64 (64-bit adds take no DPP operand).  Lanes whose source lies outside the group
// add +0.0, exact for the nonnegative times.
template <int W>
__device__ __forceinline__ double group_inclusive_scan_f64(double v) {
    auto level = [&](auto KK) __attribute__((always_inline)) {
        constexpr int k = decltype(KK)::value;
        if constexpr (k < W) {
            const uint64_t b = __double_as_longlong(v);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, 0x110 + k, 0xF, 0xF, true);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), 0x110 + k, 0xF, 0xF, true);
            double t = __longlong_as_double(((uint64_t)hi << 32) | lo);
            if constexpr (W < 16) t = __builtin_amdgcn_inverse_ballot_w64(group_tail_mask(W, k)) ? t : 0.0;
            v = v + t;
        }
    };
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    level(std::integral_constant<int, 4>{});
    level(std::integral_constant<int, 8>{});
    return v;
}

// The chunk's channel decisions as a fixed point (round 4), instead of W dependent decisions in event order.  With
// d_e = f_e(x_e) the decision of event e on the state x_e before it (decide_lo's Tlo side: F::outcome) and
// x_e = x_0 + sum_{k<e} delta(d_k), guesses g are iterated as g'_e = f_e(x_0 + sum_{k<e} delta(g_k)), all events at
// once (one lane each), starting from g_e = f_e(x_0).  By induction the first k events of the k-th iterate equal the
// sequential pass's, so at most W + 1 evaluations reach it, and a guess that reproduces itself IS the sequential
// pass's result: g_0 = f_0(x_0) = d_0, and g_k = d_k for k < e gives g_e = f_e(x_e) = d_e.  The events' count
// vectors (F::outcome's byte fields) are summed by a group prefix scan.  A chunk's state moves too little for most
// decisions to change: at config 5 (G = 2, W = 8) 96% of the chunks confirm on the second evaluation and a wave's
// slowest group needs 2.3 evaluations on average -- against 8 dependent decisions of the sequential pass.
// With K events per lane (event k W + gl in slot k) the K slots' counts are scanned side by side and slot k's prefix is
// offset by the totals of the slots before it.
// On return: mine[k] = the state before event k W + gl, st = the state after the chunk (every lane of the group), and
// cc[k] / tot[k] the cumulative rates and total of mine[k] (the last evaluation's, for the certificate).
template <int W, int K, class F>
__device__ __forceinline__ void decide_fixed_point(F& st, F* mine, const float* ulo, float (*cc)[F::NCH - 1],
                                                   float* tot) {
    uint32_t d[K], ex[K], total = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) d[k] = st.outcome(ulo[k]);
    for (int it = 0; it <= W * K; ++it) {                // <= W K + 1 evaluations (see above); exits by the break
        uint32_t incl[K];
#pragma unroll
        for (int k = 0; k < K; ++k) incl[k] = group_inclusive_scan<W>(d[k]);
        total = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            ex[k] = total + (incl[k] - d[k]);
            if (k + 1 < K) total += group_lane_dpp<W, W - 1>(incl[k]);
            else total = group_lane_dpp<W, W - 1>(ex[k] + d[k]);
        }
        bool changed = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            mine[k].advance(st, ex[k]);
            const uint32_t d2 = mine[k].outcome(ulo[k], cc[k], &tot[k]);
            changed = changed || d2 != d[k];
            d[k] = d2;
        }
        if (!__any(changed)) break;                      // wave-uniform: every group reproduced its guess
    }
    st.advance(st, total);
}

// 1/sum(a) of the state s (the reference's expressions, SsaState::rates), evaluated on the exact loop's state built
// from s's counts.  The total population N (sum(N) for the subgroups, :35 / :104 / :176) is the particle-step's
// constant the f32 state carries: (S + I) + R of any later state is the same integer, so the value is the one
// SsaState::load would compute, without re-adding the counts per event.  rates() reads no R.
template <int MODEL, int G, class F>
__device__ __forceinline__ double exact_scale(const F& s, const ChainParam& cp) {
    SsaState<MODEL, G> ex;
    if constexpr (MODEL == kSIR) {
        ex.S = (double)s.S; ex.I = (double)s.I; ex.N = s.N;
        double a0;
        return ex.rates(cp, a0);
    } else if constexpr (MODEL == kSEIR) {
        ex.S = (double)s.S; ex.E = (double)s.E; ex.I = (double)s.I; ex.N = s.N;
        double a0, a01;
        return ex.rates(cp, a0, a01);
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g) { ex.S[g] = (double)s.S(g); ex.I[g] = (double)s.I(g); }
        ex.sumN = s.sumN;
        double cum[SsaState<MODEL, G>::NCH];
        return ex.rates(cp, cum);
    }
}

// The certified clock of group_propagate<FASTCLK> (rounds 4-5).  The exact loop's tau divides every infection
// propensity by the population (IEEE), sums the propensities in order, divides the sum into 1 (IEEE) and takes glibc's
// log: its sum(a) is within (3 + n_ch)u of the real sum (three roundings per propensity, n_ch - 1 additions of positive
// terms).  Here (approx_scale)
//   * sum(a') is evaluated factored, with rN = fl(1 / N) in place of the divisions: every term positive, at most
//     2G + 2 roundings on any path, so within (2G + 2)u of the real sum;
//   * its reciprocal is v_rcp_f64 refined by two Newton steps (<= 3u relative; the IEEE quotient: 0.5u);
//   * -log(1 - U) is clock_log_impl's (epipf_device.hpp): |L' - L| <= kClockLogRel L' (+ 1u for glibc's own rounding)
//     where L' >= 2^-10, and kClockLogAbs absolute below;
// so tau' = tau (1 + e) + scale' d with |e| <= (3 + n_ch + 2G + 2 + 3.5 + 1)u + kClockLogRel + 1u <= 34u + 8u + 1u for
// G <= 4 (n_ch <= 20), inside kClockEps = 128u, and d = kClockLogAbs for the events with L' < 2^-10 (0.1%; their scale'
// is summed into the bound, `dabs`), else 0.  The times are summed per chunk by a prefix over the group
// (group_inclusive_scan_f64: <= log2 W roundings inside the chunk, one for each slot offset and one for t + prefix,
// each at most u t') where the exact loop adds them in order (one rounding per event): together < 3u per event of the
// chunk, so after n events of the step the certified clock is within D_n = (kClockEps + 4u n) t'_n + dabs of the exact
// loop's, bounded with margin by (kClockEps + 4u n) 2 tmax + dabs near tmax.  An event with t' < tmax - D is inside the
// step as in the exact loop, one with t' > tmax + D outside; in between (probability ~ D times the event rate, ~1e-9
// per particle-step) the particle-step is redone on the exact clock.
constexpr double kClockEps = 0x1.0p-46, kClockPerEvent = 0x1.0p-51;

// sum(a')'s reciprocal (see above); `ok` false when it is not a positive finite number (then the exact clock decides)
template <int MODEL, int G, class F>
__device__ __forceinline__ double approx_scale(const F& s, const ChainParam& cp, double rN, bool& ok) {
    // sum(a') factored (every term positive, each operation one rounding: <= 8u relative for G <= 4, in the budget above)
    //   SIR  I (beta S rN + gamma);  SEIR  I (beta S rN + gamma) + alpha E;
    //   subgroups  rN sum_g I_g sum_g2 beta[g][g2] S_g2 + gamma sum_g I_g
    double d;
    if constexpr (MODEL == kSIR) {
        d = (double)s.I * fma(cp.theta[0] * (double)s.S, rN, cp.theta[1]);
    } else if constexpr (MODEL == kSEIR) {
        d = fma((double)s.I, fma(cp.theta[0] * (double)s.S, rN, cp.theta[2]), cp.theta[1] * (double)s.E);
    } else {
        double Sd[G], inf = 0.0, sI = 0.0;
#pragma unroll
        for (int g = 0; g < G; ++g) Sd[g] = (double)s.S(g);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            double row = cp.theta[g * G] * Sd[0];
#pragma unroll
            for (int g2 = 1; g2 < G; ++g2) row = fma(cp.theta[g * G + g2], Sd[g2], row);
            const double Ig = (double)s.I(g);
            inf = g == 0 ? row * Ig : fma(row, Ig, inf);
            sI = g == 0 ? Ig : sI + Ig;
        }
        d = fma(inf, rN, cp.theta[G * G] * sI);
    }
    ok = d > 0x1.0p-1000 && d < 0x1.0p1000;
    // 1/d: v_rcp_f64 (~2^-26 relative) and two Newton steps, <= 3u (the IEEE division's scaling steps are not needed
    // on [2^-1000, 2^1000]; outside it `ok` sends the particle-step to the exact clock)
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    return r;
}

template <int MODEL, int G, class F>
__device__ __forceinline__ double population_of(const F& s) {
    if constexpr (MODEL == kSIR || MODEL == kSEIR) return s.N;
    else return s.sumN;
}

// One particle over [0, tmax] by its group of W lanes, K events per lane per chunk (call with the whole group
// active; every lane passes the same parent state x0).  Returns the number of events and the new state in xout, in
// every lane of the group.  Bit-identical to exact_propagate (and so to the one-lane kernel).
//
// Chunk of E = W K events, event e drawn by lane e % W in its slot e / W:
//   per lane, independent of the state: K Philox blocks, their channel uniforms uc and -log(1 - U) (glibc's log);
//   pass: E channel decisions in order, branch-free (decide_lo); lane e % W keeps the state before event e and
//          then checks that event's certificate (event_certified);
//   after: the first event whose state is extinct (ballots) -> events in the chunk; if any decision was not
//          certified, the pass is redone with the exact fallback per event;
//   per lane: each kept state's 1/sum(a) (two IEEE divisions) times its -log(1 - U) = tau (SsaState::tau_of's
//          expression);
//   clock: t + tau in event order, stop at the first t + tau > tmax.
// xch: this wave's LDS slice of K x 64 doubles, through which the clock pass reads the group's tau (one store per lane
// and shared loads instead of two DPP / swizzle moves per event, which took the place of VALU issue slots).
// Day recorder of the ABC trial (abc_kernels.hip): `days` is every event's clock in order, with the state before it.
// The filter records nothing.
// Phase timing (make phase -> lib/libepipf_phase.so, EPIPF_PHASE_TIMING): s_memtime at the phase fences of the chunk
// loop, summed per lane group; the step kernel prints each sampled wave's totals (scripts/phase_report.py).
// Scheduling fences between the chunk's phases (EPIPF_GROUP_FENCES=0 lets the compiler move work across them)
#ifndef EPIPF_GROUP_FENCES
#define EPIPF_GROUP_FENCES 1
#endif
#if EPIPF_GROUP_FENCES
#define EPIPF_GROUP_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define EPIPF_GROUP_FENCE() ((void)0)
#endif
#ifdef EPIPF_PHASE_TIMING
#define EPIPF_PHASE_MARK(v)                                  \
    const unsigned long long v = __builtin_readcyclecounter(); \
    __builtin_amdgcn_sched_barrier(0)
#else
#define EPIPF_PHASE_MARK(v)
#endif
struct NoDays {
    static constexpr bool kOn = false;
};

// FASTCLK (the filter): the certified clock above; returns -1, xout untouched, when a decision is within its bound
// (the caller then runs the particle-step again with FASTCLK = false, the exact loop's clock).
template <int MODEL, int G, int W, int K, class Days = NoDays, bool FASTCLK = false>
__device__ __forceinline__ int group_propagate(const double* x0, double* xout, const ChainParam& cp, uint32_t j,
                                               uint32_t ptag, double tmax, const LogTab* __restrict__ tab,
                                               double* xch, Days* days = nullptr, unsigned long long* ph = nullptr) {
    using F = typename GroupSsa<MODEL, G>::type;
    constexpr int C = Shape<MODEL, G>::C;
    constexpr int E = W * K;
    const int lane = (int)(threadIdx.x & 63);
    const int gl = lane & (W - 1), gb = lane - gl;
    F st;
    if (!(cp.flags & kChainFastSsa) || !st.load(x0, cp)) {
        // outside the f32 channel test's range (or EPIPF_SSA_FAST=0): the exact loop, run by every lane of the group
        // (same result in each); the lanes here all start at event 0 together, so its event index stays uniform
#pragma unroll
        for (int c = 0; c < C; ++c) xout[c] = x0[c];
        if constexpr (Days::kOn) {
            return days->exact(xout, cp, j, ptag, tmax, tab);
        } else {
            int it = 0;
            return exact_propagate<MODEL, G>(xout, cp, j, ptag, tmax, tab, it);
        }
    }
    // xout = the state s of group lane `own` (relative to the parent x0), in every lane of the group
    auto put = [&](const F& s, int own) __attribute__((always_inline)) {
        double xs[C];
#pragma unroll
        for (int c = 0; c < C; ++c) xs[c] = x0[c];
        s.save(xs);
#pragma unroll
        for (int c = 0; c < C; ++c) xout[c] = (double)__shfl((int)xs[c], gb + own, 64);
    };
    double t = 0.0;
    uint32_t base = 0;
    int nev = 0;
    if (!st.active()) {
        put(st, 0);
        return 0;
    }
    const float kB = F::kBand * cp.band_slack;           // the decision band (slack 1: kBand, exact in ulo)
    const double rN = FASTCLK ? 1.0 / population_of<MODEL, G>(st) : 0.0;   // fl(1 / N), once per particle-step
    double dabs = 0.0;                                   // FASTCLK: the clock log's absolute errors so far (bound term)
    F mine[K];                                           // mine[k]: state before event k W + gl
#pragma unroll
    for (int k = 0; k < K; ++k) mine[k] = st;            // the particle-step's constants; the counts kept per event
    for (;;) {
        EPIPF_GROUP_FENCE();
        EPIPF_PHASE_MARK(tA);
        Block r[K];
        float ulo[K];
        double L[K];
        // the Philox key opaque per chunk: its ten round keys are then formed by scalar adds here instead of being
        // hoisted out of the loop into 20 SGPRs, which the compiler spilled to VGPR lanes (v_readlane per round).
        // The key is wave-uniform for every caller (one chain per block; one key per ABC run).
        uint32_t key0 = __builtin_amdgcn_readfirstlane(cp.k0), key1 = __builtin_amdgcn_readfirstlane(cp.k1);
        asm volatile("" : "+s"(key0), "+s"(key1));
#pragma unroll
        for (int k = 0; k < K; ++k) {
            r[k] = philox(base + (uint32_t)(k * W + gl), j, ptag, cp.f, key0, key1);
            const float uc = __uint_as_float(0x3F800000u | (r[k].w >> 9)) - (1.0f - kUlpF);   // uf + 2^-24
            ulo[k] = uc - kB;
            if constexpr (FASTCLK)
                L[k] = clock_neg_log_one_minus_u01(r[k].x, r[k].y, tab);                  // within the clock's bound
            else
                L[k] = neg_log_one_minus_u01<true>(r[k].x, r[k].y, tab);                 // -log(1 - U), :62
        }
        // sched_barrier(0) fences between the phases (draws | decision pass | extinction + redo | tau | clock): the
        // scheduler otherwise hoists independent work across the latency-bound passes (measured +1% at config 5,
        // one chain; profiles/r3d_phase_timing.txt has the per-phase cycles)
        EPIPF_GROUP_FENCE();
        EPIPF_PHASE_MARK(tB);
        const F st0 = st;
        bool uncertified = false;                        // this lane's events, on the states before them
        if constexpr (F::kFixedPoint) {
            if (!(cp.flags & kChainSeqDecide)) {
                float cc[K][F::NCH - 1], tot[K];
                decide_fixed_point<W, K>(st, mine, ulo, cc, tot);
#pragma unroll
                for (int k = 0; k < K; ++k)
                    uncertified = uncertified || !(event_certified_on<F::NCH>(cc[k], tot[k], ulo[k], kB) || !mine[k].active());
            } else {
                decide_sequential<W, K>(st, mine, ulo, gl);
#pragma unroll
                for (int k = 0; k < K; ++k) uncertified = uncertified || !event_certified(mine[k], ulo[k], kB);
            }
        } else {
            decide_sequential<W, K>(st, mine, ulo, gl);
#pragma unroll
            for (int k = 0; k < K; ++k) uncertified = uncertified || !event_certified(mine[k], ulo[k], kB);
        }
        EPIPF_GROUP_FENCE();
        EPIPF_PHASE_MARK(tC);
        // events up to extinction: the first e whose state before it is extinct (the last applied event emptied it)
        int nk = E;
#pragma unroll
        for (int k = K - 1; k >= 0; --k) {
            const uint64_t dead = __ballot(!mine[k].active());
            const uint32_t bits = (uint32_t)(dead >> gb) & ((1u << W) - 1u);
            if (bits) nk = min(nk, k * W + (int)__builtin_ctz(bits));
        }
        if (__ballot(uncertified) >> gb & ((1ull << W) - 1ull)) {   // group-uniform, rare: redo with the exact fallback
            st = st0;
            nk = E;
            auto decide_exact = [&](auto I) __attribute__((always_inline)) -> bool {
                constexpr int e = decltype(I)::value;
                if (gl == e % W) mine[e / W] = st;
                const uint32_t rz = group_lane_dpp<W, e % W>(r[e / W].z), rw = group_lane_dpp<W, e % W>(r[e / W].w);
                st.apply(fast_channel(st, cp, rz, rw), 1.f);
                if (st.active()) return true;
                nk = e + 1;
                return false;
            };
            StaticFor<0, E>::run(decide_exact);
#pragma unroll
            for (int k = 0; k < K; ++k)                  // the state before event nk (< E): the extinct one
                if (k * W + gl == nk) mine[k] = st;
        }
        EPIPF_GROUP_FENCE();
        EPIPF_PHASE_MARK(tD);
        double tau[K];                                   // each event's time: the exact loop's expressions, or
        bool scale_ok = true;                            // FASTCLK's (approx_scale)
        double small = 0.0;                              // FASTCLK: sum of scale' over this lane's events with L' < 2^-10
#pragma unroll
        for (int k = 0; k < K; ++k) {
            tau[k] = 0.0;
            if (k * W + gl < nk) {
                if constexpr (FASTCLK) {
                    bool ok;
                    const double sc = approx_scale<MODEL, G>(mine[k], cp, rN, ok);
                    tau[k] = sc * L[k];
                    scale_ok = scale_ok && ok;
                    small += L[k] < 0x1.0p-10 ? sc : 0.0;
                } else {
                    tau[k] = exact_scale<MODEL, G>(mine[k], cp) * L[k];
                }
            }
        }
        if constexpr (FASTCLK) {                         // group-uniform
            if ((__ballot(!scale_ok) >> gb) & ((1ull << W) - 1ull)) return -1;
            // the clock log's absolute error on small logs (rare: ~0.1% of events), summed over the group; 4 ulps of
            // margin for the f64 sum of the positive scale' terms
            if (__any(small != 0.0)) {
                const double s = group_lane_f64<W, W - 1>(group_inclusive_scan_f64<W>(small));
                dabs = dabs + s * (kClockLogAbs * (1.0 + 0x1.0p-50));
            }
        }
        double tt = t;
        int inside = 0;
        EPIPF_GROUP_FENCE();
        EPIPF_PHASE_MARK(tE);
        if constexpr (FASTCLK && !Days::kOn) {
            // the certified clock: every event's time at once, t + its prefix over the group (no LDS, no pass in
            // event order); the first event not surely inside ends the step there, or, within the bound, the
            // particle-step goes to the exact clock
            double ttk[K];
            double off = 0.0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const double P = group_inclusive_scan_f64<W>(tau[k]);
                const double Pk = k == 0 ? P : off + P;
                ttk[k] = t + Pk;
                if (k + 1 < K) off = group_lane_f64<W, W - 1>(Pk);
            }
            const double D = (kClockEps + kClockPerEvent * (double)(nev + E)) * (2.0 * tmax) * (double)cp.clock_slack +
                             dabs;
            int first = E;
#pragma unroll
            for (int k = K - 1; k >= 0; --k) {
                const uint32_t bits = (uint32_t)(__ballot(!(ttk[k] < tmax - D)) >> gb) & ((1u << W) - 1u);
                if (bits) first = min(first, k * W + (int)__builtin_ctz(bits));
            }
            if (first == E) {
                inside = E;
                tt = group_lane_f64<W, W - 1>(ttk[K - 1]);
            } else {
                bool unsure = false;
#pragma unroll
                for (int k = 0; k < K; ++k) unsure = unsure || (k * W + gl == first && !(ttk[k] > tmax + D));
                if ((__ballot(unsure) >> gb) & ((1ull << W) - 1ull)) return -1;   // group-uniform
                inside = first;
            }
        } else {
            // the exact loop's clock: t + tau in event order (the exact loop's additions), the group's tau read from LDS
            // (one store per lane and shared loads instead of two DPP / swizzle moves per event, which took the place
            // of VALU issue slots); the step ends at the first t + tau > tmax.  Branch-free: the sum runs on through the
            // chunk (events past nk add tau = 0) and `inside` counts the events before the first overshoot -- once an
            // event overshoots, t is no longer needed (the step ends in this chunk).
#pragma unroll
            for (int k = 0; k < K; ++k) xch[k * 64 + lane] = tau[k];
            lds_sync<true>();                            // this wave's stores before its loads
            const double* xg = xch + gb;                 // tau of event e: xg[(e / W) * 64 + e % W]
            if constexpr (Days::kOn) {
                bool alive = true;
                auto clock = [&](auto I) __attribute__((always_inline)) -> bool {
                    constexpr int e = decltype(I)::value;
                    tt = tt + xg[(e / W) * 64 + e % W];
                    alive = alive && !(tt > tmax);       // :65-66
                    inside += alive ? 1 : 0;
                    if (alive && e < nk) days->passed(tt, gl == e % W, mine[e / W], x0);   // days before event e (rare)
                    return true;
                };
                StaticFor<0, E>::run(clock);
            } else {
                // The sums t + tau are nondecreasing (tau >= 0; finite on this path: f32-eligible rates and counts), so
                // every prefix is at most the chunk's total: when the total stays inside the step, so does every
                // event, and only a chunk that overshoots (the step's last) counts the events before its first
                // t + tau > tmax, adding again in the same order.
                auto clock = [&](auto I) __attribute__((always_inline)) -> bool {
                    constexpr int e = decltype(I)::value;
                    tt = tt + xg[(e / W) * 64 + e % W];
                    return true;
                };
                StaticFor<0, E>::run(clock);
                if (!(tt > tmax)) {
                    inside = E;
                } else {
                    double t2 = t;
                    bool alive = true;
                    auto recount = [&](auto I) __attribute__((always_inline)) -> bool {
                        constexpr int e = decltype(I)::value;
                        t2 = t2 + xg[(e / W) * 64 + e % W];
                        alive = alive && !(t2 > tmax);   // :65-66
                        inside += alive ? 1 : 0;
                        return true;
                    };
                    StaticFor<0, E>::run(recount);
                }
            }
        }
        EPIPF_GROUP_FENCE();
        EPIPF_PHASE_MARK(tF);
#ifdef EPIPF_PHASE_TIMING
        if (ph) {
            ph[0] += tB - tA; ph[1] += tC - tB; ph[2] += tD - tC; ph[3] += tE - tD; ph[4] += tF - tE; ph[5] += 1;
        }
#endif
        if constexpr (Days::kOn) {                       // ABC early rejection, once per chunk (group-uniform)
            if (days->template reject_now<W>()) {
                put(st, 0);
                return nev + E;
            }
        }
        const int stop = inside < nk ? inside : -1;
        t = tt;
        if (stop >= 0 || nk < E) {                       // the step ends before event `end` (past tmax or extinct)
            const int end = stop >= 0 ? stop : nk;
            F fin = st;
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (k * W + gl == end) fin = mine[k];
            put(fin, end % W);
            return nev + end;
        }
        nev += E;
        base += (uint32_t)E;
        if (!st.active()) {                              // extinct after the chunk's last event
            put(st, 0);
            return nev;
        }
    }
}

// LDS of the lane-group step kernel: log table | tau exchange [PB W / 64 waves][K][64] | red[16] | particle rows [64][C]
// int32 | block-sum prefix.  PB particles per block (64 or kGroupBlock).
inline size_t group_lds_bytes_impl(int B, int S, int C, int W, int K, int PB) {
    return step_lds_bytes_seg(B, S, 64) + sizeof(int32_t) * 64 * (size_t)C + sizeof(double) * (size_t)PB * W * K;
}

// PB particles per block: 64 (the one-lane kernel's blocks), or kGroupBlock = 16 for runs that would leave CUs idle
// (a.wg; the weight layout -- block sums, in-block prefixes -- is then one of 16-particle blocks, built by the init
// kernel the same way).  Wave 0's first PB lanes hold the block's particles in the scan/search/gather and store/weigh
// phases; the block is PB W / 64 waves.
template <int MODEL, int G, int OBS, int W, int K, int PB, int MINW>
__global__ __launch_bounds__(PB * W, MINW) void pf_step_group_kernel(StepArgs a, int p) {
    using Sh = Shape<MODEL, G>;
    constexpr int C = Sh::C;
    constexpr int PPW = 64 / W;                          // particles per wave
    static_assert(PB * W >= 64 && (PB * W) % 64 == 0, "whole waves");
    extern __shared__ __attribute__((aligned(16))) double smem[];
    LogTab* tab = reinterpret_cast<LogTab*>(smem);
    double* xch = smem + 2 * kLogTabEntries;             // the clock pass's tau exchange, [PB W / 64 waves][K][64]
    double* red = xch + PB * W * K;                      // [0]: the step's weight total, for every wave; [1]: scratch
    int32_t* rows = reinterpret_cast<int32_t*>(red + 16);
    double* seg_start = red + 16 + (64 * C + 1) / 2;
    double* seg_end = seg_start + a.nseg;
    const BlockPos bp = step_block(a);
    const int chain = bp.chain;
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    if (a.status[chain] != 0) return;
    const ChainParam cp = a.cp[chain];
    const int prev = (p - 1) & 1, cur = p & 1;
    const size_t wprev = ((size_t)prev * a.max_chains + chain) * a.wstride;
    const size_t wcur = ((size_t)cur * a.max_chains + chain) * a.wstride;
    const size_t bprev = ((size_t)prev * a.max_chains + chain) * a.bstride;
    const size_t bcur = ((size_t)cur * a.max_chains + chain) * a.bstride;
    for (int i = (int)threadIdx.x; i < kLogTabEntries; i += PB * W) tab[i] = a.logtab[i];

#ifdef EPIPF_PHASE_TIMING
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};
    const unsigned long long k0 = __builtin_readcyclecounter();
#else
    unsigned long long* ph = nullptr;
#endif
    if (wave == 0) {                                     // likelihood, resampling, gather: pf_step_kernel's code
        const int j = bp.b * PB + lane;
        const bool mine = lane < PB && j < a.N;
        double total;
        if constexpr (PB == kGroupBlock)                 // the total in the 64-particle layout's order (epipf_step.hpp)
            total = scan_block_sums16<true>(a.bsum + bprev, a.B, a.canon_per, a.seg, seg_start + a.B, seg_start,
                                            seg_start, seg_end, red + 1);
        else
            total = (a.seg == 1) ? scan_block_sums<64, true>(a.bsum + bprev, a.B, seg_start + a.B, seg_start, red)
                                 : scan_segments<true>(a.bsum + bprev, a.B, a.seg, a.nseg, seg_start, seg_end);
        if (lane == 0) red[0] = total;
        if (total > 0.0) {
            if (bp.b == 0 && lane == 0)            // pmcmc.py:183, in log space
                a.log_zeta[(size_t)chain * a.T + p] = a.log_zeta[(size_t)chain * a.T + p - 1] + log(total / (double)a.N);
            double U = 0.0;
            int anc = 0;
            bool certified = true, ambiguous = false;
            if (mine) {                                  // pmcmc.py:188-190
                const uint32_t rtag = ((uint32_t)p & 0xFFFFFFu) | kDomainResample;
                if (a.resample_mode == 0) {
                    const Block r = philox(0u, (uint32_t)j, rtag, cp.f, cp.k0, cp.k1);
                    U = u01(r.x, r.y);
                } else {
                    const Block r = philox(0u, 0u, rtag, cp.f, cp.k0, cp.k1);
                    U = ((double)j + u01(r.x, r.y)) / (double)a.N;
                }
                if (a.seg == 1)
                    anc = resample_search<PB, true>(U, seg_start + a.B, seg_start, a.B, total, a.wloc + wprev, a.N, a.cert_k,
                                              certified, a.ref_k, ambiguous);
                else
                    anc = resample_search_seg<true>(U, seg_start, seg_end, a.nseg, a.seg, a.bsum + bprev, a.B, total,
                                              a.wloc + wprev, PB, a.N, a.cert_k, certified, a.ref_k, ambiguous);
            }
            if (ambiguous) atomicAdd(counter_slot(a.counters) + 6, 1ull);
            if (__any(!certified)) {
                const int e = resample_exact_wave(!certified, U, a.wraw + wprev, a.N);
                if (!certified) {
                    anc = e;
                    atomicAdd(counter_slot(a.counters) + 1, 1ull);
                }
            }
            if (mine) {                                  // :193-199
                anc = checked_index(anc, a.N);
                a.ancestry[(size_t)chain * a.anc_stride + (size_t)p * a.N + j] = anc;
                const int32_t* hp = a.hidden + (size_t)chain * a.hist_stride + ((size_t)(p - 1) * a.N + anc) * C;
#pragma unroll
                for (int c = 0; c < C; ++c) rows[lane * C + c] = hp[c];
            }
        } else if (bp.b == 0 && lane == 0) {       // all weights 0 or NaN: :187-192
            a.status[chain] = 1;
            a.log_zeta[(size_t)chain * a.T + p] = -__builtin_inf();
        }
    }
    __syncthreads();
#ifdef EPIPF_PHASE_TIMING
    const unsigned long long k1 = __builtin_readcyclecounter();
#endif
    if (!(red[0] > 0.0)) return;                         // block-uniform

    // group SSA: wave w, group g runs particle w * PPW + g of the block
    const int gl = lane & (W - 1);
    const int pl = wave * PPW + lane / W;
    const int jg = bp.b * PB + pl;
    int nev = 0;
    double x[C];
    if (jg < a.N) {                                      // group-uniform
        double x0[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x0[c] = (double)rows[pl * C + c];
        const uint32_t ptag = ((uint32_t)p & 0xFFFFFFu) | kDomainSSA;
        constexpr bool kFastClock = true;
        nev = group_propagate<MODEL, G, W, K, NoDays, kFastClock>(x0, x, cp, (uint32_t)jg, ptag, 1.0, tab,
                                                                  xch + wave * 64 * K, (NoDays*)nullptr, ph);
        if (kFastClock && nev < 0)                       // a clock decision within the certified clock's bound (rare)
            nev = group_propagate<MODEL, G, W, K, NoDays, false>(x0, x, cp, (uint32_t)jg, ptag, 1.0, tab,
                                                                 xch + wave * 64 * K, (NoDays*)nullptr, ph);
    }
#ifdef EPIPF_PHASE_TIMING
    const unsigned long long k2 = __builtin_readcyclecounter();
#endif
    __syncthreads();                                     // every group has read its parent row
    if (jg < a.N && gl == 0) {
#pragma unroll
        for (int c = 0; c < C; ++c) rows[pl * C + c] = (int32_t)x[c];
    }
    if (a.count_events) {                                // events (no lane-use figure in this kernel)
        unsigned long long e = gl == 0 ? (unsigned long long)nev : 0ull;
        for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
        if (lane == 0) atomicAdd(counter_slot(a.counters), e);
    }
    __syncthreads();

    if (wave == 0) {                                     // store, weights for step p+1, in-block scan
        const int j = bp.b * PB + lane;
        double w = 0.0;
        if (lane < PB && j < a.N) {
            double xs[C];
#pragma unroll
            for (int c = 0; c < C; ++c) xs[c] = (double)rows[lane * C + c];
            int32_t* hc = a.hidden + (size_t)chain * a.hist_stride + ((size_t)p * a.N + j) * C;
#pragma unroll
            for (int c = 0; c < C; ++c) hc[c] = (int32_t)xs[c];                       // :222-231
            if (p + 1 < a.T)
                w = particle_weight<MODEL, G, OBS>(xs, a.Y + (size_t)p * Sh::K, cp, a.cp + chain, a.lf, a.lf_max, hc);
        }
        if (p + 1 < a.T) {
            const double loc = block_inclusive_scan<64>(w, red);
            if (lane < PB) {
                a.wraw[wcur + j] = w;
                a.wloc[wcur + j] = loc;
            }
            if (lane == PB - 1) a.bsum[bcur + bp.b] = loc;
        }
    }
#ifdef EPIPF_PHASE_TIMING
    if (lane == 0 && bp.b % 16 == 0 && (a.T < 50 || p % 20 == 0))
        printf("PH p=%d b=%d w=%d ch=%llu pre=%llu ssa=%llu bar=0 post=%llu draws=%llu decide=%llu ball=%llu tau=%llu "
               "clock=%llu nev=%d\n", p, bp.b, wave, ph[5], k1 - k0, k2 - k1, __builtin_readcyclecounter() - k2, ph[0],
               ph[1], ph[2], ph[3], ph[4], nev);
#endif
}

// ------------------------------------------------------------------------------- launch table
// The subgroup models' lane-group kernels at G >= 2 need more registers than the 4-wave bound leaves them (G = 2:
// 143 VGPRs unbounded, 128 + 13-20 spilled under the bound; G = 3: ~205 vs 128 + ~180 spilled; G = 4: ~260 vs 128 +
// ~500 spilled).  The bound pays where a launch has more waves than the unbounded kernel keeps resident (two to four
// chains of 10^4 particles); a launch with fewer -- BASELINE config 5's one chain per GPU -- gains nothing from it and
// pays the spills' scratch traffic on every chunk (7.2 MB written per launch).  So W >= 8 instances of
// those models (the widths small launches take, pick_lanes) also exist without the bound, and the host picks them by the
// launch's wave count (epipf_api.cpp, group_lone_waves).  Not in the forced-spill build (EPIPF_GROUP_MIN_WAVES).
template <int MODEL, int G, int W>
constexpr bool group_lone_instance() {
#ifdef EPIPF_GROUP_MIN_WAVES
    return false;
#else
    return group_min_waves<MODEL>() > 1 && MODEL >= kSubgroups && G >= 2 && W >= 8;
#endif
}

template <int MODEL, int G, int OBS, int W, int K, int MINW>
static void launch_group_pb(const StepArgs& a, int p, dim3 grid, size_t lds, hipStream_t s) {
    if constexpr (W >= 8) {                              // 16-particle blocks (a.wg, pick_block): W >= 8 only
        if (a.wg == kGroupBlock) {
            hipLaunchKernelGGL((pf_step_group_kernel<MODEL, G, OBS, W, K, kGroupBlock, MINW>), grid,
                               dim3(kGroupBlock * W), lds, s, a, p);
            return;
        }
    }
    hipLaunchKernelGGL((pf_step_group_kernel<MODEL, G, OBS, W, K, 64, MINW>), grid, dim3(64 * W), lds, s, a, p);
}

template <int MODEL, int G, int OBS, int W, int K>
static void launch_group_t(const StepArgs& a, int p, dim3 grid, size_t lds, hipStream_t s) {
    if constexpr (group_lone_instance<MODEL, G, W>()) {
        if (a.group_lone) {
            launch_group_pb<MODEL, G, OBS, W, K, 1>(a, p, grid, lds, s);
            return;
        }
    }
    launch_group_pb<MODEL, G, OBS, W, K, group_min_waves<MODEL>()>(a, p, grid, lds, s);
}

// (lanes per particle W, events per lane per chunk K) instantiated.  K = 2 (round 4, fixed-point pass) measured +4% at
// config 5 one chain, -1.5% at config 2, -23% at config 5 four chains (profiles/r4c_*): not instantiated, to keep the
// library's size and build time in check (the code is K-general; add X(w, 2) to bring a shape back).
#define EPIPF_GROUP_SHAPES(X) X(2, 1) X(4, 1) X(8, 1) X(16, 1)

template <int MODEL, int G, int OBS>
static GroupStepFn pick_wk(int W, int K) {
#define EPIPF_PICK(w, k) if (W == w && K == k) return launch_group_t<MODEL, G, OBS, w, k>;
    EPIPF_GROUP_SHAPES(EPIPF_PICK)
#undef EPIPF_PICK
    return nullptr;
}

template <int MODEL, int G>
static GroupStepFn pick_obs(int obs, int W, int K) {
    return obs == kBinomial ? pick_wk<MODEL, G, kBinomial>(W, K) : pick_wk<MODEL, G, kNormal>(W, K);
}

// per-model tables, one translation unit each (parallel builds)
GroupStepFn group_launcher_sir(int model, int obs, int W, int K);
GroupStepFn group_launcher_sub(int G, int obs, int W, int K);
GroupStepFn group_launcher_sub2(int G, int obs, int W, int K);

}  // namespace epipf
