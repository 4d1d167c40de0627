// epipf_fused.hpp -- the whole particle filter of one chain in ONE workgroup, for small particle counts.
//
// At N <= kFusedMaxN (the reference's own test shapes: BASELINE config 1 is N = 100, T = 50) a filter step is a few
// microseconds of work, so the step launches of epipf_kernels.hip cost more than the step: T - 1 dependent launches,
// each re-reading the weights and states the previous one left in HBM.  Here one workgroup per chain runs init and
// every step in one launch, the chain's whole working set in LDS:
//   init     Poisson initial states (init_particle), weights against Y[0], in-block scans    (pmcmc.py:156-181)
//   step p   wave 0: block-sum prefix -> total, log-likelihood                                (pmcmc.py:183)
//            waves of the particle phase: multinomial draw, certified search over the LDS prefix, exact fallback,
//            ancestor, parent row gathered from LDS                                          (pmcmc.py:185-199)
//            every wave: group SSA, W lanes per particle (group_propagate, epipf_group.hpp)  (gillespie_algo.py)
//            particle phase: store, weights against Y[p], in-block scans, block sums          (pmcmc.py:178-181, 222-231)
// with barriers between the phases instead of kernel boundaries.  The arithmetic is the step kernels' on the same
// layout -- 64-particle weight blocks, the same in-block scan, the same block-sum prefix (scan_block_sums<64>), the same
// certified search with the same certificate, the same lane-group SSA -- so states, ancestors and log-likelihoods are
// those of the multi-launch path bit for bit (tests/test_gpu_fused.py).  The history (hidden, ancestry) and the
// log-likelihoods go to HBM as the step kernels write them, for the path sampler and epipf_copy_history.
//
// A step's latency is the whole cost here (a chain is one workgroup on one CU), so what the phases read stays in LDS:
// the chain's parameters, the observations Y and, when it fits, the log n! table of the weights (a.fused_y / fused_lf:
// the host stages them when the LDS stays under kFusedLdsLimit).
//
// LDS: log table | ChainParam | tau exchange [waves][64] | red[16] | wraw, wloc [B 64] | bsum [B] | bpex [B + 64] |
//      Y [T K] | log n! [2 (lf_max + 1)] | rows [2][N][C] int32
// The weights, their in-block prefixes and the block sums are double-buffered by step parity like the rows: with one
// lane per particle (W = 1) a step has no barrier between a wave's resampling (reading step p - 1's) and its weights
// (writing step p's), so another wave may still be searching the previous ones.
#pragma once
#include "epipf_group.hpp"

namespace epipf {

constexpr int kCpDoubles = (int)((sizeof(ChainParam) + 15) / 16 * 2);
inline size_t fused_lds_bytes(int N, int C, int threads, int TK, int lf_n) {
    const int B = (N + 63) / 64;
    const size_t dbl = 2 * (size_t)kLogTabEntries + kCpDoubles + (size_t)(threads / 64) * 64 + 16 + 4 * (size_t)B * 64 +
                       2 * B + (B + 64) + (size_t)TK + (size_t)lf_n;
    return dbl * sizeof(double) + sizeof(int32_t) * 2 * (size_t)N * C;
}

// Threads of the workgroup: N W lanes for the SSA, at least one lane per particle of the 64-particle blocks
inline int fused_threads(int N, int W) {
    const int B = (N + 63) / 64;
    const int t = ((N * W + 63) / 64) * 64;
    return t > B * 64 ? t : B * 64;
}

template <int MODEL, int G, int OBS, int W>
__global__ __launch_bounds__(kFusedMaxThreads) void pf_filter_wg_kernel(StepArgs a) {
    using Sh = Shape<MODEL, G>;
    constexpr int C = Sh::C;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int nthr = (int)blockDim.x, nw = nthr >> 6;
    const int N = a.N, T = a.T, B = a.B;
    LogTab* tab = reinterpret_cast<LogTab*>(smem);
    ChainParam* cps = reinterpret_cast<ChainParam*>(smem + 2 * kLogTabEntries);   // the chain's parameters
    double* xch = smem + 2 * kLogTabEntries + kCpDoubles;   // group_propagate's tau exchange (exact clock), [nw][64]
    double* red = xch + nw * 64;                         // [0]: the step's total, for every wave
    double* wraw = red + 16;                             // weights by step parity, [2][B 64]
    double* wloc = wraw + 2 * B * 64;                    // their in-block inclusive prefixes, [2][B 64]
    double* bsum = wloc + 2 * B * 64;                    // block sums, [2][B]
    double* bpex = bsum + 2 * B;                         // exclusive prefix of the block sums [B] (+ 64 scratch)
    const int TK = a.fused_y ? T * Sh::K : 0, lf_n = a.fused_lf ? 2 * (a.lf_max + 1) : 0;
    double* ys = bpex + B + 64;                          // Y [T][K] (a.fused_y)
    double* lfs = ys + TK;                               // log n! hi [lf_max + 1], lo [lf_max + 1] (a.fused_lf)
    int32_t* rows = reinterpret_cast<int32_t*>(lfs + lf_n);   // states [2][N][C]: step parity
    const int chain = a.chain0 + (int)blockIdx.x;
    const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const ChainParam cp = a.cp[chain];
    if (tid == 0) a.status[chain] = cp.skip ? kStatusSkipped : kStatusOk;   // this run's chain status
    if (cp.skip) return;                                 // block-uniform
    for (int i = tid; i < kLogTabEntries; i += nthr) tab[i] = a.logtab[i];
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.cp + chain);
        uint32_t* dst = reinterpret_cast<uint32_t*>(cps);
        for (int i = tid; i < (int)(sizeof(ChainParam) / 4); i += nthr) dst[i] = src[i];
    }
    for (int i = tid; i < TK; i += nthr) ys[i] = a.Y[i];
    for (int i = tid; i < lf_n; i += nthr) lfs[i] = a.lf[i];
    const double* Y = a.fused_y ? ys : a.Y;
    const double* lf = a.fused_lf ? lfs : a.lf;
    __syncthreads();
    int32_t* hist = a.hidden + (size_t)chain * a.hist_stride;
    int32_t* ancg = a.ancestry + (size_t)chain * a.anc_stride;
    double* lz = a.log_zeta + (size_t)chain * T;
    const bool pt = tid < B * 64;                        // the particle phases: one lane per particle (wave-uniform)
    const int j = tid;

    // init, pmcmc.py:156-181 (pf_init_kernel's code)
    if (pt) {
        double x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = 0.0;
        double w = 0.0;
        if (j < N) {
            init_particle<MODEL, G>(a, cp, j, x);
            int32_t* h = hist + (size_t)j * C;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                h[c] = (int32_t)x[c];
                rows[j * C + c] = (int32_t)x[c];
            }
            ancg[j] = 0;
            if (T > 1) w = particle_weight<MODEL, G, OBS>(x, Y, cp, cps, lf, a.lf_max, rows + j * C);
        }
        if (T > 1) {
            const double loc = block_inclusive_scan<64>(w, nullptr);
            wraw[j] = w;
            wloc[j] = loc;
            if (lane == 63) bsum[wave] = loc;
        }
    }
    double lzp = 0.0;                                    // log_zeta[p - 1] (thread 0)
    if (tid == 0) lz[0] = 0.0;
    unsigned long long events = 0;
    const int gl = tid & (W - 1), pl = tid / W;          // SSA (W > 1): group of W lanes per particle pl
    __syncthreads();
#ifdef EPIPF_PHASE_TIMING
    unsigned long long fph[6] = {0, 0, 0, 0, 0, 0}, fm0 = __builtin_readcyclecounter(), fm1;
#define EPIPF_FUSED_MARK(k) (fm1 = __builtin_readcyclecounter(), fph[k] += fm1 - fm0, fm0 = fm1)
#else
#define EPIPF_FUSED_MARK(k) ((void)0)
#endif

    for (int p = 1; p < T; ++p) {
        const int cur = p & 1, prev = cur ^ 1;
        int32_t* rprev = rows + (size_t)prev * N * C;
        int32_t* rcur = rows + (size_t)cur * N * C;
        double* wr_prev = wraw + prev * B * 64;         // the weights step p resamples from ...
        double* wl_prev = wloc + prev * B * 64;
        double* bs_prev = bsum + prev * B;
        double* wr_cur = wraw + cur * B * 64;           // ... and the ones it produces for step p + 1
        double* wl_cur = wloc + cur * B * 64;
        double* bs_cur = bsum + cur * B;
        // (b) likelihood, pmcmc.py:183: the block-sum prefix (the step kernels' scan_block_sums<64>, S = 1)
        if (wave == 0) {
            const double total = scan_block_sums<64, true>(bs_prev, B, bpex, bs_prev, red + 1);
            if (lane == 0) red[0] = total;
        }
        __syncthreads();
        EPIPF_FUSED_MARK(0);
        const double total = red[0];
        if (!(total > 0.0)) {                            // all weights 0 or NaN: :187-192 (block-uniform)
            if (tid == 0) {
                a.status[chain] = 1;
                lz[p] = -__builtin_inf();
            }
            break;
        }
        if (tid == 0) {
            lzp = lzp + log(total / (double)N);
            lz[p] = lzp;
        }
        // (d) multinomial (or systematic) draw, certified search, exact fallback (:188-193); lanes of the particle phase
        auto draw_ancestor = [&]() __attribute__((always_inline)) -> int {
            double U = 0.0;
            int anc = 0;
            bool certified = true, ambiguous = false;
            if (j < N) {
                const uint32_t rtag = ((uint32_t)p & 0xFFFFFFu) | kDomainResample;
                if (a.resample_mode == 0) {
                    const Block r = philox(0u, (uint32_t)j, rtag, cp.f, cp.k0, cp.k1);
                    U = u01(r.x, r.y);
                } else {
                    const Block r = philox(0u, 0u, rtag, cp.f, cp.k0, cp.k1);
                    U = ((double)j + u01(r.x, r.y)) / (double)N;
                }
                // the flat in-block search (two rounds of 7 independent LDS loads instead of 6 dependent ones)
                anc = resample_search<64, true>(U, bpex, bs_prev, B, total, wl_prev, N, a.cert_k, certified, a.ref_k,
                                                ambiguous);
            }
            if (ambiguous) atomicAdd(counter_slot(a.counters) + 6, 1ull);
            if (__any(!certified)) {                     // wave-uniform
                const int e = resample_exact_wave(!certified, U, wr_prev, N);
                if (!certified) {
                    anc = e;
                    atomicAdd(counter_slot(a.counters) + 1, 1ull);
                }
            }
            anc = checked_index(anc, N);
            if (j < N) ancg[(size_t)p * N + j] = anc;
            return anc;
        };
        // store, weights for step p + 1, in-block scans (:178-181, :222-231): lane j of the particle phase, its state
        // in xs (read by the scan's other lanes only through wraw / wloc / bsum)
        auto weigh = [&](const double* xs) __attribute__((always_inline)) {
            double w = 0.0;
            if (j < N) {
                int32_t* hc = hist + ((size_t)p * N + j) * C;
#pragma unroll
                for (int c = 0; c < C; ++c) hc[c] = (int32_t)xs[c];
                if (p + 1 < T) w = particle_weight<MODEL, G, OBS>(xs, Y + (size_t)p * Sh::K, cp, cps, lf, a.lf_max,
                                                                  rcur + j * C);
            }
            if (p + 1 < T) {
                const double loc = block_inclusive_scan<64>(w, nullptr);
                wr_cur[j] = w;
                wl_cur[j] = loc;
                if (lane == 63) bs_cur[wave] = loc;
            }
        };
        const uint32_t ptag = ((uint32_t)p & 0xFFFFFFu) | kDomainSSA;
        if constexpr (W == 1) {
            // one lane per particle (pf_step_kernel's SSA): draw, gather, propagate, store and weigh on the same lane --
            // no barrier inside the step.  Lanes the certified f32 loop hands back run the exact loop (ineligible) or
            // are replayed by their whole wave (coop_replay) on their LDS row.
            double x[C];
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = 0.0;
            int nev = 0, iters = 0;
            bool fast_ok = false, eligible = false;
            const int anc = draw_ancestor();
            if (j < N) {
#pragma unroll
                for (int c = 0; c < C; ++c) x[c] = (double)rprev[anc * C + c];
                fast_ok = fast_propagate<MODEL, G>(x, cp, (uint32_t)j, ptag, 1.0, nev, iters, eligible);
            }
            const bool exact = j < N && !fast_ok;
            if (__any(exact)) {                          // wave-uniform
                if (exact && !eligible) {
                    int ex_iters = 0;
                    nev = exact_propagate<MODEL, G>(x, cp, (uint32_t)j, ptag, 1.0, tab, ex_iters);
                }
                unsigned long long pend = __ballot(exact && eligible);
                if (pend) {
                    if (j < N) {
#pragma unroll
                        for (int c = 0; c < C; ++c) rcur[j * C + c] = (int32_t)x[c];   // replayed lanes: the parent
                    }
                    lds_sync<true>();
                    while (pend) {
                        const int L = (int)__builtin_ctzll(pend);
                        pend &= pend - 1ull;
                        const uint32_t jl = __builtin_amdgcn_readlane((uint32_t)j, L);
                        const int n = coop_replay<MODEL, G, true>(rcur + (size_t)jl * C, cp, jl, ptag, 1.0, tab);
                        if (lane == L) nev = n;
                    }
                    lds_sync<true>();
                    if (j < N) {
#pragma unroll
                        for (int c = 0; c < C; ++c) x[c] = (double)rcur[j * C + c];
                    }
                }
            }
            if (j < N) {
#pragma unroll
                for (int c = 0; c < C; ++c) rcur[j * C + c] = (int32_t)x[c];
                events += (unsigned long long)nev;
            }
            EPIPF_FUSED_MARK(2);
            weigh(x);
            __syncthreads();                             // this step's states and weights before the next step
            EPIPF_FUSED_MARK(4);
        } else {
            // gather (:195-199) into this step's rows, then W lanes per particle
            if (pt) {
                const int anc = draw_ancestor();
                if (j < N) {
#pragma unroll
                    for (int c = 0; c < C; ++c) rcur[j * C + c] = rprev[anc * C + c];
                }
            }
            __syncthreads();
            EPIPF_FUSED_MARK(1);
            double x[C];
            int nev = 0;
            if (pl < N) {                                // group-uniform
                double x0[C];
#pragma unroll
                for (int c = 0; c < C; ++c) x0[c] = (double)rcur[pl * C + c];
                nev = group_propagate<MODEL, G, W, 1, NoDays, true>(x0, x, cp, (uint32_t)pl, ptag, 1.0, tab,
                                                                    xch + wave * 64);
                if (nev < 0)                             // a clock decision within the certified bound (rare)
                    nev = group_propagate<MODEL, G, W, 1, NoDays, false>(x0, x, cp, (uint32_t)pl, ptag, 1.0, tab,
                                                                         xch + wave * 64);
            }
            __syncthreads();                             // every group has read its parent row
            EPIPF_FUSED_MARK(2);
            if (pl < N && gl == 0) {
#pragma unroll
                for (int c = 0; c < C; ++c) rcur[pl * C + c] = (int32_t)x[c];
                events += (unsigned long long)nev;
            }
            __syncthreads();
            EPIPF_FUSED_MARK(3);
            if (pt) {
                double xs[C];
#pragma unroll
                for (int c = 0; c < C; ++c) xs[c] = j < N ? (double)rcur[j * C + c] : 0.0;
                weigh(xs);
            }
            __syncthreads();
            EPIPF_FUSED_MARK(4);
        }
    }
#ifdef EPIPF_PHASE_TIMING
    if (tid == 0 && blockIdx.x == 0)
        printf("FUSED T=%d N=%d W=%d cycles: scan %llu resample %llu ssa %llu writeback %llu weights %llu (sum over steps)\n",
               T, N, W, fph[0], fph[1], fph[2], fph[3], fph[4]);
#endif
    if (a.count_events) {
        unsigned long long e = events;
        for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
        if (lane == 0) atomicAdd(counter_slot(a.counters), e);
    }
}

// launch table: W lanes per particle (1, 2, 4, 8, 16), one workgroup of fused_threads(N, W) threads per chain
template <int MODEL, int G, int OBS, int W>
static void launch_fused_t(const StepArgs& a, int n_chains, int threads, size_t lds, hipStream_t s) {
    hipLaunchKernelGGL((pf_filter_wg_kernel<MODEL, G, OBS, W>), dim3(n_chains), dim3(threads), lds, s, a);
}

template <int MODEL, int G, int OBS>
static FusedFn pick_fused_w(int W) {
    switch (W) {
        case 1: return launch_fused_t<MODEL, G, OBS, 1>;
        case 2: return launch_fused_t<MODEL, G, OBS, 2>;
        case 4: return launch_fused_t<MODEL, G, OBS, 4>;
        case 8: return launch_fused_t<MODEL, G, OBS, 8>;
        case 16: return launch_fused_t<MODEL, G, OBS, 16>;
    }
    return nullptr;
}

template <int MODEL, int G>
static FusedFn pick_fused_obs(int obs, int W) {
    return obs == kBinomial ? pick_fused_w<MODEL, G, kBinomial>(W) : pick_fused_w<MODEL, G, kNormal>(W);
}

// per-model tables, one translation unit each (parallel builds)
FusedFn fused_launcher_sir(int model, int obs, int W);
FusedFn fused_launcher_sub(int G, int obs, int W);
FusedFn fused_launcher_sub2(int G, int obs, int W);

}  // namespace epipf
