// epipf_kernels.hip -- the particle-filter kernels for MI355X (gfx950) and their launchers.
//
// One filter step (pmcmc.py:177-231) is ONE kernel launch, batched over independent chains: a 1-D grid of
// (chain, particle block of WG lanes) pairs, one particle per lane, placed so that each chain's blocks share one
// XCD's L2 (step_block, epipf_step.hpp; EPIPF_XCD_MAP=0: the 2-D grid y = chain, x = block):
//
//   step p:  [scan of the previous step's block sums in LDS -> total, log-likelihood]
//            [multinomial draw U_j -> certified two-level CDF search -> ancestor a_j]   (pmcmc.py:183-193)
//            [gather parent state hidden[p-1][a_j] -> Gillespie SSA over [0,1]]          (pmcmc.py:195-220)
//            [store hidden[p][j]; weight against Y[p]; in-block scan; block sum]         (pmcmc.py:178-181, next step)
//
// so the weights, the in-block CDF and the block sums of step p are produced by the same lanes that
// produced the states, and the next launch only reads them.  The init kernel draws the Poisson initial
// states (pmcmc.py:156-175) and the first weights.
#include "epipf_step.hpp"
#include <algorithm>

#include <cstdio>

#include "epipf_internal.hpp"

#ifndef EPIPF_STEP_WAVES
#define EPIPF_STEP_WAVES 1   // minimum waves per SIMD asked of the step kernel's register allocation
#endif

namespace epipf {

template <int MODEL, int G, int OBS, int WG>
__global__ __launch_bounds__(WG) void pf_init_kernel(StepArgs a) {
    using Sh = Shape<MODEL, G>;
    constexpr int C = Sh::C;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const BlockPos bp = step_block(a);
    const int chain = bp.chain;
    // a.wg particles per block: WG (one lane each), or fewer for the lane-group runs' smaller blocks (the lanes past
    // a.wg hold no particle and weigh 0 in the scan)
    const bool mine = (int)threadIdx.x < a.wg;
    const int j = bp.b * a.wg + (int)threadIdx.x;
    const ChainParam cp = a.cp[chain];
    // the chain's status for this run: skipped or running (the step kernels read it; a degenerate step sets 1)
    if (bp.b == 0 && threadIdx.x == 0) a.status[chain] = cp.skip ? kStatusSkipped : kStatusOk;
    if (cp.skip) return;
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = 0.0;
    if (mine && j < a.N) {
        init_particle<MODEL, G>(a, cp, j, x);                  // pmcmc.py:156-175
        int32_t* h = a.hidden + (size_t)chain * a.hist_stride + (size_t)j * C;
#pragma unroll
        for (int c = 0; c < C; ++c) h[c] = (int32_t)x[c];
        a.ancestry[(size_t)chain * a.anc_stride + j] = 0;
    }
    if (bp.b == 0 && threadIdx.x == 0) a.log_zeta[(size_t)chain * a.T] = 0.0;
    if (a.T > 1) {
        double w = 0.0;
        if (mine && j < a.N)
            w = particle_weight<MODEL, G, OBS>(x, a.Y, cp, a.cp + chain, a.lf, a.lf_max,
                                               a.hidden + (size_t)chain * a.hist_stride + (size_t)j * C);
        const size_t wbase = (size_t)chain * a.wstride;            // buffer 0
        const double loc = block_inclusive_scan<WG>(w, smem);
        if (mine) {
            a.wraw[wbase + j] = w;
            a.wloc[wbase + j] = loc;
        }
        if ((int)threadIdx.x == a.wg - 1) a.bsum[(size_t)chain * a.bstride + bp.b] = loc;
    }
}

template <int MODEL, int G, int OBS, int WG>
__global__ __launch_bounds__(WG, EPIPF_STEP_WAVES) void pf_step_kernel(StepArgs a, int p) {
    using Sh = Shape<MODEL, G>;
    constexpr int C = Sh::C;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    static_assert(WG == 64, "one wave per block (scan_segments)");
    LogTab* tab = reinterpret_cast<LogTab*>(smem);       // 128 x 16 B log table (first: 16-B aligned)
    double* red = smem + 2 * kLogTabEntries;             // WG/64 (+pad)
    double* seg_start = red + 16;                        // S = 1: bsum [B] then bpex [B + WG]; else nseg + nseg
    double* seg_end = seg_start + a.nseg;
    const BlockPos bp = step_block(a);
    const int chain = bp.chain;
    const int tid = threadIdx.x;
    const int j = bp.b * WG + tid;
    if (a.status[chain] != 0) return;
    const ChainParam cp = a.cp[chain];
    const int prev = (p - 1) & 1, cur = p & 1;
    const size_t wprev = ((size_t)prev * a.max_chains + chain) * a.wstride;
    const size_t wcur = ((size_t)cur * a.max_chains + chain) * a.wstride;
    const size_t bprev = ((size_t)prev * a.max_chains + chain) * a.bstride;
    const size_t bcur = ((size_t)cur * a.max_chains + chain) * a.bstride;

    // (b) likelihood: zetas[p] = zetas[p-1] * mean(w)  (pmcmc.py:183), kept in log space
    // S = 1 (B <= kMaxSegments): the block sums and their exclusive prefix stay in LDS; else segment ends only
    const double total = (a.seg == 1) ? scan_block_sums<WG>(a.bsum + bprev, a.B, seg_start + a.B, seg_start, red)
                                      : scan_segments(a.bsum + bprev, a.B, a.seg, a.nseg, seg_start, seg_end);
    if (!(total > 0.0)) {  // all weights 0 or NaN: numpy raises ValueError -> (None, None, None), :187-192
        if (bp.b == 0 && tid == 0) {
            a.status[chain] = 1;
            a.log_zeta[(size_t)chain * a.T + p] = -__builtin_inf();
        }
        return;
    }
    if (bp.b == 0 && tid == 0)
        a.log_zeta[(size_t)chain * a.T + p] = a.log_zeta[(size_t)chain * a.T + p - 1] + log(total / (double)a.N);

    int nev = 0, iters = 0, exact = 0;
    double w = 0.0;
    // (d) multinomial (or systematic) draw and certified search, pmcmc.py:188-190
    double U = 0.0;
    int anc = 0;
    bool certified = true, ambiguous = false;
    if (j < a.N) {
        const uint32_t rtag = ((uint32_t)p & 0xFFFFFFu) | kDomainResample;
        if (a.resample_mode == 0) {
            const Block r = philox(0u, (uint32_t)j, rtag, cp.f, cp.k0, cp.k1);
            U = u01(r.x, r.y);
        } else {
            const Block r = philox(0u, 0u, rtag, cp.f, cp.k0, cp.k1);
            U = ((double)j + u01(r.x, r.y)) / (double)a.N;
        }
        if (a.seg == 1)
            anc = resample_search<WG>(U, seg_start + a.B, seg_start, a.B, total, a.wloc + wprev, a.N, a.cert_k,
                                      certified, a.ref_k, ambiguous);
        else
            anc = resample_search_seg(U, seg_start, seg_end, a.nseg, a.seg, a.bsum + bprev, a.B, total,
                                      a.wloc + wprev, WG, a.N, a.cert_k, certified, a.ref_k, ambiguous);
    }
    // reference-ambiguous draws (rare: ~1e-8 of draws at config 2; every uncertified one included), counted with
    // the other device counters (EPIPF_PROFILE_COUNTERS: bench.py's untimed counters iteration, the parity tests)
    if (ambiguous) atomicAdd(counter_slot(a.counters) + 6, 1ull);
    if (__any(!certified)) {   // wave-uniform: the whole wave resolves its uncertified draws exactly
        const int e = resample_exact_wave(!certified, U, a.wraw + wprev, a.N);
        if (!certified) {
            anc = e;
            atomicAdd(counter_slot(a.counters) + 1, 1ull);
        }
    }
    // (f) gather the parent state, (g) propagate over [0, 1], :195-220: the certified f32 loop, then the exact path
    // for the lanes it hands back.  The exact path's log table is copied to LDS only by waves that need it (~1% at
    // config 2): one wave per block, so the wave-uniform test is block-uniform and the barriers are legal.
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = 0.0;
    const uint32_t ptag = ((uint32_t)p & 0xFFFFFFu) | kDomainSSA;
    bool fast_ok = false, eligible = false;
    if (j < a.N) {
        anc = checked_index(anc, a.N);
        a.ancestry[(size_t)chain * a.anc_stride + (size_t)p * a.N + j] = anc;   // :193
        const int32_t* hp = a.hidden + (size_t)chain * a.hist_stride + ((size_t)(p - 1) * a.N + anc) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = (double)hp[c];
        fast_ok = fast_propagate<MODEL, G>(x, cp, (uint32_t)j, ptag, 1.0, nev, iters, eligible);
    }
    exact = (j < a.N && !fast_ok) ? 1 : 0;
    if (__any(exact != 0)) {
        for (int i = tid; i < kLogTabEntries; i += WG) tab[i] = a.logtab[i];
        __syncthreads();
        // lanes the f32 loop could not run (population or rates out of its range): the exact loop, per lane
        if (exact && !eligible) {
            int ex_iters = 0;
            nev = exact_propagate<MODEL, G>(x, cp, (uint32_t)j, ptag, 1.0, tab, ex_iters);
            iters += ex_iters;
        }
        // lanes it stopped at the step boundary: replayed one at a time by the whole wave (coop_replay).  The lanes'
        // states wait in their output rows meanwhile (x is not live across the replay: registers, occupancy).
        unsigned long long pend = __ballot(exact != 0 && eligible);
        if (pend) {
            int32_t* hrow = a.hidden + (size_t)chain * a.hist_stride + (size_t)p * a.N * C;
            if (j < a.N) {
#pragma unroll
                for (int c = 0; c < C; ++c) hrow[(size_t)j * C + c] = (int32_t)x[c];   // replayed lanes: the parent
            }
            __syncthreads();                                          // one wave per block: orders the rows
            while (pend) {
                const int L = (int)__builtin_ctzll(pend);
                pend &= pend - 1ull;
                const uint32_t jl = __builtin_amdgcn_readlane((uint32_t)j, L);
                const int n = coop_replay<MODEL, G>(hrow + (size_t)jl * C, cp, jl, ptag, 1.0, tab);
                if (tid == L) nev = n;
            }
            __syncthreads();
            if (j < a.N) {
#pragma unroll
                for (int c = 0; c < C; ++c) x[c] = (double)hrow[(size_t)j * C + c];
            }
        }
    }
    if (j < a.N) {
        int32_t* hc = a.hidden + (size_t)chain * a.hist_stride + ((size_t)p * a.N + j) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) hc[c] = (int32_t)x[c];                        // :222-231
        // (a) weights of the new state against Y[p], used by step p+1, :178-181
        if (p + 1 < a.T) w = particle_weight<MODEL, G, OBS>(x, a.Y + (size_t)p * Sh::K, cp, a.cp + chain, a.lf, a.lf_max, hc);
    }
    if (a.count_events) {  // accepted events; lane-iterations; wave-iterations x 64 (lane utilisation)
        unsigned long long e = (unsigned long long)nev, li = (unsigned long long)iters;
        int wmax = iters;
        for (int o = 32; o > 0; o >>= 1) {
            e += __shfl_xor(e, o, 64);
            li += __shfl_xor(li, o, 64);
            wmax = max(wmax, __shfl_xor(wmax, o, 64));
        }
        const unsigned long long ex = __ballot(exact != 0);
        if ((tid & 63) == 0) {
            unsigned long long* slot = counter_slot(a.counters);
            atomicAdd(slot, e);
            atomicAdd(slot + 2, li);
            atomicAdd(slot + 3, 64ull * (unsigned long long)wmax);
            atomicAdd(slot + 4, (unsigned long long)__popcll(ex));        // lanes on the exact SSA loop
            atomicAdd(slot + 5, ex ? 1ull : 0ull);                        // waves with at least one
        }
    }
    if (p + 1 < a.T) {
        const double loc = block_inclusive_scan<WG>(w, red);
        a.wraw[wcur + j] = w;
        a.wloc[wcur + j] = loc;
        if (tid == WG - 1) a.bsum[bcur + bp.b] = loc;
    }
}

// particle_path_sampler, pmcmc.py:236-248 (one lane per chain; T dependent loads)
__global__ void path_sample_kernel(PathArgs a) {
    const int chain = blockIdx.x * blockDim.x + threadIdx.x;
    if (chain >= a.n_chains) return;
    int32_t* out = a.traj + (size_t)chain * a.T * a.C;
    if (a.status[chain] != 0) {                      // degenerate or skipped in the last run: its history rows may be
        for (int i = 0; i < a.T * a.C; ++i) out[i] = 0;   // stale or unwritten, so it is not walked (zeros returned)
        return;
    }
    const int pick = a.chosen ? a.chosen[chain] : a.cp[chain].chosen;   // epipf_path_sample / epipf_run_sampled
    if (pick < 0) {                                  // no path asked of this chain
        for (int i = 0; i < a.T * a.C; ++i) out[i] = 0;
        return;
    }
    int chosen = checked_index(pick, a.N);
    const int32_t* hid = a.hidden + (size_t)chain * a.hist_stride;
    const int32_t* anc = a.ancestry + (size_t)chain * a.anc_stride;
    for (int c = 0; c < a.C; ++c) out[(size_t)(a.T - 1) * a.C + c] = hid[((size_t)(a.T - 1) * a.N + chosen) * a.C + c];
    for (int p = a.T - 2; p >= 0; --p) {
        chosen = checked_index(anc[(size_t)p * a.N + chosen], a.N);       // ancestry[p], as the reference
        for (int c = 0; c < a.C; ++c) out[(size_t)p * a.C + c] = hid[((size_t)p * a.N + chosen) * a.C + c];
    }
}

template <int MODEL, int G>
__global__ __launch_bounds__(256) void simulate_kernel(SimArgs a) {
    constexpr int C = Shape<MODEL, G>::C;
    __shared__ LogTab tab[kLogTabEntries];
    if (threadIdx.x < kLogTabEntries) tab[threadIdx.x] = a.logtab[threadIdx.x];
    __syncthreads();
    const int j = blockIdx.x * 256 + threadIdx.x;
    int nev = 0, iters = 0;
    if (j < a.n) {
        double x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = (double)a.in[(size_t)j * C + c];
        int exact = 0;
        nev = ssa_propagate<MODEL, G>(x, *a.cp, (uint32_t)j, (a.step & 0xFFFFFFu) | kDomainSSA, a.tmax, tab, iters, exact);
#pragma unroll
        for (int c = 0; c < C; ++c) a.out[(size_t)j * C + c] = (int32_t)x[c];
    }
    unsigned long long e = (unsigned long long)nev;
    for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(a.events, e);
}

// Full-path SSA (gillespie_algo.py *_simulate with last_values_only=False): the exact event loop -- whose clock is
// the reference's bit for bit (SsaState) -- storing every event's time and state (:68-70).  Same draws and same
// final state as simulate_kernel.  Lanes of a wave step together (the event index is wave-uniform), so event k's
// stores of the wave land in contiguous [k][...][lane] rows.
template <int MODEL, int G>
__global__ __launch_bounds__(256) void simulate_path_kernel(SimPathArgs a) {
    constexpr int C = Shape<MODEL, G>::C;
    __shared__ LogTab tab[kLogTabEntries];
    if (threadIdx.x < kLogTabEntries) tab[threadIdx.x] = a.logtab[threadIdx.x];
    __syncthreads();
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= a.n) return;
    const ChainParam cp = *a.cp;
    const uint32_t ptag = (a.step & 0xFFFFFFu) | kDomainSSA;
    double x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = (double)a.in[(size_t)j * C + c];
    SsaState<MODEL, G> st;
    st.load(x, cp);
    double t = 0.0;
    uint32_t k = 0;
    int nev = 0;
    bool alive = st.active();
    while (alive) {
        const Block r = philox(__builtin_amdgcn_readfirstlane(k), (uint32_t)j, ptag, cp.f, cp.k0, cp.k1);
        ++k;
        const bool ev = st.event(r, t, a.tmax, cp, tab);
        if (ev) {
            if (nev < a.cap) {
                double xs[C];
                st.save(xs);
                a.times[(size_t)nev * a.n + j] = t;
#pragma unroll
                for (int c = 0; c < C; ++c) a.states[((size_t)nev * C + c) * a.n + j] = (int32_t)xs[c];
            }
            ++nev;
        }
        alive = ev && st.active();
    }
    st.save(x);
#pragma unroll
    for (int c = 0; c < C; ++c) a.final_state[(size_t)j * C + c] = (int32_t)x[c];
    a.nev[j] = nev;
}

// Standalone resampler over caller-supplied weights and uniforms (same scan + search code as the filter).
template <int WG>
__global__ __launch_bounds__(WG) void resample_scan_kernel(ResampleArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int j = blockIdx.x * WG + threadIdx.x;
    const double w = (j < a.N) ? a.w[j] : 0.0;
    const double loc = block_inclusive_scan<WG>(w, smem);
    a.wraw[j] = w;
    a.wloc[j] = loc;
    if (threadIdx.x == WG - 1) a.bsum[blockIdx.x] = loc;
}

template <int WG>
__global__ __launch_bounds__(WG) void resample_search_kernel(ResampleArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* red = smem + 2 * kLogTabEntries;
    double* bsum = red + 16;
    double* bpex = bsum + a.B;
    const int j = blockIdx.x * WG + threadIdx.x;
    const double total = scan_block_sums<WG>(a.bsum, a.B, bpex, bsum, red);
    if (!(total > 0.0)) {
        if (j == 0) *a.status = 1;
        return;
    }
    const double U = (j < a.N) ? a.u[j] : 0.0;
    bool certified = true, ambiguous = false;      // standalone resampler: no reference weights, ref_k = 0
    int anc = 0;
    if (j < a.N) anc = resample_search<WG>(U, bpex, bsum, a.B, total, a.wloc, a.N, a.cert_k, certified, 0.0, ambiguous);
    if (__any(!certified)) {
        const int e = resample_exact_wave(!certified, U, a.wraw, a.N);
        if (!certified) {
            anc = e;
            atomicAdd(a.fallbacks, 1ull);
        }
    }
    if (j < a.N) a.out[j] = checked_index(anc, a.N);
}

// ------------------------------------------------------------------------------- launchers
// blocks per prefix segment: the smallest power of two with at most kMaxSegments segments
int prefix_segment(int B) {
    int S = 1;
    while ((B + S - 1) / S > kMaxSegments) S <<= 1;
    return S;
}

size_t step_lds_bytes(int B, int wg) { return step_lds_bytes_seg(B, prefix_segment(B), wg); }

size_t step_lds_bytes_seg(int B, int S, int wg) {
    if (S == 1) return sizeof(LogTab) * kLogTabEntries + sizeof(double) * (size_t)(16 + B + B + wg);
    return sizeof(LogTab) * kLogTabEntries + sizeof(double) * (size_t)(16 + 2 * ((B + S - 1) / S));
}

static size_t resample_lds_bytes(int B, int wg) {
    return sizeof(LogTab) * kLogTabEntries + sizeof(double) * (size_t)(16 + B + B + wg);
}

template <int MODEL, int G, int OBS, int WG>
static hipError_t launch_filter_t(const StepArgs& a, int n_chains, const FilterStreams& fs) {
    constexpr int C = Shape<MODEL, G>::C;
    // Chains are independent, so chain groups advance through their T steps on separate streams: one group's
    // end-of-launch tail (the last, partial round of waves) overlaps the other groups' launches.
    const size_t lds = step_lds_bytes(a.B, WG);
    const int S = std::max(1, std::min(fs.n, n_chains));
    // W lanes per particle (runs too small to fill the chip): the lane-group step kernel, epipf_group.hip
    const GroupStepFn group = a.lanes > 1 ? group_step_launcher(MODEL, G, OBS, a.lanes, a.lane_events) : nullptr;
    if (a.lanes > 1 && !group) return hipErrorInvalidValue;
    const size_t glds = group ? group_lds_bytes(a.B, a.seg, C, a.lanes, a.lane_events, a.wg) : 0;
    for (int g = 0; g < S; ++g) {
        StepArgs ag = a;
        ag.chain0 = (int)((long)n_chains * g / S);
        const int n_g = (int)((long)n_chains * (g + 1) / S) - ag.chain0;
        const hipStream_t s = fs.s[g];
        // the 1-D XCD-aware grid while its work-items fit HIP's 32-bit x extent (with room for lane-group blocks)
        ag.xcd_map = a.xcd_map && (long)a.B * n_g * WG * std::max(1, a.lanes) < (1L << 31);
        const dim3 grid = ag.xcd_map ? dim3(a.B * n_g) : dim3(a.B, n_g), block(WG);
        if (g == 0 && fs.ev_init) (void)hipEventRecord(fs.ev_init, s);
        hipLaunchKernelGGL((pf_init_kernel<MODEL, G, OBS, WG>), grid, block, lds, s, ag);
        if (g == 0 && fs.ev_step0) (void)hipEventRecord(fs.ev_step0, s);
        if (fs.g_begin[g]) (void)hipEventRecord(fs.g_begin[g], s);
        for (int p = 1; p < a.T; ++p) {
#ifdef EPIPF_ROCTX
            char msg[48];
            snprintf(msg, sizeof msg, "filter step %d group %d", p, g);
            EPIPF_RANGE_PUSH(msg);
#endif
            if (group) group(ag, p, grid, glds, s);
            else hipLaunchKernelGGL((pf_step_kernel<MODEL, G, OBS, WG>), grid, block, lds, s, ag, p);
            EPIPF_RANGE_POP();
        }
        if (fs.g_end[g]) (void)hipEventRecord(fs.g_end[g], s);
        if (g > 0) (void)hipEventRecord(fs.join[g], s);
    }
    for (int g = 1; g < S; ++g) (void)hipStreamWaitEvent(fs.s[0], fs.join[g], 0);
    if (fs.ev_end) (void)hipEventRecord(fs.ev_end, fs.s[0]);
    return hipGetLastError();
}

template <int MODEL, int G, int WG>
static hipError_t launch_obs(const StepArgs& a, int obs, int n_chains, const FilterStreams& fs) {
    return obs == kBinomial ? launch_filter_t<MODEL, G, kBinomial, WG>(a, n_chains, fs)
                            : launch_filter_t<MODEL, G, kNormal, WG>(a, n_chains, fs);
}

template <int WG>
static hipError_t launch_model(const StepArgs& a, int model, int G, int obs, int n_chains, const FilterStreams& fs) {
    switch (model) {
        case kSIR: return launch_obs<kSIR, 1, WG>(a, obs, n_chains, fs);
        case kSEIR: return launch_obs<kSEIR, 1, WG>(a, obs, n_chains, fs);
        case kSubgroups:
            switch (G) {
                case 1: return launch_obs<kSubgroups, 1, WG>(a, obs, n_chains, fs);
                case 2: return launch_obs<kSubgroups, 2, WG>(a, obs, n_chains, fs);
                case 3: return launch_obs<kSubgroups, 3, WG>(a, obs, n_chains, fs);
                case 4: return launch_obs<kSubgroups, 4, WG>(a, obs, n_chains, fs);
            }
            break;
        case kSubgroups2:
            switch (G) {
                case 1: return launch_obs<kSubgroups2, 1, WG>(a, obs, n_chains, fs);
                case 2: return launch_obs<kSubgroups2, 2, WG>(a, obs, n_chains, fs);
                case 3: return launch_obs<kSubgroups2, 3, WG>(a, obs, n_chains, fs);
                case 4: return launch_obs<kSubgroups2, 4, WG>(a, obs, n_chains, fs);
            }
            break;
    }
    return hipErrorInvalidValue;
}

// 64-thread init and step blocks; a.wg particles per block: 64, or kGroupBlock for lane-group runs of W >= 8
hipError_t launch_filter(const StepArgs& a, int model, int G, int obs, int n_chains, const FilterStreams& fs) {
    if (!(a.wg == 64 || (a.wg == kGroupBlock && a.lanes >= 8))) return hipErrorInvalidValue;
    return launch_model<64>(a, model, G, obs, n_chains, fs);
}

hipError_t launch_path_sample(const PathArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(path_sample_kernel, dim3((a.n_chains + 63) / 64), dim3(64), 0, s, a);
    return hipGetLastError();
}

template <int MODEL, int G>
static void sim_t(const SimArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((simulate_kernel<MODEL, G>), dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}

hipError_t launch_simulate(const SimArgs& a, int model, int G, hipStream_t s) {
    switch (model) {
        case kSIR: sim_t<kSIR, 1>(a, s); break;
        case kSEIR: sim_t<kSEIR, 1>(a, s); break;
        default:
            switch (G) {
                case 1: sim_t<kSubgroups, 1>(a, s); break;
                case 2: sim_t<kSubgroups, 2>(a, s); break;
                case 3: sim_t<kSubgroups, 3>(a, s); break;
                case 4: sim_t<kSubgroups, 4>(a, s); break;
                default: return hipErrorInvalidValue;
            }
    }
    return hipGetLastError();
}

template <int MODEL, int G>
static void sim_path_t(const SimPathArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((simulate_path_kernel<MODEL, G>), dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}

hipError_t launch_simulate_path(const SimPathArgs& a, int model, int G, hipStream_t s) {
    switch (model) {
        case kSIR: sim_path_t<kSIR, 1>(a, s); break;
        case kSEIR: sim_path_t<kSEIR, 1>(a, s); break;
        default:
            switch (G) {
                case 1: sim_path_t<kSubgroups, 1>(a, s); break;
                case 2: sim_path_t<kSubgroups, 2>(a, s); break;
                case 3: sim_path_t<kSubgroups, 3>(a, s); break;
                case 4: sim_path_t<kSubgroups, 4>(a, s); break;
                default: return hipErrorInvalidValue;
            }
    }
    return hipGetLastError();
}

hipError_t launch_resample(const ResampleArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(resample_scan_kernel<256>, dim3(a.B), dim3(256), sizeof(double) * 16, s, a);
    hipLaunchKernelGGL(resample_search_kernel<256>, dim3(a.B), dim3(256), resample_lds_bytes(a.B, 256), s, a);
    return hipGetLastError();
}

}  // namespace epipf
