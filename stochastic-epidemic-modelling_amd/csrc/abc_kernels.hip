// abc_kernels.hip -- ABC rejection sampling (abc_algo.py:17-109) on MI355X.
//
// abc_trials_kernel  one lane per trial t: prior draw (:35-36), initial counts (:38-39), the full SIR path
//                    (:40-45 -> gillespie_algo.py:10-75) recorded straight into the daily table the reference
//                    assembles afterwards (:47-88).
// abc_distance_kernel the distance (:89-94) with numpy's pairwise mean, one lane per trial.
// abc_select_kernel  the first `need` trials with !(distance > threshold), in trial order (:30-33 -- the
//                    reference's while loop accepts trials in exactly that order).
// abc_gather_kernel  accepted thetas and [T][4] trajectories (day, S, I, R) into the output slots.
//
// The day table needs no event history: day d holds the state after every event with time <= d (ceil(time)
// groups events into day rows, missing days repeat the previous row), so a lane writes day rows as its clock
// passes integer days.  An event past day T-1 only changes row T, which :88 truncates away: the walk stops.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "abc_device.hpp"
#include "epipf_group.hpp"
#include "epipf_internal.hpp"

namespace epipf {

__device__ __forceinline__ void write_day(int32_t* col, size_t n, int d, double S, double I, double R) {
    int32_t* p = col + (size_t)d * 3 * n;
    p[0] = (int32_t)S;
    p[n] = (int32_t)I;
    p[2 * n] = (int32_t)R;
}

// Trial t's prior (abc_algo.py:35-36) and initial counts (:38-39): theta in cp, counts in x
__device__ __forceinline__ void abc_trial_start(const AbcArgs& a, uint32_t t, ChainParam& cp, double* x) {
    const Block rp = philox(0u, t, kDomainAbcPrior, a.f, a.k0, a.k1);
    cp.theta[0] = a.prior_lo[0] + a.prior_rng[0] * u01(rp.x, rp.y);             // abc_algo.py:35
    cp.theta[1] = a.prior_lo[1] + a.prior_rng[1] * u01(rp.z, rp.w);             // :36
#pragma unroll
    for (int c = 0; c < 3; ++c) {                                               // :38-39
        const Block r = philox((uint32_t)c, t, kDomainAbcInit, a.f, a.k0, a.k1);
        x[c] = (double)poisson_mode_inversion(a.lam[c], u01(r.x, r.y), a.pm[c]);
    }
}

// The trial's SIR path from x over [0, T-1] (gillespie_algo.py:10-75 with the reference-exact clock), writing each
// day row as the clock passes it: day d holds the state after every event with time <= d.  `write`: this lane
// stores the rows (the lane-group kernel runs it on every lane of a group, one of which writes).  Returns the events;
// x holds the final state, day the first row not yet written, iters the loop iterations.
// Early rejection: `acc` sums |I_d - Y_I,d| + |R_d - Y_R,d| over the rows passed (the distance's terms,
// abc_algo.py:12); once it exceeds `reject_sum` the distance of the full table is provably above the threshold
// (epipf_abc's bound) and the walk stops with `rejected` set -- the rest of the path cannot change the
// trial's fate, and a rejected trial's table is never read.  reject_sum = INFINITY: never.
__device__ __forceinline__ int abc_exact_path(double* x, const ChainParam& cp, uint32_t t, const AbcArgs& a,
                                              const LogTab* __restrict__ tab, int32_t* col, bool write, int& day,
                                              double& next_day, int& iters, double reject_sum, bool& rejected) {
    const size_t n = (size_t)a.n;
    SsaState<kSIR, 1> st;
    st.load(x, cp);
    const double R0 = x[2];
    const double last_day = a.last_day;
    double clock = 0.0;
    uint32_t k = 0;
    int nev = 0;
    bool alive = st.active();
    double acc = 0.0;
    rejected = false;
    Block rn{0u, 0u, 0u, 0u};
    if (alive) rn = philox(0u, t, kDomainAbcSsa, a.f, a.k0, a.k1);
    while (alive) {                          // every lane enters at k = 0: k stays wave-uniform
        const Block r = rn;
        ++k;
        rn = philox(__builtin_amdgcn_readfirstlane(k), t, kDomainAbcSsa, a.f, a.k0, a.k1);
        const double S0 = st.S, I0 = st.I;
        const int rec0 = st.nrec;
        const bool ev = st.template event<true>(r, clock, last_day, cp, tab);   // false: the event lands after day T-1
        if (ev) {
            ++nev;
            while (next_day < clock) {                                   // days the event does not reach
                const double R = R0 + (double)rec0;
                if (write) write_day(col, n, day, S0, I0, R);
                acc += fabs(I0 - a.Y[3 * day + 1]) + fabs(R - a.Y[3 * day + 2]);
                ++day;
                next_day += 1.0;
            }
            rejected = acc > reject_sum;
        }
        alive = ev && st.active() && !rejected;
    }
    st.save(x);
    iters = (int)k;
    return nev;
}

// No minimum-waves bound: the loop keeps its 65 VGPRs (7 waves per SIMD) instead of spilling to fit 8, 1.8% faster
// with early rejection on (profiles/r3t_abc_waves_ab.txt)
__global__ __launch_bounds__(256) void abc_trials_kernel(AbcArgs a) {
    __shared__ LogTab tab[kLogTabEntries];
    if (threadIdx.x < kLogTabEntries) tab[threadIdx.x] = a.logtab[threadIdx.x];
    __syncthreads();
    const int g = a.g0 + (int)(blockIdx.x * 256 + threadIdx.x);    // sorted position (from g0: the lane groups below)
    int nev = 0, iters = 0;
    if (g < a.n) {
        const int i = a.perm ? a.perm[g] : g;
        const uint32_t t = a.t0 + (uint32_t)i;
        const size_t n = (size_t)a.n;
        ChainParam cp;
        double x[3];
        abc_trial_start(a, t, cp, x);
        int32_t* col = a.days + i;
        int day = 0;
        double next_day = 0.0;
        bool rejected;
        nev = abc_exact_path(x, cp, t, a, tab, col, true, day, next_day, iters, a.reject_sum, rejected);
        if (rejected) col[0] = -1;                                   // row 0's S: abc_distance_kernel's marker
        else for (; day < a.T; ++day) write_day(col, n, day, x[0], x[1], x[2]);
        a.theta[i] = cp.theta[0];
        a.theta[n + i] = cp.theta[1];
    }
    if (a.count) {
        unsigned long long e = (unsigned long long)nev, li = (unsigned long long)iters;
        int wmax = iters;
        for (int o = 32; o > 0; o >>= 1) {
            e += __shfl_xor(e, o, 64);
            li += __shfl_xor(li, o, 64);
            wmax = max(wmax, __shfl_xor(wmax, o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            unsigned long long* slot = counter_slot(a.counters);
            atomicAdd(slot, e);
            atomicAdd(slot + 2, li);
            atomicAdd(slot + 3, 64ull * (unsigned long long)wmax);
        }
    }
}

// Lane groups for the longest trials (round 3).  Sorted longest first, the first `group_end` trials are the
// explosive epidemics (~10^4 events each, a quarter of the trials holding ~70% of the events at the reference's
// setting): on one lane each they set the launch's length, a lone wave's dependent event loop.  Here W lanes run
// one trial (epipf_group.hpp's group_propagate, the filter's lane-group SSA: bit-identical to the exact loop), the
// day rows written by the lane that holds the state before each day-crossing event.  Concurrent with the one-lane
// kernel over the rest (its own stream), which fills the SIMDs the groups leave idle.
// Early rejection on lane groups (round 4): each lane sums the distance terms of the day rows it writes
// (the rows of the events it owns); after every chunk the group adds its lanes' sums and stops once the total exceeds
// reject_sum -- the same proof as abc_exact_path's (any order of summing the non-negative terms fl(|x - y|) stays
// within (1 + u)^(2T + 2) of the exact sum), so a trial stopped here is rejected, and stopping one chunk later than
// the one-lane walk changes nothing the distance kernel reads (a rejected trial's table is never read).
struct AbcDays {
    static constexpr bool kOn = true;
    int32_t* col;
    size_t n;
    int day;
    double next_day;
    bool lead;                                  // group lane 0: writes on the exact path and the tail rows
    const AbcArgs* a;
    double acc = 0.0;                           // this lane's distance terms (rows it wrote)
    bool rejected = false;                      // group-uniform
    // event at clock tt (<= T-1): the rows of the days before it hold the state before the event (owner: this lane)
    template <class F>
    __device__ __forceinline__ void passed(double tt, bool owner, const F& before, const double* x0) {
        while (next_day < tt) {
            if (owner) {
                double xs[3] = {x0[0], x0[1], x0[2]};
                before.save(xs);
                write_day(col, n, day, xs[0], xs[1], xs[2]);
                acc += fabs(xs[1] - a->Y[3 * day + 1]) + fabs(xs[2] - a->Y[3 * day + 2]);   // abc_algo.py:12
            }
            ++day;
            next_day += 1.0;
        }
    }
    // after a chunk: the group's total against reject_sum (every lane of the group gets the same answer)
    template <int W>
    __device__ __forceinline__ bool reject_now() {
        double tot = acc;
#pragma unroll
        for (int o = W / 2; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        rejected = tot > a->reject_sum;
        return rejected;
    }
    // outside the f32 test's range: the one-lane kernel's exact loop (with its early rejection), rows by the lead lane
    __device__ __forceinline__ int exact(double* x, const ChainParam& cp, uint32_t t, uint32_t, double,
                                         const LogTab* __restrict__ tab) {
        int iters = 0;
        return abc_exact_path(x, cp, t, *a, tab, col, lead, day, next_day, iters, a->reject_sum, rejected);
    }
};

template <int W>
__global__ __launch_bounds__(256) void abc_trials_group_kernel(AbcArgs a) {
    __shared__ LogTab tab[kLogTabEntries];
    __shared__ double xch[4 * 64];                                 // the clock pass's tau exchange, one slice per wave
    if (threadIdx.x < kLogTabEntries) tab[threadIdx.x] = a.logtab[threadIdx.x];
    __syncthreads();
    const int gl = (int)(threadIdx.x & (W - 1));
    const int g = (int)((blockIdx.x * 256 + threadIdx.x) / W);     // sorted position, one trial per group
    int nev = 0;
    if (g < a.group_end) {                                         // whole groups: group_end is per group
        const int i = a.perm[g];
        const uint32_t t = a.t0 + (uint32_t)i;
        const size_t n = (size_t)a.n;
        ChainParam cp{};
        double x[3];
        abc_trial_start(a, t, cp, x);
        cp.thetaf[0] = (float)cp.theta[0];
        cp.thetaf[1] = (float)cp.theta[1];
        cp.f = a.f; cp.k0 = a.k0; cp.k1 = a.k1;
        cp.flags = kChainFastSsa;
        cp.clock_slack = 1.f;
        cp.band_slack = 1.f;
        AbcDays d{a.days + i, n, 0, 0.0, gl == 0, &a};
        double xf[3];
        nev = group_propagate<kSIR, 1, W, 1, AbcDays>(x, xf, cp, t, kDomainAbcSsa, a.last_day, tab,
                                                      xch + (threadIdx.x >> 6) * 64, &d);
        if (gl == 0) {
            if (d.rejected) d.col[0] = -1;                         // row 0's S: abc_distance_kernel's marker
            else for (; d.day < a.T; ++d.day) write_day(d.col, n, d.day, xf[0], xf[1], xf[2]);
            a.theta[i] = cp.theta[0];
            a.theta[n + i] = cp.theta[1];
        } else {
            nev = 0;                                               // counted once per trial
        }
    }
    if (a.count) {
        unsigned long long e = (unsigned long long)nev;
        for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(counter_slot(a.counters), e);
    }
}

// Length ordering.  A wave costs as much as its longest trial, and trial lengths are bimodal (extinction vs a
// full epidemic: lane use 0.33 on the reference's ABC setting), so lanes are assigned trials sorted by a
// predicted event count, longest first (the long waves dispatch first, the short ones fill the tail): the prior
// draw (one Philox block) and a forward-Euler integration of the deterministic SIR from the mean initial counts,
// dt = 1/4 day, up to day T-1.  Lane use 0.87, 2.1x fewer kernel cycles.  Only the lane
// assignment changes; every output is indexed by trial.
__global__ __launch_bounds__(256) void abc_predict_kernel(AbcArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const Block rp = philox(0u, a.t0 + (uint32_t)i, kDomainAbcPrior, a.f, a.k0, a.k1);
    const float beta = (float)(a.prior_lo[0] + a.prior_rng[0] * u01(rp.x, rp.y));
    const float gamma = (float)(a.prior_lo[1] + a.prior_rng[1] * u01(rp.z, rp.w));
    float S = (float)a.lam[0], I = (float)a.lam[1];
    const float N = (float)(a.lam[0] + a.lam[1] + a.lam[2]);
    const float bN = N > 0.f ? 0.25f * beta / N : 0.f, g4 = 0.25f * gamma;
    float events = 0.f;
    for (int s = 0; s < 4 * (a.T - 1) && I >= 0.5f; ++s) {
        const float inf = fminf(bN * S * I, S), rec = g4 * I;
        S -= inf;
        I += inf - rec;
        events += inf + rec;
    }
    a.sort_keys[0][i] = (uint32_t)fminf(events * 0.25f, 65535.f);
    a.sort_vals[0][i] = i;
}

size_t abc_sort_temp_bytes(int n) {
    size_t bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const int32_t*)nullptr, (int32_t*)nullptr, n, 0, 16);
    return bytes;
}

// distance_function (abc_algo.py:9-13, :89-94) of each trial's day table; a kernel of its own so the numpy
// pairwise recursion (function calls, stack) stays out of the SSA kernel's register budget.
// T <= 128 (one pairwise block) instantiates without any call.
template <bool DEEP>
__global__ __launch_bounds__(256) void abc_distance_kernel(AbcArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const size_t n = (size_t)a.n;
    const int32_t* col = a.days + i;
    if (col[0] < 0) {                                              // rejected early by abc_trials_kernel
        a.dist[i] = INFINITY;
        return;
    }
    const AbsDiff vi{col + n, 3 * n, a.Y + 1}, vr{col + 2 * n, 3 * n, a.Y + 2};
    const double dT = (double)a.T;
    const double si = DEEP ? pairwise_sum<kAbcPairwiseDepth>(vi, 0, a.T) : pairwise_leaf(vi, 0, a.T);
    const double sr = DEEP ? pairwise_sum<kAbcPairwiseDepth>(vr, 0, a.T) : pairwise_leaf(vr, 0, a.T);
    a.dist[i] = (si / dT + sr / dT) / 2.0;
}

// One workgroup walks the batch in 1024-trial chunks: ballot + per-wave popcounts give each accepted trial its
// rank; the walk ends once `need` trials are found.
__global__ __launch_bounds__(1024) void abc_select_kernel(AbcSelectArgs a) {
    __shared__ int wsum[16];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int base = 0;
    for (int c0 = 0; c0 < a.n && base < a.need; c0 += 1024) {
        const int i = c0 + (int)threadIdx.x;
        const bool acc = i < a.n && !(a.dist[i] > a.threshold);                // :30-33
        const unsigned long long m = __ballot(acc);
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = 0, tot = 0;
        for (int q = 0; q < 16; ++q) {
            off += q < w ? wsum[q] : 0;
            tot += wsum[q];
        }
        const int pos = base + off + __popcll(m & ((1ull << lane) - 1ull));
        if (acc && pos < a.need) a.idx[pos] = i;
        base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) *a.count = min(base, a.need);
}

__global__ __launch_bounds__(256) void abc_gather_kernel(AbcGatherArgs a, int max_count) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int s = g / a.T, d = g % a.T;
    if (s >= max_count || s >= *a.count) return;
    const size_t n = (size_t)a.n;
    const int i = a.idx[s];
    const int32_t* p = a.days + (size_t)d * 3 * n + i;
    double* o = a.traj + ((size_t)(a.slot0 + s) * a.T + d) * 4;
    o[0] = (double)d;                                                          // np.ceil(time) column
    o[1] = (double)p[0];
    o[2] = (double)p[n];
    o[3] = (double)p[2 * n];
    if (d == 0) {
        a.theta_out[(size_t)(a.slot0 + s) * 2] = a.theta[i];
        a.theta_out[(size_t)(a.slot0 + s) * 2 + 1] = a.theta[n + i];
    }
}

hipError_t launch_abc_trials(const AbcArgs& a0, hipStream_t s, hipStream_t s2, hipEvent_t fork, hipEvent_t join) {
    if (a0.n <= 0) return hipSuccess;
    AbcArgs a = a0;
    a.g0 = 0;
    if (a.perm) {
        hipLaunchKernelGGL(abc_predict_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
        size_t bytes = a.sort_temp_bytes;
        hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(a.sort_temp, bytes, a.sort_keys[0], a.sort_keys[1],
                                                                    a.sort_vals[0], a.sort_vals[1], a.n, 0, 16, s);
        if (e != hipSuccess) return e;
        const int ng = (a.group_lanes > 1 && s2) ? std::min(a.group_end, a.n) : 0;
        if (ng > 0) {                           // the longest trials on lane groups, concurrently on s2
            a.group_end = ng;
            a.g0 = ng;
            (void)hipEventRecord(fork, s);
            (void)hipStreamWaitEvent(s2, fork, 0);
            const unsigned blocks = (unsigned)(((long)ng * a.group_lanes + 255) / 256);
            switch (a.group_lanes) {
                case 2: hipLaunchKernelGGL(abc_trials_group_kernel<2>, dim3(blocks), dim3(256), 0, s2, a); break;
                case 8: hipLaunchKernelGGL(abc_trials_group_kernel<8>, dim3(blocks), dim3(256), 0, s2, a); break;
                case 16: hipLaunchKernelGGL(abc_trials_group_kernel<16>, dim3(blocks), dim3(256), 0, s2, a); break;
                default: hipLaunchKernelGGL(abc_trials_group_kernel<4>, dim3(blocks), dim3(256), 0, s2, a); break;
            }
            (void)hipEventRecord(join, s2);
        }
        if (a.n > a.g0)
            hipLaunchKernelGGL(abc_trials_kernel, dim3((a.n - a.g0 + 255) / 256), dim3(256), 0, s, a);
        if (ng > 0) (void)hipStreamWaitEvent(s, join, 0);
    } else {
        hipLaunchKernelGGL(abc_trials_kernel, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    }
    if (a.T <= 128) hipLaunchKernelGGL(abc_distance_kernel<false>, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(abc_distance_kernel<true>, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_abc_select(const AbcSelectArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(abc_select_kernel, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_abc_gather(const AbcGatherArgs& a, int max_count, hipStream_t s) {
    if (max_count <= 0) return hipSuccess;
    const long total = (long)max_count * a.T;
    hipLaunchKernelGGL(abc_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a, max_count);
    return hipGetLastError();
}

}  // namespace epipf
