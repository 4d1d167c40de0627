// epipf_step.hpp -- the block-sum prefix helpers shared by the one-lane-per-particle step kernel
// (epipf_kernels.hip) and the lane-group step kernel (epipf_group.hip).
#pragma once
#include "epipf_device.hpp"
#include "epipf_internal.hpp"

namespace epipf {

// (chain, particle block) of this workgroup.  2-D grid: (blockIdx.y, blockIdx.x).  XCD-aware 1-D grid of B x chains
// (a.xcd_map): the dispatcher deals workgroups round-robin over the 8 XCDs (MI355X_MICROARCH.md, observed; which XCD
// gets block 0 is not fixed), so the blocks p = l (mod 8) share one XCD and its L2.  Label l takes a contiguous range
// of the chain-major block order -- whole chains when B x chains is a multiple of 8 chains' blocks -- so a chain's
// blocks fetch its block sums, in-block prefixes and parent states (the previous step's) into one L2 instead of
// eight, and find them already there when consecutive launches deal the label to the same XCD.  A bijection for any
// grid size (label l holds q + [l < r] blocks), so placement only changes speed.
struct BlockPos {
    int chain, b;
};
__device__ __forceinline__ BlockPos step_block(const StepArgs& a) {
    if (!a.xcd_map) return {a.chain0 + (int)blockIdx.y, (int)blockIdx.x};
    const int total = (int)gridDim.x, p = (int)blockIdx.x;
    const int q = total >> 3, r = total & 7, l = p & 7;
    const int L = l * q + min(l, r) + (p >> 3);
    const int c = L / a.B;
    return {a.chain0 + c, L - c * a.B};
}

// Initial state of particle j (pmcmc.py:156-175): per group an initial infected count Poisson(mu) by CDF inversion on
// the keyed stream (counter (g, j, 2 << 24, f)), S = population - I, the rest 0.  pf_init_kernel and the one-workgroup
// filter (epipf_fused.hpp) draw it with this code.
template <int MODEL, int G>
__device__ __forceinline__ void init_particle(const StepArgs& a, const ChainParam& cp, int j, double* x) {
    constexpr int C = Shape<MODEL, G>::C;
#pragma unroll
    for (int c = 0; c < C; ++c) x[c] = 0.0;
#pragma unroll
    for (int g = 0; g < ((MODEL >= kSubgroups) ? G : 1); ++g) {
        const Block r = philox((uint32_t)g, (uint32_t)j, kDomainInit, cp.f, cp.k0, cp.k1);
        const double U = u01(r.x, r.y);
        const double mu = a.mu[g];
        double pk = a.emu[g], F = pk;
        int k = 0;
        while (U >= F && k < a.kmax[g]) { k += 1; pk = pk * mu / (double)k; F = F + pk; }
        const double S0 = a.npop[g] - (double)k;
        if constexpr (MODEL == kSIR) { x[0] = S0; x[1] = (double)k; }
        else if constexpr (MODEL == kSEIR) { x[0] = S0; x[2] = (double)k; }
        else { x[3 * g] = S0; x[3 * g + 1] = (double)k; }
    }
}

// LDS ordering between the lanes that run a helper: the whole block (__syncthreads), or only the calling wave
// (WAVE = true: the lane-group kernel runs these on its first wave while the other waves wait at a block barrier).
template <bool WAVE>
__device__ __forceinline__ void lds_sync() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        __syncthreads();
    }
}

// exclusive prefix of the B block sums into LDS (bpex), deterministic order; returns the total.
template <int WG, bool WAVE = false>
__device__ __forceinline__ double scan_block_sums(const double* __restrict__ bsum_g, int B, double* bpex,
                                                  double* bsum, double* red) {
    const int tid = threadIdx.x;
    const int per = (B + WG - 1) / WG;
    const int beg = min(tid * per, B), end = min(beg + per, B);
    double s = 0.0;
    for (int i = beg; i < end; ++i) {
        const double v = bsum_g[i];
        bsum[i] = v;
        s = s + v;
    }
    const double incl = block_inclusive_scan<WG>(s, red);
    // exclusive offset of this thread's chunk = inclusive result of the previous thread
    double* incl_lds = bpex + B;  // scratch after bpex (allocated B + WG)
    incl_lds[tid] = incl;
    lds_sync<WAVE>();
    double e = (tid == 0) ? 0.0 : incl_lds[tid - 1];
    for (int i = beg; i < end; ++i) {
        bpex[i] = e;
        e = e + bsum[i];
    }
    lds_sync<WAVE>();
    return bpex[B - 1] + bsum[B - 1];
}

// Segmented prefix of the B block sums (64-thread block): lane l sums the blocks of segments [l*q, (l+1)*q)
// sequentially, a wave scan gives each lane its offset, and the lane writes seg_start[k] / seg_end[k] (the running
// sum before / after segment k's S blocks) to LDS.  With S = 1 this is scan_block_sums<64> exactly (seg_start =
// bpex, seg_end = bpex + bsum).  LDS holds 2 * nseg <= 400 doubles whatever N is, so one-wave blocks keep 7 waves
// per SIMD at every size (before, past ~16k particles the 2B-double table capped occupancy and 256-thread blocks
// were needed, whose four waves retire together).
template <bool WAVE = false>
__device__ __forceinline__ double scan_segments(const double* __restrict__ bsum_g, int B, int S, int nseg,
                                                double* seg_start, double* seg_end) {
    const int lane = threadIdx.x;
    const int q = (nseg + 63) / 64;
    const int k0 = min(lane * q, nseg), k1 = min(k0 + q, nseg);
    const int b0 = min(k0 * S, B), b1 = min(k1 * S, B);
    double s = 0.0;
    for (int i = b0; i < b1; ++i) s = s + bsum_g[i];
    const double inc = block_inclusive_scan<64>(s, nullptr);
    const double up = __shfl_up(inc, 1, 64);
    double e = (lane == 0) ? 0.0 : up;
    for (int k = k0; k < k1; ++k) {
        seg_start[k] = e;
        const int ie = min((k + 1) * S, B);
        for (int i = k * S; i < ie; ++i) e = e + bsum_g[i];
        seg_end[k] = e;
    }
    lds_sync<WAVE>();
    return seg_end[nseg - 1];
}

// The block-sum prefix of a run on 16-particle blocks (lane-group runs, kGroupBlock), with the step's TOTAL summed in
// the 64-particle layout's order, so that a filter's log-likelihood does not depend on which layout its launch used
// (the layout follows the number of chains sharing the launch, pick_block).  The 64-layout total is
//   c_m = the in-block scan's last lane over 64-block m = (s_4m + s_4m+1) + (s_4m+2 + s_4m+3)
// exactly: block_inclusive_scan's Hillis-Steele window at lane 63 is the balanced tree of its four aligned 16-lane
// windows, each the 16-particle block's own scan result s (lane 15, the lanes past the block adding nothing), and
// IEEE addition commutes; then lane l adds the c_m of its P consecutive 64-blocks in order (P = a.canon_per: the
// 64-layout's per-lane share, scan_block_sums / scan_segments), a wave scan gives each lane its offset, and the total is
// the last lane's running sum.  Blocks past N hold weights 0 in both layouts (sums exact).
// Outputs for the 16-particle search: flat (S16 = 1) every block's exclusive prefix and sum (bpex, bsum); segmented
// (S16 = 4 S64, whole 64-blocks per segment) seg_start / seg_end.  Inside a 64-block the 16-block prefixes are
// e, e + s0, e + (s0 + s1), e + ((s0 + s1) + s2): other roundings of the same prefixes, within the resampling
// certificate's depth bound (cert_k is taken on the 16-block layout's larger D), so the search stays certified.
// The total goes through LDS (*tot, written by the lane holding the last 64-block).
template <bool WAVE>
__device__ __forceinline__ double scan_block_sums16(const double* __restrict__ bsum_g, int B16, int P, int S16,
                                                    double* bpex, double* bsum, double* seg_start, double* seg_end,
                                                    double* tot) {
    const int lane = threadIdx.x & 63;
    const int B64 = (B16 + 3) >> 2;
    const int m0 = min(lane * P, B64), m1 = min(m0 + P, B64);
    auto sub = [&](int i) __attribute__((always_inline)) { return i < B16 ? bsum_g[i] : 0.0; };
    double s = 0.0;
    for (int m = m0; m < m1; ++m) {
        const double s0 = sub(4 * m), s1 = sub(4 * m + 1), s2 = sub(4 * m + 2), s3 = sub(4 * m + 3);
        s = s + ((s0 + s1) + (s2 + s3));
    }
    const double inc = block_inclusive_scan<64>(s, nullptr);
    const double up = __shfl_up(inc, 1, 64);
    double e = (lane == 0) ? 0.0 : up;
    for (int m = m0; m < m1; ++m) {
        const int i = 4 * m;
        const double s0 = sub(i), s1 = sub(i + 1), s2 = sub(i + 2), s3 = sub(i + 3);
        const double s01 = s0 + s1;
        if (S16 == 1) {
            bpex[i] = e;
            bsum[i] = s0;
            if (i + 1 < B16) { bpex[i + 1] = e + s0; bsum[i + 1] = s1; }
            if (i + 2 < B16) { bpex[i + 2] = e + s01; bsum[i + 2] = s2; }
            if (i + 3 < B16) { bpex[i + 3] = e + (s01 + s2); bsum[i + 3] = s3; }
        } else if (i % S16 == 0) {
            seg_start[i / S16] = e;
        }
        e = e + (s01 + (s2 + s3));
        if (S16 > 1 && ((i + 4) % S16 == 0 || m == B64 - 1)) seg_end[i / S16] = e;
        if (m == B64 - 1) *tot = e;
    }
    lds_sync<WAVE>();
    return *tot;
}

}  // namespace epipf
