// abc_device.hpp -- device pieces of the ABC rejection sampler (abc_algo.py:17-109) on gfx950.
//
// Compiled with -ffp-contract=off like the rest of libepipf: the prior draw, the Poisson walk and the
// distance are plain IEEE multiply/divide/add sequences that round exactly as the CPU restatement
// (oracle/abc_oracle.c) and the reference's numpy arithmetic do.
#pragma once
#include "epipf_device.hpp"

namespace epipf {

constexpr uint32_t kDomainAbcPrior = 3u << 24;
constexpr uint32_t kDomainAbcInit = 4u << 24;
constexpr uint32_t kDomainAbcSsa = 5u << 24;
constexpr int kAbcPairwiseDepth = 12;           // numpy pairwise recursion levels instantiated: T <= 128 * 2^12
constexpr int kAbcMaxDays = 128 << kAbcPairwiseDepth;

// Initial count of the keyed ABC stream (oracle/philox.py poisson_mode_inversion): inversion over the support
// ordered m, m+1, m-1, m+2, ... (m = floor(lam)) with the ratio recurrences p(k+1) = p(k) lam/(k+1),
// p(k-1) = p(k) k/lam; pm = P(K = m) comes from the host (glibc exp/log/lgamma).  IEEE divisions throughout.
__device__ __forceinline__ int poisson_mode_inversion(double lam, double u, double pm) {
    if (lam == 0.0) return 0;
    const int m = (int)lam;                     // integral (abc_algo.py:38 astype(int)), host-checked
    double acc = pm;
    if (u < acc) return m;
    int khi = m, klo = m;
    double phi = pm, plo = pm;
    for (;;) {
        const double prev = acc;
        phi = (phi * lam) / (double)(khi + 1);
        ++khi;
        acc = acc + phi;
        if (u < acc) return khi;
        if (klo > 0) {
            plo = (plo * (double)klo) / lam;
            --klo;
            acc = acc + plo;
            if (u < acc) return klo;
        }
        if (acc == prev) return m;
    }
}

// |x_d - y_d| of one column (abc_algo.py:12 abs(I_1 - I_2)): x from this lane's day table, y observed.
struct AbsDiff {
    const int32_t* x;    // &days[col][lane], stride between days
    size_t stride;
    const double* y;     // &Y[col], stride 3
    __device__ __forceinline__ double operator()(int d) const {
        return fabs((double)x[(size_t)d * stride] - y[3 * d]);
    }
};

// numpy pairwise_sum (numpy/_core/src/umath/loops_utils.h.src; the order of np.add.reduce, hence np.mean,
// on a contiguous float64 vector): < 8 terms sequential; <= 128 terms in 8 strided accumulators combined as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the remainder; above, split at n/2 rounded down to a multiple of 8.
__device__ __forceinline__ double pairwise_leaf(const AbsDiff& v, int off, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += v(off + i);
        return res;
    }
    double r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = v(off + k);
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] += v(off + i + k);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += v(off + i);
    return res;
}

template <int D>
__device__ __noinline__ double pairwise_sum(const AbsDiff& v, int off, int n) {
    if (n <= 128) return pairwise_leaf(v, off, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum<D - 1>(v, off, n2) + pairwise_sum<D - 1>(v, off + n2, n - n2);
}

template <>
__device__ __noinline__ double pairwise_sum<0>(const AbsDiff& v, int off, int n) {
    return pairwise_leaf(v, off, n);            // unreachable for n <= kAbcMaxDays
}

}  // namespace epipf
