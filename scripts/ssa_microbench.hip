// ssa_microbench.hip -- attribution of the Gillespie event loop's cost on gfx950 (timing-only variants).
// Each variant runs the SIR event loop over [0, 1) from the same states; events/s is reported.
// Variants replace ONE component by a cheap stand-in (results are wrong by design; only time matters):
//   0 exact (product arithmetic)       1 Philox -> 2-multiply hash      2 log -> cheap polynomial
//   3 IEEE divides -> x * rcp(y)        4 all three cheap                5 Philox via 64-bit products
//   6 fast path (approx ratios + exact fallback band), the candidate product variant
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ssa_microbench ssa_microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

struct B4 { uint32_t x, y, z, w; };

__device__ __forceinline__ B4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return B4{c0, c1, c2, c3};
}
__device__ __forceinline__ B4 philox10_64(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return B4{c0, c1, c2, c3};
}
__device__ __forceinline__ B4 cheap_hash(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    uint32_t a = (c0 ^ k0) * 0x9E3779B1u + c1, b = (c1 ^ k1 ^ c2) * 0x85EBCA77u + c0;
    return B4{a ^ (b >> 15), b ^ (a >> 13), a + b, (a ^ c3) + (b >> 7)};
}
__device__ __forceinline__ double u01(uint32_t lo, uint32_t hi) {
    return (double)((((uint64_t)hi << 32) | lo) >> 11) * 0x1.0p-53;
}

template <int V>
__global__ __launch_bounds__(256) void ssa_kernel(const int* st, int* out, int n, double beta, double gamma,
                                                  unsigned long long* events, unsigned long long* fallbacks) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    int nev = 0, nfb = 0;
    if (j < n) {
        double S = st[3 * j], I = st[3 * j + 1], R = st[3 * j + 2];
        const double N = (S + I) + R;
        const double invN = 1.0 / N;
        double t = 0.0;
        uint32_t k = 0;
        while (I > 0.0) {
            B4 r;
            if constexpr (V == 1 || V == 4) r = cheap_hash(k, j, 7u, 3u, 11u, 13u);
            else if constexpr (V == 5) r = philox10_64(k, j, 7u, 3u, 11u, 13u);
            else r = philox10(k, j, 7u, 3u, 11u, 13u);
            ++k;
            const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
            double a0, as, tau;
            bool second;
            if constexpr (V == 3 || V == 4) {
                a0 = ((beta * S) * I) * invN;
                const double a1 = gamma * I;
                as = a0 + a1;
                const double ri = __builtin_amdgcn_rcp(as);
                const double L = (V == 4) ? -(u1 * (1.0 + u1 * (0.5 + u1 * 0.33))) : log(1.0 - u1);
                tau = ri * (-L);
                second = (a0 * ri) <= u2;
            } else if constexpr (V == 6) {
                // fast path: approximate ratio with an error band, exact reference arithmetic inside the band
                a0 = ((beta * S) * I) * invN;
                const double a1 = gamma * I;
                as = a0 + a1;
                double ri = __builtin_amdgcn_rcp(as);
                ri = fma(fma(-as, ri, 1.0), ri, ri);
                tau = ri * (-log(1.0 - u1));
                const double q = a0 * ri;
                if (fabs(q - u2) <= 0x1.0p-40) {
                    ++nfb;
                    const double e0 = ((beta * S) * I) / N, e1 = gamma * I, es = e0 + e1;
                    const double p0 = e0 / es, p1 = e1 / es;
                    second = (p0 / (p0 + p1)) <= u2;
                } else {
                    second = q <= u2;
                }
            } else {
                a0 = ((beta * S) * I) / N;
                const double a1 = gamma * I;
                as = a0 + a1;
                const double L = (V == 2) ? -(u1 * (1.0 + u1 * (0.5 + u1 * 0.33))) : log(1.0 - u1);
                tau = (1.0 / as) * (-L);
                const double p0 = a0 / as, p1 = a1 / as;
                second = (p0 / (p0 + p1)) <= u2;
            }
            if (t + tau > 1.0) break;
            t = t + tau;
            if (second) { I -= 1.0; R += 1.0; } else { S -= 1.0; I += 1.0; }
            ++nev;
        }
        out[3 * j] = (int)S; out[3 * j + 1] = (int)I; out[3 * j + 2] = (int)R;
    }
    unsigned long long e = nev, f = nfb;
    for (int o = 32; o > 0; o >>= 1) { e += __shfl_xor(e, o, 64); f += __shfl_xor(f, o, 64); }
    if ((threadIdx.x & 63) == 0) { atomicAdd(events, e); atomicAdd(fallbacks, f); }
}

template <int V>
void run(const char* name, const int* dst, int* dout, int n, unsigned long long* dev) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(ssa_kernel<V>, dim3((n + 255) / 256), dim3(256), 0, 0, dst, dout, n, 0.25, 0.1, dev, dev + 1);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(dev, 0, 16));
    const int reps = 5;
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(ssa_kernel<V>, dim3((n + 255) / 256), dim3(256), 0, 0, dst, dout, n, 0.25, 0.1, dev, dev + 1);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long h[2];
    CHECK(hipMemcpy(h, dev, 16, hipMemcpyDeviceToHost));
    printf("variant %d %-34s %8.3f ms/launch  %.3e events/s  fallbacks/event %.2e\n", V, name, ms / reps,
           h[0] / (ms / 1e3), (double)h[1] / (double)h[0]);
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 327680;
    std::vector<int> st(3 * n);
    srand(1);
    for (int j = 0; j < n; ++j) {
        int I = 200 + rand() % 600, R = rand() % 2000;
        st[3 * j] = 10000 - I - R; st[3 * j + 1] = I; st[3 * j + 2] = R;
    }
    int *dst, *dout;
    unsigned long long* dev;
    CHECK(hipMalloc(&dst, 12 * (size_t)n)); CHECK(hipMalloc(&dout, 12 * (size_t)n)); CHECK(hipMalloc(&dev, 16));
    CHECK(hipMemcpy(dst, st.data(), 12 * (size_t)n, hipMemcpyHostToDevice));
    printf("lanes %d\n", n);
    run<0>("exact (product)", dst, dout, n, dev);
    run<1>("Philox -> cheap hash", dst, dout, n, dev);
    run<2>("log -> cheap poly", dst, dout, n, dev);
    run<3>("divides -> rcp mul", dst, dout, n, dev);
    run<4>("all cheap", dst, dout, n, dev);
    run<5>("Philox 64-bit products", dst, dout, n, dev);
    run<6>("fast ratio + exact band", dst, dout, n, dev);
    return 0;
}
