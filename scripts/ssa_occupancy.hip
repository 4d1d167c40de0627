// ssa_occupancy.hip -- does the SIR event loop gain from more waves per SIMD?  (timing-only diagnostic)
// Runs the product's ssa_propagate<kSIR> (csrc/epipf_device.hpp) and stripped variants at 1, 2, 4 and 8
// waves per SIMD, and reports cycles per wave-iteration per SIMD (lower = better; flat = throughput-bound,
// halving with 2x waves = latency-bound).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I stochastic-epidemic-modelling_amd/csrc -o occ scripts/ssa_occupancy.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "epipf_device.hpp"

using namespace epipf;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

struct Out { unsigned long long events, wave_iters, lane_iters, ticks, rticks, pad[11]; };

__device__ __forceinline__ void mulhilo(uint32_t a, uint32_t m, uint32_t& hi, uint32_t& lo) {
    asm("v_mul_hi_u32 %0, %2, %3\n\tv_mul_lo_u32 %1, %2, %3" : "=&v"(hi), "=&v"(lo) : "v"(a), "v"(m));
}

__device__ __forceinline__ Block philox_split(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = __builtin_amdgcn_readfirstlane(0xD2511F53u), M1 = __builtin_amdgcn_readfirstlane(0xCD9E8D57u);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, lo0, hi1, lo1;
        mulhilo(c0, M0, hi0, lo0);
        mulhilo(c2, M1, hi1, lo1);
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return Block{c0, c1, c2, c3};
}

template <int V>
__global__ __launch_bounds__(256) void occ_kernel(const int* st, int* out, int n, ChainParam cp, Out* o) {
    __shared__ LogTab tab[kLogTabEntries];
    if (threadIdx.x < kLogTabEntries) log_table_entry(tab, threadIdx.x);
    __syncthreads();
    const int j = blockIdx.x * 256 + threadIdx.x;
    int nev = 0, iters = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (j < n) {
        double x[3] = {(double)st[3 * j], (double)st[3 * j + 1], (double)st[3 * j + 2]};
        if constexpr (V == 0) {
            nev = ssa_propagate<kSIR, 1>(x, cp, (uint32_t)j, 5u, 1.0, tab, iters);
        } else if constexpr (V == 1) {
            // Philox + uniforms only, fixed 100 iterations (no data-dependent exit, no f64 state logic)
            double acc = 0.0;
            for (uint32_t k = 0; k < 100; ++k) {
                const Block r = philox(k, j, 5u, cp.f, cp.k0, cp.k1);
                acc += u01(r.x, r.y) + u01(r.z, r.w);
            }
            x[0] += acc; iters = 100;
        } else if constexpr (V == 4 || V == 5) {
            // V4: Philox with split v_mul_hi/v_mul_lo (no v_mad_u64_u32 carry-out SGPR writes)
            // V5: product Philox with a per-lane (non-uniform) counter so no round runs on the scalar unit
            double acc = 0.0;
            const uint32_t z = (uint32_t)(j >> 30);
            for (uint32_t k = 0; k < 100; ++k) {
                const Block r = (V == 4) ? philox_split(k ^ z, j, 5u, cp.f, cp.k0, cp.k1)
                                         : philox(k ^ z, j, 5u, cp.f, cp.k0, cp.k1);
                acc += u01(r.x, r.y) + u01(r.z, r.w);
            }
            x[0] += acc; iters = 100;
        } else if constexpr (V == 6) {
            // Philox only, no uniform conversion (xor-accumulate)
            uint32_t acc = 0;
            for (uint32_t k = 0; k < 100; ++k) {
                const Block r = philox(k, j, 5u, cp.f, cp.k0, cp.k1);
                acc ^= r.x ^ r.y ^ r.z ^ r.w;
            }
            x[0] += (double)acc; iters = 100;
        } else if constexpr (V == 7) {
            // Philox ILP 4: four independent blocks per loop iteration (25 iterations = 100 blocks)
            uint32_t acc = 0;
            const uint32_t z = (uint32_t)(j >> 30);
            for (uint32_t k = 0; k < 25; ++k) {
                const Block r0 = philox(k ^ z, j, 5u, cp.f, cp.k0, cp.k1);
                const Block r1 = philox((k + 25) ^ z, j, 5u, cp.f, cp.k0, cp.k1);
                const Block r2 = philox((k + 50) ^ z, j, 5u, cp.f, cp.k0, cp.k1);
                const Block r3 = philox((k + 75) ^ z, j, 5u, cp.f, cp.k0, cp.k1);
                acc ^= r0.x ^ r0.y ^ r0.z ^ r0.w ^ r1.x ^ r1.y ^ r1.z ^ r1.w ^ r2.x ^ r2.y ^ r2.z ^ r2.w ^ r3.x ^ r3.y ^ r3.z ^ r3.w;
            }
            x[0] += (double)acc; iters = 100;
        } else if constexpr (V == 8) {
            // 8 independent multiply-xor chains with data-dependent multiplicands, 20 steps = one Philox block's muls
            uint32_t a[8];
            for (int i = 0; i < 8; ++i) a[i] = j * 2654435761u + i;
            for (uint32_t k = 0; k < 100; ++k) {
#pragma unroll
                for (int r = 0; r < 20; r += 8) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const uint64_t p = (uint64_t)0xD2511F53u * a[i];
                        a[i] = (uint32_t)(p >> 32) ^ (uint32_t)p ^ k;
                    }
                }
            }
            uint32_t acc = 0;
            for (int i = 0; i < 8; ++i) acc ^= a[i];
            x[0] += (double)acc; iters = 100;
        } else if constexpr (V == 2) {
            // f64 event arithmetic only (uniforms from a cheap LCG), same exit structure as the product
            const double beta = cp.theta[0], gamma = cp.theta[1];
            double S = x[0], I = x[1], R = x[2];
            const double invN = 1.0 / ((S + I) + R);
            double t = 0.0;
            uint32_t s = j * 747796405u + 1u;
            while (I > 0.0) {
                s = s * 1664525u + 1013904223u; const double u1 = (double)(s >> 8) * 0x1.0p-24;
                s = s * 1664525u + 1013904223u; const double u = (double)(s >> 8) * 0x1.0p-24;
                ++iters;
                const double a0 = ((beta * S) * I) * invN;
                const double as = a0 + gamma * I;
                const double ri = recip(as);
                const double tau = ri * (-fast_log(1.0 - u1, tab));
                const bool second = a0 * ri <= u;
                if (t + tau > 1.0) break;
                t = t + tau;
                if (second) { I -= 1.0; R += 1.0; } else { S -= 1.0; I += 1.0; }
                ++nev;
            }
            x[0] = S; x[1] = I; x[2] = R;
        } else if constexpr (V == 3) {
            // V0 without the exact-channel fallback call and with a branch-free state update
            const double beta = cp.theta[0], gamma = cp.theta[1];
            double S = x[0], I = x[1], R = x[2];
            const double invN = 1.0 / ((S + I) + R);
            double t = 0.0;
            uint32_t k = 0;
            while (I > 0.0) {
                const Block r = philox(k, j, 5u, cp.f, cp.k0, cp.k1);
                ++k;
                const double a0 = ((beta * S) * I) * invN;
                const double as = a0 + gamma * I;
                const double ri = recip(as);
                const double tau = ri * (-fast_log(1.0 - u01(r.x, r.y), tab));
                const double u = u01(r.z, r.w);
                const bool second = a0 * ri <= u;
                const double tn = t + tau;
                if (tn > 1.0) break;
                t = tn;
                const double ds = second ? 0.0 : -1.0, dr = second ? 1.0 : 0.0;
                S += ds; R += dr; I = I - ds - dr;
                ++nev;
            }
            iters = (int)k;
            x[0] = S; x[1] = I; x[2] = R;
        }
        out[3 * j] = (int)x[0]; out[3 * j + 1] = (int)x[1]; out[3 * j + 2] = (int)x[2];
    }
    unsigned long long e = nev, li = iters;
    int wm = iters;
    for (int of = 32; of > 0; of >>= 1) {
        e += __shfl_xor(e, of, 64); li += __shfl_xor(li, of, 64); wm = max(wm, __shfl_xor(wm, of, 64));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {   // spread over 64 slots: same-address atomics serialise (~10 ns each)
        Out* q = o + ((blockIdx.x * 4 + (threadIdx.x >> 6)) & 63);
        atomicAdd(&q->ticks, t1 - t0); atomicAdd(&q->rticks, r1 - r0);
        atomicAdd(&q->events, e); atomicAdd(&q->lane_iters, li); atomicAdd(&q->wave_iters, (unsigned long long)wm);
    }
}

template <int V>
void run(const char* name, int wps, const int* dst, int* dout, Out* dev, const ChainParam& cp) {
    const int waves = 1024 * wps, n = waves * 64, blocks = n / 256;
    hipLaunchKernelGGL(occ_kernel<V>, dim3(blocks), dim3(256), 0, 0, dst, dout, n, cp, dev);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(dev, 0, 64 * sizeof(Out)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    const int reps = 5;
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(occ_kernel<V>, dim3(blocks), dim3(256), 0, 0, dst, dout, n, cp, dev);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    Out hs[64], h{};
    CHECK(hipMemcpy(hs, dev, sizeof hs, hipMemcpyDeviceToHost));
    for (auto& q : hs) { h.events += q.events; h.wave_iters += q.wave_iters; h.lane_iters += q.lane_iters; h.ticks += q.ticks; h.rticks += q.rticks; }
    const double us = ms / reps * 1e3;
    const double wave_iters_per_simd = (double)h.wave_iters / reps / 1024.0;
    const double ghz = (double)h.ticks / ((double)h.rticks / 100.0) / 1e3;
    const double wave_life_us = (double)h.rticks / 100.0 / (waves * (double)reps);
    printf("V%d %-28s waves/SIMD=%d  %9.1f us  %.3e ev/s  lane-use %.3f  %7.1f ns/wave-iter/SIMD  clk %.2f GHz -> %.0f cyc  wave life %.1f us\n",
           V, name, wps, us, h.events / (ms / 1e3), (double)h.lane_iters / (64.0 * h.wave_iters),
           us * 1e3 / wave_iters_per_simd, ghz, us * 1e3 / wave_iters_per_simd * ghz, wave_life_us);
}

int main() {
    const int nmax = 1024 * 8 * 64;
    std::vector<int> st(3 * nmax);
    srand(1);
    for (int j = 0; j < nmax; ++j) {   // config-2-like states: pop 1e4, I ~ 300
        int I = 250 + rand() % 100, R = 3000 + rand() % 200;
        st[3 * j] = 10000 - I - R; st[3 * j + 1] = I; st[3 * j + 2] = R;
    }
    int *dst, *dout;
    Out* dev;
    CHECK(hipMalloc(&dst, 12 * (size_t)nmax)); CHECK(hipMalloc(&dout, 12 * (size_t)nmax)); CHECK(hipMalloc(&dev, 64 * sizeof(Out)));
    CHECK(hipMemcpy(dst, st.data(), 12 * (size_t)nmax, hipMemcpyHostToDevice));
    ChainParam cp{};
    cp.theta[0] = 0.25; cp.theta[1] = 0.1; cp.k0 = 7; cp.k1 = 9; cp.f = 3;
    if (getenv("OCC_ONLY_NEW") == nullptr) {
    for (int w : {1, 2, 4, 8}) run<0>("product ssa_propagate", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<1>("philox+u01 only (100 it)", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<2>("f64 arithmetic only", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<3>("no fallback, branch-free upd", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<4>("philox split mul_hi/lo", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<5>("philox lane-varying counter", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<6>("philox only, no u01", w, dst, dout, dev, cp);
    }
    for (int w : {1, 2, 4, 8}) run<7>("philox ILP4", w, dst, dout, dev, cp);
    for (int w : {1, 2, 4, 8}) run<8>("8 mul chains x 24 muls/iter", w, dst, dout, dev, cp);
    return 0;
}
