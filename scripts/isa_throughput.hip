// isa_throughput.hip -- cycles per wave64 instruction on gfx950 for the instructions of the SSA event
// loop (throughput: 8 independent chains per lane, 8 waves/SIMD; latency: 1 dependent chain, 1 wave/SIMD).
// Timing-only microbenchmark (results meaningless); build:
//   hipcc --offload-arch=gfx950 -O3 -o isa_tp isa_throughput.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kIters = 4096;

#define OP_KERNEL(NAME, T, INIT, ASM, ...)                                                               \
    template <int ILP>                                                                                   \
    __global__ __launch_bounds__(256) void NAME(T* out, unsigned long long* clk) {                       \
        T a[ILP];                                                                                        \
        _Pragma("unroll") for (int i = 0; i < ILP; ++i) a[i] = (T)(INIT + threadIdx.x + i);              \
        unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();     \
        for (int it = 0; it < kIters; ++it) {                                                            \
            _Pragma("unroll") for (int i = 0; i < ILP; ++i) { asm volatile(ASM : "+v"(a[i]) __VA_ARGS__); } \
        }                                                                                                \
        unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();     \
        T s = a[0];                                                                                      \
        _Pragma("unroll") for (int i = 1; i < ILP; ++i) s = (T)(s + a[i]);                               \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                                         \
        if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }                 \
    }

OP_KERNEL(k_xor, uint32_t, 1, "v_xor_b32 %0, %0, %1", : "v"(0x1234u))
OP_KERNEL(k_add_u32, uint32_t, 1, "v_add_u32 %0, %0, %1", : "v"(0x1234u))
OP_KERNEL(k_mul_lo, uint32_t, 1, "v_mul_lo_u32 %0, %0, %1", : "v"(0xD2511F53u))
OP_KERNEL(k_mul_hi, uint32_t, 1, "v_mul_hi_u32 %0, %0, %1", : "v"(0xD2511F53u))
OP_KERNEL(k_mul_u24, uint32_t, 1, "v_mul_u32_u24 %0, %0, %1", : "v"(0x1F53u))
OP_KERNEL(k_mulhi_u24, uint32_t, 1, "v_mul_hi_u32_u24 %0, %0, %1", : "v"(0x1F53u))
OP_KERNEL(k_mad_u64, uint64_t, 1, "v_mad_u64_u32 %0, vcc, %1, %2, %0", : "v"(0xD2511F53u), "v"(0x1234567u) : "vcc")
OP_KERNEL(k_lshr64, uint64_t, 1, "v_lshrrev_b64 %0, 1, %0", )
OP_KERNEL(k_fma_f32, float, 1.0f, "v_fma_f32 %0, %0, %1, %1", : "v"(0.999f))
OP_KERNEL(k_log_f32, float, 1.0f, "v_log_f32 %0, %0", )
OP_KERNEL(k_rcp_f32, float, 1.0f, "v_rcp_f32 %0, %0", )
OP_KERNEL(k_fma_f64, double, 1.0, "v_fma_f64 %0, %0, %1, %1", : "v"(0.999))
OP_KERNEL(k_mul_f64, double, 1.0, "v_mul_f64 %0, %0, %1", : "v"(0.999))
OP_KERNEL(k_add_f64, double, 1.0, "v_add_f64 %0, %0, %1", : "v"(0.999))
OP_KERNEL(k_rcp_f64, double, 1.0, "v_rcp_f64 %0, %0", )
OP_KERNEL(k_ldexp_f64, double, 1.0, "v_ldexp_f64 %0, %0, 1", )
OP_KERNEL(k_frexp_f64, double, 1.0, "v_frexp_mant_f64 %0, %0", )
OP_KERNEL(k_fract_f64, double, 1.0, "v_fract_f64 %0, %0", )
OP_KERNEL(k_cvt_f64_f32, double, 1.0, "v_cvt_f64_f32 %0, %1", : "v"(1.5f))
OP_KERNEL(k_cvt_f32_f64, float, 1.0f, "v_cvt_f32_f64 %0, %1", : "v"(1.5))
OP_KERNEL(k_cvt_f64_u32, double, 1.0, "v_cvt_f64_u32 %0, %1", : "v"(7u))
OP_KERNEL(k_cmp_f64, uint32_t, 1, "v_cmp_lt_f64 vcc, %1, %2\n\tv_cndmask_b32 %0, %0, 0, vcc", : "v"(1.0), "v"(2.0) : "vcc")
OP_KERNEL(k_cndmask, uint32_t, 1, "v_cmp_lt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, 0, vcc", : "v"(7u) : "vcc")
OP_KERNEL(k_pk_fma_f32, double, 1.0, "v_pk_fma_f32 %0, %0, %1, %1", : "v"(0.999))

template <template <int> class K>
struct Runner;

template <class T, int ILP>
using KFn = void (*)(T*, unsigned long long*);

template <class T, int ILP>
void run(const char* name, KFn<T, ILP> k, int blocks, double ns_xor) {
    T* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, sizeof(T) * blocks * 256));
    CHECK(hipMalloc(&clk, 16));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk);
    CHECK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    const int reps = 10;
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    unsigned long long h[2];
    CHECK(hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost));
    const double waves = blocks * 4.0;
    const double winst = waves * kIters * ILP;                   // wave-instructions per launch
    const double per_simd = winst / 1024.0;                      // 256 CUs x 4 SIMDs
    const double ghz = (double)h[0] / ((double)h[1] / 100.0) / 1e3;   // s_memtime ticks per us / 1e3
    const double cyc = (ms / reps) * 1e-3 * ghz * 1e9 / per_simd;
    const double in_kernel_cyc = (double)h[0] / (kIters * ILP);  // one wave's view (latency mode)
    printf("%-14s ILP=%d blocks=%5d  %8.3f us/launch  clk %.2f GHz  %6.2f cyc/wave-inst/SIMD  (wave0: %6.2f cyc/inst)\n",
           name, ILP, blocks, ms / reps * 1e3, ghz, cyc, in_kernel_cyc);
    CHECK(hipFree(out)); CHECK(hipFree(clk));
    (void)ns_xor;
}

#define BOTH(K, T)                                                      \
    run<T, 8>(#K, K<8>, 256 * 4 * 8 / 4, 0.0);                          \
    run<T, 1>(#K, K<1>, 256, 0.0);

int main() {
    BOTH(k_xor, uint32_t)
    BOTH(k_add_u32, uint32_t)
    BOTH(k_mul_lo, uint32_t)
    BOTH(k_mul_hi, uint32_t)
    BOTH(k_mul_u24, uint32_t)
    BOTH(k_mulhi_u24, uint32_t)
    BOTH(k_mad_u64, uint64_t)
    BOTH(k_lshr64, uint64_t)
    BOTH(k_fma_f32, float)
    BOTH(k_log_f32, float)
    BOTH(k_rcp_f32, float)
    BOTH(k_fma_f64, double)
    BOTH(k_mul_f64, double)
    BOTH(k_add_f64, double)
    BOTH(k_rcp_f64, double)
    BOTH(k_ldexp_f64, double)
    BOTH(k_frexp_f64, double)
    BOTH(k_fract_f64, double)
    BOTH(k_cvt_f64_f32, double)
    BOTH(k_cvt_f32_f64, float)
    BOTH(k_cvt_f64_u32, double)
    BOTH(k_cmp_f64, uint32_t)
    BOTH(k_cndmask, uint32_t)
    BOTH(k_pk_fma_f32, double)
    return 0;
}
