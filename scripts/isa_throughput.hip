// isa_throughput.hip -- cycles per wave64 instruction on gfx950 for the instructions of the SSA event
// loop (throughput: 8 independent chains per lane, 8 waves/SIMD; latency: 1 dependent chain, 1 wave/SIMD).
// Timing-only microbenchmark (results meaningless); build:
//   hipcc --offload-arch=gfx950 -O3 -o isa_tp isa_throughput.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kIters = 1024;

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
OP_KERNEL(k_xor3, uint32_t, 1, "v_add3_u32 %0, %0, %1, %1", : "v"(0x1234u))
OP_KERNEL(k_xor3_s, uint32_t, 1, "v_add3_u32 %0, %0, %1, %0", : "s"(0x1234u))
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
OP_KERNEL(k_bitop3, uint32_t, 1, "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96", : "v"(0x1234u))
OP_KERNEL(k_bitop3_s, uint32_t, 1, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96", : "s"(0x1234u))
OP_KERNEL(k_mul_f32, float, 1.0f, "v_mul_f32 %0, %0, %1", : "v"(0.999f))
OP_KERNEL(k_add_f32, float, 1.0f, "v_add_f32 %0, %0, %1", : "v"(0.999f))
OP_KERNEL(k_cvt_f32_u32, float, 1.0f, "v_cvt_f32_u32 %0, %1", : "v"(7u))
OP_KERNEL(k_pk_mul_f32, double, 1.0, "v_pk_mul_f32 %0, %0, %1", : "v"(0.999))
OP_KERNEL(k_pk_add_f32, double, 1.0, "v_pk_add_f32 %0, %0, %1", : "v"(0.999))
OP_KERNEL(k_exp_f32, float, 1.0f, "v_exp_f32 %0, %0", )
// random-operand probes: the value stays a full-width random word (each is 2 instructions: op + xor-fold)
#define RND(NAME, OPASM) OP_KERNEL(NAME, uint32_t, 0x9E3779B9u * 7, OPASM "\n\tv_xor_b32 %0, %0, v44", : "v"(0xD2511F53u) : "v44")
RND(k_r_mulhi, "v_mul_hi_u32 v44, %0, %1")
RND(k_r_mullo, "v_mul_lo_u32 v44, %0, %1")
RND(k_r_mulu24, "v_mul_u32_u24 v44, %0, %1")
RND(k_r_mulhiu24, "v_mul_hi_u32_u24 v44, %0, %1")
RND(k_r_xor, "v_add_u32 v44, %0, %1")
OP_KERNEL(k_r_mad, uint32_t, 0x9E3779B9u * 7, "v_mad_u64_u32 v[44:45], vcc, %0, %1, 0\n\tv_xor_b32 %0, v45, v44", : "v"(0xD2511F53u) : "v44", "v45", "vcc")
OP_KERNEL(k_r_fma64, double, 0.6180339887, "v_fma_f64 %0, %0, %1, %2\n\tv_fract_f64 %0, %0", : "v"(3.7320508075688772), "v"(0.1234567))

// scalar-unit and mixed probes (uniform operands)
#define SOP_KERNEL(NAME, ASM, ...)                                                                       \
    template <int ILP>                                                                                   \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, unsigned long long* clk) {                \
        uint32_t a[ILP];                                                                                 \
        _Pragma("unroll") for (int i = 0; i < ILP; ++i) a[i] = __builtin_amdgcn_readfirstlane(blockIdx.x + i); \
        uint32_t v = threadIdx.x;                                                                        \
        unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();     \
        for (int it = 0; it < kIters; ++it) {                                                            \
            _Pragma("unroll") for (int i = 0; i < ILP; ++i) { asm volatile(ASM : "+s"(a[i]), "+v"(v) __VA_ARGS__); } \
        }                                                                                                \
        unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();     \
        uint32_t s = v;                                                                                  \
        _Pragma("unroll") for (int i = 0; i < ILP; ++i) s += a[i];                                       \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                                         \
        if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }                 \
    }
SOP_KERNEL(k_s_xor, "s_xor_b32 %0, %0, 0x1234", )
SOP_KERNEL(k_s_mul, "s_mul_i32 %0, %0, 0xD2511F53", )
SOP_KERNEL(k_s_mulhi, "s_mul_hi_u32 %0, %0, 0xD2511F53", : : "scc")
SOP_KERNEL(k_mad_sgpr, "v_mad_u64_u32 v[40:41], s[40:41], %1, %0, 0\n\tv_xor_b32 %1, %1, v41", : : "v40", "v41", "s40", "s41")
SOP_KERNEL(k_cmp_saveexec, "v_cmp_lt_u32 vcc, %1, %0\n\ts_and_saveexec_b64 s[40:41], vcc\n\tv_add_u32 %1, 1, %1\n\ts_or_b64 exec, exec, s[40:41]", : : "vcc", "s40", "s41")
SOP_KERNEL(k_branch, "s_cmp_eq_u32 %0, 7\n\ts_cbranch_scc1 1f\n\tv_add_u32 %1, 1, %1\n1:\n\ts_add_u32 %0, %0, 1", : : "scc")

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
    fflush(stdout);
    CHECK(hipFree(out)); CHECK(hipFree(clk));
    (void)ns_xor;
}

#define BOTH(K, T)                                                      \
    run<T, 8>(#K, K<8>, 256 * 4 * 8 / 4, 0.0);                          \
    run<T, 1>(#K, K<1>, 256, 0.0);

#define LAT_SCALING(K, T)                                                                 \
    for (int w : {1, 2, 4, 8}) run<T, 1>(#K " dep", K<1>, 256 * w, 0.0);                   \
    for (int w : {1, 2, 4, 8}) run<T, 2>(#K " ilp2", K<2>, 256 * w, 0.0);

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'r') {   // random operands, 8 waves/SIMD, ILP 8 (2 instructions per op)
        for (int w : {1, 8}) {
            const int b = 256 * w;
            run<uint32_t, 8>("r add+xor", k_r_xor<8>, b, 0.0);
            run<uint32_t, 8>("r mullo+xor", k_r_mullo<8>, b, 0.0);
            run<uint32_t, 8>("r mulhi+xor", k_r_mulhi<8>, b, 0.0);
            run<uint32_t, 8>("r mulu24+xor", k_r_mulu24<8>, b, 0.0);
            run<uint32_t, 8>("r mulhiu24+xor", k_r_mulhiu24<8>, b, 0.0);
            run<uint32_t, 8>("r mad64+xor", k_r_mad<8>, b, 0.0);
            run<double, 8>("r fma64+fract", k_r_fma64<8>, b, 0.0);
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'b') {   // gfx950 three-input bitop and f32 candidates for the event loop
        BOTH(k_xor, uint32_t)
        BOTH(k_bitop3, uint32_t)
        BOTH(k_bitop3_s, uint32_t)
        BOTH(k_mul_f32, float)
        BOTH(k_add_f32, float)
        BOTH(k_fma_f32, float)
        BOTH(k_cvt_f32_u32, float)
        BOTH(k_pk_mul_f32, double)
        BOTH(k_pk_add_f32, double)
        BOTH(k_pk_fma_f32, double)
        BOTH(k_log_f32, float)
        BOTH(k_exp_f32, float)
        BOTH(k_rcp_f32, float)
        BOTH(k_mad_u64, uint64_t)
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {   // loop-body size probe at 8 waves/SIMD (kIters scaled by the host)
        run<uint32_t, 8>("xor vop2 x8", k_xor<8>, 2048, 0.0);
        run<uint32_t, 32>("xor vop2 x32", k_xor<32>, 2048, 0.0);
        run<uint32_t, 96>("xor vop2 x96", k_xor<96>, 2048, 0.0);
        run<uint32_t, 8>("xor3 vop3 x8", k_xor3<8>, 2048, 0.0);
        run<uint32_t, 32>("xor3 vop3 x32", k_xor3<32>, 2048, 0.0);
        run<uint32_t, 96>("xor3 vop3 x96", k_xor3<96>, 2048, 0.0);
        run<uint32_t, 8>("xor3 sgpr x8", k_xor3_s<8>, 2048, 0.0);
        run<uint32_t, 96>("xor3 sgpr x96", k_xor3_s<96>, 2048, 0.0);
        run<uint64_t, 8>("mad_u64 x8", k_mad_u64<8>, 2048, 0.0);
        run<uint64_t, 48>("mad_u64 x48", k_mad_u64<48>, 2048, 0.0);
        return 0;
    }
    if (argc > 1) {   // overlap test: dependent chains at 1, 2, 4, 8 waves per SIMD
        LAT_SCALING(k_xor, uint32_t)
        LAT_SCALING(k_fma_f64, double)
        LAT_SCALING(k_mad_u64, uint64_t)
        return 0;
    }
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
