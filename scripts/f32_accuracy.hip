// f32_accuracy.hip -- exhaustive error of the gfx950 hardware v_log_f32 / v_rcp_f32 (and the f32 event-time
// recipe of the SSA fast path) against f64 references, to size the certification bounds.
//   log: every float x in [2^-20, 1): |log2_hw(x) - log2(x)| as a multiple of |log2 x| (relative) and absolute
//   rcp: every float mantissa at exponents -60..60 (step 4): relative error
// Build: hipcc --offload-arch=gfx950 -O3 -o f32_acc f32_accuracy.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

__device__ void atomic_max_f64(double* p, double v) {
    unsigned long long* a = (unsigned long long*)p;
    unsigned long long old = *a;
    while (v > __longlong_as_double((long long)old)) {
        unsigned long long prev = atomicCAS(a, old, (unsigned long long)__double_as_longlong(v));
        if (prev == old) break;
        old = prev;
    }
}

// x = float with bits base + i
__global__ void log_kernel(uint32_t base, uint32_t n, double* out) {
    double rel = 0.0, ab = 0.0, relx = 0.0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __uint_as_float(base + i);
        const float l = __builtin_amdgcn_logf(x);            // v_log_f32: log2
        const double ref = log2((double)x);
        const double e = fabs((double)l - ref);
        if (ref != 0.0) rel = fmax(rel, e / fabs(ref));
        ab = fmax(ab, e);
        // error relative to (1 - x) scale: what the event clock sees when x = 1 - U is near 1
        relx = fmax(relx, e / fmax(1.0 - (double)x, 1e-300));
    }
    for (int o = 32; o > 0; o >>= 1) {
        rel = fmax(rel, __shfl_xor(rel, o, 64));
        ab = fmax(ab, __shfl_xor(ab, o, 64));
        relx = fmax(relx, __shfl_xor(relx, o, 64));
    }
    if ((threadIdx.x & 63) == 0) { atomic_max_f64(out, rel); atomic_max_f64(out + 1, ab); atomic_max_f64(out + 2, relx); }
}

__global__ void rcp_kernel(int e0, int e1, double* out) {
    double rel = 0.0;
    for (int e = e0; e <= e1; e += 4) {
        for (uint32_t m = blockIdx.x * blockDim.x + threadIdx.x; m < (1u << 23); m += gridDim.x * blockDim.x) {
            const float x = ldexpf(1.0f + (float)m * 0x1.0p-23f, e);
            const float r = __builtin_amdgcn_rcpf(x);
            const double ref = 1.0 / (double)x;
            rel = fmax(rel, fabs((double)r - ref) / ref);
        }
    }
    for (int o = 32; o > 0; o >>= 1) rel = fmax(rel, __shfl_xor(rel, o, 64));
    if ((threadIdx.x & 63) == 0) atomic_max_f64(out + 3, rel);
}

int main() {
    double* d;
    CHECK(hipMalloc(&d, 8 * sizeof(double)));
    CHECK(hipMemset(d, 0, 8 * sizeof(double)));
    const uint32_t lo = 0x35800000u;   // 2^-20
    const uint32_t hi = 0x3F800000u;   // 1.0
    hipLaunchKernelGGL(log_kernel, dim3(4096), dim3(256), 0, 0, lo, hi - lo, d);
    hipLaunchKernelGGL(rcp_kernel, dim3(4096), dim3(256), 0, 0, -60, 60, d);
    CHECK(hipDeviceSynchronize());
    double h[8];
    CHECK(hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost));
    printf("v_log_f32 on [2^-20, 1): max |err|/|log2 x| = %.3e (= %.2f x 2^-24)   max |err| = %.3e (= %.2f x 2^-24)   "
           "max |err|/(1-x) = %.3e\n", h[0], h[0] / 0x1.0p-24, h[1], h[1] / 0x1.0p-24, h[2]);
    printf("v_rcp_f32 on 2^[-60,60]: max rel err = %.3e (= %.2f x 2^-24)\n", h[3], h[3] / 0x1.0p-24);
    return 0;
}
