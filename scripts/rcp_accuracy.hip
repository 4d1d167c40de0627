// rcp_accuracy.hip -- max ulp error of v_rcp_f64 and of 1 / 2 Newton steps against IEEE 1/x (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
__global__ void k(double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t s = 0x9E3779B97F4A7C15ull * (i + 1);
    s ^= s >> 29; s *= 0xBF58476D1CE4E5B9ull; s ^= s >> 32;
    const double x = ldexp(1.0 + (double)(s >> 11) * 0x1.0p-53, (int)(s % 40) - 10);
    const double e = 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
    const double r0 = r;
    r = fma(fma(-x, r, 1.0), r, r);
    const double r1 = r;
    r = fma(fma(-x, r, 1.0), r, r);
    const double ulp = ldexp(1.0, ilogb(e) - 52);
    out[3 * i] = fabs(r0 - e) / ulp; out[3 * i + 1] = fabs(r1 - e) / ulp; out[3 * i + 2] = fabs(r - e) / ulp;
}
int main() {
    const int n = 1 << 22;
    double* d; hipMalloc(&d, 24 * (size_t)n);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, n);
    double* h = new double[3 * (size_t)n];
    hipMemcpy(h, d, 24 * (size_t)n, hipMemcpyDeviceToHost);
    double m[3] = {0, 0, 0}; long cnt[3] = {0, 0, 0};
    for (long i = 0; i < n; ++i) for (int j = 0; j < 3; ++j) { m[j] = fmax(m[j], h[3 * i + j]); cnt[j] += h[3 * i + j] > 0; }
    printf("max ulp error: rcp %.3g  1 NR %.3g  2 NR %.3g ; inexact fraction: %.4f %.4f %.4f\n", m[0], m[1], m[2],
           cnt[0] / (double)n, cnt[1] / (double)n, cnt[2] / (double)n);
    return 0;
}
