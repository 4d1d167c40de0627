// census.hip -- where and when do waves run?  Each wave records its XCC / SE / CU / SIMD (hardware id
// registers) and its start / end time (s_memrealtime, 100 MHz); the host reports distinct CUs and SIMDs used,
// the peak and mean number of co-resident waves, and the device properties.  Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -o census scripts/census.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); exit(1); } } while (0)

struct Rec { unsigned hwid, xcc; unsigned long long t0, t1; };

__device__ __forceinline__ uint32_t mix(uint32_t a, uint32_t k) {
    const uint64_t p = (uint64_t)0xD2511F53u * a;
    return (uint32_t)(p >> 32) ^ (uint32_t)p ^ k;
}

__global__ __launch_bounds__(256) void work(Rec* rec, uint32_t* out, int iters) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t a = blockIdx.x * 256 + threadIdx.x, b = a * 7 + 1;
    for (int i = 0; i < iters; ++i) { a = mix(a, i); b = mix(b, a); }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b;
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        Rec r{hw, xcc, t0, t1};
        rec[blockIdx.x * 4 + (threadIdx.x >> 6)] = r;
    }
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    printf("device %s gcnArch %s CUs %d clock %d kHz maxThreadsPerCU %d regsPerBlock %d l2 %d\n", p.name, p.gcnArchName,
           p.multiProcessorCount, p.clockRate, p.maxThreadsPerMultiProcessor, p.regsPerBlock, p.l2CacheSize);
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    for (int blocks : {64, 256, 1024, 2048}) {
        const int waves = blocks * 4;
        Rec* drec;
        uint32_t* dout;
        CHECK(hipMalloc(&drec, sizeof(Rec) * waves));
        CHECK(hipMalloc(&dout, sizeof(uint32_t) * blocks * 256));
        hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, 0, drec, dout, iters);
        CHECK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, 0, drec, dout, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        std::vector<Rec> h(waves);
        CHECK(hipMemcpy(h.data(), drec, sizeof(Rec) * waves, hipMemcpyDeviceToHost));
        std::set<unsigned> cus, simds, xccs;
        unsigned long long tmin = ~0ull, tmax = 0;
        double life = 0;
        std::vector<std::pair<unsigned long long, int>> ev;
        for (auto& r : h) {
            const unsigned wave = r.hwid & 0xF, simd = (r.hwid >> 4) & 3, cu = (r.hwid >> 8) & 0xF,
                           sh = (r.hwid >> 12) & 1, se = (r.hwid >> 13) & 7;
            (void)wave;
            const unsigned cuk = (r.xcc << 12) | (se << 8) | (sh << 4) | cu;
            cus.insert(cuk);
            simds.insert((cuk << 2) | simd);
            xccs.insert(r.xcc);
            tmin = std::min(tmin, r.t0);
            tmax = std::max(tmax, r.t1);
            life += (double)(r.t1 - r.t0);
            ev.push_back({r.t0, 1});
            ev.push_back({r.t1, -1});
        }
        std::sort(ev.begin(), ev.end());
        int cur = 0, peak = 0;
        for (auto& e : ev) { cur += e.second; peak = std::max(peak, cur); }
        const double span = (double)(tmax - tmin);
        printf("blocks %5d waves %5d: %.1f us (event)  span %.1f us  mean wave life %.1f us  XCCs %zu CUs %zu SIMDs %zu  "
               "peak co-resident waves %d  mean %.0f\n",
               blocks, waves, ms * 1e3, span / 100.0, life / waves / 100.0, xccs.size(), cus.size(), simds.size(), peak,
               life / span);
        CHECK(hipFree(drec)); CHECK(hipFree(dout));
    }
    return 0;
}
