// loop_ceiling.hip -- the attainable issue rate of the step kernels' SSA event loop (bench.py's VALU roofline peak).
//
// Runs the library's own certified f32 event loop (fast_propagate, csrc/epipf_device.hpp, the same code the step
// kernels and the one-workgroup filter inline) over one day (tmax = 1, as every filter step) from a mid-epidemic state of
// each BASELINE config, on grids that fill every SIMD.  Variant "uniform": every lane of a wave runs the same particle
// (same stream index j), so every lane is busy for every event -- the loop's instruction stream at lane use 1 with no
// per-step phases (weights, scan, search, gather) and no launch tails: the ceiling the step kernel's loop can reach on
// this chip.  Variant "distinct": lane i runs particle i (the step kernel's divergence, still no per-step phases).
// Timing only: the states are discarded.  One JSON line per (config, variant): lane-events/s over HIP events.
// scripts/loop_ceiling.sh adds a rocprofv3 PMC pass (wave64 VALU instructions per second of the same dispatches).
//
// build (scripts/loop_ceiling.sh): hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math
//        -I stochastic-epidemic-modelling_amd/csrc -I stochastic-epidemic-modelling_amd/lib -o <out> loop_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "epipf_device.hpp"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

using namespace epipf;

struct State { double x[12]; };

template <int MODEL, int G>
__global__ __launch_bounds__(64) void loop_ceiling_kernel(ChainParam cp, State s0, int reps, int distinct,
                                                          unsigned long long* events) {
    constexpr int C = (MODEL == kSIR) ? 3 : (MODEL == kSEIR) ? 4 : 3 * G;
    const uint32_t lane = blockIdx.x * 64u + threadIdx.x;
    const uint32_t j = distinct ? lane : blockIdx.x;       // one wave per block: "uniform" = one particle per wave
    extern __shared__ unsigned char occupancy_pad[];       // dynamic LDS, sized by the host to cap waves per SIMD
    if (reps < 0) occupancy_pad[threadIdx.x] = 0;
    unsigned long long tot = 0;
    for (int r = 0; r < reps; ++r) {
        double x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = s0.x[c];
        int nev = 0, iters = 0;
        bool eligible = false;
        if (fast_propagate<MODEL, G>(x, cp, j, (uint32_t)r, 1.0, nev, iters, eligible)) tot += (unsigned long long)nev;
    }
    events[lane] = tot;
}

struct Cfg {
    int cfg, model, G;
    std::vector<double> theta, x;
};

template <int MODEL, int G>
static void run(const Cfg& c, int blocks, int reps, int distinct, int repeats, int waves_per_simd) {
    ChainParam cp;
    memset(&cp, 0, sizeof(cp));
    for (size_t i = 0; i < c.theta.size(); ++i) { cp.theta[i] = c.theta[i]; cp.thetaf[i] = (float)c.theta[i]; }
    cp.k0 = 0x1234567u; cp.k1 = 0x89abcdefu; cp.f = 0;
    cp.flags = kChainFastSsa;
    cp.clock_slack = 1.f; cp.band_slack = 1.f;
    State s0;
    memset(&s0, 0, sizeof(s0));
    for (size_t i = 0; i < c.x.size(); ++i) s0.x[i] = c.x[i];
    const size_t lanes = (size_t)blocks * 64;
    unsigned long long* d_ev;
    CHECK(hipMalloc(&d_ev, lanes * sizeof(unsigned long long)));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    // waves_per_simd > 0: dynamic LDS per one-wave block so that a CU (160 KiB, 4 SIMDs) holds at most that many
    const size_t lds = waves_per_simd > 0 ? (size_t)(163840 / (4 * waves_per_simd)) / 512 * 512 : 0;
    loop_ceiling_kernel<MODEL, G><<<blocks, 64, lds>>>(cp, s0, 2, distinct, d_ev);   // warm-up
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> ev(lanes);
    double best = 0, best_ms = 0, per_call = 0;
    for (int k = 0; k < repeats; ++k) {
        CHECK(hipEventRecord(a));
        loop_ceiling_kernel<MODEL, G><<<blocks, 64, lds>>>(cp, s0, reps, distinct, d_ev);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        CHECK(hipMemcpy(ev.data(), d_ev, lanes * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        double tot = 0;
        for (auto v : ev) tot += (double)v;
        const double rate = tot / (ms * 1e-3);
        if (rate > best) { best = rate; best_ms = ms; per_call = tot / (double)lanes / reps; }
    }
    printf("{\"config\": %d, \"variant\": \"%s\", \"lane_events_per_s\": %.6e, \"ms\": %.3f, \"events_per_call\": %.2f, "
           "\"waves\": %d, \"calls_per_lane\": %d, \"waves_per_simd_cap\": %d}\n", c.cfg, distinct ? "distinct" : "uniform",
           best, best_ms, per_call, blocks, reps, waves_per_simd);
    fflush(stdout);
    CHECK(hipFree(d_ev));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    // BASELINE configs' models and parameters (epipf/datasets.py benchmark_dataset) and a mid-epidemic state whose
    // event rate is near each config's measured events per particle-step (bench detail: 6 / 90 / 150 / 504 / 545)
    const Cfg cfgs[] = {
        {1, kSIR, 1, {2.0, 1.0}, {100, 3, 97}},
        {2, kSIR, 1, {0.25, 0.1}, {5000, 400, 4600}},
        {3, kSEIR, 1, {0.5, 0.2, 0.1}, {4000, 200, 400, 5400}},
        {4, kSIR, 1, {2.0, 1.0}, {2000, 250, 2570}},
        {5, kSubgroups, 2, {4.0, 1.0, 1.0, 4.0, 1.0}, {1000, 100, 930, 1500, 150, 1390}},
    };
    const char* only = argc > 1 ? argv[1] : "";
    const int blocks = argc > 2 ? atoi(argv[2]) : 8192;    // waves: 8 per SIMD requested (occupancy caps what runs)
    const int cap = argc > 3 ? atoi(argv[3]) : 0;         // waves per SIMD cap (0: the kernel's own occupancy)
    const int repeats = 3;
    for (const Cfg& c : cfgs) {
        char tag[8];
        snprintf(tag, sizeof(tag), "%d", c.cfg);
        if (*only && !strstr(only, tag)) continue;
        // about 8e9 lane-events per launch: ~20-60 ms at the measured rates
        const int reps = (int)(8e9 / ((double)blocks * 64 * (c.cfg == 1 ? 6 : c.cfg == 2 ? 90 : c.cfg == 3 ? 150 : 520)));
        for (int distinct = 0; distinct < 2; ++distinct) {
            if (c.model == kSIR) run<kSIR, 1>(c, blocks, reps, distinct, repeats, cap);
            else if (c.model == kSEIR) run<kSEIR, 1>(c, blocks, reps, distinct, repeats, cap);
            else run<kSubgroups, 2>(c, blocks, reps, distinct, repeats, cap);
        }
    }
    return 0;
}
