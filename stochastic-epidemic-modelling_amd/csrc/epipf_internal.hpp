// epipf_internal.hpp -- kernel argument blocks and launchers shared by epipf_kernels.hip and epipf_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "epipf_device.hpp"

namespace epipf {

// Device counters are spread over kCounterSlots cache lines: same-address atomics from every wave serialise
// (~10 ns each on MI355X), which at 5k waves per launch cost more than the launch itself.
constexpr int kCounterSlots = 64;
constexpr int kCounterStride = 16;   // u64 per slot = 128 B
constexpr int kNumCounters = 4;

__device__ __forceinline__ unsigned long long* counter_slot(unsigned long long* base) {
    return base + (size_t)((blockIdx.x + 7u * blockIdx.y) & (kCounterSlots - 1)) * kCounterStride;
}

// HBM layout (per context, sized at create for max_chains x t_max x n_particles):
//   hidden   int32 [max_chains][t_max][N][C]      particle states (the reference's hidden_process)
//   ancestry int32 [max_chains][t_max][N]         resampled parent indices (row 0 zeros)
//   wraw     f64   [2][max_chains][B*WG]          raw weights of the last produced step (double buffer)
//   wloc     f64   [2][max_chains][B*WG]          in-block inclusive prefix of wraw
//   bsum     f64   [2][max_chains][B]             block totals
//   log_zeta f64   [max_chains][T]
//   Y        f64   [T][K];  lf f64 [lf_max+1] = lgamma(n+1)
struct StepArgs {
    int N, T, B, wg, max_chains, resample_mode, count_events, lf_max;
    size_t hist_stride, anc_stride, wstride, bstride;
    double cert_k;                // K = N + 2D + 8 of the resampling certificate (epipf_device.hpp)
    const double* Y;
    const double* lf;
    const LogTab* logtab;         // fast_log table [kLogTabEntries] (context-resident)
    const ChainParam* cp;
    int32_t* hidden;
    int32_t* ancestry;
    double* wraw;
    double* wloc;
    double* bsum;
    double* log_zeta;
    int32_t* status;
    unsigned long long* counters;  // [kCounterSlots][kCounterStride]: [0] events, [1] resample fallbacks,
                                   // [2] SSA lane-iterations, [3] wave-iterations x 64 (summed on the host)
    double npop[kMaxG], mu[kMaxG], emu[kMaxG];
    int kmax[kMaxG];
};

struct PathArgs {
    int n_chains, N, T, C;
    size_t hist_stride, anc_stride;
    const int32_t* hidden;
    const int32_t* ancestry;
    const int32_t* chosen;
    int32_t* traj;
};

struct SimArgs {
    const LogTab* logtab;
    int n;
    uint32_t step;
    double tmax;
    const ChainParam* cp;
    const int32_t* in;
    int32_t* out;
    unsigned long long* events;
};

struct ResampleArgs {
    int N, B;
    double cert_k;
    const double* w;
    const double* u;
    double* wraw;
    double* wloc;
    double* bsum;
    int32_t* out;
    int32_t* status;
    unsigned long long* fallbacks;
};

size_t step_lds_bytes(int B, int wg);
hipError_t launch_filter(const StepArgs& a, int model, int G, int obs, int n_chains, hipStream_t s,
                         hipEvent_t ev_init, hipEvent_t ev_step0, hipEvent_t ev_end);
hipError_t launch_path_sample(const PathArgs& a, hipStream_t s);
hipError_t launch_log_table(LogTab* tab, hipStream_t s);
hipError_t launch_simulate(const SimArgs& a, int model, int G, hipStream_t s);
hipError_t launch_resample(const ResampleArgs& a, hipStream_t s);

}  // namespace epipf
