// epipf_internal.hpp -- kernel argument blocks and launchers shared by epipf_kernels.hip and epipf_api.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "epipf_device.hpp"

// roctx ranges (the debug build, EPIPF_ROCTX): one around each epipf_run (an MH iteration's filter) and one around
// the enqueue of each filter step, so a rocprofv3 --marker-trace timeline shows which host call a kernel belongs to
#ifdef EPIPF_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#define EPIPF_RANGE_PUSH(msg) roctxRangePushA(msg)
#define EPIPF_RANGE_POP() roctxRangePop()
#else
#define EPIPF_RANGE_PUSH(msg) ((void)0)
#define EPIPF_RANGE_POP() ((void)0)
#endif

namespace epipf {

// Device counters are spread over kCounterSlots cache lines: same-address atomics from every wave serialise
// (~10 ns each on MI355X), which at 5k waves per launch cost more than the launch itself.
constexpr int kCounterSlots = 64;
constexpr int kCounterStride = 16;   // u64 per slot = 128 B
constexpr int kNumCounters = 7;

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
//   Y        f64   [T][K];  lf f64 [2][lf_max+1] = log n! as hi, then lo (binary128 on the host, logfact.cpp)
struct StepArgs {
    int N, T, B, wg, max_chains, resample_mode, count_events, lf_max;   // wg: particles per block of the weight
                                                                        // layout (64; kGroupBlock for some lane runs)
    int chain0;                   // first chain of this launch (chain groups run on separate streams)
    int lanes;                    // lanes per particle in the SSA: 1 = pf_step_kernel, 2..16 = pf_step_group_kernel
    int lane_events;              // pf_step_group_kernel: events per lane per chunk
    int xcd_map;                  // 1: 1-D grid of B x chains, each chain's blocks on one XCD (step_block); 0: 2-D grid
    int seg, nseg;                // block-sum prefix: S blocks per segment, ceil(B / S) segments (<= kMaxSegments)
    int canon_per;                // 64-particle blocks per lane of the canonical total's scan (scan_block_sums16):
                                  // the 64-layout's share, ceil(ceil(B64 / S64) / 64) S64, S64 = prefix_segment(B64)
    size_t hist_stride, anc_stride, wstride, bstride;
    double cert_k;                // K = N + 2D + 8 of the resampling certificate (epipf_device.hpp)
    double ref_k;                 // 2E (1 + 2^-10): reference-ambiguity bracket (ref_halfwidth)
    const double* Y;
    const double* lf;             // log n!, n = 0..lf_max: hi parts, then lo parts (binom_logpmf_plain)
    const LogTab* logtab;         // glibc log table [kLogTabEntries] (context-resident)
    const ChainParam* cp;
    int32_t* hidden;
    int32_t* ancestry;
    double* wraw;
    double* wloc;
    double* bsum;
    double* log_zeta;
    int32_t* status;
    unsigned long long* counters;  // [kCounterSlots][kCounterStride]: [0] events, [1] resample fallbacks,
                                   // [2] SSA lane-iterations, [3] wave-iterations x 64, [4] particle-steps on
                                   // the exact SSA loop, [5] waves with one, [6] reference-ambiguous draws
                                   // (summed on the host)
    double npop[kMaxG], mu[kMaxG], emu[kMaxG];
    int kmax[kMaxG];
    int fused_y, fused_lf;        // one-workgroup filter: Y / the log n! table staged in LDS (epipf_fused.hpp)
    int group_lone;               // lane-group kernel: 1 = its instance without the minimum-waves register bound
                                  // (group_lone_instance, epipf_group.hpp), for launches too small to need the waves
};

struct PathArgs {
    int n_chains, N, T, C;
    size_t hist_stride, anc_stride;
    const int32_t* hidden;
    const int32_t* ancestry;
    const int32_t* chosen;      // per chain, or null: ChainParam::chosen (epipf_run_sampled)
    const ChainParam* cp;
    const int32_t* status;      // the last run's chain status: only EPIPF_STATUS_OK chains are walked
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

// full-path SSA (epipf_simulate_path): event-major outputs, so each loop iteration's stores are coalesced
struct SimPathArgs {
    const LogTab* logtab;
    int n, cap;
    uint32_t step;
    double tmax;
    const ChainParam* cp;
    const int32_t* in;
    double* times;               // [cap][n]
    int32_t* states;             // [cap][C][n]
    int32_t* nev;                // [n]
    int32_t* final_state;        // [n][C]
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

// ABC rejection (abc_algo.py:17-109).  One lane per trial; HBM layout per batch of n trials:
//   days  int32 [T][3][n]   S, I, R at each day 0..T-1 (the reference's daily table, day column implicit)
//   theta f64   [2][n]      beta, gamma;   dist f64 [n]
struct AbcArgs {
    const LogTab* logtab;
    const double* Y;             // [T][3] observed (S, I, R)
    int T, n, count;             // days, trials this launch, profiling counters on
    int g0;                      // abc_trials_kernel: first sorted position it runs (the ones before: lane groups)
    int group_end, group_lanes;  // the first group_end sorted trials on group_lanes lanes each (1: none)
    // length-ordered lanes (one lane per trial): predicted-length keys sorted with their trial offsets, lane g
    // runs trial perm[g].  NULL: lane g runs trial g.
    const int32_t* perm;
    uint32_t* sort_keys[2];
    int32_t* sort_vals[2];
    void* sort_temp;
    size_t sort_temp_bytes;
    uint32_t t0, f, k0, k1;      // first trial index, run index, Philox key
    double last_day;             // T - 1 as a kernel argument (an SGPR pair; a VALU int->f64 convert would not be)
    double prior_lo[2], prior_rng[2];   // lo and hi - lo (numpy uniform's range)
    double lam[3], pm[3];        // initial-count means Y[0].astype(int) and their mode probabilities
    // early rejection (epipf_abc only): a one-lane trial stops once its running sum of |I_d - Y_I,d| + |R_d - Y_R,d|
    // over the days passed exceeds this bound, which proves distance > threshold; INFINITY: off
    double reject_sum;
    int32_t* days;
    double* theta;
    double* dist;
    unsigned long long* counters;  // [0] events, [2] lane-iterations, [3] wave-iterations x 64
};

struct AbcSelectArgs {
    const double* dist;
    int n, need;
    double threshold;
    int32_t* idx;                // [need] accepted trial offsets, in trial order
    int32_t* count;              // [1] accepted (<= need)
};

struct AbcGatherArgs {
    const int32_t* days;
    const double* theta;
    const int32_t* idx;
    const int32_t* count;
    int n, T, slot0;
    double* traj;                // [samples][T][4]: day, S, I, R (abc_algo.py:56-62 column order)
    double* theta_out;           // [samples][2]
};

// Streams of one filter run: group g of the chains runs on s[g]; s[0] is the context stream, the others have
// waited for its inputs.  join[g] (g > 0) is recorded at the end of group g, and s[0] waits for all of them.
constexpr int kMaxFilterStreams = 8;
struct FilterStreams {
    int n;
    hipStream_t s[kMaxFilterStreams];
    hipEvent_t join[kMaxFilterStreams];
    hipEvent_t ev_init, ev_step0, ev_end;   // timing (profiling on) or null
    hipEvent_t g_begin[kMaxFilterStreams], g_end[kMaxFilterStreams];   // per-group step-kernel span, or null
};

// logfact.cpp (host, binary128): log n! and log p / log1p(-p) split into hi + lo doubles
void logfact_table(int n_max, double* out);
void log_p_split(double p, double* logp_hi, double* logp_lo, double* log1mp_hi, double* log1mp_lo);

size_t step_lds_bytes(int B, int wg);
size_t step_lds_bytes_seg(int B, int S, int wg);   // with S blocks per prefix segment (1: block sums in LDS)
// lane-group step kernel (epipf_group.hip): W lanes per particle, launched as grid (B, chains) x 64 W threads
using GroupStepFn = void (*)(const StepArgs& a, int p, dim3 grid, size_t lds, hipStream_t s);
GroupStepFn group_step_launcher(int model, int G, int obs, int W, int K);
bool group_shape_supported(int W, int K);
size_t group_lds_bytes(int B, int S, int C, int W, int K, int PB);
int prefix_segment(int B);
constexpr int kMaxSegments = 200;
// lane-group runs on 16-particle blocks keep every block sum and its prefix in LDS (S = 1) up to this many blocks
// (2 x 8 B each): a chain of 10^4 particles is 626 blocks, whose segmented prefix (S = 4) cost each workgroup's
// resampling search a dependent global load of its segment's block sums
constexpr int kMaxFlatGroupBlocks = 1280;
constexpr int kGroupBlock = 16;   // particles per block of the lane-group runs that spread a chain over every CU
hipError_t launch_filter(const StepArgs& a, int model, int G, int obs, int n_chains, const FilterStreams& fs);
// the one-workgroup filter (epipf_fused.hpp): init and every step of a chain in one launch, for N <= kFusedMaxN;
// one workgroup of fused_threads(N, W) threads per chain, W lanes per particle in the SSA
constexpr int kFusedMaxThreads = 512;    // 8 waves: up to 256 VGPRs a lane (2 waves per SIMD)
constexpr int kFusedMaxN = 512;     // N lanes of one particle each in a 512-thread workgroup
constexpr size_t kFusedLdsLimit = 64 * 1024;    // the default dynamic LDS limit of a launch
using FusedFn = void (*)(const StepArgs& a, int n_chains, int threads, size_t lds, hipStream_t s);
FusedFn fused_launcher(int model, int G, int obs, int W);
size_t fused_lds_bytes_of(int N, int C, int threads, int TK, int lf_n);   // TK / lf_n: doubles staged (0: none)
int fused_threads_of(int N, int W);
hipError_t launch_path_sample(const PathArgs& a, hipStream_t s);
hipError_t launch_simulate(const SimArgs& a, int model, int G, hipStream_t s);
hipError_t launch_simulate_path(const SimPathArgs& a, int model, int G, hipStream_t s);
hipError_t launch_resample(const ResampleArgs& a, hipStream_t s);
hipError_t launch_abc_trials(const AbcArgs& a, hipStream_t s, hipStream_t s2, hipEvent_t fork, hipEvent_t join);
size_t abc_sort_temp_bytes(int n);
hipError_t launch_abc_select(const AbcSelectArgs& a, hipStream_t s);
hipError_t launch_abc_gather(const AbcGatherArgs& a, int max_count, hipStream_t s);

}  // namespace epipf
