// epipf_api.cpp -- the C ABI of libepipf.so (declared in include/epipf.h).
//
// A context owns every device buffer for one (model, G, N, t_max, max_chains) shape and one HIP
// stream; the observations, the log-factorial table and the whole particle history stay resident in
// HBM across calls, so an MH iteration moves only the chain parameters (host->device, ~200 B per
// chain) and the log-likelihoods + status (device->host) over PCIe.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/epipf.h"
#include "abc_device.hpp"
#include "epipf_internal.hpp"

using namespace epipf;

namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return fail(EPIPF_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

template <class T>
int dalloc(T** p, size_t n) {
    if (n == 0) n = 1;
    if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) {
        *p = nullptr;
        return fail(EPIPF_ENOMEM, "hipMalloc of %zu bytes failed", n * sizeof(T));
    }
    return 0;
}

int default_wg(int N) {
    // One wave per block at every N: the block-sum prefix is segmented (scan_segments), so a block's LDS does
    // not grow with N.
    (void)N;
    return 64;
}
}  // namespace

namespace epipf {
// the host MH draws (host_mh.cpp) report their argument errors through the same per-thread message
int set_error(int code, const char* msg) { return fail(code, "%s", msg); }
}  // namespace epipf

struct epipf_ctx {
    int device = 0, model = 0, G = 1, C = 3, K = 3, N = 0, Tmax = 0, max_chains = 0, wg = 64, B = 0;
    hipStream_t stream = nullptr;
    size_t hist_stride = 0, anc_stride = 0, wstride = 0, bstride = 0;
    int32_t *hidden = nullptr, *ancestry = nullptr, *status = nullptr, *chosen = nullptr, *traj = nullptr;
    // status [max_chains] | counters | log_zeta [max_chains][t_max] in one block (device and pinned host), so that a
    // run's results come back in one copy; status, counters and log_zeta point into it
    void* res = nullptr;
    void* h_res = nullptr;
    size_t res_counters = 0, res_lz = 0;   // byte offsets of counters and log_zeta in the block
    int32_t* h_traj = nullptr;             // pinned staging of epipf_run_sampled's trajectories
    double *wraw = nullptr, *wloc = nullptr, *bsum = nullptr, *log_zeta = nullptr, *Y = nullptr, *lf = nullptr;
    ChainParam* cp = nullptr;
    LogTab* logtab = nullptr;
    unsigned long long* counters = nullptr;
    // pinned staging
    ChainParam* h_cp = nullptr;
    int32_t* h_status = nullptr;
    double* h_lz = nullptr;
    unsigned long long* h_counters = nullptr;
    int T = 0, lf_max = -1, lf_cap = 0, last_chains = 0, last_T = 0;
    bool have_Y = false, have_pop = false, have_run = false;
    int profiling = 0;   // EPIPF_PROFILE_* level
    double npop[kMaxG] = {0}, mu[kMaxG] = {0}, emu[kMaxG] = {0};
    int kmax[kMaxG] = {0};
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    epipf_stats stats{};
    // scratch for epipf_simulate / epipf_resample (grown on demand)
    size_t scratch_bytes = 0;
    void* scratch = nullptr;
    // ABC buffers (grown on demand): days, theta, dist for one batch; Y; accepted idx/count; output slots
    size_t abc_bytes = 0;
    void* abc = nullptr;
    bool abc_order = true;   // length-ordered ABC lanes (EPIPF_ABC_ORDER=0 disables)
    // lanes per trial for the longest ABC trials: 0 = automatic (abc_launch_trials), EPIPF_ABC_LANES overrides (1 = off)
    int abc_lanes = 0;
    double abc_frac = -1.0;  // share of the sorted trials on lane groups: < 0 automatic, EPIPF_ABC_GROUP_FRAC overrides
    bool fast_ssa = true;    // certified f32 event loop (EPIPF_SSA_FAST=0 disables; results are identical)
    bool seq_decide = false; // lane groups: the sequential decision pass instead of the fixed-point one
                             // (EPIPF_GROUP_DECIDE=seq; results are identical, A/B and tests)
    float clock_slack = 1.f; // EPIPF_CLOCK_SLACK >= 1 widens its clock band: replays on purpose (stress tests)
    float band_slack = 1.f;  // EPIPF_BAND_SLACK >= 1 widens the channel decision's band: exact decisions and redone
                             // lane-group chunks on purpose (stress tests)
    double tie_scale = 1.0;  // EPIPF_TIE_SCALE >= 1 widens particle_weight's tie band: the all-columns pass on purpose
    int n_streams = 4;   // chain groups on concurrent streams (EPIPF_STREAMS overrides, 1..kMaxFilterStreams)
    hipStream_t aux[kMaxFilterStreams] = {};
    hipEvent_t join[kMaxFilterStreams] = {};
    hipEvent_t fork = nullptr;
    hipEvent_t gb[kMaxFilterStreams] = {};   // per-group step spans (timing)
    hipEvent_t ge[kMaxFilterStreams] = {};
    int last_groups = 1;
    int lanes = 0;           // SSA lanes per particle: 0 = automatic (pick_lanes), else 1/2/4/8/16 (EPIPF_LANES)
    int lane_events = 0;     // events per lane per chunk of the lane-group kernel: 0 = automatic (EPIPF_LANE_EVENTS)
    int lane_blocks = 1280;  // automatic choice: lane groups up to this many particle blocks per launch
    int group_block = 0;     // lane-group runs' particles per block: 0 = automatic (pick_block), 16 or 64 (EPIPF_GROUP_BLOCK)
    int xcd_map = 1;         // XCD-aware placement of the step launches' blocks (EPIPF_XCD_MAP=0: 2-D grid)
    int group_lone = -1;     // lane-group runs' unbounded instance: -1 = by the launch's waves (pick_group_lone),
                             // 0 / 1 = never / wherever it exists (EPIPF_GROUP_LONE)
    // one-workgroup filter for N <= kFusedMaxN when the lanes are automatic: -1 = measured per batch size (FusedTune),
    // 1 = always, 0 = never (EPIPF_FUSED)
    int fused = -1;
    int fused_lanes = 0;     // its SSA lanes per particle: 0 = automatic (pick_fused), EPIPF_FUSED_LANES = 1/2/4/8/16
    uint64_t y_hash = 0;     // FNV-1a of the observations (epipf_set_observations): part of the path choice's key
    double split_p = -1.0;   // probs of the cached hi/lo split of log p, log1p(-p) (chains usually share probs)
    double split[4] = {0, 0, 0, 0};
};

// Lanes per particle for a run of n_chains filters.  The one-lane kernel needs ~20k waves per launch to fill the
// chip; below 8 chains of 10^4 particles (n_chains x B <= 1280 particle blocks) the lane-group kernel with W = 4
// runs each particle-step 1.6-2.1x faster (1-8 chains, BASELINE configs 2 and 5: profiles/r2e_lanes_sweep*.jsonl;
// W = 2, 16 and K > 1 measured no better).  Up to 640 blocks (4 chains of 10^4) W = 8 is faster since round 3's
// mask-based decision pass and swizzle broadcasts (one chain: configs 2 / 3 / 5 +10% / +8% / +9%, four chains
// +3% / 0% / +9%; at 8 chains W = 4 leads by 16-29%: profiles/r3k_lanes_sweep_chains.jsonl).  Since round 4's
// fixed-point decision pass (a chunk's decisions cost ~2.3 evaluations instead of W dependent ones) and the clock pass
// through LDS, W = 16 leads up to two chains of 10^4 (320 blocks; one chain: configs 2 / 3 / 5 +12% / +16% / +18%
// over W = 8, two chains +9% / +10% / +12%), W = 8 from three (profiles/r4i_*, r4k_*).  With W = 16 on 16-particle
// blocks (pick_block) the subgroup models keep W = 16 up to four chains (+27% over W = 8 at three and four) and SIR /
// SEIR take W = 8 up to six (+11% / +7% over W = 4 at six; profiles/r4aa_lanes_sweep.txt).
static int pick_lanes(const epipf_ctx* c, int n_chains) {
    if (c->lanes > 0) return c->lanes;
    const long blocks = (long)n_chains * c->B, lb = c->lane_blocks;
    if (c->model == EPIPF_SIR || c->model == EPIPF_SEIR)
        return blocks <= lb / 4 ? 16 : blocks <= lb * 3 / 4 ? 8 : blocks <= lb ? 4 : 1;
    // the W = 16 rule was measured on G = 2, whose decisions run as a fixed point (FastSubgroupsPacked::kFixedPoint,
    // G <= 2); G = 3, 4 keep the sequential pass (W dependent decisions per chunk) and round 3's W = 8
    if (c->G > 2) return blocks <= lb / 2 ? 8 : blocks <= lb ? 4 : 1;
    // round 5 (certified group clock): W = 16 leads up to six chains of 10^4 (+10% over W = 4 at six), W = 4 at eight
    // (profiles/r5l_lanes_pick_sweep.jsonl)
    return blocks <= lb * 3 / 4 ? 16 : blocks <= lb ? 4 : 1;
}

// Particles per block of a run's weight layout (block sums, in-block prefixes): 64, one wave of the one-lane kernel, or
// for W = 16 lane-group runs (at most two chains of 10^4, pick_lanes) kGroupBlock = 16 -- a chain of 10^4 particles is
// then 626 workgroups of 4 waves instead of 157 of 16 waves, spread over all 256 CUs.  Measured A/B
// (profiles/r4o_block_clock_ab.txt): W = 16, configs 2 / 3 / 5, one chain +1-2% / +4-6% / +18-20%, two chains 0-2% /
// 0-5% / +19%; at W = 8 the redundant block-sum scan per workgroup mostly costs more than the spread gains (-2% to -8%).
// EPIPF_GROUP_BLOCK = 16 / 64 forces either layout for W >= 8.
static int pick_block(const epipf_ctx* c, int W) {
    if (W < 8) return c->wg;
    if (c->group_block > 0) return c->group_block;
    return W >= 16 ? kGroupBlock : c->wg;
}

// The lane-group kernel's instance without the minimum-waves bound (epipf_group.hpp, group_lone_instance: subgroup
// models, G >= 2, W >= 8) when the launch's waves all stay resident at the unbounded kernel's occupancy -- 3 waves per
// SIMD at G = 2 (143 VGPRs), 2 at G = 3, 1 at G = 4 -- on the chip's 1024 SIMDs: BASELINE config 5's one chain of 10^4
// particles at W = 16 is 2,500 waves (2.4 per SIMD).  Larger launches keep the bounded instance (more waves resident, a
// few spills: +7% / +14% at two / four chains, profiles/README.md).
static int pick_group_lone(const epipf_ctx* c, const StepArgs& a, int n_chains) {
    if (a.lanes < 8 || c->model < EPIPF_SIR_SUBGROUPS || c->G < 2) return 0;
    if (c->group_lone >= 0) return c->group_lone;
    const long waves = (long)n_chains * a.B * ((long)a.wg * a.lanes / 64);
    const long per_simd = c->G == 2 ? 3 : c->G == 3 ? 2 : 1;
    return waves <= per_simd * 1024 ? 1 : 0;
}

// Lanes per particle of the one-workgroup filter (epipf_fused.hpp), or 0 when the run takes the step launches: N <=
// kFusedMaxN with the lanes automatic (an explicit epipf_set_lanes / EPIPF_LANES keeps the step kernels it names) and
// the chain's LDS within the default launch limit.  W: EPIPF_FUSED_LANES where its N W lanes fit one workgroup, else 1.
static int pick_fused(const epipf_ctx* c) {
    if (!c->fused || c->lanes > 0 || c->N > kFusedMaxN) return 0;
    const int W = (c->fused_lanes > 0 && c->N * c->fused_lanes <= kFusedMaxThreads) ? c->fused_lanes : 1;
    if (fused_lds_bytes_of(c->N, c->C, fused_threads_of(c->N, W), 0, 0) > kFusedLdsLimit) return 0;
    return W;
}

// Which path is faster depends on the events per particle-step, which the host cannot see ahead: one workgroup per
// chain wins where a step is little work or many chains fill the chip (config 1, N = 100, 6 events: 3.1x at 256
// chains, 1.3x at one), the step launches where one chain's many events want more than one CU (N = 100 at config
// 2's 90 events: 2.2x the other way).  So a workload's first runs time both (the filter's device span, HIP events;
// results identical either way) and the faster one stays.
//
// The choice is PER PROCESS, keyed on the workload (device, model, observation model, N, T, chains per run, the
// observations and the population), not per context: contexts that run concurrently on one GPU (run_pipelined's chain
// groups) pool their timed runs into one decision and all take the same path.  Each context deciding alone from
// timings taken while the others ran let them settle on different paths.  A new dataset, T or population
// is a new key, so epipf_set_observations / epipf_set_population start a fresh choice.
struct FusedKey {
    int device, model, G, obs, N, T, n_chains;
    uint64_t data;
    bool operator<(const FusedKey& o) const {
        if (device != o.device) return device < o.device;
        if (model != o.model) return model < o.model;
        if (G != o.G) return G < o.G;
        if (obs != o.obs) return obs < o.obs;
        if (N != o.N) return N < o.N;
        if (T != o.T) return T < o.T;
        if (n_chains != o.n_chains) return n_chains < o.n_chains;
        return data < o.data;
    }
};
struct FusedTune {
    int issued = 0;                    // tuning runs handed out (they alternate the paths)
    int runs = 0;                      // tuning runs recorded
    double best[2] = {1e300, 1e300};   // fastest timed run: [0] step launches, [1] one-workgroup filter
    int choice = -1;
};
static std::mutex g_tune_mu;
static std::map<FusedKey, FusedTune> g_tune;

static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}

static FusedKey fused_key(const epipf_ctx* c, int obs, int n_chains) {
    const uint64_t h = fnv1a(c->y_hash, c->npop, sizeof(double) * c->G);
    return FusedKey{c->device, c->model, c->G, obs, c->N, c->T, n_chains, fnv1a(h, c->mu, sizeof(double) * c->G)};
}

// EPIPF_FUSED=auto (the default): the first 8 runs of a workload in this process alternate the paths (fused first, each
// path's first run untimed), then each path's fastest of three timed runs decides, the step launches only by a 15%
// margin (concurrent contexts share the device while they time, which spreads both paths' times).  *timed: this run's
// device span is recorded; *tuning: the choice is still open.
static bool fused_decide(const epipf_ctx* c, int obs, int n_chains, bool& timed, bool& tuning) {
    timed = tuning = false;
    if (c->fused >= 0) return c->fused == 1;
    std::lock_guard<std::mutex> lk(g_tune_mu);
    FusedTune& t = g_tune[fused_key(c, obs, n_chains)];
    if (t.choice >= 0) return t.choice == 1;
    tuning = true;
    const int r = t.issued++;
    timed = r >= 2;                                      // runs 0, 1: warm-up of each path
    return (r & 1) == 0;                                 // even runs: fused
}

static void fused_record(const epipf_ctx* c, int obs, int n_chains, bool fused, double seconds) {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    FusedTune& t = g_tune[fused_key(c, obs, n_chains)];
    t.best[fused ? 1 : 0] = std::min(t.best[fused ? 1 : 0], seconds);
    if (++t.runs >= 8 && t.choice < 0) t.choice = t.best[0] < 0.85 * t.best[1] ? 0 : 1;
}

static hipError_t launch_fused_run(const StepArgs& a, const epipf_ctx* c, int obs, int n_chains, const FilterStreams& fs) {
    const FusedFn f = fused_launcher(c->model, c->G, obs, a.lanes);
    if (!f) return hipErrorInvalidValue;
    const int threads = fused_threads_of(a.N, a.lanes);
    const size_t lds = fused_lds_bytes_of(a.N, c->C, threads, a.fused_y ? a.T * c->K : 0,
                                          a.fused_lf ? 2 * (a.lf_max + 1) : 0);
    const hipStream_t s = fs.s[0];
    if (fs.ev_init) (void)hipEventRecord(fs.ev_init, s);
    if (fs.ev_step0) (void)hipEventRecord(fs.ev_step0, s);    // init runs inside the one launch: its time is in step_ms
    if (fs.g_begin[0]) (void)hipEventRecord(fs.g_begin[0], s);
    EPIPF_RANGE_PUSH("one-workgroup filter");
    f(a, n_chains, threads, lds, s);
    EPIPF_RANGE_POP();
    if (fs.g_end[0]) (void)hipEventRecord(fs.g_end[0], s);
    if (fs.ev_end) (void)hipEventRecord(fs.ev_end, s);
    return hipGetLastError();
}

static int pick_lane_events(const epipf_ctx* c, int W) {
    if (W <= 1) return 1;
    if (c->lane_events > 0 && group_shape_supported(W, c->lane_events)) return c->lane_events;
    return 1;                                       // K > 1 measured no faster (profiles/r2e_lanes_sweep.jsonl)
}

// K = N + 2D + 8 of the resampling certificate (epipf_device.hpp): D bounds the depth of the parallel
// reduction tree behind every prefix: in-block scan (6 shuffle levels + <=4 wave offsets + 1) = 11 <= 16,
// block-sum scan 16 + 2 * ceil(B / WG) sequential chunk adds, +2 for the final adds.
static double cert_k(int N, int B, int S, int wg) {
    const int nseg = (B + S - 1) / S;
    const int per = ((nseg + wg - 1) / wg) * S;          // sequential block-sum adds per lane (scan_segments)
    const int D = 34 + 2 * per;
    return (double)N + 2.0 * D + 8.0;
}

// E: the relative error by which the reference's weights (scipy binom.pmf / norm.pdf) may differ from the device's.
// Binomial: scipy's Boost evaluation measured against 200-bit truth (scripts/scipy_pmf_envelope.py,
// profiles/r3_scipy_pmf_envelope.json: at most ~0.6 of this envelope over n <= 2e5, all p) plus the device's own
// <= 2 ulps; normal: numpy's exp vs the device's plus the divisions, 2^-48 (16 ulps).  An envelope, measured, not
// proven: the count it drives (resample_ref_ambiguous) is a diagnostic, never a decision.
static double ref_pmf_envelope(int obs_model, int n_max) {
    if (obs_model == EPIPF_OBS_NORMAL) return 0x1.0p-48;
    return 4e-12 + 1e-16 * (double)std::max(n_max, 0);
}

static int theta_dim(int model, int G) { return model == EPIPF_SIR ? 2 : model == EPIPF_SEIR ? 3 : G * G + 1; }

static void free_ctx(epipf_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* dev[] = {c->hidden, c->ancestry, c->res, c->chosen, c->traj, c->wraw, c->wloc, c->bsum,
                   c->Y, c->lf, c->cp, c->logtab, c->scratch, c->abc};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    void* host[] = {c->h_cp, c->h_res, c->h_traj};
    for (void* p : host)
        if (p) (void)hipHostFree(p);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->join)
        if (e) (void)hipEventDestroy(e);
    for (int g = 0; g < kMaxFilterStreams; ++g) {
        if (c->gb[g]) (void)hipEventDestroy(c->gb[g]);
        if (c->ge[g]) (void)hipEventDestroy(c->ge[g]);
    }
    if (c->fork) (void)hipEventDestroy(c->fork);
    for (auto& st : c->aux)
        if (st) { (void)hipStreamSynchronize(st); (void)hipStreamDestroy(st); }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// Streams and events of chain groups 0..n-1 (group 0 runs on c->stream), created on first use.
static bool ensure_streams(epipf_ctx* c, int n) {
    for (int g = 0; g < n; ++g) {
        if (!c->gb[g] && hipEventCreate(&c->gb[g]) != hipSuccess) return false;
        if (!c->ge[g] && hipEventCreate(&c->ge[g]) != hipSuccess) return false;
        if (g == 0) continue;
        if (!c->aux[g] && hipStreamCreateWithFlags(&c->aux[g], hipStreamNonBlocking) != hipSuccess) return false;
        if (!c->join[g] && hipEventCreateWithFlags(&c->join[g], hipEventDisableTiming) != hipSuccess) return false;
    }
    return true;
}

extern "C" {

const char* epipf_last_error(void) { return g_err.c_str(); }
int epipf_abi_version(void) { return EPIPF_ABI_VERSION; }
static_assert(kStatusOk == EPIPF_STATUS_OK && kStatusDegenerate == EPIPF_STATUS_DEGENERATE &&
              kStatusSkipped == EPIPF_STATUS_SKIPPED, "device status codes");
const char* epipf_build_id(void) {
#ifdef EPIPF_BUILD_ID
    return EPIPF_BUILD_ID;
#else
    return "unknown";
#endif
}
int epipf_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int epipf_create(epipf_ctx** out, int device, int model, int groups, int n_particles, int t_max, int max_chains) {
    if (!out) return fail(EPIPF_EINVAL, "out is NULL");
    *out = nullptr;
    if (model < EPIPF_SIR || model > EPIPF_SIR_SUBGROUPS2) return fail(EPIPF_EINVAL, "unknown model %d", model);
    const int G = model >= EPIPF_SIR_SUBGROUPS ? groups : 1;
    if (G < 1 || G > kMaxG) return fail(EPIPF_EINVAL, "groups must be in [1, %d], got %d", kMaxG, groups);
    if (n_particles < 1 || t_max < 1 || max_chains < 1) return fail(EPIPF_EINVAL, "n_particles, t_max, max_chains must be >= 1");
    if (t_max > (1 << 24)) return fail(EPIPF_EINVAL, "t_max must be < 2^24 (Philox step field)");
    int ndev = epipf_device_count();
    if (device < 0 || device >= ndev) return fail(EPIPF_EINVAL, "device %d not present (%d HIP devices)", device, ndev);
    epipf_ctx* c = new epipf_ctx();
    c->device = device;
    c->model = model;
    c->G = G;
    c->C = model == EPIPF_SIR ? 3 : model == EPIPF_SEIR ? 4 : 3 * G;
    c->K = model == EPIPF_SIR_SUBGROUPS2 ? 3 : c->C;
    c->N = n_particles;
    c->Tmax = t_max;
    c->max_chains = max_chains;
    c->wg = default_wg(n_particles);
    if (const char* e = getenv("EPIPF_SSA_FAST")) c->fast_ssa = atoi(e) != 0;
    if (const char* e = getenv("EPIPF_GROUP_DECIDE")) c->seq_decide = strcmp(e, "seq") == 0;
    if (const char* e = getenv("EPIPF_CLOCK_SLACK")) c->clock_slack = std::max(1.0f, std::min(1e12f, (float)atof(e)));
    if (const char* e = getenv("EPIPF_BAND_SLACK")) c->band_slack = std::max(1.0f, std::min(1e4f, (float)atof(e)));
    if (const char* e = getenv("EPIPF_TIE_SCALE")) c->tie_scale = std::max(1.0, std::min(1e300, atof(e)));
    if (const char* e = getenv("EPIPF_STREAMS")) c->n_streams = std::max(1, std::min(kMaxFilterStreams, atoi(e)));
    if (const char* e = getenv("EPIPF_LANES")) {
        const int w = atoi(e);
        if (w == 0 || w == 1 || w == 2 || w == 4 || w == 8 || w == 16) c->lanes = w;
    }
    if (const char* e = getenv("EPIPF_LANE_BLOCKS")) c->lane_blocks = std::max(0, atoi(e));
    if (const char* e = getenv("EPIPF_LANE_EVENTS")) c->lane_events = std::max(0, atoi(e));
    if (const char* e = getenv("EPIPF_GROUP_BLOCK")) {
        const int b = atoi(e);
        if (b == 0 || b == kGroupBlock || b == 64) c->group_block = b;
    }
    if (const char* e = getenv("EPIPF_XCD_MAP")) c->xcd_map = atoi(e) != 0;
    if (const char* e = getenv("EPIPF_GROUP_LONE")) c->group_lone = strcmp(e, "auto") == 0 ? -1 : atoi(e) != 0;
    if (const char* e = getenv("EPIPF_FUSED")) c->fused = strcmp(e, "auto") == 0 ? -1 : atoi(e) != 0;
    if (const char* e = getenv("EPIPF_FUSED_LANES")) {
        const int w = atoi(e);
        if (w == 0 || w == 1 || w == 2 || w == 4 || w == 8 || w == 16) c->fused_lanes = w;
    }
    c->B = (n_particles + c->wg - 1) / c->wg;
    if (step_lds_bytes(c->B, c->wg) > 160 * 1024) {
        free_ctx(c);
        return fail(EPIPF_EINVAL, "n_particles %d too large for one LDS block-sum table", n_particles);
    }
    c->hist_stride = (size_t)t_max * n_particles * c->C;
    c->anc_stride = (size_t)t_max * n_particles;
    c->wstride = (size_t)c->B * c->wg;
    // block sums for the lane-group runs' 16-particle blocks too (pick_block, kGroupBlock)
    c->bstride = std::max((size_t)c->B, (size_t)((n_particles + kGroupBlock - 1) / kGroupBlock));
    int rc = 0;
    if (hipSetDevice(device) != hipSuccess) { free_ctx(c); return fail(EPIPF_EHIP, "hipSetDevice(%d) failed", device); }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        free_ctx(c);
        return fail(EPIPF_EHIP, "hipStreamCreate failed");
    }
    rc |= dalloc(&c->hidden, (size_t)max_chains * c->hist_stride);
    rc |= dalloc(&c->ancestry, (size_t)max_chains * c->anc_stride);
    c->res_counters = ((sizeof(int32_t) * (size_t)max_chains + 127) / 128) * 128;
    c->res_lz = c->res_counters + sizeof(unsigned long long) * (size_t)kCounterSlots * kCounterStride;
    const size_t res_bytes = c->res_lz + sizeof(double) * (size_t)max_chains * t_max;
    rc |= dalloc(reinterpret_cast<char**>(&c->res), res_bytes);
    rc |= dalloc(&c->chosen, (size_t)max_chains);
    rc |= dalloc(&c->traj, (size_t)max_chains * t_max * c->C);
    rc |= dalloc(&c->wraw, 2 * (size_t)max_chains * c->wstride);
    rc |= dalloc(&c->wloc, 2 * (size_t)max_chains * c->wstride);
    rc |= dalloc(&c->bsum, 2 * (size_t)max_chains * c->bstride);
    rc |= dalloc(&c->cp, (size_t)max_chains);
    rc |= dalloc(&c->logtab, (size_t)kLogTabEntries);
    if (rc) { free_ctx(c); return EPIPF_ENOMEM; }
    c->status = static_cast<int32_t*>(c->res);
    c->counters = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->res) + c->res_counters);
    c->log_zeta = reinterpret_cast<double*>(static_cast<char*>(c->res) + c->res_lz);
    if (hipHostMalloc((void**)&c->h_cp, sizeof(ChainParam) * max_chains) != hipSuccess ||
        hipHostMalloc(&c->h_res, res_bytes) != hipSuccess ||
        hipHostMalloc((void**)&c->h_traj, sizeof(int32_t) * (size_t)max_chains * t_max * c->C) != hipSuccess) {
        free_ctx(c);
        return fail(EPIPF_ENOMEM, "hipHostMalloc failed");
    }
    c->h_status = static_cast<int32_t*>(c->h_res);
    c->h_counters = reinterpret_cast<unsigned long long*>(static_cast<char*>(c->h_res) + c->res_counters);
    c->h_lz = reinterpret_cast<double*>(static_cast<char*>(c->h_res) + c->res_lz);
    for (auto& e : c->ev)
        if (hipEventCreate(&e) != hipSuccess) { free_ctx(c); return fail(EPIPF_EHIP, "hipEventCreate failed"); }
    if (hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess) {
        free_ctx(c);
        return fail(EPIPF_EHIP, "hipEventCreate failed");
    }
    // on the context stream (a NULL-stream copy would take one of the process's hardware queues, which the
    // chain-group streams then share: two groups serialised, -14% at config 2)
    LogTab lt[kLogTabEntries];                 // synchronised below, before it goes out of scope
    glibc_log_table(lt);
    if (hipMemcpyAsync(c->logtab, lt, sizeof lt, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * (size_t)kCounterSlots * kCounterStride, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        free_ctx(c);
        return fail(EPIPF_EHIP, "counter init failed");
    }
    *out = c;
    return EPIPF_OK;
}

void epipf_destroy(epipf_ctx* ctx) { free_ctx(ctx); }

int epipf_set_observations(epipf_ctx* c, const double* Y, int T, int K) {
    if (!c || !Y) return fail(EPIPF_EINVAL, "NULL argument");
    if (T < 1 || T > c->Tmax) return fail(EPIPF_EINVAL, "T=%d outside [1, t_max=%d]", T, c->Tmax);
    if (K != c->K) return fail(EPIPF_EINVAL, "K=%d but the model observes %d columns", K, c->K);
    HIP_TRY(hipSetDevice(c->device));
    if (c->Y) { HIP_TRY(hipStreamSynchronize(c->stream)); (void)hipFree(c->Y); c->Y = nullptr; }
    if (dalloc(&c->Y, (size_t)T * K)) return EPIPF_ENOMEM;
    HIP_TRY(hipMemcpyAsync(c->Y, Y, sizeof(double) * (size_t)T * K, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->T = T;
    c->y_hash = fnv1a(0xcbf29ce484222325ull ^ (uint64_t)T, Y, sizeof(double) * (size_t)T * K);
    c->have_Y = true;
    return EPIPF_OK;
}

int epipf_set_population(epipf_ctx* c, const double* n_population, const double* mu) {
    if (!c || !n_population || !mu) return fail(EPIPF_EINVAL, "NULL argument");
    double tot = 0.0;
    for (int g = 0; g < c->G; ++g) {
        const double np_ = n_population[g], m = mu[g];
        if (!(np_ >= 0.0) || np_ != std::floor(np_) || np_ > 1e8)
            return fail(EPIPF_EINVAL, "n_population[%d]=%g must be an integer in [0, 1e8]", g, np_);
        if (!(m >= 0.0) || m > 700.0) return fail(EPIPF_EINVAL, "mu[%d]=%g must be in [0, 700]", g, m);
        c->npop[g] = np_;
        c->mu[g] = m;
        c->emu[g] = std::exp(-m);                                        // host glibc, as the oracle
        c->kmax[g] = (int)std::ceil(m + 40.0 * std::sqrt(m) + 60.0);
        tot += np_;
    }
    const int need = (int)tot;
    HIP_TRY(hipSetDevice(c->device));
    if (need + 1 > c->lf_cap) {
        if (c->lf) { HIP_TRY(hipStreamSynchronize(c->stream)); (void)hipFree(c->lf); c->lf = nullptr; }
        if (dalloc(&c->lf, 2 * ((size_t)need + 1))) return EPIPF_ENOMEM;
        c->lf_cap = need + 1;
    }
    if (need != c->lf_max) {
        std::vector<double> lf(2 * ((size_t)need + 1));
        logfact_table(need, lf.data());                      // log n!: hi parts, then lo parts (binom_logpmf)
        HIP_TRY(hipMemcpyAsync(c->lf, lf.data(), sizeof(double) * lf.size(), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        c->lf_max = need;
    }
    c->have_pop = true;
    return EPIPF_OK;
}

static int run_impl(epipf_ctx* c, int n_chains, const double* theta, int d, int obs_model, const double* probs,
                    const uint64_t* keys, const uint32_t* filter_index, const int32_t* active, int resample_mode,
                    const int32_t* chosen, double* log_zetas_out, int32_t* status_out, int32_t* traj_out) {
    if (!c || !theta || !probs || !keys || !filter_index || !status_out) return fail(EPIPF_EINVAL, "NULL argument");
    if ((chosen == nullptr) != (traj_out == nullptr)) return fail(EPIPF_EINVAL, "chosen and traj_out go together");
    if (!c->have_Y) return fail(EPIPF_ESTATE, "epipf_set_observations was not called");
    if (!c->have_pop) return fail(EPIPF_ESTATE, "epipf_set_population was not called");
    if (n_chains < 1 || n_chains > c->max_chains) return fail(EPIPF_EINVAL, "n_chains=%d outside [1, %d]", n_chains, c->max_chains);
    if (d != theta_dim(c->model, c->G)) return fail(EPIPF_EINVAL, "theta has %d entries per chain, model needs %d", d, theta_dim(c->model, c->G));
    if (obs_model != EPIPF_OBS_BINOMIAL && obs_model != EPIPF_OBS_NORMAL) return fail(EPIPF_EINVAL, "bad obs_model %d", obs_model);
    if (resample_mode != EPIPF_RESAMPLE_MULTINOMIAL && resample_mode != EPIPF_RESAMPLE_SYSTEMATIC)
        return fail(EPIPF_EINVAL, "bad resample_mode %d", resample_mode);
    int n_active = 0;
    for (int ch = 0; ch < n_chains; ++ch) {
        const bool on = !active || active[ch];
        ChainParam& q = c->h_cp[ch];
        memset(&q, 0, sizeof q);
        for (int i = 0; i < d; ++i) {
            const double v = theta[(size_t)ch * d + i];
            if (on && !(v >= 0.0 && v < INFINITY))
                return fail(EPIPF_EINVAL, "theta[%d][%d]=%g: parameters must be finite and >= 0 (pmcmc.py:333)", ch, i, v);
            q.theta[i] = v;
            q.thetaf[i] = (float)v;
        }
        q.probs = probs[ch];
        if (!(probs[ch] == c->split_p) && !(std::isnan(probs[ch]) && std::isnan(c->split_p))) {   // binary128: ~2 us
            log_p_split(probs[ch], &c->split[0], &c->split[1], &c->split[2], &c->split[3]);
            c->split_p = probs[ch];
        }
        q.logp = c->split[0]; q.logp_lo = c->split[1]; q.log1mp = c->split[2]; q.log1mp_lo = c->split[3];
        // particle_weight's tie tolerance: 8x a bound on its plain column logs' error, ~8 roundings of at most half
        // an ulp of the sum of their terms' magnitudes, 2 log n! + n (|log p| + |log1p(-p)|) at n = the population
        const double nmax = (double)std::max(c->lf_max, 0);
        q.tie_tol = (2.0 * std::lgamma(nmax + 1.0) * 1.01 + nmax * (std::fabs(q.logp) + std::fabs(q.log1mp)) + 1.0) *
                    0x1.0p-46 * c->tie_scale;
        q.k0 = (uint32_t)keys[ch];
        q.k1 = (uint32_t)(keys[ch] >> 32);
        q.f = filter_index[ch];
        q.flags = (c->fast_ssa ? kChainFastSsa : 0u) | (c->seq_decide ? kChainSeqDecide : 0u);
        q.clock_slack = c->clock_slack;
        q.band_slack = c->band_slack;
        q.skip = on ? 0 : 1;                            // the first kernel writes the chain's status from it
        q.chosen = -1;
        if (chosen && on) {
            if (chosen[ch] >= c->N) return fail(EPIPF_EINVAL, "chosen[%d]=%d outside [0, N)", ch, chosen[ch]);
            q.chosen = chosen[ch] < 0 ? -1 : chosen[ch];
        }
        n_active += on;
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(c->cp, c->h_cp, sizeof(ChainParam) * n_chains, hipMemcpyHostToDevice, c->stream));

    StepArgs a{};
    a.N = c->N; a.T = c->T; a.max_chains = c->max_chains;
    bool tune_timed = false, tuning = false;
    const int fusedW = pick_fused(c) && fused_decide(c, obs_model, n_chains, tune_timed, tuning) ? pick_fused(c) : 0;
    a.lanes = fusedW ? fusedW : pick_lanes(c, n_chains);
    a.wg = fusedW ? 64 : pick_block(c, a.lanes);
    a.B = (c->N + a.wg - 1) / a.wg;
    a.group_lone = fusedW ? 0 : pick_group_lone(c, a, n_chains);
    a.resample_mode = resample_mode; a.count_events = c->profiling >= EPIPF_PROFILE_COUNTERS ? 1 : 0; a.lf_max = c->lf_max;
    a.hist_stride = c->hist_stride; a.anc_stride = c->anc_stride; a.wstride = c->wstride; a.bstride = c->bstride;
    // S blocks per prefix segment: 1 (every block sum in LDS) for lane-group runs on 16-particle blocks up to
    // kMaxFlatGroupBlocks, else the smallest power of two with at most kMaxSegments segments
    // The 16-particle layout sums the step total in the 64-particle layout's order (scan_block_sums16): its segments are
    // whole segments of that layout (S16 = 4 S64, the same as prefix_segment(B16) wherever it segments), and canon_per
    // is that layout's 64-blocks per lane, so the log-likelihood is the same whichever layout the chain count picks.
    const int B64 = (c->N + 63) / 64, S64 = prefix_segment(B64);
    a.canon_per = ((B64 + S64 - 1) / S64 + 63) / 64 * S64;
    a.seg = fusedW ? 1 : (a.lanes > 1 && a.wg == kGroupBlock) ? (a.B <= kMaxFlatGroupBlocks ? 1 : 4 * S64) : prefix_segment(a.B);
    a.nseg = (a.B + a.seg - 1) / a.seg;
    a.cert_k = cert_k(c->N, a.B, a.seg, 64);              // the block-sum scans run on 64 lanes whatever the layout
    // the reference-ambiguity test runs with the other device counters (bench.py's untimed counters iteration, the
    // parity tests); ref_k = 0 switches it off in the timed, production launches
    a.ref_k = a.count_events ? 2.0 * ref_pmf_envelope(obs_model, c->lf_max) * (1.0 + 0x1.0p-10) : 0.0;
    a.Y = c->Y; a.lf = c->lf; a.logtab = c->logtab; a.cp = c->cp; a.hidden = c->hidden; a.ancestry = c->ancestry;
    a.wraw = c->wraw; a.wloc = c->wloc; a.bsum = c->bsum; a.log_zeta = c->log_zeta; a.status = c->status;
    a.counters = c->counters;
    a.lane_events = pick_lane_events(c, a.lanes);
    a.xcd_map = c->xcd_map;
    if (a.lanes > 1 && !group_shape_supported(a.lanes, a.lane_events))
        return fail(EPIPF_EINVAL, "no lane-group kernel for %d lanes x %d events", a.lanes, a.lane_events);
    c->stats.last_lanes = a.lanes;
    c->stats.last_lane_events = a.lane_events;
    c->stats.last_fused = fusedW ? 1 : 0;
    if (fusedW) {   // stage Y, then the log n! table, in LDS while the launch stays within the default dynamic LDS limit
        const int threads = fused_threads_of(a.N, a.lanes);
        const size_t base = fused_lds_bytes_of(a.N, c->C, threads, 0, 0);
        const size_t yb = sizeof(double) * (size_t)a.T * c->K, lb = sizeof(double) * 2 * (size_t)(a.lf_max + 1);
        a.fused_y = base + yb <= kFusedLdsLimit;
        a.fused_lf = a.lf_max >= 0 && base + (a.fused_y ? yb : 0) + lb <= kFusedLdsLimit;
    }
    for (int g = 0; g < kMaxG; ++g) { a.npop[g] = c->npop[g]; a.mu[g] = c->mu[g]; a.emu[g] = c->emu[g]; a.kmax[g] = c->kmax[g]; }

    EPIPF_RANGE_PUSH("epipf_run");
    struct RangeEnd { ~RangeEnd() { EPIPF_RANGE_POP(); } } range_end;
    FilterStreams fs{};
    fs.n = fusedW ? 1 : std::min(c->n_streams, n_chains);
    // Created on first use, not with the context: HIP maps streams onto its few hardware queues in creation order,
    // so contexts that each run one group (run_pipelined) get one stream each and land on different queues.
    if (!ensure_streams(c, fs.n)) return fail(EPIPF_EHIP, "auxiliary stream creation failed");
    fs.s[0] = c->stream;
    if (fs.n > 1) HIP_TRY(hipEventRecord(c->fork, c->stream));    // the groups' inputs are on c->stream
    for (int g = 1; g < fs.n; ++g) {
        fs.s[g] = c->aux[g];
        fs.join[g] = c->join[g];
        HIP_TRY(hipStreamWaitEvent(c->aux[g], c->fork, 0));
    }
    fs.ev_init = (c->profiling || tuning) ? c->ev[0] : nullptr;   // the path choice times the device span
    fs.ev_step0 = c->profiling ? c->ev[1] : nullptr;
    fs.ev_end = (c->profiling || tuning) ? c->ev[2] : nullptr;
    for (int g = 0; g < fs.n; ++g) {
        fs.g_begin[g] = c->profiling ? c->gb[g] : nullptr;
        fs.g_end[g] = c->profiling ? c->ge[g] : nullptr;
    }
    c->last_groups = fs.n;
    hipError_t le = fusedW ? launch_fused_run(a, c, obs_model, n_chains, fs)
                           : launch_filter(a, c->model, c->G, obs_model, n_chains, fs);
    if (le != hipSuccess) return fail(EPIPF_EHIP, "kernel launch failed: %s", hipGetErrorString(le));
    if (chosen) {   // the path sampler (pmcmc.py:236-248) after the filter, on the same stream: no second round trip
        PathArgs pa{};
        pa.n_chains = n_chains; pa.N = c->N; pa.T = c->T; pa.C = c->C;
        pa.hist_stride = c->hist_stride; pa.anc_stride = c->anc_stride;
        pa.hidden = c->hidden; pa.ancestry = c->ancestry; pa.chosen = nullptr; pa.cp = c->cp; pa.status = c->status;
        pa.traj = c->traj;
        hipError_t pe = launch_path_sample(pa, c->stream);
        if (pe != hipSuccess) return fail(EPIPF_EHIP, "path kernel launch failed: %s", hipGetErrorString(pe));
        HIP_TRY(hipMemcpyAsync(c->h_traj, c->traj, sizeof(int32_t) * (size_t)n_chains * c->T * c->C,
                               hipMemcpyDeviceToHost, c->stream));
    }
    // status, counters and the log-likelihoods: one copy of the result block's prefix
    HIP_TRY(hipMemcpyAsync(c->h_res, c->res, c->res_lz + sizeof(double) * (size_t)n_chains * c->T, hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (tuning) {   // the filter's device span, init to the last step (host threads contending for the GIL do not
                    // enter it, as they would a wall clock)
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[2]));
        fused_record(c, obs_model, n_chains, fusedW != 0, tune_timed ? (double)ms : 1e300);
    }
    if (chosen) memcpy(traj_out, c->h_traj, sizeof(int32_t) * (size_t)n_chains * c->T * c->C);
    memcpy(status_out, c->h_status, sizeof(int32_t) * n_chains);
    if (log_zetas_out) {
        memcpy(log_zetas_out, c->h_lz, sizeof(double) * (size_t)n_chains * c->T);
        // steps after a degenerate step were never run: report -inf there (zetas = 0)
        for (int ch = 0; ch < n_chains; ++ch) {
            if (c->h_status[ch] == EPIPF_STATUS_OK) continue;
            bool dead = false;
            for (int p = 0; p < c->T; ++p) {
                double& v = log_zetas_out[(size_t)ch * c->T + p];
                if (c->h_status[ch] == EPIPF_STATUS_SKIPPED) { v = NAN; continue; }
                if (dead) v = -INFINITY;
                else if (v == -INFINITY) dead = true;
            }
        }
    }
    if (c->profiling) {
        float ms_init = 0.f, ms_step = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms_init, c->ev[0], c->ev[1]));
        HIP_TRY(hipEventElapsedTime(&ms_step, c->ev[1], c->ev[2]));
        c->stats.init_ms += ms_init;
        c->stats.init_launches += 1;
        c->stats.step_ms += ms_step;
        c->stats.step_launches += fusedW ? 1 : c->T - 1;   // the one-workgroup filter: one launch per run
        for (int g = 0; g < c->last_groups; ++g) {        // each group's back-to-back step kernels on its stream
            float ms_g = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms_g, c->gb[g], c->ge[g]));
            c->stats.step_kernel_ms += ms_g;
            c->stats.step_kernel_launches += fusedW ? 1 : c->T - 1;
        }
    }
    unsigned long long tot[kNumCounters] = {};
    for (int sl = 0; sl < kCounterSlots; ++sl)
        for (int k = 0; k < kNumCounters; ++k) tot[k] += c->h_counters[(size_t)sl * kCounterStride + k];
    c->stats.events = (int64_t)tot[0];
    c->stats.resample_fallbacks = (int64_t)tot[1];
    c->stats.lane_iterations = (int64_t)tot[2];
    c->stats.wave_lane_slots = (int64_t)tot[3];
    c->stats.ssa_exact_lanes = (int64_t)tot[4];
    c->stats.ssa_exact_waves = (int64_t)tot[5];
    c->stats.resample_ref_ambiguous = (int64_t)tot[6];
    c->stats.particle_steps += (int64_t)n_active * c->N * c->T;
    c->stats.filters += n_active;
    c->last_chains = n_chains;
    c->last_T = c->T;
    c->have_run = true;
    return EPIPF_OK;
}

int epipf_run(epipf_ctx* c, int n_chains, const double* theta, int d, int obs_model, const double* probs,
              const uint64_t* keys, const uint32_t* filter_index, const int32_t* active, int resample_mode,
              double* log_zetas_out, int32_t* status_out) {
    return run_impl(c, n_chains, theta, d, obs_model, probs, keys, filter_index, active, resample_mode, nullptr,
                    log_zetas_out, status_out, nullptr);
}

int epipf_run_sampled(epipf_ctx* c, int n_chains, const double* theta, int d, int obs_model, const double* probs,
                      const uint64_t* keys, const uint32_t* filter_index, const int32_t* active, int resample_mode,
                      const int32_t* chosen, double* log_zetas_out, int32_t* status_out, int32_t* traj_out) {
    if (!chosen || !traj_out) return fail(EPIPF_EINVAL, "NULL argument");
    return run_impl(c, n_chains, theta, d, obs_model, probs, keys, filter_index, active, resample_mode, chosen,
                    log_zetas_out, status_out, traj_out);
}

int epipf_copy_history(epipf_ctx* c, int n_chains, int32_t* hidden_out, int32_t* ancestry_out) {
    if (!c) return fail(EPIPF_EINVAL, "NULL context");
    if (!c->have_run) return fail(EPIPF_ESTATE, "no filter has run on this context");
    if (n_chains < 1 || n_chains > c->last_chains) return fail(EPIPF_EINVAL, "n_chains=%d outside [1, %d]", n_chains, c->last_chains);
    HIP_TRY(hipSetDevice(c->device));
    const size_t T = (size_t)c->last_T;
    if (hidden_out)
        HIP_TRY(hipMemcpy2DAsync(hidden_out, T * c->N * c->C * sizeof(int32_t), c->hidden, c->hist_stride * sizeof(int32_t),
                                 T * c->N * c->C * sizeof(int32_t), n_chains, hipMemcpyDeviceToHost, c->stream));
    if (ancestry_out)
        HIP_TRY(hipMemcpy2DAsync(ancestry_out, T * c->N * sizeof(int32_t), c->ancestry, c->anc_stride * sizeof(int32_t),
                                 T * c->N * sizeof(int32_t), n_chains, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EPIPF_OK;
}

int epipf_path_sample(epipf_ctx* c, int n_chains, const int32_t* chosen, int32_t* traj_out) {
    if (!c || !chosen || !traj_out) return fail(EPIPF_EINVAL, "NULL argument");
    if (!c->have_run) return fail(EPIPF_ESTATE, "no filter has run on this context");
    if (n_chains < 1 || n_chains > c->last_chains) return fail(EPIPF_EINVAL, "n_chains=%d outside [1, %d]", n_chains, c->last_chains);
    for (int ch = 0; ch < n_chains; ++ch)
        if (chosen[ch] < 0 || chosen[ch] >= c->N) return fail(EPIPF_EINVAL, "chosen[%d]=%d outside [0, N)", ch, chosen[ch]);
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(c->chosen, chosen, sizeof(int32_t) * n_chains, hipMemcpyHostToDevice, c->stream));
    PathArgs a{};
    a.n_chains = n_chains; a.N = c->N; a.T = c->last_T; a.C = c->C;
    a.hist_stride = c->hist_stride; a.anc_stride = c->anc_stride;
    a.hidden = c->hidden; a.ancestry = c->ancestry; a.chosen = c->chosen; a.cp = c->cp; a.status = c->status;
    a.traj = c->traj;
    hipError_t le = launch_path_sample(a, c->stream);
    if (le != hipSuccess) return fail(EPIPF_EHIP, "path kernel launch failed: %s", hipGetErrorString(le));
    HIP_TRY(hipMemcpyAsync(traj_out, c->traj, sizeof(int32_t) * (size_t)n_chains * a.T * a.C, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EPIPF_OK;
}

static int ensure_scratch(epipf_ctx* c, size_t bytes) {
    if (bytes <= c->scratch_bytes) return 0;
    if (c->scratch) { (void)hipStreamSynchronize(c->stream); (void)hipFree(c->scratch); c->scratch = nullptr; c->scratch_bytes = 0; }
    if (hipMalloc(&c->scratch, bytes) != hipSuccess) return fail(EPIPF_ENOMEM, "scratch hipMalloc(%zu) failed", bytes);
    c->scratch_bytes = bytes;
    return 0;
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Scratch above this stays allocated only for the call that needed it (a one-off long full-path batch must not pin
// gigabytes on a context get_engine caches for the whole process); the stream is synchronised by then.
constexpr size_t kScratchKeepBytes = (size_t)64 << 20;
static void trim_scratch(epipf_ctx* c) {
    if (c->scratch && c->scratch_bytes > kScratchKeepBytes) {
        (void)hipFree(c->scratch);
        c->scratch = nullptr;
        c->scratch_bytes = 0;
    }
}

int epipf_simulate(epipf_ctx* c, int n, const int32_t* states_in, const double* theta, int d, double max_time,
                   uint64_t key, uint32_t filter_index, uint32_t step, int32_t* states_out, int64_t* events_out) {
    if (!c || !states_in || !theta || !states_out) return fail(EPIPF_EINVAL, "NULL argument");
    if (n < 0) return fail(EPIPF_EINVAL, "n < 0");
    if (d != theta_dim(c->model, c->G)) return fail(EPIPF_EINVAL, "theta needs %d entries", theta_dim(c->model, c->G));
    if (!(max_time >= 0.0)) return fail(EPIPF_EINVAL, "max_time must be >= 0");
    for (int i = 0; i < d; ++i)
        if (!(theta[i] >= 0.0 && theta[i] < INFINITY)) return fail(EPIPF_EINVAL, "theta[%d] must be finite and >= 0", i);
    for (size_t i = 0; i < (size_t)n * c->C; ++i)
        if (states_in[i] < 0) return fail(EPIPF_EINVAL, "states must be non-negative");
    if (n == 0) { if (events_out) *events_out = 0; return EPIPF_OK; }
    HIP_TRY(hipSetDevice(c->device));
    const size_t sb = align256((size_t)n * c->C * sizeof(int32_t));
    const size_t need = align256(sizeof(ChainParam)) + 2 * sb + 256;
    if (ensure_scratch(c, need)) return EPIPF_ENOMEM;
    char* base = (char*)c->scratch;
    ChainParam* dcp = (ChainParam*)base;
    int32_t* din = (int32_t*)(base + align256(sizeof(ChainParam)));
    int32_t* dout = (int32_t*)((char*)din + sb);
    unsigned long long* dev_events = (unsigned long long*)((char*)dout + sb);
    ChainParam q;
    memset(&q, 0, sizeof q);
    for (int i = 0; i < d; ++i) { q.theta[i] = theta[i]; q.thetaf[i] = (float)theta[i]; }
    q.k0 = (uint32_t)key; q.k1 = (uint32_t)(key >> 32); q.f = filter_index;
    q.flags = (c->fast_ssa ? kChainFastSsa : 0u) | (c->seq_decide ? kChainSeqDecide : 0u);
    q.clock_slack = c->clock_slack;
    q.band_slack = c->band_slack;
    HIP_TRY(hipMemcpyAsync(dcp, &q, sizeof q, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(din, states_in, sizeof(int32_t) * (size_t)n * c->C, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(dev_events, 0, sizeof(unsigned long long), c->stream));
    SimArgs a{};
    a.logtab = c->logtab; a.n = n; a.step = step; a.tmax = max_time; a.cp = dcp; a.in = din; a.out = dout; a.events = dev_events;
    hipError_t le = launch_simulate(a, c->model, c->G, c->stream);
    if (le != hipSuccess) return fail(EPIPF_EHIP, "simulate launch failed: %s", hipGetErrorString(le));
    unsigned long long ev = 0;
    HIP_TRY(hipMemcpyAsync(states_out, dout, sizeof(int32_t) * (size_t)n * c->C, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&ev, dev_events, sizeof ev, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (events_out) *events_out = (int64_t)ev;
    return EPIPF_OK;
}

int epipf_simulate_path(epipf_ctx* c, int n, const int32_t* states_in, const double* theta, int d, double max_time,
                        uint64_t key, uint32_t filter_index, uint32_t step, int max_events, double* times_out,
                        int32_t* states_out, int32_t* n_events_out, int32_t* final_out) {
    if (!c || !states_in || !theta || !n_events_out) return fail(EPIPF_EINVAL, "NULL argument");
    if (n < 0 || max_events < 0) return fail(EPIPF_EINVAL, "n and max_events must be >= 0");
    if (max_events > 0 && (!times_out || !states_out)) return fail(EPIPF_EINVAL, "NULL path output");
    if (d != theta_dim(c->model, c->G)) return fail(EPIPF_EINVAL, "theta needs %d entries", theta_dim(c->model, c->G));
    if (!(max_time >= 0.0)) return fail(EPIPF_EINVAL, "max_time must be >= 0");
    for (int i = 0; i < d; ++i)
        if (!(theta[i] >= 0.0 && theta[i] < INFINITY)) return fail(EPIPF_EINVAL, "theta[%d] must be finite and >= 0", i);
    for (size_t i = 0; i < (size_t)n * c->C; ++i)
        if (states_in[i] < 0) return fail(EPIPF_EINVAL, "states must be non-negative");
    if (n == 0) return EPIPF_OK;
    HIP_TRY(hipSetDevice(c->device));
    const int C = c->C;
    const size_t cap = (size_t)max_events;
    const size_t sb = align256((size_t)n * C * sizeof(int32_t));
    const size_t tb = align256(cap * n * sizeof(double)), xb = align256(cap * n * C * sizeof(int32_t));
    const size_t nb = align256((size_t)n * sizeof(int32_t));
    const size_t need = align256(sizeof(ChainParam)) + 2 * sb + tb + xb + nb;
    if (ensure_scratch(c, need)) return EPIPF_ENOMEM;
    char* base = (char*)c->scratch;
    ChainParam* dcp = (ChainParam*)base;
    int32_t* din = (int32_t*)(base + align256(sizeof(ChainParam)));
    int32_t* dfin = (int32_t*)((char*)din + sb);
    double* dt = (double*)((char*)dfin + sb);
    int32_t* dx = (int32_t*)((char*)dt + tb);
    int32_t* dnev = (int32_t*)((char*)dx + xb);
    ChainParam q;
    memset(&q, 0, sizeof q);
    for (int i = 0; i < d; ++i) { q.theta[i] = theta[i]; q.thetaf[i] = (float)theta[i]; }
    q.k0 = (uint32_t)key; q.k1 = (uint32_t)(key >> 32); q.f = filter_index;
    q.clock_slack = 1.f;
    q.band_slack = 1.f;
    HIP_TRY(hipMemcpyAsync(dcp, &q, sizeof q, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(din, states_in, sizeof(int32_t) * (size_t)n * C, hipMemcpyHostToDevice, c->stream));
    SimPathArgs a{};
    a.logtab = c->logtab; a.n = n; a.cap = max_events; a.step = step; a.tmax = max_time; a.cp = dcp; a.in = din;
    a.times = dt; a.states = dx; a.nev = dnev; a.final_state = dfin;
    hipError_t le = launch_simulate_path(a, c->model, c->G, c->stream);
    if (le != hipSuccess) return fail(EPIPF_EHIP, "simulate_path launch failed: %s", hipGetErrorString(le));
    HIP_TRY(hipMemcpyAsync(n_events_out, dnev, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    if (final_out)
        HIP_TRY(hipMemcpyAsync(final_out, dfin, sizeof(int32_t) * (size_t)n * C, hipMemcpyDeviceToHost, c->stream));
    std::vector<double> ht;
    std::vector<int32_t> hx;
    if (cap > 0) {
        ht.resize(cap * n);
        hx.resize(cap * n * C);
        HIP_TRY(hipMemcpyAsync(ht.data(), dt, sizeof(double) * cap * n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(hx.data(), dx, sizeof(int32_t) * cap * n * C, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int j = 0; j < n; ++j) {                       // event-major device rows -> one row per trajectory
        const size_t m = std::min<size_t>(cap, (size_t)std::max(n_events_out[j], 0));
        for (size_t e = 0; e < m; ++e) {
            times_out[(size_t)j * cap + e] = ht[e * n + j];
            for (int k = 0; k < C; ++k) states_out[((size_t)j * cap + e) * C + k] = hx[(e * C + k) * n + j];
        }
    }
    trim_scratch(c);
    return EPIPF_OK;
}

int epipf_glibc_log(int64_t n, const double* x, double* out) {
    if (n < 0 || (n > 0 && (!x || !out))) return fail(EPIPF_EINVAL, "NULL argument");
    LogTab lt[kLogTabEntries];
    glibc_log_table(lt);
    for (int64_t i = 0; i < n; ++i) out[i] = glibc_log_impl(x[i], lt);
    return EPIPF_OK;
}

int epipf_clock_log(int64_t n, const double* x, double* out) {
    if (n < 0 || (n > 0 && (!x || !out))) return fail(EPIPF_EINVAL, "NULL argument");
    LogTab lt[kLogTabEntries];
    glibc_log_table(lt);
    for (int64_t i = 0; i < n; ++i) out[i] = clock_log_impl(x[i], lt);
    return EPIPF_OK;
}

int epipf_resample(epipf_ctx* c, int n, const double* w, const double* u, int32_t* out, int64_t* fallbacks_out) {
    if (!c || !w || !u || !out) return fail(EPIPF_EINVAL, "NULL argument");
    if (n < 1) return fail(EPIPF_EINVAL, "n must be >= 1");
    const int B = (n + 255) / 256;
    if (step_lds_bytes(B, 256) > 160 * 1024) return fail(EPIPF_EINVAL, "n too large");
    for (int i = 0; i < n; ++i)
        if (!(u[i] >= 0.0 && u[i] < 1.0)) return fail(EPIPF_EINVAL, "uniforms must lie in [0, 1)");
    HIP_TRY(hipSetDevice(c->device));
    const size_t nw = align256(sizeof(double) * (size_t)B * 256);
    const size_t need = 4 * nw + align256(sizeof(double) * B) + align256(sizeof(int32_t) * (size_t)n) + 512;
    if (ensure_scratch(c, need)) return EPIPF_ENOMEM;
    char* p = (char*)c->scratch;
    ResampleArgs a{};
    a.N = n; a.B = B; a.cert_k = cert_k(n, B, prefix_segment(B), 256);
    double* dw = (double*)p; p += nw;
    double* du = (double*)p; p += nw;
    a.wraw = (double*)p; p += nw;
    a.wloc = (double*)p; p += nw;
    a.bsum = (double*)p; p += align256(sizeof(double) * B);
    a.out = (int32_t*)p; p += align256(sizeof(int32_t) * (size_t)n);
    a.status = (int32_t*)p; p += 256;
    a.fallbacks = (unsigned long long*)p;
    a.w = dw; a.u = du;
    HIP_TRY(hipMemcpyAsync(dw, w, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(du, u, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(a.status, 0, 256 + sizeof(unsigned long long), c->stream));
    hipError_t le = launch_resample(a, c->stream);
    if (le != hipSuccess) return fail(EPIPF_EHIP, "resample launch failed: %s", hipGetErrorString(le));
    int32_t st = 0;
    unsigned long long fb = 0;
    HIP_TRY(hipMemcpyAsync(out, a.out, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&st, a.status, sizeof st, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(&fb, a.fallbacks, sizeof fb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (fallbacks_out) *fallbacks_out = (int64_t)fb;
    return st ? EPIPF_STATUS_DEGENERATE : EPIPF_OK;
}

// ------------------------------------------------------------------------------- ABC rejection
namespace {
struct AbcPlan {
    AbcArgs args{};
    double* Ydev = nullptr;
    int32_t* idx = nullptr;
    int32_t* count = nullptr;
    double* traj = nullptr;
    double* theta_out = nullptr;
};

// Validates the reference-level arguments and fills the launch constants (abc_algo.py:35-39).
int abc_prepare(epipf_ctx* c, const double* Y, int T, const double* priors, uint64_t key, uint32_t run_index,
                AbcArgs& a) {
    if (!c || !Y || !priors) return fail(EPIPF_EINVAL, "NULL argument");
    if (T < 1 || T > kAbcMaxDays) return fail(EPIPF_EINVAL, "T=%d outside [1, %d]", T, kAbcMaxDays);
    for (int q = 0; q < 4; ++q)
        if (!(priors[q] >= 0.0 && priors[q] < INFINITY))
            return fail(EPIPF_EINVAL, "priors[%d]=%g: prior bounds must be finite and >= 0", q, priors[q]);
    for (int q = 0; q < 3 * T; ++q)
        if (!std::isfinite(Y[q])) return fail(EPIPF_EINVAL, "observed_data[%d][%d] is not finite", q / 3, q % 3);
    memset(&a, 0, sizeof a);
    for (int j = 0; j < 2; ++j) {
        a.prior_lo[j] = priors[2 * j];
        a.prior_rng[j] = priors[2 * j + 1] - priors[2 * j];           // numpy uniform: low + (high - low) * U
    }
    for (int q = 0; q < 3; ++q) {
        const double lam = std::trunc(Y[q]);                           // Y[0].astype(int), :38
        if (lam < 0.0) return fail(EPIPF_EINVAL, "observed_data[0][%d]=%g: Poisson lam < 0 (numpy raises)", q, Y[q]);
        if (lam > 1e9) return fail(EPIPF_EINVAL, "observed_data[0][%d]=%g: initial count above 1e9", q, Y[q]);
        a.lam[q] = lam;
        a.pm[q] = lam > 0.0 ? std::exp(-lam + lam * std::log(lam) - std::lgamma(lam + 1.0)) : 0.0;   // host glibc
    }
    a.T = T;
    a.reject_sum = INFINITY;                                           // early rejection: epipf_abc turns it on
    a.last_day = (double)(T - 1);
    a.f = run_index;
    a.k0 = (uint32_t)key;
    a.k1 = (uint32_t)(key >> 32);
    a.logtab = c->logtab;
    a.counters = c->counters;
    a.count = c->profiling >= EPIPF_PROFILE_COUNTERS ? 1 : 0;
    c->abc_order = true;
    if (const char* e = getenv("EPIPF_ABC_ORDER")) c->abc_order = atoi(e) != 0;
    // lane groups for the longest trials (abc_trials_group_kernel): W lanes each for the first `abc_frac` of
    // the sorted trials; EPIPF_ABC_LANES = 1 turns them off (results are identical either way)
    a.group_lanes = c->abc_lanes;                                      // 0: chosen per launch (abc_launch_trials)
    if (const char* e = getenv("EPIPF_ABC_LANES")) {
        const int w = atoi(e);
        if (w == 1 || w == 2 || w == 4 || w == 8 || w == 16) a.group_lanes = w;
    }
    c->abc_frac = -1.0;
    if (const char* e = getenv("EPIPF_ABC_GROUP_FRAC")) c->abc_frac = atof(e) < 0.0 ? -1.0 : std::min(1.0, atof(e));
    return 0;
}

// Carves the ABC buffers for batches of up to `batch` trials and `samples` output slots.
int abc_buffers(epipf_ctx* c, int T, int batch, int samples, AbcPlan& p) {
    const size_t b = (size_t)batch;
    const size_t sz_days = align256(sizeof(int32_t) * 3 * (size_t)T * b), sz_theta = align256(sizeof(double) * 2 * b),
                 sz_dist = align256(sizeof(double) * b), sz_Y = align256(sizeof(double) * 3 * (size_t)T),
                 sz_idx = align256(sizeof(int32_t) * (size_t)(samples + 1)), sz_cnt = 256,
                 sz_traj = align256(sizeof(double) * 4 * (size_t)T * samples), sz_to = align256(sizeof(double) * 2 * (size_t)samples);
    const size_t sz_key = align256(sizeof(uint32_t) * b), sz_tmp = align256(abc_sort_temp_bytes(batch));
    const size_t need = sz_days + sz_theta + sz_dist + sz_Y + sz_idx + sz_cnt + sz_traj + sz_to + 4 * sz_key + sz_tmp;
    if (need > c->abc_bytes) {
        if (c->abc) { (void)hipStreamSynchronize(c->stream); (void)hipFree(c->abc); c->abc = nullptr; c->abc_bytes = 0; }
        if (hipMalloc(&c->abc, need) != hipSuccess) return fail(EPIPF_ENOMEM, "ABC buffers hipMalloc(%zu) failed", need);
        c->abc_bytes = need;
    }
    char* q = (char*)c->abc;
    p.args.days = (int32_t*)q; q += sz_days;
    p.args.theta = (double*)q; q += sz_theta;
    p.args.dist = (double*)q; q += sz_dist;
    p.Ydev = (double*)q; q += sz_Y;
    p.idx = (int32_t*)q; q += sz_idx;
    p.count = (int32_t*)q; q += sz_cnt;
    p.traj = (double*)q; q += sz_traj;
    p.theta_out = (double*)q; q += sz_to;
    for (int k = 0; k < 2; ++k) {
        p.args.sort_keys[k] = (uint32_t*)q; q += sz_key;
        p.args.sort_vals[k] = (int32_t*)q; q += sz_key;
    }
    p.args.sort_temp = q;
    p.args.sort_temp_bytes = sz_tmp;
    p.args.perm = c->abc_order ? p.args.sort_vals[1] : nullptr;
    p.args.Y = p.Ydev;
    return 0;
}

// Launches of up to this many trials put the longest half on lane groups of 4 (automatic mode).  Measured at the
// reference's setting (profiles/r3_abc_lane_groups.jsonl): 64k-trial launches 5.0 -> 3.1 ms (+61% end to end), 128k
// +14%, 192k +3.5%.  Larger launches are throughput-bound and take lane groups only for the longest few percent: with
// round 4's lane-group kernel (fixed-point decisions, early rejection on groups) W = 16 on the longest 4% of a 256k
// launch runs the reference's setting at 3.06-3.08e7 trials/s against 2.90-2.93e7 one lane (3-8%: 3.0-3.07e7; W = 4
// or 8, 10% and more lose; profiles/r4q_abc_groups.txt).
constexpr int kAbcGroupMaxTrials = 196608;
constexpr int kAbcLongLanes = 16;
constexpr double kAbcLongFrac = 0.04;

int abc_launch_trials(epipf_ctx* c, AbcArgs& a0, uint32_t t0, int n) {
    AbcArgs& a = a0;
    a.t0 = t0;
    a.n = n;
    const int lanes = a.group_lanes;
    if (lanes == 0) a.group_lanes = n <= kAbcGroupMaxTrials ? 4 : kAbcLongLanes;
    const double frac = c->abc_frac >= 0.0 ? c->abc_frac : n <= kAbcGroupMaxTrials ? 0.5 : kAbcLongFrac;
    a.group_end = (a.group_lanes > 1 && a.perm) ? (int)std::llround(frac * n) : 0;
    if (a.group_end > 0 && !ensure_streams(c, 2)) return fail(EPIPF_EHIP, "auxiliary stream creation failed");
    if (c->profiling) HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    hipError_t le = launch_abc_trials(a, c->stream, a.group_end > 0 ? c->aux[1] : nullptr, c->fork, c->join[1]);
    a.group_lanes = lanes;                                             // automatic again for the next launch
    if (le != hipSuccess) return fail(EPIPF_EHIP, "ABC trial kernel launch failed: %s", hipGetErrorString(le));
    if (c->profiling) HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    return 0;
}

int abc_account(epipf_ctx* c, int n) {
    if (c->profiling) {
        HIP_TRY(hipEventSynchronize(c->ev[1]));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        c->stats.abc_ms += ms;
    }
    c->stats.abc_launches += 1;
    c->stats.abc_trials += n;
    return 0;
}

int abc_read_counters(epipf_ctx* c) {
    if (c->profiling < EPIPF_PROFILE_COUNTERS) return 0;
    HIP_TRY(hipMemcpyAsync(c->h_counters, c->counters, sizeof(unsigned long long) * (size_t)kCounterSlots * kCounterStride,
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    unsigned long long tot[kNumCounters] = {};
    for (int sl = 0; sl < kCounterSlots; ++sl)
        for (int k = 0; k < kNumCounters; ++k) tot[k] += c->h_counters[(size_t)sl * kCounterStride + k];
    c->stats.events = (int64_t)tot[0];
    c->stats.lane_iterations = (int64_t)tot[2];
    c->stats.wave_lane_slots = (int64_t)tot[3];
    return 0;
}
}  // namespace

int epipf_abc_trials(epipf_ctx* c, const double* Y, int T, const double* priors, uint64_t key, uint32_t run_index,
                     uint32_t t0, int n, double* theta_out, int32_t* rows_out, double* dist_out, int64_t* events_out) {
    AbcPlan p;
    if (int rc = abc_prepare(c, Y, T, priors, key, run_index, p.args)) return rc;
    if (!theta_out) return fail(EPIPF_EINVAL, "theta_out is NULL");
    if (n < 0 || (uint64_t)t0 + (uint64_t)n > (1ull << 32)) return fail(EPIPF_EINVAL, "trials [t0, t0+n) must lie in [0, 2^32)");
    if (n == 0) { if (events_out) *events_out = 0; return EPIPF_OK; }
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = abc_buffers(c, T, n, 1, p)) return rc;
    AbcArgs a = p.args;
    HIP_TRY(hipMemcpyAsync(p.Ydev, Y, sizeof(double) * 3 * (size_t)T, hipMemcpyHostToDevice, c->stream));
    unsigned long long ev_before = 0;
    const bool counting = a.count != 0;
    if (counting) {
        if (int rc = abc_read_counters(c)) return rc;
        ev_before = (unsigned long long)c->stats.events;
    }
    if (int rc = abc_launch_trials(c, a, t0, n)) return rc;
    std::vector<double> th((size_t)2 * n);
    HIP_TRY(hipMemcpyAsync(th.data(), a.theta, sizeof(double) * 2 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    if (dist_out) HIP_TRY(hipMemcpyAsync(dist_out, a.dist, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    std::vector<int32_t> days;
    if (rows_out) {
        days.resize((size_t)3 * T * n);
        HIP_TRY(hipMemcpyAsync(days.data(), a.days, sizeof(int32_t) * days.size(), hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (int rc = abc_account(c, n)) return rc;
    for (int i = 0; i < n; ++i) {
        theta_out[2 * (size_t)i] = th[i];
        theta_out[2 * (size_t)i + 1] = th[(size_t)n + i];
    }
    if (rows_out)   // device [T][3][n] -> caller [n][T][3]
        for (int d = 0; d < T; ++d)
            for (int q = 0; q < 3; ++q)
                for (int i = 0; i < n; ++i)
                    rows_out[((size_t)i * T + d) * 3 + q] = days[((size_t)d * 3 + q) * n + i];
    if (events_out) {
        *events_out = -1;
        if (counting) {
            if (int rc = abc_read_counters(c)) return rc;
            *events_out = (int64_t)((unsigned long long)c->stats.events - ev_before);
        }
    }
    return EPIPF_OK;
}

int epipf_abc(epipf_ctx* c, const double* Y, int T, int no_of_samples, double threshold, const double* priors,
              uint64_t key, uint32_t run_index, int64_t max_trials, int batch, double* theta_out, double* traj_out,
              int64_t* trials_out, int32_t* accepted_out) {
    AbcPlan p;
    if (int rc = abc_prepare(c, Y, T, priors, key, run_index, p.args)) return rc;
    if (!theta_out || !traj_out || !trials_out || !accepted_out) return fail(EPIPF_EINVAL, "NULL output pointer");
    if (no_of_samples < 0) return fail(EPIPF_EINVAL, "no_of_samples < 0");
    if (std::isnan(threshold)) return fail(EPIPF_EINVAL, "threshold is NaN");
    if (max_trials < 0 || max_trials > (int64_t)(1ull << 32)) return fail(EPIPF_EINVAL, "max_trials must lie in [0, 2^32]");
    if (batch < 0) return fail(EPIPF_EINVAL, "batch < 0");
    *trials_out = 0;
    *accepted_out = 0;
    if (no_of_samples == 0) return EPIPF_OK;
    // batch sizes: fixed, or 256k trials first, then 1.25x the trials the observed acceptance rate predicts for
    // the samples still missing (x4 while nothing is accepted), within [256k, 1M] and a day table < 4 GiB.  A launch
    // lasts at least as long as its longest trials (~5 ms at the reference's setting), and below ~4 waves per SIMD
    // the exact f64 trial loop is latency-bound: 64k trials take 5.2 ms, 256k 7.0 ms (1.27e7 vs 3.74e7 trials/s,
    // profiles/r2p_abc_batch_sweep.jsonl), so a smaller batch saves nothing and a second launch costs a whole floor.
    const int64_t cap_days = ((int64_t)1 << 32) / (12 * (int64_t)T);
    const int max_batch = (int)std::max<int64_t>(256, std::min<int64_t>(batch > 0 ? batch : (1 << 20), cap_days));
    const int min_batch = std::min(1 << 18, max_batch);
    int cur = batch > 0 ? std::min(batch, max_batch) : min_batch;
    HIP_TRY(hipSetDevice(c->device));
    if (int rc = abc_buffers(c, T, max_batch, no_of_samples, p)) return rc;
    AbcArgs a = p.args;
    // Early rejection: the device distance is fl(fl(fl(si/T) + fl(sr/T))/2) with si, sr numpy-pairwise
    // sums of the non-negative terms fl(|x_d - y_d|), so it is at least the exact (sum_I + sum_R)/(2T) times
    // (1-u)^(T+4), and a lane's running sum `acc` of the same terms is at most that exact sum times (1+u)^(2T+2)
    // (u = 2^-53).  acc > 2T threshold (1 + 1e-9) therefore proves distance > threshold (for T <= kAbcMaxDays,
    // (3T+8)u < 2e-10), i.e. the trial is rejected (abc_algo.py:30-33).  Only for a threshold well inside the normal
    // range (no subnormal quotients); EPIPF_ABC_EARLY=0 turns it off (the results are identical either way).
    bool early = threshold >= 1e-200 && threshold <= 1e200;
    if (const char* e = getenv("EPIPF_ABC_EARLY")) early = early && atoi(e) != 0;
    if (early) a.reject_sum = 2.0 * (double)T * threshold * (1.0 + 1e-9);
    HIP_TRY(hipMemcpyAsync(p.Ydev, Y, sizeof(double) * 3 * (size_t)T, hipMemcpyHostToDevice, c->stream));
    int have = 0;
    int64_t t = 0, last = -1;
    int32_t* h_cnt = c->h_status;   // pinned staging (>= 1 entry)
    while (have < no_of_samples && t < max_trials) {
        const int nb = (int)std::min<int64_t>(cur, max_trials - t);
        if (int rc = abc_launch_trials(c, a, (uint32_t)t, nb)) return rc;
        AbcSelectArgs s{};
        s.dist = a.dist; s.n = nb; s.need = no_of_samples - have; s.threshold = threshold; s.idx = p.idx; s.count = p.count;
        hipError_t le = launch_abc_select(s, c->stream);
        if (le != hipSuccess) return fail(EPIPF_EHIP, "ABC select launch failed: %s", hipGetErrorString(le));
        AbcGatherArgs g{};
        g.days = a.days; g.theta = a.theta; g.idx = p.idx; g.count = p.count; g.n = nb; g.T = T; g.slot0 = have;
        g.traj = p.traj; g.theta_out = p.theta_out;
        le = launch_abc_gather(g, no_of_samples - have, c->stream);
        if (le != hipSuccess) return fail(EPIPF_EHIP, "ABC gather launch failed: %s", hipGetErrorString(le));
        HIP_TRY(hipMemcpyAsync(h_cnt, p.count, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (int rc = abc_account(c, nb)) return rc;
        const int got = h_cnt[0];
        if (got > 0) {
            HIP_TRY(hipMemcpyAsync(h_cnt, p.idx + got - 1, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(hipStreamSynchronize(c->stream));
            last = t + h_cnt[0];
        }
        have += got;
        t += nb;
        if (batch <= 0) {
            const double want = have > 0 ? 1.25 * (double)(no_of_samples - have) * (double)t / (double)have
                                              : 4.0 * cur;
            cur = (int)std::max<double>(std::min<double>(want + 1024.0, (double)max_batch), (double)min_batch);
        }
    }
    if (have > 0) {
        HIP_TRY(hipMemcpyAsync(theta_out, p.theta_out, sizeof(double) * 2 * (size_t)have, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(traj_out, p.traj, sizeof(double) * 4 * (size_t)T * have, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    if (int rc = abc_read_counters(c)) return rc;
    *accepted_out = have;
    *trials_out = have == no_of_samples ? last + 1 : t;
    return EPIPF_OK;
}

int epipf_set_profiling(epipf_ctx* c, int enable) {
    if (!c) return fail(EPIPF_EINVAL, "NULL context");
    if (enable < EPIPF_PROFILE_OFF || enable > EPIPF_PROFILE_COUNTERS) return fail(EPIPF_EINVAL, "bad profiling level %d", enable);
    c->profiling = enable;
    return EPIPF_OK;
}

int epipf_set_streams(epipf_ctx* c, int n_streams) {
    if (!c) return fail(EPIPF_EINVAL, "NULL context");
    if (n_streams < 1 || n_streams > kMaxFilterStreams)
        return fail(EPIPF_EINVAL, "n_streams %d outside [1, %d]", n_streams, kMaxFilterStreams);
    c->n_streams = n_streams;     // streams are created at the first run that uses them
    return EPIPF_OK;
}

int epipf_set_lanes(epipf_ctx* c, int lanes, int events_per_lane) {
    if (!c) return fail(EPIPF_EINVAL, "NULL context");
    if (!(lanes == 0 || lanes == 1 || lanes == 2 || lanes == 4 || lanes == 8 || lanes == 16))
        return fail(EPIPF_EINVAL, "lanes %d not in {0 (automatic), 1, 2, 4, 8, 16}", lanes);
    if (events_per_lane < 0) return fail(EPIPF_EINVAL, "events_per_lane %d < 0", events_per_lane);
    if (lanes > 1 && events_per_lane > 0 && !group_shape_supported(lanes, events_per_lane))
        return fail(EPIPF_EINVAL, "no lane-group kernel for %d lanes x %d events per lane", lanes, events_per_lane);
    c->lanes = lanes;
    c->lane_events = events_per_lane;
    return EPIPF_OK;
}

int epipf_get_stats(epipf_ctx* c, epipf_stats* out) {
    if (!c || !out) return fail(EPIPF_EINVAL, "NULL argument");
    *out = c->stats;
    return EPIPF_OK;
}

int epipf_reset_stats(epipf_ctx* c) {
    if (!c) return fail(EPIPF_EINVAL, "NULL context");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * (size_t)kCounterSlots * kCounterStride, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    memset(&c->stats, 0, sizeof c->stats);
    return EPIPF_OK;
}

}  // extern "C"
