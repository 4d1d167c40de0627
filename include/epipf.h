/*
 * epipf.h -- C ABI of the MI355X particle-filter engine (libepipf.so).
 *
 * The reference (GeorgeEfstathiadis/Stochastic-Epidemic-Modelling) is pure Python and has no FFI;
 * its seams are plain Python calls.  These entry points replace, one for one:
 *
 *   epipf_run            pmcmc.py:123-233  particle_filter(Y, type_model, theta_proposal, observations,
 *                                          probs, n_particles, n_population, mu, jobs)
 *                        -- batched over independent chains; the per-particle joblib dispatch of
 *                           pmcmc.py:200-220 becomes one GPU lane per particle.
 *   epipf_copy_history   pmcmc.py:151-152,233  the hidden_process [T,N,C] / ancestry_matrix [T,N] outputs
 *   epipf_path_sample    pmcmc.py:236-248  particle_path_sampler(hidden_process, ancestry_matrix)
 *                        (the uniform pick np.random.randint(0, N) stays on the host RNG: `chosen`)
 *   epipf_simulate       gillespie_algo.py:10-75 / 78-146 / 148-233  sir_simulate / seir_simulate /
 *                        sir_subgroups_simulate(..., last_values_only=True), batched over states
 *   epipf_simulate_path  the same functions with last_values_only=False (event times + states)
 *   epipf_resample       pmcmc.py:185-190  normalise + np.random.choice(range(N), N, p=w/sum(w)) with
 *                        caller-supplied uniforms (bit-exact to numpy's legacy choice)
 *   epipf_abc            abc_algo.py:17-109  abc_algo(observed_data, no_of_samples, threshold, priors)
 *                        -- the rejection loop batched: one GPU lane per trial, trials accepted in trial order
 *   epipf_abc_trials     abc_algo.py:33-94  one pass of the while-loop body per trial (prior draw, initial
 *                        counts, sir_simulate(..., False), daily table, distance_function) for trials [t0, t0+n)
 *
 * The host wrapper (stochastic-epidemic-modelling_amd/epipf/) binds these with ctypes and keeps
 * the reference's Python signatures.  Conventions:
 *   - all pointers are HOST pointers to C-contiguous arrays owned by the caller; the context owns and
 *     reuses every device buffer (observations and history stay resident in HBM across calls);
 *   - return value 0 = EPIPF_OK, negative = error (message via epipf_last_error()); nothing throws;
 *   - one context per device; calls on one context must be serialised by the caller;
 *   - random numbers come from the keyed Philox4x32-10 stream documented in DESIGN.md §3
 *     (key = 64-bit seed per chain, filter_index = one per particle-filter call).
 */
#ifndef EPIPF_H
#define EPIPF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EPIPF_ABI_VERSION 8

/* return codes */
#define EPIPF_OK 0
#define EPIPF_EINVAL (-1)   /* bad argument / shape */
#define EPIPF_EHIP (-2)     /* HIP runtime error */
#define EPIPF_ENOMEM (-3)   /* device allocation failed */
#define EPIPF_ESTATE (-4)   /* call order (e.g. path sample before any run) */

/* per-chain status written by epipf_run */
#define EPIPF_STATUS_OK 0
#define EPIPF_STATUS_DEGENERATE 1 /* all weights 0 or NaN at some step: reference returns (None, None, None) */
#define EPIPF_STATUS_SKIPPED 2    /* chain was inactive in this call (active[c] == 0) */

/* models: pmcmc.py:116-120 ModelType */
#define EPIPF_SIR 0
#define EPIPF_SEIR 1
#define EPIPF_SIR_SUBGROUPS 2
#define EPIPF_SIR_SUBGROUPS2 3

/* observation models: pmcmc.py:178-181 (observations=False / True) */
#define EPIPF_OBS_BINOMIAL 0
#define EPIPF_OBS_NORMAL 1

/* resampling: multinomial is the reference's (pmcmc.py:188); systematic is opt-in and changes results */
#define EPIPF_RESAMPLE_MULTINOMIAL 0
#define EPIPF_RESAMPLE_SYSTEMATIC 1

typedef struct epipf_ctx epipf_ctx;

typedef struct {
    double step_ms;              /* HIP-event time of the fused resample+propagate+weight kernels (profiling on) */
    int64_t step_launches;       /* number of such launches timed */
    double init_ms;              /* HIP-event time of the init kernels (profiling on) */
    int64_t init_launches;
    int64_t events;              /* accepted Gillespie events (profiling on) */
    int64_t particle_steps;      /* N x T_obs x chains that ran a filter */
    int64_t filters;             /* chain-filters run */
    int64_t resample_fallbacks;  /* draws resolved by the sequential bit-exact path */
    int64_t lane_iterations;     /* SSA loop iterations summed over lanes (profiling on) */
    int64_t wave_lane_slots;     /* SSA loop iterations x 64 summed over waves: lane_iterations / this = SIMD lane use */
    double abc_ms;               /* HIP-event time of the ABC trial kernels (profiling on) */
    int64_t abc_launches;        /* ABC trial kernel launches */
    int64_t abc_trials;          /* ABC trials simulated (accepted or not) */
    int64_t ssa_exact_lanes;     /* filter particle-steps simulated on the exact f64 SSA loop (profiling counters) */
    int64_t ssa_exact_waves;     /* filter wave-steps with at least one such particle-step */
    double step_kernel_ms;       /* summed span of each chain group's back-to-back step kernels, HIP events on the
                                    group's own stream (profiling on) */
    int64_t step_kernel_launches;/* their number: one step of all chains (step_ms) is one launch per chain group on
                                    concurrent streams (EPIPF_STREAMS, default 4) */
    int64_t last_lanes;          /* SSA lanes per particle of the last epipf_run (1: one-lane step kernel; 2..16: the
                                    lane-group step kernel, epipf_set_lanes) */
    int64_t last_lane_events;    /* events per lane per chunk of that run's lane-group kernel (1 for the one-lane one) */
    int64_t resample_ref_ambiguous; /* resampling draws whose uniform lies so close to a CDF boundary that scipy's own
                                       weights (within the measured envelope of their error) could pick
                                       a neighbouring ancestor: a diagnostic count, always on; the draw itself is the
                                       numpy answer over the device's weights */
    int64_t last_fused;          /* 1: the last epipf_run ran each chain's whole filter in one workgroup launch (N <= 512
                                    with the lanes automatic); 0: one launch per filter step */
} epipf_stats;

/* groups: G for the subgroup models (1 <= G <= 4), ignored (1) for SIR/SEIR.
 * t_max: largest T (observation rows) a run may use; max_chains: largest batch of independent filters. */
int epipf_create(epipf_ctx** out, int device, int model, int groups, int n_particles, int t_max,
                 int max_chains);
void epipf_destroy(epipf_ctx* ctx);

/* Y: [T*K] row-major observed counts (K = C, or 3 for SIR_SUBGROUPS2).  Uploaded once, kept in HBM. */
int epipf_set_observations(epipf_ctx* ctx, const double* Y, int T, int K);

/* n_population, mu: [G] (pmcmc.py:129-131; G = 1 for SIR/SEIR).  n_population must be integral. */
int epipf_set_population(epipf_ctx* ctx, const double* n_population, const double* mu);

/* Run n_chains independent particle filters (one per chain) over the resident observations.
 *   theta  [n_chains*d]: SIR (beta, gamma); SEIR (beta, alpha, gamma); subgroups beta[G][G] row-major + gamma
 *   probs  [n_chains]   : binomial detection probability, or the normal-noise ratio (observations=True)
 *   keys   [n_chains]   : Philox key per chain;  filter_index [n_chains]: stream index of this call
 *   active [n_chains] or NULL: 0 marks a chain that runs nothing this call (status SKIPPED)
 *   log_zetas_out [n_chains*T] or NULL: log of the reference's zetas (zetas = exp(log_zetas))
 *   status_out [n_chains]: EPIPF_STATUS_*                                                               */
int epipf_run(epipf_ctx* ctx, int n_chains, const double* theta, int d, int obs_model, const double* probs,
              const uint64_t* keys, const uint32_t* filter_index, const int32_t* active, int resample_mode,
              double* log_zetas_out, int32_t* status_out);

/* epipf_run, then the path sampler of epipf_path_sample on the same stream before the results come back: one round
 * trip per MH iteration instead of two (pmcmc.py:360-362 -- particle_filter, then particle_path_sampler).
 *   chosen [n_chains]: the final particle of each chain's sampled path (the host's np.random.randint(0, N) draw,
 *                      taken before the filter -- epipf.pmcmc peeks it off the RandomState without consuming it),
 *                      or -1 for none
 *   traj_out [n_chains*T*C] int32: the sampled trajectories; zeros for chains with chosen -1 or a status other than
 *                      EPIPF_STATUS_OK (the reference draws no path after a degenerate filter) */
int epipf_run_sampled(epipf_ctx* ctx, int n_chains, const double* theta, int d, int obs_model, const double* probs,
                      const uint64_t* keys, const uint32_t* filter_index, const int32_t* active, int resample_mode,
                      const int32_t* chosen, double* log_zetas_out, int32_t* status_out, int32_t* traj_out);

/* Copy the last run's history: hidden [n_chains*T*N*C] int32 (compartment counts), ancestry [n_chains*T*N]
 * int32 (row 0 zeros, as pmcmc.py:152).  Either pointer may be NULL. */
int epipf_copy_history(epipf_ctx* ctx, int n_chains, int32_t* hidden_out, int32_t* ancestry_out);

/* On-device particle_path_sampler (pmcmc.py:236-248, including its ancestry[p] indexing) for each chain of
 * the last run; chosen [n_chains] is the host's np.random.randint(0, N) draw.  traj_out [n_chains*T*C].
 * A chain whose last run was not EPIPF_STATUS_OK (degenerate or skipped) gets zeros: its history is not walked. */
int epipf_path_sample(epipf_ctx* ctx, int n_chains, const int32_t* chosen, int32_t* traj_out);

/* Batched last-value SSA from n states [n*C] over [0, max_time] (gillespie_algo.py *_simulate with
 * last_values_only=True).  State j draws SSA event k from counter (k, j, step, filter_index). */
int epipf_simulate(epipf_ctx* ctx, int n, const int32_t* states_in, const double* theta, int d,
                   double max_time, uint64_t key, uint32_t filter_index, uint32_t step, int32_t* states_out,
                   int64_t* events_out);

/* Batched full-path SSA (gillespie_algo.py *_simulate with last_values_only=False, :68-75 / :139-146 /
 * :218-233): the same draws and final states as epipf_simulate, plus every event's time and the state after it.
 * Trajectory j keeps its first max_events events: times_out [n*max_events] (row j: its event times, ascending),
 * states_out [n*max_events*C]; n_events_out [n] is its full event count (> max_events: the rows hold the first
 * max_events only, call again with a larger buffer); final_out [n*C] (or NULL) its last state.  The event times
 * are the reference's clock bit for bit.  The initial state (time 0.0) is the caller's input. */
int epipf_simulate_path(epipf_ctx* ctx, int n, const int32_t* states_in, const double* theta, int d,
                        double max_time, uint64_t key, uint32_t filter_index, uint32_t step, int max_events,
                        double* times_out, int32_t* states_out, int32_t* n_events_out, int32_t* final_out);

/* Standalone resampler: out[j] = numpy legacy choice(range(n), n, p=w/sum(w)) given uniforms u[j].
 * Returns EPIPF_STATUS_DEGENERATE (as a positive value) where numpy raises ValueError. */
int epipf_resample(epipf_ctx* ctx, int n, const double* w, const double* u, int32_t* out,
                   int64_t* fallbacks_out);

/* ABC rejection sampling, abc_algo.py:17-109, for the SIR model (any context works; its model is ignored).
 *   Y [T*3]: observed_data (S, I, R per day); initial counts ~ Poisson(Y[0].astype(int)), abc_algo.py:38-39
 *   priors [4]: beta lo, hi, gamma lo, hi (uniform priors, abc_algo.py:35-36)
 * Trial t of run `run_index` draws from the keyed ABC stream: prior (0, t, 3<<24, run),
 * initial count c (c, t, 4<<24, run), SSA event k (k, t, 5<<24, run).  t < 2^32.
 *
 * epipf_abc: the first no_of_samples trials with distance <= threshold, in trial order (the reference's
 * sequential while loop).  theta_out [no_of_samples*2] (beta, gamma); traj_out [no_of_samples*T*4] rows
 * (day, S, I, R) exactly as abc_algo returns them.  At most max_trials trials are run (the reference loops
 * forever when the threshold is unreachable): *accepted_out < no_of_samples then.  *trials_out = the trial
 * count the reference reports (index of the last accepted trial + 1; max_trials when short).
 * batch <= 0 picks batch sizes automatically (growing from 16k trials to 1M).                              */
int epipf_abc(epipf_ctx* ctx, const double* Y, int T, int no_of_samples, double threshold, const double* priors,
              uint64_t key, uint32_t run_index, int64_t max_trials, int batch, double* theta_out, double* traj_out,
              int64_t* trials_out, int32_t* accepted_out);

/* Trials [t0, t0+n): theta_out [n*2]; rows_out [n*T*3] int32 (S, I, R per day) or NULL; dist_out [n] or NULL. */
int epipf_abc_trials(epipf_ctx* ctx, const double* Y, int T, const double* priors, uint64_t key, uint32_t run_index,
                     uint32_t t0, int n, double* theta_out, int32_t* rows_out, double* dist_out, int64_t* events_out);

/* The device's restatement of glibc's log (the reference's math.log / numpy legacy exponential),
 * evaluated on the host CPU with the same code and table: out[i] = log(x[i]) bit for bit for normal x[i] > 0.
 * For tests of that restatement; no GPU involved. */
int epipf_glibc_log(int64_t n, const double* x, double* out);

/* The lane-group filter's certified-clock log (clock_log_impl, csrc/epipf_device.hpp: glibc's table path without its
 * close-to-1 branch), on the host CPU with the same code and table: out[i] ~ log(x[i]) within the bound its clock
 * certificate assumes (tests/test_glibc_log.py measures it).  For tests; no GPU involved. */
int epipf_clock_log(int64_t n, const double* x, double* out);

/* Profiling levels: OFF; TIMING = HIP events around the init / step kernels (step_ms, init_ms), no effect on
 * the kernels; COUNTERS = TIMING + device counters of SSA events and lane use (a few atomics per wave). */
#define EPIPF_PROFILE_OFF 0
#define EPIPF_PROFILE_TIMING 1
#define EPIPF_PROFILE_COUNTERS 2
int epipf_set_profiling(epipf_ctx* ctx, int level);

/* Chain groups of one epipf_run on concurrent HIP streams (1..8, default 4 or EPIPF_STREAMS): each group's T-1
   step kernels run back to back on its own stream so that one group's launch tail overlaps the others' work.
   Engine tuning only, no reference counterpart; results do not depend on it.  A host that runs several contexts
   from separate threads (MH iterations pipelined with the device, epipf.pmcmc.run_pipelined) sets 1 each. */
int epipf_set_streams(epipf_ctx* ctx, int n_streams);
/* Lanes per particle in the step kernel's SSA: 0 = automatic (default; EPIPF_LANES overrides), 1 = one lane per
   particle (throughput: batches that fill the chip), 2/4/8/16 = a group of lanes draws consecutive events' Philox
   blocks in parallel and runs only the sequential decisions event by event (latency: a single chain or a few chains,
   DESIGN.md §12).  events_per_lane: events each lane of a group draws per chunk (0 = automatic).  Engine tuning only,
   no reference counterpart; results are identical for every value. */
int epipf_set_lanes(epipf_ctx* ctx, int lanes, int events_per_lane);
int epipf_get_stats(epipf_ctx* ctx, epipf_stats* out);
int epipf_reset_stats(epipf_ctx* ctx);

/* Host side of a many-chain MH iteration (epipf.pmcmc.ChainSampler, pmcmc.py:325-406 per chain), in C: each chain's
 * numpy legacy RandomState draws made on its MT19937 state in place (mt_states[c]: the bit generator's
 * ctypes.state_address, numpy's mt19937_state), bit-identical to numpy's own and in the reference's order.  No device
 * work; status codes as the rest of the ABI.
 * epipf_mh_propose: props_out[c] = multivariate_normal(means[c], .) of pmcmc.py:330 = standard_normal(d) (even d, empty
 *   gaussian cache) times factors[c] ([d][d], mvn_factor) by dgemv (numpy's own cblas_dgemv, a function pointer:
 *   the product numpy computes for np.dot) plus means[c].
 * epipf_mh_decide: for the n chains listed in chains[] (their filters succeeded), in order: chosen_out[c] =
 *   randint(0, n_particles) (the path sampler's pick, pmcmc.py:241), then accept_out[c] = random_sample() <
 *   min(1, exp(min(lz_new[c] - lz_old[c], 0))) (the log-space acceptance, 0 for NaN). */
int epipf_mh_propose(int n_chains, int d, void* const* mt_states, const double* factors, const double* means,
                     double* props_out, void* dgemv);
int epipf_mh_decide(int n, const int32_t* chains, void* const* mt_states, int n_particles, const double* lz_new,
                    const double* lz_old, int32_t* chosen_out, int32_t* accept_out);
/* epipf_mh_peek: chosen_out[c] = the randint(0, n_particles) the next epipf_mh_decide draws for each listed chain,
 * read on a copy of its state (nothing consumed): the path sampler's picks for epipf_run_sampled, before the filter. */
int epipf_mh_peek(int n, const int32_t* chains, void* const* mt_states, int n_particles, int32_t* chosen_out);

const char* epipf_last_error(void);
int epipf_abi_version(void);
/* Hash of the library's sources and build flags (16 hex digits; "...-debug" for libepipf_debug.so).  Profiles taken
 * on one build are trusted by bench.py only for the same id. */
const char* epipf_build_id(void);
int epipf_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* EPIPF_H */
