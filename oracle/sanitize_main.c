/* sanitize_main.c -- runs the C oracle (test infrastructure) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (SURVEY.md §5 "host ASan/UBSan build of the C-ABI and the CPU restatement").  `make -C oracle asan` builds it;
 * tests/test_sanitizers.py runs it.  It exercises every exported oracle entry point on small and edge-case inputs
 * (N = 1, T = 1, extinct starts, degenerate weights, every model, full-path buffers at their exact capacity and one
 * short); numerics are checked elsewhere (tests/test_oracle.py against the reference's goldens) -- this driver is
 * about memory and UB.  Exit status 0 and no sanitizer report = clean. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t key, uint32_t* out);
int oracle_simulate(int model, int G, int n, const int32_t* states_in, const double* theta, int d, double max_time,
                    uint64_t key, uint32_t f, uint32_t step, int32_t* states_out, int64_t* events_out);
int oracle_simulate_path(int model, int G, int n, const int32_t* states_in, const double* theta, int d,
                         double max_time, uint64_t key, uint32_t f, uint32_t step, long cap, double* times,
                         int32_t* states, int32_t* nev, int32_t* final_state);
int oracle_resample(int n, const double* w, const double* u, int32_t* out);
int oracle_particle_filter(int model, int G, int N, int T, int K, const double* Y, const double* theta, int d,
                           int obs, double probs, const double* npop, const double* mu, uint64_t key, uint32_t f,
                           int resample_mode, double* log_zeta, double* zeta, int32_t* hidden, int32_t* ancestry,
                           int64_t* events_out);
void oracle_set_num_threads(int n);
void oracle_log_batch(long n, const double* x, double* out);
double oracle_binom_pmf(double k, double n, double p);
double oracle_norm_pdf(double y, double x, double probs);
double oracle_pairwise_sum(const double* a, long n);
double oracle_poisson_mode_pmf(double lam);
long oracle_poisson_mode_inversion(double lam, double u, double pm);
int oracle_abc_trials(const double* Y, int T, const double* priors, const double* lams, const double* pms,
                      uint64_t key, uint32_t run_index, uint32_t t0, int n, double* theta_out, int32_t* rows_out,
                      double* dist_out, int64_t* events_out);

static int C_of(int model, int G) { return model == 0 ? 3 : model == 1 ? 4 : 3 * G; }
static int K_of(int model, int G) { return model == 3 ? 3 : C_of(model, G); }

static void filter_case(int model, int G, int N, int T, int obs, double mu0, double probs) {
    const int C = C_of(model, G), K = K_of(model, G);
    const int d = model == 0 ? 2 : model == 1 ? 3 : G * G + 1;
    double* Y = malloc(sizeof(double) * (size_t)T * K);
    for (int t = 0; t < T; ++t)                          /* about probs x (S, I, R) of the initial states */
        for (int k = 0; k < K; ++k) {
            const int c = k % (model == 1 ? 4 : 3);
            const double x = c == 0 ? 2000.0 : (c == (model == 1 ? 2 : 1) ? mu0 + t : (double)t);
            Y[t * K + k] = floor((probs > 0 && probs <= 1 ? probs : 0.1) * x * (model == 3 ? G : 1));
        }
    double theta[17];
    for (int i = 0; i < d; ++i) theta[i] = 0.5 + 0.25 * i;
    double npop[4] = {2000, 3000, 1500, 1200}, mu[4] = {mu0, mu0, mu0, mu0};
    int32_t* hidden = malloc(sizeof(int32_t) * (size_t)T * N * C);
    int32_t* ancestry = malloc(sizeof(int32_t) * (size_t)T * N);
    double* lz = malloc(sizeof(double) * (size_t)T);
    double* z = malloc(sizeof(double) * (size_t)T);
    int64_t events = 0;
    const int status = oracle_particle_filter(model, G, N, T, K, Y, theta, d, obs, probs, npop, mu, 7, 3, N % 2, lz, z,
                                              hidden, ancestry, &events);
    printf("filter model=%d G=%d N=%d T=%d obs=%d mu=%g: status=%d events=%lld\n", model, G, N, T, obs, mu0, status,
           (long long)events);
    free(Y); free(hidden); free(ancestry); free(lz); free(z);
}

int main(void) {
    oracle_set_num_threads(2);
    uint32_t r[4];
    oracle_philox(1, 2, 3, 4, 0x123456789abcdefull, r);
    /* filters: every model, both observation types, N = 1 and ragged N, T = 1 and 2, extinct starts (mu = 0),
       degenerate weights (probs = 0 with positive counts), NaN weights (probs outside [0, 1]) */
    for (int model = 0; model < 4; ++model)
        for (int G = 1; G <= (model >= 2 ? 3 : 1); ++G) {
            filter_case(model, G, 1, 3, 0, 20, 0.1);
            filter_case(model, G, 65, 4, model < 2, 20, 0.3);
            filter_case(model, G, 7, 1, 0, 20, 0.1);
            filter_case(model, G, 9, 2, 0, 0, 0.1);
        }
    filter_case(0, 1, 33, 5, 0, 20, 0.0);
    filter_case(0, 1, 33, 5, 0, 20, 1.5);
    filter_case(0, 1, 200, 6, 1, 20, 0.5);
    /* last-value and full-path SSA, buffers at exact capacity and one event short */
    {
        const int n = 5;
        int32_t in[5 * 6], out[5 * 6], nev[5], fin[5 * 6];
        for (int j = 0; j < n; ++j) { in[3 * j] = 90 - j; in[3 * j + 1] = 10 + j; in[3 * j + 2] = 0; }
        const double th[2] = {2.0, 1.0};
        int64_t ev = 0;
        oracle_simulate(0, 1, n, in, th, 2, 1.5, 11, 0, 0, out, &ev);
        const long cap = 400;
        double* times = malloc(sizeof(double) * cap * n);
        int32_t* states = malloc(sizeof(int32_t) * cap * n * 3);
        int rc = oracle_simulate_path(0, 1, n, in, th, 2, 1.5, 11, 0, 0, cap, times, states, nev, fin);
        long mx = 0;
        for (int j = 0; j < n; ++j) mx = nev[j] > mx ? nev[j] : mx;
        printf("path rc=%d max events %ld (last-value events %lld)\n", rc, mx, (long long)ev);
        if (mx > 1) rc = oracle_simulate_path(0, 1, n, in, th, 2, 1.5, 11, 0, 0, mx - 1, times, states, nev, fin);
        printf("path short rc=%d\n", rc);
        free(times); free(states);
    }
    /* resampling: positive, tied, all-zero and single weights */
    {
        double w[8] = {0.1, 0.2, 0.2, 0.0, 0.5, 0.0, 1e-300, 3.0}, u[8] = {0, 0.1, 0.2, 0.3, 0.5, 0.7, 0.99, 0.999999};
        int32_t out[8];
        printf("resample %d", oracle_resample(8, w, u, out));
        double z[3] = {0, 0, 0};
        printf(" %d", oracle_resample(3, z, u, out));
        printf(" %d\n", oracle_resample(1, w, u, out));
    }
    /* scalar helpers at their edges */
    {
        double x[6] = {1.0, 0x1p-1074, 0x1p-1022, 1e308, 0.9999999999999999, 2.0}, y[6];
        oracle_log_batch(6, x, y);
        printf("pmf %g %g %g %g pdf %g\n", oracle_binom_pmf(3, 10, 0.1), oracle_binom_pmf(0, 0, 0.5),
               oracle_binom_pmf(11, 10, 0.1), oracle_binom_pmf(2, 10, -0.1), oracle_norm_pdf(10, 12, 0.1));
        double a[300];
        for (int i = 0; i < 300; ++i) a[i] = 1.0 / (i + 1);
        printf("pairwise %g %g %g\n", oracle_pairwise_sum(a, 300), oracle_pairwise_sum(a, 1), oracle_pairwise_sum(a, 0));
        printf("poisson %g %ld %ld\n", oracle_poisson_mode_pmf(3.0), oracle_poisson_mode_inversion(3.0, 0.5, 0.224),
               oracle_poisson_mode_inversion(0.0, 0.5, 1.0));
    }
    /* ABC trials: T = 1 and T = 15, with and without day rows */
    for (int T = 1; T <= 15; T += 14) {
        double Y[15 * 3];
        for (int i = 0; i < T; ++i) { Y[3 * i] = 4800 - 10 * i; Y[3 * i + 1] = 20 + 5 * i; Y[3 * i + 2] = 5 * i; }
        const double priors[4] = {0, 5, 0, 5}, lams[3] = {4800, 20, 0};
        double pms[3];
        for (int c = 0; c < 3; ++c) pms[c] = oracle_poisson_mode_pmf(lams[c]);
        const int n = 64;
        double th[2 * 64], dist[64];
        int32_t* rows = malloc(sizeof(int32_t) * (size_t)n * T * 3);
        int64_t ev = 0;
        int rc = oracle_abc_trials(Y, T, priors, lams, pms, 5, 1, 0, n, th, rows, dist, &ev);
        int rc2 = oracle_abc_trials(Y, T, priors, lams, pms, 5, 1, 64, n, th, NULL, dist, &ev);
        printf("abc T=%d rc=%d/%d events %lld\n", T, rc, rc2, (long long)ev);
        free(rows);
    }
    printf("sanitize_main: done\n");
    return 0;
}
