/*
 * abc_oracle.c -- CPU restatement of the reference ABC rejection sampler (TEST INFRASTRUCTURE).
 *
 * THIS IS THE ORACLE, NOT THE PRODUCT.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it (built into oracle/build/liboracle.so next to epipf_oracle.c).
 *
 * It restates /root/reference/abc_algo.py:17-109 (abc_algo) on the keyed ABC stream of oracle/philox.py:
 *   :35-36  beta, gamma = np.random.uniform(lo, hi)    -> lo + (hi - lo) * U, counter (0, t, 3<<24, f)
 *   :38-39  n_start = np.random.poisson(Y[0].astype(int)) -> poisson_mode_inversion, counter (c, t, 4<<24, f)
 *   :40-45  sir_simulate(list(n_start), [beta, gamma], T, False), gillespie_algo.py:10-75, event k drawn
 *           from counter (k, t, 5<<24, f)
 *   :47-87  the daily table: row d (0 <= d < T) = [d, S, I, R] of the state after every event with
 *           time <= d (ceil(time) groups events into day rows; missing days copy the previous row)
 *   :89-94  distance_function = (mean|I - Y[:,1]| + mean|R - Y[:,2]|) / 2, np.mean = numpy pairwise sum / T
 *   :30-33  accept when not (distance > threshold); samples are the first accepted trials in trial order
 * Events with time in (T-1, T] only touch day T, which :88 truncates away, so the walk stops at T-1.
 *
 * Compile with -ffp-contract=off (see Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

enum { DOM_ABC_PRIOR = 3, DOM_ABC_INIT = 4, DOM_ABC_SSA = 5 };

void oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint64_t key, uint32_t* out);

static double u01(uint32_t lo, uint32_t hi) {
    uint64_t x = ((uint64_t)hi << 32) | lo;
    return (double)(x >> 11) * (1.0 / 9007199254740992.0);
}

/* numpy/_core/src/umath/loops_utils.h.src pairwise_sum (PW_BLOCKSIZE 128), the order np.add.reduce and so
 * np.mean use on a contiguous float64 vector; pinned against numpy in tests/test_abc.py. */
static double pairwise_sum(const double* a, long n) {
    if (n < 8) {
        double res = 0.0;
        for (long i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        long i;
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

double oracle_pairwise_sum(const double* a, long n) { return pairwise_sum(a, n); }

/* oracle/philox.py poisson_mode_inversion: inversion over m, m+1, m-1, m+2, ... with ratio recurrences. */
static long poisson_mode_inversion(double lam, double u, double pm) {
    if (lam == 0.0) return 0;
    const long m = (long)floor(lam);
    double acc = pm;
    if (u < acc) return m;
    long khi = m, klo = m;
    double phi = pm, plo = pm;
    for (;;) {
        const double prev = acc;
        phi = (phi * lam) / (double)(khi + 1);
        ++khi;
        acc = acc + phi;
        if (u < acc) return khi;
        if (klo > 0) {
            plo = (plo * (double)klo) / lam;
            --klo;
            acc = acc + plo;
            if (u < acc) return klo;
        }
        if (acc == prev) return m;
    }
}

/* mode probability exp(-lam + m log lam - lgamma(m+1)) (oracle/philox.py poisson_mode_pmf) */
double oracle_poisson_mode_pmf(double lam) {
    const double m = floor(lam);
    return exp(-lam + m * log(lam) - lgamma(m + 1.0));
}

long oracle_poisson_mode_inversion(double lam, double u, double pm) { return poisson_mode_inversion(lam, u, pm); }

/* One trial: prior draw, initial counts, SSA with daily rows.  rows [T*3] (S, I, R per day) -- the reference's
 * row d is [d, S, I, R].  work [2*T] scratch.  Returns the distance; theta[2], *events filled. */
static double abc_trial(const double* Y, int T, const double* priors, const double* lams, const double* pms,
                        uint64_t key, uint32_t f, uint32_t t, double* theta, int32_t* rows, double* work,
                        long* events) {
    uint32_t r[4];
    oracle_philox(0, t, (uint32_t)DOM_ABC_PRIOR << 24, f, key, r);
    const double beta = priors[0] + (priors[1] - priors[0]) * u01(r[0], r[1]);     /* abc_algo.py:35 */
    const double gamma = priors[2] + (priors[3] - priors[2]) * u01(r[2], r[3]);    /* :36 */
    theta[0] = beta;
    theta[1] = gamma;
    double x[3];
    for (int c = 0; c < 3; ++c) {                                                  /* :38-39 */
        oracle_philox((uint32_t)c, t, (uint32_t)DOM_ABC_INIT << 24, f, key, r);
        x[c] = (double)poisson_mode_inversion(lams[c], u01(r[0], r[1]), pms[c]);
    }
    double S = x[0], I = x[1], R = x[2];
    const double N = (S + I) + R;                                                  /* gillespie_algo.py:35 */
    const double last_day = (double)(T - 1);
    double time = 0.0;
    int day = 0;  /* next day row to record */
    long nev = 0;
    uint32_t k = 0;
    while (I > 0.0) {                                                              /* :48 */
        const double a0 = ((beta * S) * I) / N, a1 = gamma * I;                    /* :38-39 */
        const double as = a0 + a1;
        oracle_philox(k++, t, (uint32_t)DOM_ABC_SSA << 24, f, key, r);
        const double tau = (1.0 / as) * (-log(1.0 - u01(r[0], r[1])));            /* :62 */
        const double p0 = a0 / as, p1 = a1 / as, c1 = p0 + p1;
        const int ch = ((p0 / c1) <= u01(r[2], r[3])) ? 1 : 0;                     /* :63 */
        if (time + tau > (double)T) break;                                         /* :65-66, max_time = T */
        time = time + tau;                                                         /* :68 */
        if (time > last_day) break;  /* the event lands on day T: no row < T changes */
        while ((double)day < time) {                                               /* rows of days before it */
            rows[3 * day] = (int32_t)S; rows[3 * day + 1] = (int32_t)I; rows[3 * day + 2] = (int32_t)R;
            ++day;
        }
        if (ch == 0) { S -= 1.0; I += 1.0; } else { I -= 1.0; R += 1.0; }
        ++nev;
    }
    for (; day < T; ++day) {
        rows[3 * day] = (int32_t)S; rows[3 * day + 1] = (int32_t)I; rows[3 * day + 2] = (int32_t)R;
    }
    for (int d = 0; d < T; ++d) {                                                  /* :89-94 */
        work[d] = fabs((double)rows[3 * d + 1] - Y[3 * d + 1]);
        work[T + d] = fabs((double)rows[3 * d + 2] - Y[3 * d + 2]);
    }
    *events = nev;
    return (pairwise_sum(work, T) / (double)T + pairwise_sum(work + T, T) / (double)T) / 2.0;
}

/* Trials [t0, t0 + n) of run f.  Y [T*3]; priors [4] = beta lo, hi, gamma lo, hi; lams/pms [3] from Y[0].
 * theta_out [n*2], rows_out [n*T*3] or NULL, dist_out [n]. */
int oracle_abc_trials(const double* Y, int T, const double* priors, const double* lams, const double* pms,
                      uint64_t key, uint32_t f, uint32_t t0, int n, double* theta_out, int32_t* rows_out,
                      double* dist_out, int64_t* events_out) {
    if (T < 1 || n < 0) return -1;
    long total = 0;
#pragma omp parallel reduction(+ : total)
    {
        double* work = (double*)malloc(sizeof(double) * 2 * (size_t)T);
        int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)T);
#pragma omp for schedule(dynamic, 4)
        for (int i = 0; i < n; ++i) {
            long ev = 0;
            dist_out[i] = abc_trial(Y, T, priors, lams, pms, key, f, t0 + (uint32_t)i, theta_out + 2 * (size_t)i,
                                    rows, work, &ev);
            if (rows_out)
                for (int q = 0; q < 3 * T; ++q) rows_out[(size_t)i * 3 * T + q] = rows[q];
            total += ev;
        }
        free(work);
        free(rows);
    }
    if (events_out) *events_out = total;
    return 0;
}
