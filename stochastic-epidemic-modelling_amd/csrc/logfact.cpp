// logfact.cpp -- host tables for the compensated binomial weight (epipf_device.hpp: binom_logpmf).
//
// The reference's weight is scipy.stats.binom.pmf (pmcmc.py:179).  The device evaluates
//   log pmf = (log n! - log k! - log (n-k)!) + (k log p + (n-k) log1p(-p))
// as an unevaluated sum hi + lo of doubles, from log-factorials and log p / log1p(-p) rounded from binary128
// (libquadmath) to a hi double plus a lo double.  The table carries ~106 significant bits, so the weight's
// only rounding errors left are exp's and one multiply-add.
// Built with g++ (binary128 is a host type; nothing here runs on the GPU).
#include <quadmath.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <thread>
#include <vector>

namespace {

inline void split(__float128 q, double* hi, double* lo) {
    const double h = (double)q;
    *hi = h;
    *lo = std::isfinite(h) ? (double)(q - (__float128)h) : 0.0;
}

void fill(int from, int to, double* hi, double* lo) {
    for (int n = from; n < to; ++n) split(lgammaq((__float128)n + 1), &hi[n], &lo[n]);
}

}  // namespace

namespace epipf {

namespace {

void fill_threaded(int from, int to, double* hi, double* lo) {
    const int n = to - from;
    const int threads = n > 65536 ? (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency())) : 1;
    if (threads == 1) {
        fill(from, to, hi, lo);
        return;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back(fill, from + (int)((long)n * t / threads), from + (int)((long)n * (t + 1) / threads), hi, lo);
    for (auto& th : pool) th.join();
}

// Process-wide cache of the table (every entry is a function of n alone, so a table for a larger population holds
// every smaller one as its prefix): contexts and populations share it, and a larger population only computes the
// entries past the cached ones.  lgammaq costs ~2 us per entry, so the cache turns repeated set_population calls
// (one per sampler / particle_filter rebinding, several contexts per process) into copies.  Tables above
// kLogfactCacheMax entries (268 MB of host memory) are built per call and not kept.
constexpr int kLogfactCacheMax = 1 << 24;
std::mutex g_lf_mu;
std::vector<double> g_lf_hi, g_lf_lo;

}  // namespace

// out[n] = hi and out[n_max + 1 + n] = lo of log(n!) for n = 0..n_max (lgammaq: ~2 us per entry, threaded above
// 64k entries; cached up to kLogfactCacheMax entries)
void logfact_table(int n_max, double* out) {
    const int n = n_max + 1;
    double* lo = out + n;
    if (n > kLogfactCacheMax) {
        fill_threaded(0, n, out, lo);
        return;
    }
    // the lock covers the copies only: the missing entries (seconds for millions of them) are computed outside it, so
    // other contexts' set_population calls are not held behind a long fill; entries depend on n alone, so concurrent
    // fills of the same range write the same values and whichever extends the cache first wins
    int have;
    {
        std::lock_guard<std::mutex> lock(g_lf_mu);
        have = std::min((int)g_lf_hi.size(), n);
        std::copy(g_lf_hi.begin(), g_lf_hi.begin() + have, out);
        std::copy(g_lf_lo.begin(), g_lf_lo.begin() + have, lo);
    }
    if (have == n) return;
    fill_threaded(have, n, out, lo);
    std::lock_guard<std::mutex> lock(g_lf_mu);
    const int cur = (int)g_lf_hi.size();
    if (cur < n) {
        g_lf_hi.insert(g_lf_hi.end(), out + cur, out + n);
        g_lf_lo.insert(g_lf_lo.end(), lo + cur, lo + n);
    }
}

// hi/lo of log(p) and log1p(-p) (the weight's per-chain constants)
void log_p_split(double p, double* logp_hi, double* logp_lo, double* log1mp_hi, double* log1mp_lo) {
    split(logq((__float128)p), logp_hi, logp_lo);
    split(log1pq(-(__float128)p), log1mp_hi, log1mp_lo);
}

}  // namespace epipf
