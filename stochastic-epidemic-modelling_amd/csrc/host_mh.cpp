// host_mh.cpp -- the host side of a many-chain MH iteration (epipf.pmcmc.ChainSampler) in C: each chain's numpy
// legacy RandomState draws -- the proposal's standard_normal(d), the path sampler's randint(0, N), the acceptance
// uniform -- made on the chain's own MT19937 state in place, in the reference's order (pmcmc.py:330, :361, :393).
//
// With 256 chains of BASELINE config 1 (N = 100) the device filter of a whole MH iteration takes ~0.4 ms and the
// Python per-chain calls ~0.6 ms; here they take a few microseconds.  Bit-identical to numpy 2.2's legacy
// RandomState by construction, and checked against it (tests/test_host_rng.py):
//   MT19937         mt19937_gen / mt19937_next32 (numpy/random/src/mt19937), the state numpy's bit generator exposes
//                   (bit_generator.ctypes.state_address: uint32 key[624], int pos)
//   random_sample   legacy_double = mt19937_next_double: (a >> 5, b >> 6) -> (a 2^26 + b) / 2^53
//   standard_normal legacy_gauss: the polar method, pairs (f x2 returned, f x1 cached).  Only even d, with an empty
//                   cache on entry (has_gauss = 0, which ChainSampler checks once): a call then uses whole pairs and
//                   leaves the cache empty, as numpy's own would -- so the RandomState's cached-gaussian fields, which
//                   live in the Python object and not in the MT state, stay right without being touched
//   randint(0, N)   masked rejection on 32-bit words (random_bounded_uint64_fill's buffered_bounded_masked_uint32)
//   multivariate_normal's np.dot(z, factor): the same OpenBLAS routine numpy calls for a (1, d) x (d, d) product
//                   (cblas_dgemv, row-major, transposed), passed in by the caller from numpy's own library
// epipf_mh_peek: the randint(0, N) the next epipf_mh_decide will draw, without consuming it (a copy of the state),
// so that the path sampler can ride on the filter's launch (epipf_run_sampled) for any number of chains.
// Compiled without FMA contraction (-ffp-contract=off), like numpy's baseline build of these functions.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/epipf.h"

namespace {

constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

struct MTState {   // numpy's mt19937_state
    uint32_t key[kN];
    int pos;
};

void mt_gen(MTState* s) {
    uint32_t y;
    int i;
    for (i = 0; i < kN - kM; i++) {
        y = (s->key[i] & kUpper) | (s->key[i + 1] & kLower);
        s->key[i] = s->key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    for (; i < kN - 1; i++) {
        y = (s->key[i] & kUpper) | (s->key[i + 1] & kLower);
        s->key[i] = s->key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    y = (s->key[kN - 1] & kUpper) | (s->key[0] & kLower);
    s->key[kN - 1] = s->key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    s->pos = 0;
}

inline uint32_t next32(MTState* s) {
    if (s->pos == kN) mt_gen(s);
    uint32_t y = s->key[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

inline double next_double(MTState* s) {
    const int32_t a = (int32_t)(next32(s) >> 5), b = (int32_t)(next32(s) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

// legacy_gauss with an empty cache: one pair, the returned value first, the cached one second
inline void gauss_pair(MTState* s, double& first, double& second) {
    double f, x1, x2, r2;
    do {
        x1 = 2.0 * next_double(s) - 1.0;
        x2 = 2.0 * next_double(s) - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    f = std::sqrt(-2.0 * std::log(r2) / r2);
    first = f * x2;
    second = f * x1;
}

inline int32_t bounded(MTState* s, uint32_t rng) {   // randint(0, rng + 1), rng < 2^31 here
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = next32(s) & mask) > rng) {
    }
    return (int32_t)v;
}

using Dgemv = void (*)(int order, int trans, int64_t m, int64_t n, double alpha, const double* a, int64_t lda,
                       const double* x, int64_t incx, double beta, double* y, int64_t incy);
constexpr int kRowMajor = 101, kTrans = 112;   // CBLAS_ORDER / CBLAS_TRANSPOSE
constexpr int kMaxD = 32;

}  // namespace

namespace epipf {
int set_error(int code, const char* msg);   // epipf_api.cpp: epipf_last_error()'s message for this thread
}

extern "C" {

int epipf_mh_propose(int n_chains, int d, void* const* mt_states, const double* factors, const double* means,
                     double* props_out, void* dgemv) {
    if (n_chains < 0 || d < 2 || d > kMaxD || (d & 1) || !mt_states || !factors || !means || !props_out || !dgemv)
        return epipf::set_error(EPIPF_EINVAL, "epipf_mh_propose: n_chains < 0, d outside the even values 2..32, or a "
                                              "NULL argument");
    const Dgemv gemv = reinterpret_cast<Dgemv>(dgemv);
    double z[kMaxD], y[kMaxD];
    for (int c = 0; c < n_chains; ++c) {
        MTState* s = static_cast<MTState*>(mt_states[c]);
        for (int k = 0; k < d; k += 2) gauss_pair(s, z[k], z[k + 1]);            // standard_normal(d)
        gemv(kRowMajor, kTrans, d, d, 1.0, factors + (size_t)c * d * d, d, z, 1, 0.0, y, 1);   // np.dot(z, factor)
        for (int k = 0; k < d; ++k) props_out[(size_t)c * d + k] = y[k] + means[(size_t)c * d + k];   // += mean
    }
    return EPIPF_OK;
}

int epipf_mh_peek(int n, const int32_t* chains, void* const* mt_states, int n_particles, int32_t* chosen_out) {
    if (n < 0 || n_particles < 1 || !chains || !mt_states || !chosen_out)
        return epipf::set_error(EPIPF_EINVAL, "epipf_mh_peek: n < 0, n_particles < 1 or a NULL argument");
    const uint32_t rng = (uint32_t)(n_particles - 1);
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    for (int i = 0; i < n; ++i) {
        const int c = chains[i];
        const MTState* s = static_cast<const MTState*>(mt_states[c]);
        int32_t v = -1;
        if (rng == 0) v = 0;
        for (int p = s->pos; v < 0 && p < kN; ++p) {     // the words ahead, read in place and tempered as next32 would
            uint32_t y = s->key[p];
            y ^= (y >> 11);
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= (y >> 18);
            if ((y & mask) <= rng) v = (int32_t)(y & mask);
        }
        if (v < 0) {                                      // the draw regenerates the state first: on a copy
            MTState copy;
            memcpy(&copy, s, sizeof copy);
            v = bounded(&copy, rng);
        }
        chosen_out[c] = v;
    }
    return EPIPF_OK;
}

int epipf_mh_decide(int n, const int32_t* chains, void* const* mt_states, int n_particles, const double* lz_new,
                    const double* lz_old, int32_t* chosen_out, int32_t* accept_out) {
    if (n < 0 || n_particles < 1 || !chains || !mt_states || !lz_new || !lz_old || !chosen_out || !accept_out)
        return epipf::set_error(EPIPF_EINVAL, "epipf_mh_decide: n < 0, n_particles < 1 or a NULL argument");
    for (int i = 0; i < n; ++i) {
        const int c = chains[i];
        MTState* s = static_cast<MTState*>(mt_states[c]);
        chosen_out[c] = bounded(s, (uint32_t)(n_particles - 1));                 // randint(0, N), pmcmc.py:241
        const double u = next_double(s);                                           // random_sample, :393
        const double lr = lz_new[c] - lz_old[c];                                   // _log_ratio
        const double prob = std::isnan(lr) ? 0.0 : std::fmin(1.0, std::exp(lr < 0.0 ? lr : 0.0));
        accept_out[c] = u < prob ? 1 : 0;
    }
    return EPIPF_OK;
}

}  // extern "C"
