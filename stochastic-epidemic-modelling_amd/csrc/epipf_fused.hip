// epipf_fused.hip -- launch table of the one-workgroup filter (epipf_fused.hpp): SIR and SEIR here, the subgroup models
// in epipf_fused_sub.hip / epipf_fused_sub2.hip (one translation unit each: they build in parallel).
#include "epipf_fused.hpp"

namespace epipf {

size_t fused_lds_bytes_of(int N, int C, int threads, int TK, int lf_n) { return fused_lds_bytes(N, C, threads, TK, lf_n); }
int fused_threads_of(int N, int W) { return fused_threads(N, W); }

FusedFn fused_launcher_sir(int model, int obs, int W) {
    return model == kSIR ? pick_fused_obs<kSIR, 1>(obs, W) : pick_fused_obs<kSEIR, 1>(obs, W);
}

FusedFn fused_launcher(int model, int G, int obs, int W) {
    switch (model) {
        case kSIR:
        case kSEIR: return fused_launcher_sir(model, obs, W);
        case kSubgroups: return fused_launcher_sub(G, obs, W);
        case kSubgroups2: return fused_launcher_sub2(G, obs, W);
    }
    return nullptr;
}

}  // namespace epipf
