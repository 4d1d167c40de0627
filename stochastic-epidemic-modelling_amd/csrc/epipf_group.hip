// epipf_group.hip -- launch table of the lane-group step kernel (epipf_group.hpp): SIR and SEIR here, the subgroup
// models in epipf_group_sub.hip / epipf_group_sub2.hip (one translation unit each: they build in parallel).
#include "epipf_group.hpp"

namespace epipf {

size_t group_lds_bytes(int B, int S, int C, int W, int K, int PB) { return group_lds_bytes_impl(B, S, C, W, K, PB); }

bool group_shape_supported(int W, int K) {
#define EPIPF_HAS(w, k) if (W == w && K == k) return true;
    EPIPF_GROUP_SHAPES(EPIPF_HAS)
#undef EPIPF_HAS
    return false;
}

GroupStepFn group_launcher_sir(int model, int obs, int W, int K) {
    return model == kSIR ? pick_obs<kSIR, 1>(obs, W, K) : pick_obs<kSEIR, 1>(obs, W, K);
}

GroupStepFn group_step_launcher(int model, int G, int obs, int W, int K) {
    switch (model) {
        case kSIR:
        case kSEIR: return group_launcher_sir(model, obs, W, K);
        case kSubgroups: return group_launcher_sub(G, obs, W, K);
        case kSubgroups2: return group_launcher_sub2(G, obs, W, K);
    }
    return nullptr;
}

}  // namespace epipf
