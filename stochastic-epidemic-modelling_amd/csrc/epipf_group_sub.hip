// epipf_group_sub.hip -- lane-group step kernels of the subgroup model (epipf_group.hpp)
#include "epipf_group.hpp"

namespace epipf {

GroupStepFn group_launcher_sub(int G, int obs, int W, int K) {
    switch (G) {
        case 1: return pick_obs<kSubgroups, 1>(obs, W, K);
        case 2: return pick_obs<kSubgroups, 2>(obs, W, K);
        case 3: return pick_obs<kSubgroups, 3>(obs, W, K);
        case 4: return pick_obs<kSubgroups, 4>(obs, W, K);
    }
    return nullptr;
}

}  // namespace epipf
