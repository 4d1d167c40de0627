// epipf_group_sub2.hip -- lane-group step kernels of the group-summed subgroup model (epipf_group.hpp)
#include "epipf_group.hpp"

namespace epipf {

GroupStepFn group_launcher_sub2(int G, int obs, int W, int K) {
    switch (G) {
        case 1: return pick_obs<kSubgroups2, 1>(obs, W, K);
        case 2: return pick_obs<kSubgroups2, 2>(obs, W, K);
        case 3: return pick_obs<kSubgroups2, 3>(obs, W, K);
        case 4: return pick_obs<kSubgroups2, 4>(obs, W, K);
    }
    return nullptr;
}

}  // namespace epipf
