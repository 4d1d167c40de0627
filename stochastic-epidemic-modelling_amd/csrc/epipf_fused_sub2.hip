// epipf_fused_sub2.hip -- one-workgroup filter kernels of the subgroup-2 model (epipf_fused.hpp)
#include "epipf_fused.hpp"

namespace epipf {

FusedFn fused_launcher_sub2(int G, int obs, int W) {
    switch (G) {
        case 1: return pick_fused_obs<kSubgroups2, 1>(obs, W);
        case 2: return pick_fused_obs<kSubgroups2, 2>(obs, W);
        case 3: return pick_fused_obs<kSubgroups2, 3>(obs, W);
        case 4: return pick_fused_obs<kSubgroups2, 4>(obs, W);
    }
    return nullptr;
}

}  // namespace epipf
