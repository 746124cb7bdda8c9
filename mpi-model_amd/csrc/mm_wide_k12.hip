// mm_wide_k12.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 12:
// 3 level(s) per wave, 4 waves per workgroup.
#include "mm_wide.hpp"

namespace mm {

hipError_t wide_launch_k12(bool red, const PassArgs& a, hipStream_t s, int v) {
    return wide_launch2<4, 1, 3, 4, MM_WIDE_MIN_WAVES>(red, a, s, v);
}

int wide_blocks_k12(bool red, int nt) { return wide_blocks<4, 1, 3, 4, MM_WIDE_MIN_WAVES>(red, nt); }


}  // namespace mm
