// mm_wide_k4.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 4:
// 1 level(s) per wave, 4 waves per workgroup.
#include "mm_wide.hpp"

namespace mm {

hipError_t wide_launch_k4(bool red, const PassArgs& a, hipStream_t s, int v) {
    return wide_launch2<4, 1, 1, 4, MM_WIDE_MIN_WAVES>(red, a, s, v);
}

int wide_blocks_k4(bool red, int nt) { return wide_blocks<4, 1, 1, 4, MM_WIDE_MIN_WAVES>(red, nt); }


}  // namespace mm
