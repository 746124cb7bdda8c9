// mm_wide8_k8.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 8
// with 8 columns per lane: 2 level(s) per wave (ascending, no pend registers), 4 waves per
// workgroup, two waves per SIMD.
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 2
#endif
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 1
#endif
#include "mm_wide.hpp"

namespace mm {

hipError_t wide8_launch_k8(bool red, const PassArgs& a, hipStream_t s, int v) {
    return wide_launch2<8, 2, 4, 2>(red, a, s, v);
}

int wide8_blocks_k8(bool red, int nt) { return wide_blocks<8, 2, 4, 2>(red, nt); }

}  // namespace mm
