// mm_wide_k16.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 16:
// 4 level(s) per wave, 4 waves per workgroup.
// Tuning (tools/libsweep.py, profiles/r03/sweep_w16): 2 input rows prefetched by the first
// wave (243 VGPRs, no spill; 4 rows: 256 VGPRs with a spill) -- 1.5 % faster at 32768^2.
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#include "mm_wide.hpp"

namespace mm {

hipError_t wide_launch_k16(bool red, const PassArgs& a, hipStream_t s, int v) {
    return wide_launch2<4, 1, 4, 4, MM_WIDE_MIN_WAVES>(red, a, s, v);
}

int wide_blocks_k16(bool red, int nt) { return wide_blocks<4, 1, 4, 4, MM_WIDE_MIN_WAVES>(red, nt); }


}  // namespace mm
