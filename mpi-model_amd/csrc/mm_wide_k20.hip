// mm_wide_k20.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 20:
// 5 level(s) per wave, 4 waves per workgroup.
// Tuning (tools/libsweep.py, profiles/r03/var_k20): levels in ascending order (no pend
// registers: VGPR spills 504 -> 27) and 2 input rows prefetched -- 7 % faster at 32768^2
// than the pend hand-off with 4 rows (8260 vs 8891 us per 20-step pass on one box).
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 1
#endif
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_K20_KW
#define MM_K20_KW 5  // levels per wave (20 / MM_K20_KW waves per workgroup)
#endif
#include "mm_wide.hpp"

namespace mm {

hipError_t wide_launch_k20(bool red, const PassArgs& a, hipStream_t s, int v) {
    return wide_launch2<4, 1, MM_K20_KW, 20 / MM_K20_KW, MM_WIDE_MIN_WAVES>(red, a, s, v);
}

int wide_blocks_k20(bool red, int nt) {
    return wide_blocks<4, 1, MM_K20_KW, 20 / MM_K20_KW, MM_WIDE_MIN_WAVES>(red, nt);
}

int wide_waves_k20() { return 20 / MM_K20_KW; }

}  // namespace mm
