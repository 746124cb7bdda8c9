// mm_widea_k8.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 8
// and several attributes (config C5: four, with transfer chains): 2 columns per lane,
// 1 level per wave, 8 waves per workgroup, rows handed on in groups of 2 (the LDS ring
// of a group of 4 rows holds 224 KiB per workgroup).
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 2
#endif
#include "mm_wide.hpp"

namespace mm {

hipError_t widea_launch_k8(int na, bool red, const PassArgs& a, hipStream_t s, int v) {
    if (na == 4) return wide_launch2<2, 4, 1, 8, 2>(red, a, s, v);
    return hipErrorInvalidValue;
}

int widea_blocks_k8(int na, bool red, int nt) {
    return na == 4 ? wide_blocks<2, 4, 1, 8, 2>(red, nt) : 0;
}

}  // namespace mm
