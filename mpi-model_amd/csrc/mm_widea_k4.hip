// mm_widea_k4.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 4
// and several attributes (config C5: four, with transfer chains): 2 columns per lane,
// 1 level per wave, 4 waves per workgroup, rows handed on in groups of 2 (the LDS ring
// of a group of 4 rows holds 96 KiB per workgroup). Pre- and post-chains with run-time
// operands (chain_asm: the first n slots of a chain run, a scalar branch inside the asm
// skips the rest; outflows leaving the system land on the pad pair).
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 2
#endif
#define MM_CHAIN_ASM 1
#define MM_CHAIN_POST 1
#include "mm_wide.hpp"

namespace mm {

hipError_t widea_launch_k4(int na, bool red, const PassArgs& a, hipStream_t s, int v) {
    if (na == 4) return wide_launch2<2, 4, 1, 4, 2>(red, a, s, v & 1);
    return hipErrorInvalidValue;
}

int widea_blocks_k4(int na, bool red, int nt) {
    return na == 4 ? wide_blocks<2, 4, 1, 4, 2>(red, nt & 1) : 0;
}

}  // namespace mm
