// mm_wide_k8.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 8:
// 2 level(s) per wave, 4 waves per workgroup.
// Tuning (tools/libsweep.py, profiles/r04/k8): barrier groups of 2 rows (2 prefetched):
// the pipeline fill of the 108-row segments of C2 (4096^2) is 6 iterations shorter per
// wave, 85.0 / 84.3 vs 87.2 / 86.6 us per 8-step pass in two sweeps; groups of 1 row
// 101 us; an LDS-DMA input ring 8 / 12 rows deep 86.0 / 86.5 us.
// Three workgroups per CU (168 VGPRs, `MM_WIDE_MIN_WAVES 3`): with the GEN / EDGE bodies and
// the MID-body pipeline fill of round 5 the instance took 188 VGPRs, two per CU, and C2
// fell from 1564 to 1435 GCUPS with longer segments; at 168 the steady loops are
// unchanged (no scratch, tools/asm_steady.py), the spills sit in the GEN paths.
// Levels in ascending order (round 6, with the box-sum step): no pend registers, and the
// wave offset D = 2 KW + B is even, so the middle waves share one instance; the pend
// hand-off (D = 7) takes C2 from 1722-1808 to 1531-1607 GCUPS on one box (profiles/r06/ab).
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 1
#endif
#ifndef MM_WIDE_MIN_WAVES
#define MM_WIDE_MIN_WAVES 3
#endif
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 2
#endif
#include "mm_wide.hpp"

namespace mm {

hipError_t wide_launch_k8(bool red, const PassArgs& a, hipStream_t s, int v) {
    return wide_launch2<4, 1, 2, 4, MM_WIDE_MIN_WAVES>(red, a, s, v);
}

int wide_blocks_k8(bool red, int nt) { return wide_blocks<4, 1, 2, 4, MM_WIDE_MIN_WAVES>(red, nt); }


}  // namespace mm
