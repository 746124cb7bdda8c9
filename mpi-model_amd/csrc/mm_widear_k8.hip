// mm_widear_k8.hip -- the four-attribute level-split K-step kernel (mm_widea_k8.hip) for
// programs whose pre-chain is the ring of transfers t -> t+1 mod 4 and that have no
// post-chain (config C5's topology): the chain's operands are compile-time registers
// instead of an indexed register vector, and every attribute diffuses. The engine checks
// the pattern (wring).
// Levels in ascending order, two input rows prefetched (round 6: C5 365-368 GCUPS against
// 327 with the pend hand-off and one row, profiles/r06/ab)
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 1
#endif
#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 2
#endif
#ifndef MM_WIDEAR_KW
// levels per wave (P = 8 / KW waves per workgroup): two levels on 4 waves run the C5 pass
// in 504-512 us against 595-604 for one level on 8 (same box, bit-identical states;
// profiles/r03/c5var); 4 waves also halve the LDS (48 KiB: two workgroups per CU)
#define MM_WIDEAR_KW 2
#endif
#define MM_CHAIN_RING 1
// per-column GEN weights: the row-factor GEN body takes this instance from 239 VGPRs and no
// scratch to 256 + 20 bytes of scratch (the C5 pass 349 -> 374 us on two boxes)
#define MM_WIDE_GEN_ROW 0
#define MM_ND 4  // every attribute diffuses (the engine checks)
#include "mm_wide.hpp"

namespace mm {

hipError_t widear_launch_k8(int na, bool red, const PassArgs& a, hipStream_t s, int v) {
    if (na == 4) return wide_launch2<2, 4, MM_WIDEAR_KW, 8 / MM_WIDEAR_KW, 2>(red, a, s, v);
    return hipErrorInvalidValue;
}

int widear_waves_k8() { return 8 / MM_WIDEAR_KW; }

int widear_blocks_k8(int na, bool red, int nt) {
    return na == 4 ? wide_blocks<2, 4, MM_WIDEAR_KW, 8 / MM_WIDEAR_KW, 2>(red, nt) : 0;
}

}  // namespace mm
