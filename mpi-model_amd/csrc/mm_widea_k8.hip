// mm_widea_k8.hip -- instances of the level-split K-step kernel (mm_wide.hpp) for K = 8
// and four attributes (config C5 and any other one-pass program of transfer chains and
// diffusions): 2 columns per lane, 2 levels per wave on 4 waves (the ring instance's
// layout, mm_widear_k8.hip), rows handed on in groups of 2, non-temporal stores. Chains
// with run-time operands at the ring's cost (chain_asm: the s_set_gpr_idx mode indexes the
// fp64 instructions' own operands).
//
// Compiled once per instance by the Makefile: MM_ND = N (attributes 0..N-1 diffuse, the
// others pass through; the engine relabels the attributes so that the diffusing ones come
// first) and MM_CHAIN_POST = P (the pass has a post-chain), into widea8_launch_nN_pP /
// widea8_blocks_nN_pP.
#ifndef MM_ND
#error "MM_ND (1..4) is set per object by the Makefile"
#endif
#ifndef MM_CHAIN_POST
#error "MM_CHAIN_POST (0 / 1) is set per object by the Makefile"
#endif
#define MM_WIDE_U 1
#define MM_WIDE_B 2
// levels in ascending order (round 6): no pend registers -- the sums instance spilled 455
// VGPRs with the pend hand-off and the box-sum step, 29 without
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 1
#endif
#define MM_CHAIN_ASM 1
#define MM_WIDE_GEN_ROW 0  // per-column GEN weights: the row-factor body spills here (n4 p1: 125 -> 379)
#include "mm_wide.hpp"

#define MM_CAT3(a, b, c) a##b##c
#define MM_NAME(f, n, p) MM_CAT3(f, n, p)
#define MM_LAUNCH MM_NAME(widea8_launch_n, MM_ND, MM_NAME(_p, MM_CHAIN_POST, ))
#define MM_BLOCKS MM_NAME(widea8_blocks_n, MM_ND, MM_NAME(_p, MM_CHAIN_POST, ))

namespace mm {

hipError_t MM_LAUNCH(bool red, const PassArgs& a, hipStream_t s) {
    return wide_launch3<2, 4, 2, 4, 2, 1>(red, a, s);
}

int MM_BLOCKS(bool red) {
    return red ? wide_blocks_v<2, 4, 2, 4, 2, true, 1>() : wide_blocks_v<2, 4, 2, 4, 2, false, 1>();
}

}  // namespace mm
