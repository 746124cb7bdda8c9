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

// One object per instance (sums or not x non-temporal stores or not): the Makefile builds
// this unit with MM_PART_RED / MM_PART_NT set for each of the four instances (they compile
// in parallel), and once without them for the dispatcher below.
#define MM_K20_P (20 / MM_K20_KW)
#define MM_CAT4(a, b, c, d) a##b##c##d
#define MM_PN(f, r, n) MM_CAT4(f, r, _n, n)

namespace mm {

#if defined(MM_PART_RED) && defined(MM_PART_NT)

hipError_t MM_PN(wide_launch_k20_r, MM_PART_RED, MM_PART_NT)(const PassArgs& a, hipStream_t s) {
    return wide_launch4<4, 1, MM_K20_KW, MM_K20_P, MM_WIDE_MIN_WAVES, MM_PART_RED != 0,
                        MM_PART_NT>(a, s);
}

int MM_PN(wide_blocks_k20_r, MM_PART_RED, MM_PART_NT)() {
    return wide_blocks_v<4, 1, MM_K20_KW, MM_K20_P, MM_WIDE_MIN_WAVES, MM_PART_RED != 0,
                         MM_PART_NT>();
}

#else

#define MM_K20_DECL(r, n)                                                                 \
    hipError_t wide_launch_k20_r##r##_n##n(const PassArgs& a, hipStream_t s);              \
    int wide_blocks_k20_r##r##_n##n();
MM_K20_DECL(0, 0)
MM_K20_DECL(0, 1)
MM_K20_DECL(1, 0)
MM_K20_DECL(1, 1)
#undef MM_K20_DECL

hipError_t wide_launch_k20(bool red, const PassArgs& a, hipStream_t s, int v) {
    if (red) return (v & 1) ? wide_launch_k20_r1_n1(a, s) : wide_launch_k20_r1_n0(a, s);
    return (v & 1) ? wide_launch_k20_r0_n1(a, s) : wide_launch_k20_r0_n0(a, s);
}

int wide_blocks_k20(bool red, int nt) {
    if (red) return nt ? wide_blocks_k20_r1_n1() : wide_blocks_k20_r1_n0();
    return nt ? wide_blocks_k20_r0_n1() : wide_blocks_k20_r0_n0();
}

int wide_waves_k20() { return MM_K20_P; }

#endif

}  // namespace mm
