// mm_passk_k2.hip -- instances of the K-step kernel (mm_passk.hpp) for K = 2.
// Tuning (tools/libsweep.py --program c5, profiles/r02/libsweep_c5.log): the 3- and
// 4-attribute instances fit two waves per SIMD (<= 256 registers) with one row of the
// attributes prefetched; at the default 2 rows the 4-attribute K = 2 instance needs 257
// registers, one wave per SIMD, and runs 1.7x slower.
#ifndef MM_PASSK_MIN_WAVES
#define MM_PASSK_MIN_WAVES 2
#endif
#ifndef MM_SEG_UN
#define MM_SEG_UN 1
#endif
#include "mm_passk.hpp"

namespace mm {

hipError_t passk_launch_k2(int na, bool red, const PassArgs& a, hipStream_t s, int v) {
    switch (na) {
        case 1: return launch_k2<2, 1, false>(red, a, s, v);
        case 2: return launch_k2<2, 2, true>(red, a, s, v);
        case 3: return launch_k2<2, 3, true>(red, a, s, v);
        case 4: return launch_k2<2, 4, true>(red, a, s, v);
        default: return hipErrorInvalidValue;
    }
}

int passk_waves_k2(int na, bool red, int nt) {
    switch (na) {
        case 1: return seg_blocks_per_cu<2, 1, false>(red, nt) * kWavesPerBlock;
        case 2: return seg_blocks_per_cu<2, 2, true>(red, nt) * kWavesPerBlock;
        case 3: return seg_blocks_per_cu<2, 3, true>(red, nt) * kWavesPerBlock;
        case 4: return seg_blocks_per_cu<2, 4, true>(red, nt) * kWavesPerBlock;
        default: return 0;
    }
}

}  // namespace mm
