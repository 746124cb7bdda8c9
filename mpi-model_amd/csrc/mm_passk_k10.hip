// mm_passk_k10.hip -- instances of the K-step kernel (mm_passk.hpp) for K = 10 (one attribute).
// Tuning (tools/libsweep.py, profiles/r02): two waves per SIMD (<= 256 VGPRs) and 4 rows
// prefetched per wave; with the register file's other half a second
// wave hides the K-level VALU chains.
#ifndef MM_PASSK_MIN_WAVES
#define MM_PASSK_MIN_WAVES 2
#endif
#ifndef MM_SEG_U1
#define MM_SEG_U1 4
#endif
// scheduling barrier every second row of the steady loop (1.5 % faster than every row at
// 32768^2, profiles/r02_end/rowbarrier; K = 8 prefers every row)
#ifndef MM_ROW_BARRIER
#define MM_ROW_BARRIER 2
#endif
#include "mm_passk.hpp"

namespace mm {

hipError_t passk_launch_k10(int na, bool red, const PassArgs& a, hipStream_t s, int v) {
    switch (na) {
        case 1: return launch_k2<10, 1, false>(red, a, s, v);
        default: return hipErrorInvalidValue;
    }
}

int passk_waves_k10(int na, bool red, int nt) {
    switch (na) {
        case 1: return seg_blocks_per_cu<10, 1, false>(red, nt) * kWavesPerBlock;
        default: return 0;
    }
}

}  // namespace mm
