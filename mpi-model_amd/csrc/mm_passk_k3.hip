// mm_passk_k3.hip -- instances of the K-step kernel (mm_passk.hpp) for K = 3.
#include "mm_passk.hpp"

namespace mm {

hipError_t passk_launch_k3(int na, bool red, const PassArgs& a, hipStream_t s, int v) {
    switch (na) {
        case 1: return launch_k2<3, 1, false>(red, a, s, v);
        default: return hipErrorInvalidValue;
    }
}

int passk_waves_k3(int na, bool red, int nt) {
    switch (na) {
        case 1: return seg_blocks_per_cu<3, 1, false>(red, nt) * kWavesPerBlock;
        default: return 0;
    }
}

}  // namespace mm
