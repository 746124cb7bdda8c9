// mm_kernels_k.hip -- dispatch of the K-step kernels (templates: mm_passk.hpp and
// mm_wide.hpp, instances: mm_passk_k1..10.hip, mm_wide_k*.hip) and the fixed-order
// level-sum finalize kernel.
#include "mm_wide.hpp"

namespace mm {

namespace {

// Fixed-order sums of the levels in `mask` of partials[n][k][na] -> one history entry of
// na sums per level, slots from the device counter (graph-replayable). One workgroup per
// (level of the mask, attribute), all in parallel: workgroup b sums level j = the e-th set
// bit of mask (e = b / na) of attribute a = b % na -- each thread a strided run of the n
// partials, then a tree over the 256 threads (the order of the single-workgroup kernel
// this replaces, which walked the K x NA sums one after another: 37.8 us per C5 pass,
// profiles/r03/r3q). Partials slot a holds attribute (perm >> 2a) & 3 (the engine's
// relabelled passes). Every workgroup reads the slot counter hist_n[0]; the last one to
// finish (hist_n[1] counts them, agent-scope atomics: the workgroups run on every XCD)
// advances it and resets the count for the next launch.
__global__ __launch_bounds__(256) void mm_level_sums_kernel(const double* partials, long long n,
                                                            int k, int na, int mask,
                                                            double* hist,
                                                            unsigned long long* hist_n,
                                                            long long cap, int perm) {
    __shared__ double red[256];
    const int e = (int)blockIdx.x / na, a = (int)blockIdx.x % na;
    int j = 0;
    for (int c = -1; j < k; ++j)
        if (((mask >> j) & 1) && ++c == e) break;
    double s = 0.0;
    for (long long i = threadIdx.x; i < n; i += 256) s = s + partials[(i * k + j) * na + a];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int m = 128; m >= 1; m >>= 1) {
        if ((int)threadIdx.x < m) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + m];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const unsigned long long slot =
            __hip_atomic_load(hist_n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const long long idx = (long long)slot + e;
        if (idx < cap) hist[idx * na + ((perm >> (2 * a)) & 3)] = red[0];
        // the slot is read before this workgroup counts itself done (acq_rel orders them)
        const unsigned long long done = __hip_atomic_fetch_add(
            hist_n + 1, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (unsigned long long)gridDim.x - 1) {
            const int entries = __builtin_popcount((unsigned)mask);
            __hip_atomic_store(hist_n, slot + (unsigned long long)entries, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(hist_n + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

hipError_t launch_finalize_levels(const double* partials, long long n, int k, int na, int mask,
                                  double* hist, unsigned long long* hist_n, long long cap,
                                  hipStream_t s, int perm) {
    const int entries = __builtin_popcount((unsigned)mask);
    if (entries == 0) return hipSuccess;
    hipLaunchKernelGGL(mm_level_sums_kernel, dim3((unsigned)(entries * na)), dim3(256), 0, s,
                       partials, n, k, na, mask, hist, hist_n, cap, perm);
    return hipGetLastError();
}

int passk_out_cols(int k) { return kStripCols - 4 * ((k + 1) / 2); }

int passk_max_steps(int na) { return na == 1 ? kMaxSteps : 2; }

long long passk_max_rows(int k, long long pitch) {
    // every buffer offset of a wave (rows x pitch x 8 B, plus the OOB marker) stays < 2^31
    return (1LL << 31) / (pitch * 8) - (3 * k + 2 * seg_prefetch<1>() + 8);
}

int passk_waves_per_cu(int k, int na, bool red, int nt) {
    switch (k) {
        case 1: return passk_waves_k1(na, red, nt);
        case 2: return passk_waves_k2(na, red, nt);
        case 3: return passk_waves_k3(na, red, nt);
        case 4: return passk_waves_k4(na, red, nt);
        case 5: return passk_waves_k5(na, red, nt);
        case 6: return passk_waves_k6(na, red, nt);
        case 7: return passk_waves_k7(na, red, nt);
        case 8: return passk_waves_k8(na, red, nt);
        case 9: return passk_waves_k9(na, red, nt);
        case 10: return passk_waves_k10(na, red, nt);
        default: return 0;
    }
}

// A pass of no work is not launched -- unless waves_a < 0 marks it as mm_prepare's
// priming dispatch: one workgroup that leaves at its first instruction (waves_total = 0),
// which loads the kernel and sizes the queue's scratch for it ahead of the run.
hipError_t launch_passk(int k, int na, bool red, const PassArgs& a, hipStream_t s, int variant) {
    if (a.waves_total <= 0 && a.waves_a >= 0) return hipSuccess;
    switch (k) {
        case 1: return passk_launch_k1(na, red, a, s, variant);
        case 2: return passk_launch_k2(na, red, a, s, variant);
        case 3: return passk_launch_k3(na, red, a, s, variant);
        case 4: return passk_launch_k4(na, red, a, s, variant);
        case 5: return passk_launch_k5(na, red, a, s, variant);
        case 6: return passk_launch_k6(na, red, a, s, variant);
        case 7: return passk_launch_k7(na, red, a, s, variant);
        case 8: return passk_launch_k8(na, red, a, s, variant);
        case 9: return passk_launch_k9(na, red, a, s, variant);
        case 10: return passk_launch_k10(na, red, a, s, variant);
        default: return hipErrorInvalidValue;
    }
}

bool wide_has(int k, int c, int na) {
    if (na > 1) return na == 4 && c == 2 && (k == 4 || k == 8);
    return c == 4 && (k == 4 || k == 8 || k == 12 || k == 16 || k == 20);
}

int wide_out_cols(int k, int c, int na) {
    (void)na;
    return 64 * c - 2 * c * ((k + c - 1) / c);  // 64 lanes less ceil(K / C) halo lanes a side
}

int wide_waves_per_block(int k, int c, int na, bool ring) {
    if (!wide_has(k, c, na)) return 0;
    if (na > 1 && k == 8 && ring) return widear_waves_k8();
    if (na == 1 && k == 20) return wide_waves_k20();  // MM_K20_KW levels per wave
    // one attribute: K / 4 levels per wave, 4 level groups; four attributes: mm_widea_k4
    // 1 level per wave, mm_widea_k8 2
    return 4;
}

namespace {

// The K = 8 four-attribute instance of a variant: (nd - 1) * 2 + post, -1 if none.
int widea8_index(int variant) {
    const int nd = (variant >> 4) & 7, post = (variant >> 2) & 1;
    return nd >= 1 && nd <= 4 ? (nd - 1) * 2 + post : -1;
}

}  // namespace

int wide_blocks_per_cu(int k, int c, int na, bool red, int nt) {
    if (!wide_has(k, c, na)) return 0;
    if (na > 1 && k == 8 && (nt & 2)) return widear_blocks_k8(na, red, nt & 1);
    if (na > 1 && k == 4) return widea_blocks_k4(na, red, nt & 1);
    if (na > 1) {
        switch (widea8_index(nt)) {
            case 0: return widea8_blocks_n1_p0(red);
            case 1: return widea8_blocks_n1_p1(red);
            case 2: return widea8_blocks_n2_p0(red);
            case 3: return widea8_blocks_n2_p1(red);
            case 4: return widea8_blocks_n3_p0(red);
            case 5: return widea8_blocks_n3_p1(red);
            case 6: return widea8_blocks_n4_p0(red);
            case 7: return widea8_blocks_n4_p1(red);
            default: return 0;
        }
    }
    nt &= 1;
    switch (k) {
        case 4: return wide_blocks_k4(red, nt);
        case 8: return wide_blocks_k8(red, nt);
        case 12: return wide_blocks_k12(red, nt);
        case 16: return wide_blocks_k16(red, nt);
        default: return wide_blocks_k20(red, nt);
    }
}

hipError_t launch_wide(int k, int c, int na, bool red, const PassArgs& a, hipStream_t s,
                       int variant) {
    if (a.waves_total <= 0 && a.waves_a >= 0) return hipSuccess;  // (waves_a < 0: priming)
    if (!wide_has(k, c, na)) return hipErrorInvalidValue;
    if (na > 1 && k == 8 && (variant & 2)) return widear_launch_k8(na, red, a, s, variant & 1);
    if (na > 1 && k == 4) return widea_launch_k4(na, red, a, s, variant & 1);
    if (na > 1) {
        switch (widea8_index(variant)) {
            case 0: return widea8_launch_n1_p0(red, a, s);
            case 1: return widea8_launch_n1_p1(red, a, s);
            case 2: return widea8_launch_n2_p0(red, a, s);
            case 3: return widea8_launch_n2_p1(red, a, s);
            case 4: return widea8_launch_n3_p0(red, a, s);
            case 5: return widea8_launch_n3_p1(red, a, s);
            case 6: return widea8_launch_n4_p0(red, a, s);
            case 7: return widea8_launch_n4_p1(red, a, s);
            default: return hipErrorInvalidValue;
        }
    }
    switch (k) {
        case 4: return wide_launch_k4(red, a, s, variant);
        case 8: return wide_launch_k8(red, a, s, variant);
        case 12: return wide_launch_k12(red, a, s, variant);
        case 16: return wide_launch_k16(red, a, s, variant);
        default: return wide_launch_k20(red, a, s, variant);
    }
}

}  // namespace mm
