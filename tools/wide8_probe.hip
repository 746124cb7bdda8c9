// wide8_probe.hip -- diagnostic: the level-split kernel at K = 8 with 4 and with 8 columns
// per lane on a 32768^2 grid (no sums, non-temporal stores), HIP-event timed, for rocprofv3
// counter passes. Not part of the product.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I mpi-model_amd/csrc \
//         -I include -mllvm -pragma-unroll-threshold=200000 tools/wide8_probe.hip -o tools/wide8_probe
//   tools/wide8_probe [cols: 4|8|0=both] [reps]
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef MM_WIDE_U
#define MM_WIDE_U 2
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 2
#endif
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 1
#endif
#include "mm_wide.hpp"

using namespace mm;

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));      \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

template <int C, int KW, int MW, int GB = MM_WIDE_B>
double run(double* in, double* out, long long H, long long W, long long pitch, int reps) {
    constexpr int P = 4, K = KW * P;
    constexpr int LH = (K + C - 1) / C, OC = 64 * C - 2 * C * LH;
    PassArgs A;
    std::memset(&A, 0, sizeof A);
    A.in[0] = in;
    A.out[0] = out;
    A.H = H;
    A.W = W;
    A.pitch = pitch;
    A.drate[0] = 0.1;
    A.diffuse_mask = 1;
    A.seg = 1;
    A.nstrips = (int)((W + OC - 1) / OC);
    const int blocks_per_cu = [] {
        hipFuncAttributes fa;
        CHECK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(
            mm_wide_kernel<C, 1, KW, P, MW, MM_WIDE_U, GB, false, 1>)));
        const int regs = (fa.numRegs + 7) / 8 * 8;
        int b = std::min(8, 512 / regs) * 4 / P;
        return std::min(b, (int)(160 * 1024 / fa.sharedSizeBytes));
    }();
    // segments: ~4 resident block waves, edge strips at half length
    const long long want = 4LL * 256 * std::max(1, blocks_per_cu);
    const double units = (A.nstrips - 2) + 2.0 / 0.5;
    long long r = (long long)(H * units / want) + 1;
    A.th = (int)r;
    A.th_edge = (int)std::max<long long>(8, r / 2);
    A.ra0 = 0;
    A.ra1 = (int)H;
    const long long nbe = (H + A.th_edge - 1) / A.th_edge, nb = (H + r - 1) / r;
    A.waves_a = A.waves_total = 2 * nbe + (A.nstrips - 2) * nb;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    auto launch = [&] {
        hipLaunchKernelGGL((mm_wide_kernel<C, 1, KW, P, MW, MM_WIDE_U, GB, false, 1>),
                           dim3((unsigned)A.waves_total), dim3(64 * P), 0, 0, A);
        return hipGetLastError();
    };
    CHECK(launch());  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) CHECK(launch());
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"B\": %d, \"cols\": %d, \"K\": %d, \"strips\": %d, \"rows_per_block\": %lld, \"blocks\": %lld, "
                "\"blocks_per_cu\": %d, \"pass_us\": %.1f}\n",
                GB, C, K, A.nstrips, r, (long long)A.waves_total, blocks_per_cu, 1e3 * ms / reps);
    return ms / reps;
}

int main(int argc, char** argv) {
    const int which = argc > 1 ? std::atoi(argv[1]) : 0;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const long long H = 32768, W = 32768, pitch = 32768, ghost = 20;
    const size_t n = (size_t)(H + 2 * ghost) * pitch;
    double *b0, *b1;
    CHECK(hipMalloc(&b0, n * sizeof(double)));
    CHECK(hipMalloc(&b1, n * sizeof(double)));
    std::vector<double> row(pitch, 1.0);
    CHECK(hipMemset(b0, 0, n * sizeof(double)));
    CHECK(hipMemset(b1, 0, n * sizeof(double)));
    for (long long i = 0; i < H; i += 4096)  // some non-zero data
        CHECK(hipMemcpy(b0 + (ghost + i) * pitch, row.data(), pitch * sizeof(double), hipMemcpyHostToDevice));
    CHECK(hipDeviceSynchronize());
    double* in = b0 + ghost * pitch;
    double* out = b1 + ghost * pitch;
    if (which == 4) run<4, 2, 2>(in, out, H, W, pitch, reps);

    if (which == 16) run<4, 4, 2>(in, out, H, W, pitch, reps);
    if (which == 20) run<4, 5, 2>(in, out, H, W, pitch, reps);
    if (which == 164) run<4, 4, 2, 4>(in, out, H, W, pitch, reps);
    if (which == 204) run<4, 5, 2, 4>(in, out, H, W, pitch, reps);
    CHECK(hipFree(b0));
    CHECK(hipFree(b1));
    return 0;
}
