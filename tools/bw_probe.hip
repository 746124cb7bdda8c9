// bw_probe.hip -- HBM ceiling on this box for the access shape of the step kernel:
// a 16-B-per-lane streaming copy (read N bytes + write N bytes), plain and
// non-temporal, at the C2 (268 MB total) and C3-like (8.6 GB total) sizes.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double dv2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void copy2(const double2* __restrict__ a, double2* __restrict__ b, long long n) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    long long stride = (long long)gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        if (NT) {
            dv2 v = __builtin_nontemporal_load((const dv2*)(a + i));
            __builtin_nontemporal_store(v, (dv2*)(b + i));
        } else {
            b[i] = a[i];
        }
    }
}

template <bool NT>
float run(const double2* a, double2* b, long long n, int blocks, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(copy2<NT>, dim3(blocks), dim3(256), 0, 0, a, b, n);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(copy2<NT>, dim3(blocks), dim3(256), 0, 0, i & 1 ? (const double2*)b : a, i & 1 ? (double2*)a : b, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

// The step kernel's memory pattern without its arithmetic: a wave walks down a strip of
// 128 columns (16 B per lane per row) for TH rows with U row loads in flight.
// STRIP_MAJOR: the strip's rows are contiguous ([strip][row][128]) instead of row-major.
template <int U, bool NT, bool STRIP_MAJOR>
__global__ __launch_bounds__(256) void walk(const double* in, double* out, long long H, long long W,
                                            int TH) {
    const int lane = threadIdx.x & 63;
    const long long wid = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long long nstrips = W / 128;
    const long long strip = wid % nstrips, rb = wid / nstrips;
    const long long r0 = rb * TH;
    if (r0 >= H) return;
    const int rows = (int)(r0 + TH <= H ? TH : H - r0);  // rows of this wave, never past H
    auto off = [&](long long r) {
        return STRIP_MAJOR ? (strip * H + r) * 128 + 2 * lane : r * W + strip * 128 + 2 * lane;
    };
    dv2 buf[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
        if (k < rows)
            buf[k] = NT ? __builtin_nontemporal_load((const dv2*)(in + off(r0 + k)))
                        : *(const dv2*)(in + off(r0 + k));
    for (int r = 0; r < rows; r += U) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (r + k >= rows) break;
            dv2 v = buf[k];
            if (r + k + U < rows)
                buf[k] = NT ? __builtin_nontemporal_load((const dv2*)(in + off(r0 + r + k + U)))
                            : *(const dv2*)(in + off(r0 + r + k + U));
            v = v * 0.5;
            if (NT)
                __builtin_nontemporal_store(v, (dv2*)(out + off(r0 + r + k)));
            else
                *(dv2*)(out + off(r0 + r + k)) = v;
        }
    }
}

template <int U, bool NT, bool SM>
float run_walk(const double* a, double* b, long long H, long long W, int TH, int reps) {
    const long long waves = (W / 128) * ((H + TH - 1) / TH);
    const unsigned blocks = (unsigned)((waves + 3) / 4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((walk<U, NT, SM>), dim3(blocks), dim3(256), 0, 0, a, b, H, W, TH);
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((walk<U, NT, SM>), dim3(blocks), dim3(256), 0, 0, i & 1 ? (const double*)b : a, i & 1 ? (double*)a : b, H, W, TH);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

void walks(long long H, long long W) {
    double *a, *b;
    CK(hipMalloc(&a, H * W * 8)); CK(hipMalloc(&b, H * W * 8));
    CK(hipMemset(a, 0, H * W * 8)); CK(hipMemset(b, 0, H * W * 8));
    const double bytes = 16.0 * H * W;
    for (int TH : {8, 16, 32, 64, 256}) {
        float t[6] = {run_walk<8, false, false>(a, b, H, W, TH, 10), run_walk<8, true, false>(a, b, H, W, TH, 10),
                      run_walk<8, false, true>(a, b, H, W, TH, 10), run_walk<8, true, true>(a, b, H, W, TH, 10),
                      run_walk<16, true, false>(a, b, H, W, TH, 10), run_walk<16, true, true>(a, b, H, W, TH, 10)};
        printf("walk %lldx%lld TH=%d GB/s: rowmajor %.0f rowmajor-nt %.0f stripmajor %.0f stripmajor-nt %.0f | U16 rowmajor-nt %.0f stripmajor-nt %.0f\n",
               H, W, TH, bytes / t[0] / 1e6, bytes / t[1] / 1e6, bytes / t[2] / 1e6, bytes / t[3] / 1e6,
               bytes / t[4] / 1e6, bytes / t[5] / 1e6);
    }
    CK(hipFree(a)); CK(hipFree(b));
}

int main() {
    walks(16384, 16384);
    walks(4096, 4096);
    walks(32768, 32768);
    long long sizes[] = {4096LL * 4096, 16384LL * 16384, 32768LL * 16384};
    for (long long cells : sizes) {
        long long n = cells / 2;
        double2 *a, *b;
        CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16));
        CK(hipMemset(a, 0, n * 16)); CK(hipMemset(b, 0, n * 16));
        for (int blocks : {2048, 4096, 8192, (int)std::min<long long>(n / 256, 1 << 20)}) {
            float t0 = run<false>(a, b, n, blocks, 20);
            float t1 = run<true>(a, b, n, blocks, 20);
            double bytes = 2.0 * cells * 8;
            printf("cells=%lld blocks=%d plain %.1f us %.0f GB/s | nt %.1f us %.0f GB/s\n", cells, blocks,
                   t0 * 1e3, bytes / t0 / 1e6, t1 * 1e3, bytes / t1 / 1e6);
        }
        CK(hipFree(a)); CK(hipFree(b));
    }
    return 0;
}
