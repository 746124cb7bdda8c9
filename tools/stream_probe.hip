// stream_probe.hip -- what limits a long-lived streaming wave on MI355X HBM?
//
// The K-step kernel (csrc/mm_passk.hpp) runs ~2000-row segments per wave and moves
// ~5.1 TB/s; short 8-row waves of the same shape reach ~6.2 TB/s (profiles/r01/bw_probe.log).
// This probe isolates the memory pattern (no arithmetic): a wave copies a 1-KiB-wide strip
// (16 B per lane, buffer loads / non-temporal stores, U rows in flight) down R rows.
//   layout 0: wave = (row segment, strip), strips fastest (the production segment plan)
//   layout 1: "lockstep": wave (group g, strip s) handles rows g, g+G, g+2G, ... so the
//             resident waves all work in one band of G rows that moves down the grid
// occupancy is limited with dynamic LDS (blocks of 4 waves per CU: lds_kb per block).
// mode: 0 copy, 1 loads only (one store per wave), 2 stores only.
// Build: hipcc --offload-arch=gfx950 -O3 tools/stream_probe.hip -o tools/stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                          \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Args {
    const double* in;
    double* out;
    long long H, W;
    int R;          // rows per wave (layout 0) / row groups G (layout 1)
    long long nstrips, waves;
    int layout, mode;
    long long pitch;  // row stride in doubles (>= W)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const double* p, long long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, (int)bytes, 0x00020000);
}

template <int U, int LAUX = 0, int SAUX = 2>
__global__ __launch_bounds__(256) void walk(Args a) {
    extern __shared__ double lds_pad[];
    const int lane = threadIdx.x & 63;
    const long long wid = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wid >= a.waves) return;
    const long long strip = wid % a.nstrips, q = wid / a.nstrips;
    long long r0, rstep;
    int n;
    if (a.layout == 0) {
        r0 = q * a.R;
        rstep = 1;
        n = (int)((r0 + a.R <= a.H) ? a.R : a.H - r0);
    } else {
        r0 = q;  // group q of G = a.R groups
        rstep = a.R;
        n = (int)((a.H - q + a.R - 1) / a.R);
    }
    const long long rowb = a.pitch * 8;
    const unsigned voff = (unsigned)((strip * 128 + 2 * lane) * 8);
    const unsigned step = (unsigned)(rstep * rowb);
    // descriptors rebuilt every U rows at the current row: offsets stay below 2^31
    auto desc = [&](const double* base, int r) {
        const long long rem = (long long)(n - r) * rstep * rowb;
        return rsrc(base + (long long)r * rstep * a.pitch + r0 * a.pitch, rem < 0x7fffffffLL ? rem : 0x7fffffffLL);
    };
    __amdgpu_buffer_rsrc_t ri = desc(a.in, 0), ro = desc(a.out, 0);
    dv2 buf[U];
    if (a.mode != 2) {
#pragma unroll
        for (int k = 0; k < U; ++k)
            buf[k] = __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(ri, voff + k * step, 0, LAUX));
    }
    dv2 acc = {0.0, 0.0};
    for (int r = 0; r < n; r += U) {
        ri = desc(a.in, r);
        ro = desc(a.out, r);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            dv2 v;
            if (a.mode != 2) {
                v = buf[k];
                buf[k] = __builtin_bit_cast(
                    dv2, __builtin_amdgcn_raw_buffer_load_b128(ri, voff + (unsigned)(k + U) * step, 0, LAUX));
            } else {
                v.x = (double)(r + k);
                v.y = v.x;
            }
            if (a.mode == 1) {
                acc = acc + v;
            } else {
                v = v * 0.5;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro,
                                                       voff + (unsigned)k * step, 0, SAUX);
            }
        }
    }
    if (a.mode == 1)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc),
                                               rsrc(a.out + r0 * a.pitch, rowb), voff, 0, 2);
    if (lane == 64) lds_pad[0] = acc.x;  // keep the LDS allocation (never executed)
}

template <int U, int LAUX = 0, int SAUX = 2>
float run(const Args& a0, int lds_kb, int reps) {
    CK(hipFuncSetAttribute((const void*)walk<U, LAUX, SAUX>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           160 * 1024));
    const unsigned blocks = (unsigned)((a0.waves + 3) / 4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    Args a = a0;
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL((walk<U, LAUX, SAUX>), dim3(blocks), dim3(256), lds_kb * 1024, 0, a);
    CK(hipGetLastError());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) {
        Args b = a0;
        if (i & 1) {
            b.in = a0.out;
            b.out = const_cast<double*>(a0.in);
        }
        hipLaunchKernelGGL((walk<U, LAUX, SAUX>), dim3(blocks), dim3(256), lds_kb * 1024, 0, b);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}


// Decoupled stores: a workgroup of NP producer waves (one strip each, loads only, U rows
// in flight) and NC consumer waves. A producer copies each loaded (scaled) row into its
// LDS ring of S slots and publishes it with a counter; a consumer polls the counters of its
// producers, reads the rows back from LDS and issues the global stores. The producers'
// vmcnt then counts loads only; the consumers never wait on their stores.
template <int U, int NP, int NC, int S>
__global__ __launch_bounds__(64 * (NP + NC)) void walk_split(Args a) {
    __shared__ dv2 ring[NP][S][64];
    __shared__ int full[NP], used[NP];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < NP) {
        full[threadIdx.x] = 0;
        used[threadIdx.x] = 0;
    }
    __syncthreads();
    const long long rowb = a.W * 8;
    const long long seg = blockIdx.x / ((a.nstrips + NP - 1) / NP);
    const long long sgrp = blockIdx.x % ((a.nstrips + NP - 1) / NP);
    const long long r0 = seg * a.R;
    const int n = (int)((r0 + a.R <= a.H) ? a.R : a.H - r0);
    if (wave < NP) {
        const long long strip = sgrp * NP + wave;
        const bool live = strip < a.nstrips;
        const unsigned voff = live ? (unsigned)((strip * 128 + 2 * lane) * 8) : 0x80000000u;
        auto desc = [&](int r) {
            const long long rem = (long long)(n - r) * rowb;
            return rsrc(a.in + (r0 + r) * a.W, rem < 0x7fffffffLL ? rem : 0x7fffffffLL);
        };
        __amdgpu_buffer_rsrc_t ri = desc(0);
        dv2 buf[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            buf[k] = __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(ri, voff + k * (unsigned)rowb, 0, 0));
        for (int r = 0; r < n; r += U) {
            ri = desc(r);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                dv2 v = buf[k] * 0.5;
                buf[k] = __builtin_bit_cast(
                    dv2, __builtin_amdgcn_raw_buffer_load_b128(ri, voff + (unsigned)(k + U) * (unsigned)rowb, 0, 0));
                const int t = r + k;
                if (t >= n) break;
                // wait for a free slot: the consumer has taken row t - S
                for (int spin = 0; spin < (1 << 20) &&
                     __hip_atomic_load(&used[wave], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < t - S + 1;
                     ++spin)
                    __builtin_amdgcn_s_sleep(1);  // bounded: a bug shows as wrong data, never a hang
                ring[wave][t % S][lane] = v;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0)
                    __hip_atomic_store(&full[wave], t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    } else {
        const int c = wave - NP;
        for (int t = 0; t < n; ++t) {
            for (int p = c; p < NP; p += NC) {
                const long long strip = sgrp * NP + p;
                for (int spin = 0; spin < (1 << 20) &&
                     __hip_atomic_load(&full[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < t + 1;
                     ++spin)
                    __builtin_amdgcn_s_sleep(1);
                const dv2 v = ring[p][t % S][lane];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0)
                    __hip_atomic_store(&used[p], t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (strip < a.nstrips)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(u32x4, v), rsrc(a.out + (r0 + t) * a.W, rowb),
                        (unsigned)((strip * 128 + 2 * lane) * 8), 0, 2);
            }
        }
    }
}

template <int U, int NP, int NC, int S>
float run_split(const Args& a0, int reps) {
    const long long sg = (a0.nstrips + NP - 1) / NP;
    const unsigned blocks = (unsigned)(sg * ((a0.H + a0.R - 1) / a0.R));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((walk_split<U, NP, NC, S>), dim3(blocks), dim3(64 * (NP + NC)), 0, 0, a0);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) {
        Args b = a0;
        if (i & 1) {
            b.in = a0.out;
            b.out = const_cast<double*>(a0.in);
        }
        hipLaunchKernelGGL((walk_split<U, NP, NC, S>), dim3(blocks), dim3(64 * (NP + NC)), 0, 0, b);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const long long H = argc > 1 ? atoll(argv[1]) : 32768, W = argc > 2 ? atoll(argv[2]) : 32768;
    double *a, *b;
    const long long maxpitch = W + (argc > 4 ? 32768 : 4096);
    CK(hipMalloc(&a, H * maxpitch * 8));
    CK(hipMalloc(&b, H * maxpitch * 8));
    CK(hipMemset(a, 0, H * maxpitch * 8));
    CK(hipMemset(b, 0, H * maxpitch * 8));
    if (argc > 3 && std::string(argv[3]) == "pitch") {
        std::vector<int> pads;
        for (int i = 4; i < argc; ++i) pads.push_back(atoi(argv[i]));
        if (pads.empty()) pads = {0, 64, 128, 256, 1024, 4096};
        for (int pad : pads)
            for (int mode : {0, 2})
                for (int R : {8, 2048}) {
                    Args a0{a, b, H, W, R, W / 128, (W / 128) * ((H + R - 1) / R), 0, mode, W + pad};
                    const float t = run<8>(a0, 0, 6);
                    const double bytes = (mode == 0 ? 16.0 : 8.0) * H * W;
                    std::printf("pitch W+%d R=%d mode=%s : %.1f us %.0f GB/s\n", pad, R,
                                mode == 0 ? "copy" : "store", t * 1e3, bytes / t / 1e6);
                }
        if (argc > 4) return 0;
        for (int pad : {0, 128, 1024})
            for (int R : {512, 2048}) {
                Args a0{a, b, H, W, R, W / 128, (W / 128) * ((H + R - 1) / R), 0, 0, W + pad};
                const float t = run<32>(a0, 160, 6);
                std::printf("pitch W+%d R=%d U=32 lds_kb=160 copy : %.1f us %.0f GB/s\n", pad, R,
                            t * 1e3, 16.0 * H * W / t / 1e6);
            }
        return 0;
    }
    const long long ns = W / 128;
    const char* mname[] = {"copy", "load", "store"};
    std::printf("grid %lldx%lld, GB/s counted as 16 B per cell (copy), 8 B (load/store only)\n", H, W);
    struct Cfg { int layout, R, U, lds_kb, mode; };
    std::vector<Cfg> cfgs;
    for (int mode : {0, 1, 2})
        for (int R : {8, 64, 512, 2048}) cfgs.push_back({0, R, 8, 0, mode});
    for (int lds : {40, 80, 160})  // 16, 8, 4 waves per CU
        for (int R : {512, 2048}) cfgs.push_back({0, R, lds >= 160 ? 32 : (lds >= 80 ? 16 : 8), lds, 0});
    for (int G : {8, 16, 64})
        for (int lds : {0, 80}) cfgs.push_back({1, G, lds >= 80 ? 16 : 8, lds, 0});
    for (const Cfg& c : cfgs) {
        Args a0{a, b, H, W, c.R, ns, 0, c.layout, c.mode, W};
        a0.waves = c.layout == 0 ? ns * ((H + c.R - 1) / c.R) : ns * c.R;
        float t = c.U == 8 ? run<8>(a0, c.lds_kb, 6) : (c.U == 16 ? run<16>(a0, c.lds_kb, 6) : run<32>(a0, c.lds_kb, 6));
        const double bytes = (c.mode == 0 ? 16.0 : 8.0) * H * W;
        std::printf("layout=%d %s=%d U=%d lds_kb=%d mode=%s waves=%lld : %.1f us %.0f GB/s\n", c.layout,
                    c.layout ? "G" : "R", c.R, c.U, c.lds_kb, mname[c.mode], a0.waves, t * 1e3,
                    bytes / t / 1e6);
    }
    // decoupled stores (producer / consumer waves through LDS)
    auto split = [&](const char* name, float (*f)(const Args&, int), int R) {
        Args a0{a, b, H, W, R, ns, 0, 0, 0, W};
        const float t = f(a0, 6);
        std::printf("split %s R=%d : %.1f us %.0f GB/s\n", name, R, t * 1e3, 16.0 * H * W / t / 1e6);
    };
    for (int R : {512, 2048}) {
        split("U8 P6 C2 S8", run_split<8, 6, 2, 8>, R);
        split("U8 P3 C1 S8", run_split<8, 3, 1, 8>, R);
        split("U16 P6 C2 S8", run_split<16, 6, 2, 8>, R);
        split("U8 P4 C4 S8", run_split<8, 4, 4, 8>, R);
        split("U8 P12 C4 S4", run_split<8, 12, 4, 4>, R);
    }
    if (argc > 3) return 0;
    // cache policy of the loads / stores (aux bits: 1 sc0, 2 nt, 16 sc1) on long copies
    std::printf("policy sweep: layout 0, R=2048, copy\n");
    auto pol = [&](const char* name, float (*f)(const Args&, int, int), int U, int lds) {
        Args a0{a, b, H, W, 2048, ns, ns * ((H + 2047) / 2048), 0, 0, W};
        const float t = f(a0, lds, 6);
        std::printf("policy %s U=%d lds_kb=%d : %.1f us %.0f GB/s\n", name, U, lds, t * 1e3,
                    16.0 * H * W / t / 1e6);
    };
#define POL(L, S)                                                   \
    pol("load" #L "_store" #S, run<8, L, S>, 8, 0);                 \
    pol("load" #L "_store" #S, run<32, L, S>, 32, 160);
    POL(0, 2) POL(0, 0) POL(0, 1) POL(0, 3) POL(0, 16) POL(0, 17) POL(0, 18) POL(0, 19)
    POL(2, 2) POL(16, 2) POL(1, 2) POL(2, 0) POL(18, 18)
    return 0;
}
