// mm_kernels_k.hip -- K fused Exponencial steps per HBM pass (temporal blocking), gfx950.
//
// The headline path (one attribute, one whole-grid Exponencial flow; SURVEY.md 8a, the
// generalisation of src/Model.hpp:176-235 + src/Exponencial.hpp:18-20). A pass reads
// every cell once, advances it K steps in registers and writes it once, so HBM moves
// 16/K B per cell-update instead of 16 B.
//
// Overlapped strips. A wave owns a strip of 128 LOADED columns (lane l: columns
// c0+2l, c0+2l+1 as one 16-B buffer load) but outputs only the inner 128-4L columns,
// L = ceil(K/2) lanes on each side. Every level of the K-step pipeline computes all 64
// lanes with exactly the same instructions; the y+-1 neighbours come from the adjacent
// lanes through DPP wave_shr:1 / wave_shl:1, and the lanes at the wave's edges receive
// garbage that moves one column inward per level -- after K levels it has reached
// columns < K from each edge, i.e. the L halo lanes, whose results are discarded. There
// are no edge-column loads and no per-lane special cases; the price is 4L/128 extra
// (L2-resident) column reads.
//
// Rows. The wave slides down its strip: input rows rA-K .. rB+K-1 arrive one by one
// (U rows prefetched), and level j (1..K) keeps a three-row window (shares of the row
// above, shares and u - out of the current row) in registers. Level j emits row
// rA-K+i-j at input i and feeds it to level j+1; level K's rows rA..rB-1 are stored.
// Levels j < K compute K-j extra rows above and below the block (recomputed by the
// neighbouring row block as well).
//
// Every level uses exactly the single-step arithmetic of oracle/mm_oracle.h, so K fused
// steps are bit-identical to K single steps (built with -ffp-contract=off).
#include "mm_internal.hpp"

#ifndef MM_SCHED_BARRIER
#define MM_SCHED_BARRIER 1
#endif

namespace mm {

namespace {

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr unsigned kOOBk = 0x80000000u;  // voffset past any num_records: load 0 / drop store

__device__ __forceinline__ double dpp_lower(double src) {
    // lane i <- lane i-1 (wave_shr:1); lane 0 keeps its own value (a halo lane)
    const long long s = __double_as_longlong(src);
    const int lo = __builtin_amdgcn_update_dpp((int)s, (int)s, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(s >> 32), (int)(s >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double dpp_upper(double src) {
    // lane i <- lane i+1 (wave_shl:1); lane 63 keeps its own value (a halo lane)
    const long long s = __double_as_longlong(src);
    const int lo = __builtin_amdgcn_update_dpp((int)s, (int)s, 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(s >> 32), (int)(s >> 32), 0x130, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1 + (i > 0) + (i < n-1) inside [0, n), 0 outside: cnt = span(x)*span(y) - 1
__device__ __forceinline__ int span3k(long long n, long long i) {
    return (i >= 0 && i < n) ? 1 + (i > 0) + (i < n - 1) : 0;
}

__device__ __forceinline__ double share_k(double out, int cnt) {
    return cnt == 8 ? out * 0.125 : (cnt > 0 ? out / (double)cnt : 0.0);
}

// Descriptor of `rows` consecutive rows starting at `first` (pointer already offset):
// row k of the range is at byte offset k*pitch*8 (added to the lane's voffset), offsets
// past the range -- later rows, or lanes whose voffset is kOOBk -- load 0 / drop stores.
// One descriptor per wave instead of one per row keeps the unrolled rows from holding
// dozens of scalar descriptors (which spilled SGPRs into VGPR lanes).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const double* first, int rows,
                                                            long long pitch) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(first), 0,
                                             rows > 0 ? (int)(rows * pitch * 8) : 0, 0x00020000);
}

// One level's three-row window: shares of the row above (p), shares and u - out of the
// current row (c).
struct Win {
    double sp0, sp1, sc0, sc1, dc0, dc1;
};

// out = rate*u, s = out/cnt, d = u - out for this lane's two columns of row gx
// (src/Exponencial.hpp:18-20, src/Model.hpp:199); cells outside the grid emit nothing.
template <bool FAST>
__device__ __forceinline__ void proc_k(long long H, long long gx, bool fast_cols, double rate,
                                       int sy0, int sy1, double u0, double u1, double& s0,
                                       double& s1, double& d0, double& d1) {
    const int sx = FAST ? 3 : span3k(H, gx);
    if (FAST || (sx == 3 && fast_cols)) {  // interior row, interior strip: cnt == 8 everywhere
        const double o0 = rate * u0, o1 = rate * u1;
        s0 = o0 * 0.125;
        s1 = o1 * 0.125;
        d0 = u0 - o0;
        d1 = u1 - o1;
        return;
    }
    if (sx == 0) {  // row outside the grid
        s0 = s1 = 0.0;
        d0 = u0;
        d1 = u1;
        return;
    }
    const int c0 = sy0 ? sx * sy0 - 1 : 0;
    const int c1 = sy1 ? sx * sy1 - 1 : 0;
    const double o0 = c0 > 0 ? rate * u0 : 0.0;
    const double o1 = c1 > 0 ? rate * u1 : 0.0;
    s0 = share_k(o0, c0);
    s1 = share_k(o1, c1);
    d0 = u0 - o0;
    d1 = u1 - o1;
}

// v' = (u - out) + nb, nb = (c3(y-1) + c3(y+1)) + p with p = s(x-1) + s(x+1) and
// c3 = p + s(x) (src/Model.hpp:206-211,234; the order fixed by oracle/mm_oracle.h).
__device__ __forceinline__ void emit_k(const Win& w, double sn0, double sn1, double& w0,
                                       double& w1) {
    const double p0 = w.sp0 + sn0, p1 = w.sp1 + sn1;
    const double c0 = p0 + w.sc0, c1 = p1 + w.sc1;
    const double left = dpp_lower(c1);   // c3 at column y0-1 (lane-1's second column)
    const double right = dpp_upper(c0);  // c3 at column y0+2 (lane+1's first column)
    w0 = w.dc0 + ((left + c1) + p0);
    w1 = w.dc1 + ((c0 + right) + p1);
}

__device__ __forceinline__ double wave_sum_k(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
    return v;
}

// The row pipeline of one wave (see the file comment). FAST: every cell this wave
// touches is interior, so the neighbour-count cases compile away.
template <int K, int TH, int U, bool RED, int NT, bool FAST>
__device__ __forceinline__ void passk_body(const PassArgs& A, long long wid, int lane, int rA,
                                           int rB, unsigned voff, unsigned soff, int sy0, int sy1,
                                           bool fast_cols, bool own0, bool own1) {
    constexpr int NI = TH + 2 * K;  // input rows per wave
    const long long H = A.H;
    const double rate = A.drate[0];
    const long long gx0 = A.x_init;
    double acc[K];
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j] = 0.0;

    // input rows rA-K .. rB+K-1 (input i at offset i*rowb), output rows rA .. rB-1
    const unsigned rowb = (unsigned)(A.pitch * 8);
    const __amdgpu_buffer_rsrc_t rin =
        rows_rsrc(A.in[0] + (long long)(rA - K) * A.pitch, rB - rA + 2 * K, A.pitch);
    const __amdgpu_buffer_rsrc_t rout =
        rows_rsrc(A.out[0] + (long long)rA * A.pitch, rB - rA, A.pitch);
    dv2 raw[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
        raw[k] = __builtin_bit_cast(
            dv2, __builtin_amdgcn_raw_buffer_load_b128(rin, voff + k * rowb, 0, 0));
    Win win[K];

#pragma unroll
    for (int i = 0; i < NI; ++i) {
        double u0 = raw[i % U].x, u1 = raw[i % U].y;
        if (i + U < NI)
            raw[i % U] = __builtin_bit_cast(
                dv2, __builtin_amdgcn_raw_buffer_load_b128(rin, voff + (i + U) * rowb, 0, 0));
#pragma unroll
        for (int j = 1; j <= K; ++j) {
            const int m = i - 2 * (j - 1);  // rows level j has received before this one
            if (m < 0) break;               // compile-time under full unrolling
            const int r_in = rA - K + i - (j - 1);  // row of level j's input
            double sn0, sn1, dn0, dn1;
            proc_k<FAST>(H, gx0 + r_in, fast_cols, rate, sy0, sy1, u0, u1, sn0, sn1, dn0, dn1);
            Win& wj = win[j - 1];
            if (m == 0) {
                wj.sp0 = sn0;
                wj.sp1 = sn1;
                break;
            }
            if (m == 1) {
                wj.sc0 = sn0;
                wj.sc1 = sn1;
                wj.dc0 = dn0;
                wj.dc1 = dn1;
                break;
            }
            double w0, w1;
            emit_k(wj, sn0, sn1, w0, w1);
            wj.sp0 = wj.sc0;
            wj.sp1 = wj.sc1;
            wj.sc0 = sn0;
            wj.sc1 = sn1;
            wj.dc0 = dn0;
            wj.dc1 = dn1;
            const int r_out = r_in - 1;  // level j's output row
            // r_out - rA = i - K - j: rows of the block are known at compile time, only
            // the end of a short last block (rB) is not
            if (RED && i - K - j >= 0 && i - K - j < TH) {
                const bool own = r_out < rB;  // wave-uniform
                acc[j - 1] = acc[j - 1] + ((own && own0) ? w0 : 0.0);
                acc[j - 1] = acc[j - 1] + ((own && own1) ? w1 : 0.0);
                // materialise the sum here: otherwise LLVM sinks the whole chain of adds
                // to the kernel exit and keeps every row's values live until then
                asm volatile("" : "+v"(acc[j - 1]));
            }
            if (j == K) {
                dv2 v;
                v.x = w0;
                v.y = w1;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v),
                                                       rout, soff + (i - 2 * K) * rowb, 0,
                                                       (NT & 1) ? 2 : 0);
            }
            u0 = w0;
            u1 = w1;
        }
#if MM_SCHED_BARRIER
        // keep the row order: the scheduler would otherwise hoist and sink whole rows
        // (values stay live across the unrolled loop and the VGPR count explodes)
        __builtin_amdgcn_sched_barrier(0);
#endif
    }

    if (RED) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double t = wave_sum_k(acc[j]);
            if (lane == 0) A.partials[(A.partial_base + wid) * K + j] = t;
        }
    }
}


// The same pipeline with the levels SKEWED by one input row: at iteration i level j
// consumes what level j-1 emitted at iteration i-1 (held in pend[j-2]), so the K levels
// of one iteration are independent and interleave, instead of forming one K-deep
// dependent chain per input row. Level j's m-th input is row rA-K+(j-1)+m and arrives
// at iteration m + 3(j-1); level K's last row leaves at iteration TH + 3K - 2.
template <int K, int TH, int U, bool RED, int NT, bool FAST>
__device__ __forceinline__ void passk_body_skew(const PassArgs& A, long long wid, int lane,
                                                int rA, int rB, unsigned voff, unsigned soff,
                                                int sy0, int sy1, bool fast_cols, bool own0,
                                                bool own1) {
    constexpr int NI = TH + 2 * K;       // input rows per wave
    constexpr int NIT = TH + 3 * K - 1;  // iterations
    const long long H = A.H;
    const double rate = A.drate[0];
    const long long gx0 = A.x_init;
    double acc[K];
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j] = 0.0;

    const unsigned rowb = (unsigned)(A.pitch * 8);
    const __amdgpu_buffer_rsrc_t rin =
        rows_rsrc(A.in[0] + (long long)(rA - K) * A.pitch, rB - rA + 2 * K, A.pitch);
    const __amdgpu_buffer_rsrc_t rout =
        rows_rsrc(A.out[0] + (long long)rA * A.pitch, rB - rA, A.pitch);
    dv2 raw[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
        raw[k] = __builtin_bit_cast(
            dv2, __builtin_amdgcn_raw_buffer_load_b128(rin, voff + k * rowb, 0, 0));
    Win win[K];
    double pend0[K], pend1[K];  // level j's output of the previous iteration: pend[j-1]

#pragma unroll
    for (int i = 0; i < NIT; ++i) {
#pragma unroll
        for (int j = K; j >= 1; --j) {  // descending: pend[j-2] is read before it is refilled
            const int m = i - 3 * (j - 1);
            if (m < 0 || m >= NI - 2 * (j - 1)) continue;  // compile-time
            double u0, u1;
            if (j == 1) {
                u0 = raw[i % U].x;
                u1 = raw[i % U].y;
                if (i + U < NI)
                    raw[i % U] = __builtin_bit_cast(
                        dv2, __builtin_amdgcn_raw_buffer_load_b128(rin, voff + (i + U) * rowb, 0, 0));
            } else {
                u0 = pend0[j - 2];
                u1 = pend1[j - 2];
            }
            const int r_in = rA - K + (j - 1) + m;
            double sn0, sn1, dn0, dn1;
            proc_k<FAST>(H, gx0 + r_in, fast_cols, rate, sy0, sy1, u0, u1, sn0, sn1, dn0, dn1);
            Win& wj = win[j - 1];
            if (m == 0) {
                wj.sp0 = sn0;
                wj.sp1 = sn1;
                continue;
            }
            if (m == 1) {
                wj.sc0 = sn0;
                wj.sc1 = sn1;
                wj.dc0 = dn0;
                wj.dc1 = dn1;
                continue;
            }
            double w0, w1;
            emit_k(wj, sn0, sn1, w0, w1);
            wj.sp0 = wj.sc0;
            wj.sp1 = wj.sc1;
            wj.sc0 = sn0;
            wj.sc1 = sn1;
            wj.dc0 = dn0;
            wj.dc1 = dn1;
            const int orow = m + j - K - 2;  // output row - rA (compile-time)
            if (RED && orow >= 0 && orow < TH) {
                const bool own = rA + orow < rB;  // wave-uniform
                acc[j - 1] = acc[j - 1] + ((own && own0) ? w0 : 0.0);
                acc[j - 1] = acc[j - 1] + ((own && own1) ? w1 : 0.0);
                asm volatile("" : "+v"(acc[j - 1]));
            }
            if (j == K) {
                dv2 v;
                v.x = w0;
                v.y = w1;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rout,
                                                       soff + orow * rowb, 0, (NT & 1) ? 2 : 0);
            } else {
                pend0[j - 1] = w0;
                pend1[j - 1] = w1;
            }
        }
#if MM_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
    }

    if (RED) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double t = wave_sum_k(acc[j]);
            if (lane == 0) A.partials[(A.partial_base + wid) * K + j] = t;
        }
    }
}

// K steps per pass; TH output rows per wave; U input rows prefetched; RED: per-level
// sums of the owned cells into partials[(partial_base + wave) * K + level]; NT & 1:
// non-temporal stores.
template <int K, int TH, int U, bool RED, int NT, bool SKEW>
__global__ __launch_bounds__(kBlock) void mm_passk_kernel(const PassArgs A) {
    constexpr int L = (K + 1) / 2;               // halo lanes per side
    constexpr int OC = kStripCols - 4 * L;       // output columns per strip
    constexpr int NI = TH + 2 * K;               // input rows per wave
    static_assert(U <= NI, "prefetch deeper than the input rows");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-aware block order: hardware block b runs on XCD b % 8; logical block
    // (b % 8) * per + b / 8 gives every XCD a contiguous run of tiles, so vertically
    // adjacent row blocks (which share K halo rows) meet in the same L2.
    long long blk = blockIdx.x;
    if (A.xcd_remap) {
        const long long per = gridDim.x / 8;
        blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const long long wid = blk * kWavesPerBlock + wave;
    if (wid >= A.waves_total) return;

    int rlo, rhi;
    long long w = wid;
    if (w < A.waves_a) {
        rlo = A.ra0;
        rhi = A.ra1;
    } else {
        w -= A.waves_a;
        rlo = A.rb0;
        rhi = A.rb1;
    }
    const int strip = (int)(w % A.nstrips);
    const int rb = (int)(w / A.nstrips);
    const int rA = rlo + rb * TH;
    const int rB = min(rA + TH, rhi);  // output rows [rA, rB)

    const long long W = A.W, H = A.H;
    const long long c0 = (long long)strip * OC - 2 * L;  // first loaded column (even)
    const long long y0 = c0 + 2 * lane;
    const bool in_row = y0 >= 0 && y0 < A.pitch;  // y0 even, pitch a multiple of 128
    const unsigned voff = in_row ? (unsigned)(y0 * 8) : kOOBk;
    const bool store_lane = lane >= L && lane < 64 - L && y0 < W;
    // columns past W inside the pitch are padding: writing them is harmless
    const unsigned soff = store_lane ? (unsigned)(y0 * 8) : kOOBk;
    const int sy0 = span3k(W, y0), sy1 = span3k(W, y0 + 1);
    const bool fast_cols = c0 >= 1 && c0 + kStripCols <= W - 1;  // loaded cols in [1, W-2]
    const bool own0 = store_lane, own1 = store_lane && y0 + 1 < W;
    const long long gx0 = A.x_init;

    // a wave whose input rows and loaded columns are all interior (cnt == 8 everywhere)
    // runs the branch-free body; edge waves run the general one
    const bool fast_wave = fast_cols && gx0 + rA - K >= 1 && gx0 + rB + K - 1 <= H - 2;
    if (SKEW) {
        if (fast_wave)
            passk_body_skew<K, TH, U, RED, NT, true>(A, wid, lane, rA, rB, voff, soff, sy0, sy1,
                                                     fast_cols, own0, own1);
        else
            passk_body_skew<K, TH, U, RED, NT, false>(A, wid, lane, rA, rB, voff, soff, sy0,
                                                      sy1, fast_cols, own0, own1);
    } else {
        if (fast_wave)
            passk_body<K, TH, U, RED, NT, true>(A, wid, lane, rA, rB, voff, soff, sy0, sy1,
                                                fast_cols, own0, own1);
        else
            passk_body<K, TH, U, RED, NT, false>(A, wid, lane, rA, rB, voff, soff, sy0, sy1,
                                                 fast_cols, own0, own1);
    }
}

template <int K, int TH, int U, int NT, bool SKEW>
hipError_t launch_k3(bool red, const PassArgs& a, hipStream_t s) {
    long long blocks = (a.waves_total + kWavesPerBlock - 1) / kWavesPerBlock;
    if (a.xcd_remap) blocks = (blocks + 7) / 8 * 8;
    const dim3 g((unsigned)blocks), b(kBlock);
    if (red)
        hipLaunchKernelGGL((mm_passk_kernel<K, TH, U, true, NT, SKEW>), g, b, 0, s, a);
    else
        hipLaunchKernelGGL((mm_passk_kernel<K, TH, U, false, NT, SKEW>), g, b, 0, s, a);
    return hipGetLastError();
}

// variant bit 0: non-temporal stores; bit 2: unskewed level schedule (one dependent
// chain per input row)
template <int K, int TH, int U>
hipError_t launch_k3v(bool red, const PassArgs& a, hipStream_t s, int v) {
    switch (v & 5) {
        case 0: return launch_k3<K, TH, U, 0, true>(red, a, s);
        case 1: return launch_k3<K, TH, U, 1, true>(red, a, s);
        case 4: return launch_k3<K, TH, U, 0, false>(red, a, s);
        default: return launch_k3<K, TH, U, 1, false>(red, a, s);
    }
}

template <int K>
hipError_t launch_k2(bool red, const PassArgs& a, hipStream_t s, int v) {
    switch (a.th) {
        case 4: return launch_k3<K, 4, 4, 0, true>(red, a, s);  // border rows of a split pass
        case 16: return launch_k3v<K, 16, 8>(red, a, s, v);
        case 32: return launch_k3v<K, 32, 8>(red, a, s, v);
        default: return hipErrorInvalidValue;
    }
}

// Fixed-order sums of the levels in `mask` of partials[n][k] -> one history entry each
// (one attribute), slots from the device counter (graph-replayable).
__global__ __launch_bounds__(256) void mm_finalize_levels_kernel(const double* partials,
                                                                 long long n, int k, int mask,
                                                                 double* hist,
                                                                 unsigned long long* hist_n,
                                                                 long long cap) {
    __shared__ double red[256];
    __shared__ unsigned long long slot;
    if (threadIdx.x == 0) slot = *hist_n;
    __syncthreads();
    unsigned long long e = 0;
    for (int j = 0; j < k; ++j) {
        if (!(mask & (1 << j))) continue;
        double s = 0.0;
        for (long long i = threadIdx.x; i < n; i += 256) s = s + partials[i * k + j];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int m = 128; m >= 1; m >>= 1) {
            if ((int)threadIdx.x < m) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + m];
            __syncthreads();
        }
        const long long idx = (long long)(slot + e);
        if (threadIdx.x == 0 && idx < cap) hist[idx] = red[0];
        ++e;
        __syncthreads();
    }
    if (threadIdx.x == 0) *hist_n = slot + e;
}

}  // namespace

hipError_t launch_finalize_levels(const double* partials, long long n, int k, int mask,
                                  double* hist, unsigned long long* hist_n, long long cap,
                                  hipStream_t s) {
    hipLaunchKernelGGL(mm_finalize_levels_kernel, dim3(1), dim3(256), 0, s, partials, n, k, mask,
                       hist, hist_n, cap);
    return hipGetLastError();
}

int passk_out_cols(int k) { return kStripCols - 4 * ((k + 1) / 2); }

hipError_t launch_passk(int k, bool red, const PassArgs& a, hipStream_t s, int variant) {
    if (a.waves_total <= 0) return hipSuccess;
    switch (k) {
        case 1: return launch_k2<1>(red, a, s, variant);
        case 2: return launch_k2<2>(red, a, s, variant);
        case 3: return launch_k2<3>(red, a, s, variant);
        case 4: return launch_k2<4>(red, a, s, variant);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace mm
