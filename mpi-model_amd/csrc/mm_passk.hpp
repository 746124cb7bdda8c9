// mm_passk.hpp -- K fused flow-program steps per HBM pass (temporal blocking), gfx950.
//
// The hot path: the generalisation of src/Model.hpp:176-235 +
// src/Exponencial.hpp:18-20 to every cell and every step -- one whole-grid Exponencial
// flow per attribute, with optional same-cell transfer chains before / after it (config
// C5). A pass reads every cell once, advances it K steps in registers and writes it once,
// so HBM moves 16/K B per cell-update and attribute instead of 16 B.
//
// Overlapped strips. A wave owns a strip of 128 LOADED columns (lane l: columns
// c0+2l, c0+2l+1 as one 16-B buffer load per attribute) but outputs only the inner
// 128-4L columns, L = ceil(K/2) lanes on each side. Every level of the K-step pipeline
// computes all 64 lanes with exactly the same instructions; the y+-1 neighbours come from
// the adjacent lanes through DPP wave_shr:1 / wave_shl:1, and the lanes at the wave's
// edges receive garbage that moves one column inward per level -- after K levels it has
// reached columns < K from each edge, i.e. the L halo lanes, whose results are
// discarded. No edge-column loads, no per-lane special cases; the price is 4L/128 extra
// (L2-resident) column reads.
//
// Rows. The wave slides down its strip, input rows rA-K .. rB+K-1 one by one (U rows
// prefetched). Level j (1..K) keeps a three-row window per attribute in registers
// (shares of the row above; shares and u - out of the current row) and emits one row
// per input row. The levels are SKEWED: at iteration i level j consumes the row level
// j-1 emitted at iteration i-1, so the K levels of one iteration are independent
// instruction streams that interleave (instead of one K-deep dependent chain per input
// row). Level j's m-th input is row rA-K+(j-1)+m, at iteration m + 3(j-1); it emits row
// rA-K-2j+1+i. Level K's rows rA..rB-1 are stored; lower levels compute K-j rows beyond
// the segment on each side (recomputed by the neighbouring segment).
//
// Two schedules of that pipeline:
//   * SEGMENT (interior and whole-slab passes): a wave runs a tall segment of rows (row
//     counts at run time, sized so the chip's wave slots hold every wave at once). A
//     compile-time prologue fills the levels, then a runtime loop streams the segment with
//     all K levels active: the row overhead of temporal blocking is K(K-1) level-rows per
//     segment. The two edge strips (their first / last grid column has 5 or 3
//     neighbours: true divisions, the slow body) get shorter segments and are dispatched
//     first, so the waves of a launch finish together;
//   * BLOCK: 4 rows, fully unrolled -- the border rows of a halo-split pass.
//
// Every level uses exactly the single-step arithmetic of oracle/mm_oracle.h (transfers
// in declared order, then the weights w = u * 8/cnt, the row-paired column triples, the
// column-paired box sum S and v' = fma(fma(u, -(8 + 8/cnt), S), r/8, u)), so K fused steps
// are bit-identical to K single steps (built with -ffp-contract=off; the fma explicit).
//
// This header holds the kernel templates; mm_passk_k<K>.hip instantiate them (one
// translation unit per K so the builds run in parallel) and mm_kernels_k.hip dispatches.
#pragma once

#include <algorithm>

#include "mm_internal.hpp"

namespace mm {

// per-K entry points (mm_passk_k1.hip .. mm_passk_k8.hip); na outside the TU's set is
// hipErrorInvalidValue / 0
#define MM_PASSK_DECL(K)                                                                  \
    hipError_t passk_launch_k##K(int na, bool red, const PassArgs& a, hipStream_t s, int v); \
    int passk_waves_k##K(int na, bool red, int nt);
MM_PASSK_DECL(1)
MM_PASSK_DECL(2)
MM_PASSK_DECL(3)
MM_PASSK_DECL(4)
MM_PASSK_DECL(5)
MM_PASSK_DECL(6)
MM_PASSK_DECL(7)
MM_PASSK_DECL(8)
MM_PASSK_DECL(9)
MM_PASSK_DECL(10)
#undef MM_PASSK_DECL

namespace {


typedef double dv2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr unsigned kOOBk = 0x80000000u;  // voffset past any num_records: load 0 / drop store
constexpr int kSeg = 0;                  // MODE value of the segment schedule

#ifndef MM_PASSK_MIN_WAVES
#define MM_PASSK_MIN_WAVES 1  // __launch_bounds__ minimum waves per SIMD (caps VGPRs)
#endif

// input rows prefetched per wave: 8 KiB in flight for one attribute, ~8 KiB for more
#ifndef MM_LEVEL_BARRIER
#define MM_LEVEL_BARRIER 0  // scheduling barrier after every this many levels (0: none)
#endif
#ifndef MM_ROW_BARRIER
#define MM_ROW_BARRIER 1  // steady loop: scheduling barrier after every this many rows (0: none)
#endif
#ifndef MM_SEG_U1
#define MM_SEG_U1 8  // rows prefetched per wave, one attribute
#endif
#ifndef MM_SEG_UN
#define MM_SEG_UN 2  // rows prefetched per wave, three or four attributes
#endif
template <int NA>
constexpr int seg_prefetch() {
    return NA == 1 ? MM_SEG_U1 : (NA == 2 ? 4 : MM_SEG_UN);
}

// mov_dpp has no tied "old" operand, so the result can land in a fresh register without
// first copying the source; lanes without a source lane read 0 (bound_ctrl) -- only the
// halo lanes at the wave's edges, whose results are discarded.
__device__ __forceinline__ double dpp_lower(double src) {
    // lane i <- lane i-1 (wave_shr:1)
    const long long s = __double_as_longlong(src);
    const int lo = __builtin_amdgcn_mov_dpp((int)s, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(s >> 32), 0x138, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double dpp_upper(double src) {
    // lane i <- lane i+1 (wave_shl:1)
    const long long s = __double_as_longlong(src);
    const int lo = __builtin_amdgcn_mov_dpp((int)s, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(s >> 32), 0x130, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The same two shifts through the LDS crossbar (ds_bpermute_b32: no LDS memory, the DS
// pipe instead of the VALU). A DPP shift of a double is two VALU moves, 4 of the 18 VALU
// instructions of a level-row of two columns; ds_bpermute moves them to the otherwise idle
// DS pipe. `addr` = 4 * source lane (wraps around the wave: the halo lanes get garbage
// instead of 0, and their results are discarded either way).
#ifndef MM_SHIFT_LDS
#define MM_SHIFT_LDS 0
#endif
__device__ __forceinline__ double lds_shift(double src, int addr) {
    const long long s = __double_as_longlong(src);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)s);
    const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(s >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// A prefetched row is copied out of its ring slot where it is consumed (U rows after its
// load was issued). Without the copy the slot's registers become the level's d = u - out
// (v_fmac works in place), every reload lands in fresh registers, and the loop's back edge
// copies them into the slots right after the last load -- a vmcnt(0) wait that exposes the
// full memory latency once per U rows. The early clobber keeps the copy out of the slot.
#ifndef MM_LOAD_COPY
#define MM_LOAD_COPY 1
#endif
__device__ __forceinline__ double vcopy(double x) {
    double y;
    asm volatile("v_mov_b64 %0, %1" : "=&v"(y) : "v"(x));
    return y;
}

// 1 + (i > 0) + (i < n-1) inside [0, n), 0 outside: cnt = span(x)*span(y) - 1
__device__ __forceinline__ int span3k(long long n, long long i) {
    return (i >= 0 && i < n) ? 1 + (i > 0) + (i < n - 1) : 0;
}

// A neighbour's weight factor 8/cnt (oracle/mm_oracle.c c8_of: w = u * 8/cnt, 1 for an
// interior cell, 0 outside the grid): the correctly rounded quotients as constants.
__device__ __forceinline__ double c8k(int cnt) {
    return cnt == 8 ? 1.0
                    : (cnt == 5 ? 8.0 / 5.0
                                : (cnt == 3 ? 8.0 / 3.0
                                            : (cnt == 2 ? 4.0 : (cnt == 1 ? 8.0 : 0.0))));
}

// The own-weight coefficient -(8 + 8/cnt) of the box sum (oracle/mm_oracle.c m_of): -9 for
// an interior cell, 0 for a cell without neighbours (it keeps its value) or outside the grid.
constexpr double kM8 = -9.0;
constexpr double kM5 = -(8.0 + 8.0 / 5.0);
__device__ __forceinline__ double m8k(int cnt) {
    return cnt == 8 ? kM8
                    : (cnt == 5 ? kM5
                                : (cnt == 3 ? -(8.0 + 8.0 / 3.0)
                                            : (cnt == 2 ? -12.0 : (cnt == 1 ? -16.0 : 0.0))));
}

// Descriptor of `rows` consecutive rows starting at `first` (pointer already offset):
// row k of the range is at byte offset k*pitch*8 (added to the lane's voffset), offsets
// past the range -- later rows, or lanes whose voffset is kOOBk -- load 0 / drop stores.
// One descriptor per wave and attribute instead of one per row keeps the unrolled rows
// from holding dozens of scalar descriptors (which spilled SGPRs into VGPR lanes). The
// engine keeps every offset below 2^31 (passk_max_rows).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const double* first, int rows,
                                                            long long pitch) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(first), 0,
                                             rows > 0 ? (int)(rows * pitch * 8) : 0, 0x00020000);
}

#ifndef MM_LOAD_NT
#define MM_LOAD_NT 0  // 1: input rows loaded non-temporal (aux nt)
#endif
__device__ __forceinline__ dv2 load_row(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, MM_LOAD_NT ? 2 : 0));
}

template <int NT>
__device__ __forceinline__ void store_row(__amdgpu_buffer_rsrc_t r, unsigned off, double w0,
                                          double w1) {
    dv2 v;
    v.x = w0;
    v.y = w1;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0,
                                           (NT & 1) ? 2 : 0);
}

// One level's three-row window of one attribute: the weights of the row above (wa; before
// an odd row is emitted, the pair sum of the row above and the current row) and of the
// current row (wm), the current row's values (um).
struct Win {
    double wa0, wa1, wm0, wm1, um0, um1;
};

// What every level of one wave needs besides its windows.
struct Lane {
    long long H, gx0;  // grid rows, global row of local row 0
    int sy0, sy1;      // column spans of this lane's two columns
    bool fast_cols;    // all loaded columns interior
    bool own0, own1;   // this lane's columns are output cells of this wave
    int from_lower, from_upper;  // ds_bpermute byte addresses of lanes i-1, i+1 (MM_SHIFT_LDS)
};

// Transfers of a chain, in declared order, on one cell's attribute values: out = r*u_a;
// u_a -= out; u_b += out (b < 0: the outflow leaves the system). a and b are wave-uniform
// kernel arguments. The values sit in one 8-element register vector for the chain -- at
// that width LLVM indexes it with s_set_gpr_idx (two v_mov per access) instead of a
// select over every attribute per operand (36 v_cndmask per transfer and column) -- and a
// pad slot takes the outflows that leave the system.
typedef double dv8 __attribute__((ext_vector_type(8)));
#ifndef MM_CHAIN_CAP
#define MM_CHAIN_CAP kMaxChain  // transfers a chain may hold (tuning: fewer unrolled slots)
#endif
template <int NA>
__device__ __forceinline__ void chain_k(double (&u)[NA], int n, const signed char* ta,
                                        const signed char* tb, const double* tr) {
    static_assert(NA < 8, "one pad slot");
    dv8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = k < NA ? u[k] : 0.0;
#pragma unroll
    for (int t = 0; t < MM_CHAIN_CAP; ++t) {
        if (t >= n) break;  // wave-uniform
        const int a = ta[t];
        const int b = tb[t] >= 0 ? tb[t] : 7;
        const double out = tr[t] * v[a];
        v[a] = v[a] - out;
        v[b] = v[b] + out;
    }
#pragma unroll
    for (int k = 0; k < NA; ++k) u[k] = v[k];
}

// Pre-chain, then per diffusing attribute the weights w = u * 8/cnt of this lane's two
// columns of row gx (oracle/mm_oracle.c w_row: each neighbour's share out/cnt = (r/8) * w,
// src/Exponencial.hpp:18-20, src/Model.hpp:199); cells outside the grid weigh 0;
// attributes that do not diffuse pass through (w = 0).
template <int NA, bool FAST, bool CHAIN>
__device__ __forceinline__ void proc_n(const PassArgs& A, const Lane& c, long long gx,
                                       double (&u0)[NA], double (&u1)[NA], double (&w0)[NA],
                                       double (&w1)[NA]) {
    if (CHAIN && A.npre) {
        chain_k<NA>(u0, A.npre, A.pre_a, A.pre_b, A.pre_r);
        chain_k<NA>(u1, A.npre, A.pre_a, A.pre_b, A.pre_r);
    }
    const int sx = FAST ? 3 : span3k(c.H, gx);
    const bool inner = FAST || (sx == 3 && c.fast_cols);  // wave-uniform
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        if (NA > 1 && !((A.diffuse_mask >> a) & 1)) {
            w0[a] = w1[a] = 0.0;
        } else if (inner) {  // interior row, interior strip: cnt == 8, w = u
            w0[a] = u0[a];
            w1[a] = u1[a];
        } else {  // a column outside the grid (span 0: its pitch padding) weighs 0 by select,
                  // so no value it holds reaches a cell
            w0[a] = c.sy0 == 0 ? 0.0 : u0[a] * c8k(sx * c.sy0 - 1);
            w1[a] = c.sy1 == 0 ? 0.0 : u1[a] * c8k(sx * c.sy1 - 1);
        }
    }
}

// Level input row m = 0 or 1 (global row gx): fill the windows. e1: parity of the level's
// first emitted row (row gx at m = 1): odd, the window holds the pair sum of rows m = 0, 1.
template <int NA, bool FAST, bool CHAIN>
__device__ __forceinline__ void level_fill(const PassArgs& A, const Lane& c, long long gx, int m,
                                           int e1, Win (&w)[NA], double (&u0)[NA],
                                           double (&u1)[NA]) {
    double w0[NA], w1[NA];
    proc_n<NA, FAST, CHAIN>(A, c, gx, u0, u1, w0, w1);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        if (m == 0) {
            w[a].wa0 = w0[a];
            w[a].wa1 = w1[a];
        } else {
            if (e1) {
                w[a].wa0 = w[a].wa0 + w0[a];
                w[a].wa1 = w[a].wa1 + w1[a];
            }
            w[a].wm0 = w0[a];
            w[a].wm1 = w1[a];
            w[a].um0 = u0[a];
            w[a].um1 = u1[a];
        }
    }
}

// Level input row m >= 2 (global row gx): emit the windows' current row (then the
// post-chain) and slide the windows. e: parity of the emitted row gx - 1 (a constant where
// the iteration is unrolled). Even: the pair sum of this row and the next, p = wm + wn,
// gives the column triple wa + p and stays in wa for the odd row after it, whose triple is
// p + wn; the box sum of the lane's even / odd column: cw(y-1) + (cw(y) + cw(y+1)) /
// (cw(y-1) + cw(y)) + cw(y+1); v' = fma(fma(u, -(8 + 8/cnt), S), r/8, u)
// (src/Model.hpp:206-211,234; the order fixed by oracle/mm_oracle.h); a cell without
// neighbours (a 1 x 1 grid) keeps its value.
template <int NA, bool FAST, bool CHAIN>
__device__ __forceinline__ void level_emit(const PassArgs& A, const Lane& c, long long gx, int e,
                                           Win (&w)[NA], double (&u0)[NA], double (&u1)[NA],
                                           double (&o0)[NA], double (&o1)[NA]) {
    double wn0[NA], wn1[NA];
    proc_n<NA, FAST, CHAIN>(A, c, gx, u0, u1, wn0, wn1);
    const int sxm = FAST ? 3 : span3k(c.H, gx - 1);  // the emitted row
    const double m0 = FAST ? kM8 : m8k(sxm * c.sy0 - 1);
    const double m1 = FAST ? kM8 : m8k(sxm * c.sy1 - 1);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        double na0, na1;  // the window's next wa
        if (NA > 1 && !((A.diffuse_mask >> a) & 1)) {
            o0[a] = w[a].um0;
            o1[a] = w[a].um1;
            na0 = w[a].wm0;
            na1 = w[a].wm1;
        } else {
            double c0, c1;
            if (e == 0) {
                na0 = w[a].wm0 + wn0[a];
                na1 = w[a].wm1 + wn1[a];
                c0 = w[a].wa0 + na0;
                c1 = w[a].wa1 + na1;
            } else {
                c0 = w[a].wa0 + wn0[a];
                c1 = w[a].wa1 + wn1[a];
                na0 = w[a].wm0;
                na1 = w[a].wm1;
            }
#if MM_SHIFT_LDS
            const double left = lds_shift(c1, c.from_lower);
            const double right = lds_shift(c0, c.from_upper);
#else
            const double left = dpp_lower(c1);   // cw at column y0-1 (lane-1's second column)
            const double right = dpp_upper(c0);  // cw at column y0+2 (lane+1's first column)
#endif
            const double r8 = A.drate[a] * 0.125;
            const double pk = c0 + c1;
            o0[a] = __builtin_fma(__builtin_fma(w[a].um0, m0, left + pk), r8, w[a].um0);
            o1[a] = __builtin_fma(__builtin_fma(w[a].um1, m1, pk + right), r8, w[a].um1);
        }
        w[a].wa0 = na0;
        w[a].wa1 = na1;
        w[a].wm0 = wn0[a];
        w[a].wm1 = wn1[a];
        w[a].um0 = u0[a];
        w[a].um1 = u1[a];
    }
    if (CHAIN && A.npost) {
        chain_k<NA>(o0, A.npost, A.post_a, A.post_b, A.post_r);
        chain_k<NA>(o1, A.npost, A.post_a, A.post_b, A.post_r);
    }
}

// Add an emitted row's owned cells to a level sum. The empty asm materialises the sum
// here: otherwise LLVM sinks the whole chain of adds to the kernel exit and keeps every
// row's values live until then.
__device__ __forceinline__ void accum(double& acc, bool own, const Lane& c, double w0, double w1) {
    acc = acc + ((own && c.own0) ? w0 : 0.0);
    acc = acc + ((own && c.own1) ? w1 : 0.0);
    asm volatile("" : "+v"(acc));
}

__device__ __forceinline__ double wave_sum_k(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
    return v;
}

template <int K, int NA>
__device__ __forceinline__ void write_sums(const PassArgs& A, long long wid, int lane,
                                           double (&acc)[K][NA]) {
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const double t = wave_sum_k(acc[j][a]);
            if (lane == 0) A.partials[((A.partial_base + wid) * K + j) * NA + a] = t;
        }
}

// The per-wave buffers of one pass: NA input and output row ranges.
template <int K, int NA>
struct Bufs {
    __amdgpu_buffer_rsrc_t in[NA], out[NA];
    __device__ __forceinline__ Bufs(const PassArgs& A, int rA, int rB) {
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            in[a] = rows_rsrc(A.in[a] + (long long)(rA - K) * A.pitch, rB - rA + 2 * K, A.pitch);
            out[a] = rows_rsrc(A.out[a] + (long long)rA * A.pitch, rB - rA, A.pitch);
        }
    }
};

// BLOCK schedule: TH rows, every iteration unrolled at compile time (level fill states,
// row offsets, block ownership and, per GP = the parity of the first input row, the rows'
// parities are all constants).
template <int K, int TH, int U, bool RED, int NT, bool FAST, int NA, bool CHAIN, int GP>
__device__ __forceinline__ void passk_block(const PassArgs& A, const Lane& c, long long wid,
                                            int lane, int rA, int rB, unsigned voff,
                                            unsigned soff) {
    constexpr int NI = TH + 2 * K;       // input rows
    constexpr int NIT = TH + 3 * K - 1;  // iterations
    double acc[K][NA];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[j][a] = 0.0;
    const unsigned rowb = (unsigned)(A.pitch * 8);
    const Bufs<K, NA> B(A, rA, rB);
    dv2 raw[U][NA];
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
        for (int a = 0; a < NA; ++a) raw[k][a] = load_row(B.in[a], voff + k * rowb);
    Win win[K][NA];
    double pend0[K][NA], pend1[K][NA];  // level j's row of the previous iteration: pend[j-1]

#pragma unroll
    for (int i = 0; i < NIT; ++i) {
#pragma unroll
        for (int j = K; j >= 1; --j) {  // descending: pend[j-2] is read before it is refilled
            const int m = i - 3 * (j - 1);
            if (m < 0 || m >= NI - 2 * (j - 1)) continue;  // compile-time
            double u0[NA], u1[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                if (j == 1) {
                    u0[a] = raw[i % U][a].x;
                    u1[a] = raw[i % U][a].y;
                    if (i + U < NI) raw[i % U][a] = load_row(B.in[a], voff + (i + U) * rowb);
                } else {
                    u0[a] = pend0[j - 2][a];
                    u1[a] = pend1[j - 2][a];
                }
            }
            const long long gx = c.gx0 + rA - K + (j - 1) + m;
            if (m < 2) {
                level_fill<NA, FAST, CHAIN>(A, c, gx, m, (GP + j) & 1, win[j - 1], u0, u1);
                continue;
            }
            double w0[NA], w1[NA];
            level_emit<NA, FAST, CHAIN>(A, c, gx, (GP + j + m) & 1, win[j - 1], u0, u1, w0, w1);
            const int orow = m + j - K - 2;  // output row - rA (compile-time)
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                if (RED && orow >= 0 && orow < TH)
                    accum(acc[j - 1][a], rA + orow < rB, c, w0[a], w1[a]);
                if (j == K) {
                    store_row<NT>(B.out[a], soff + orow * rowb, w0[a], w1[a]);
                } else {
                    pend0[j - 1][a] = w0[a];
                    pend1[j - 1][a] = w1[a];
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the row order: bounds the live registers
    }
    if (RED) write_sums<K, NA>(A, wid, lane, acc);
}

// Steady state of the SEGMENT schedule, iterations [b0, b1) (b0 = I0 mod U): every level
// emits one row per iteration, level K's row rA + (i - I0) is stored. FAST: every row the
// levels read in these iterations is an interior row of an interior strip.
// rG: the segment's geometry start (rA, or rA - 1 for a shifted segment, passk_segment),
// whose first input row is even: level j's row emitted at iteration i, rG - K - 2j + 1 + i,
// has the parity of i + 1.
template <int K, int U, bool RED, int NT, bool FAST, int NA, bool CHAIN>
__device__ __forceinline__ void seg_steady(const PassArgs& A, const Lane& c, const Bufs<K, NA>& B,
                                           int rG, int rA, int rB, unsigned voff, unsigned soff,
                                           unsigned rowb, int b0, int b1, dv2 (&raw)[U][NA],
                                           Win (&win)[K][NA], double (&pend0)[K][NA],
                                           double (&pend1)[K][NA], double (&acc)[K][NA]) {
    constexpr int I0 = 3 * K - 1;
    const __amdgpu_buffer_rsrc_t none = rows_rsrc(A.out[0], 0, A.pitch);
    for (int base = b0; base < b1; base += U) {
#pragma unroll
        for (int t = 0; t < U; ++t) {
            const int i = base + t;
            const int slot = (I0 + t) % U;  // base = I0 (mod U)
#pragma unroll
            for (int j = K; j >= 1; --j) {
                double u0[NA], u1[NA];
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    if (j == 1) {
#if MM_LOAD_COPY
                        u0[a] = vcopy(raw[slot][a].x);
                        u1[a] = vcopy(raw[slot][a].y);
#else
                        u0[a] = raw[slot][a].x;
                        u1[a] = raw[slot][a].y;
#endif
                        raw[slot][a] = load_row(B.in[a], voff + (unsigned)(i + U) * rowb);
                    } else {
                        u0[a] = pend0[j - 2][a];
                        u1[a] = pend1[j - 2][a];
                    }
                }
                const long long gx = c.gx0 + rG - K + i - 2 * (j - 1);
                double w0[NA], w1[NA];
                // an even U keeps base = I0 (mod 2): the parity is a constant per unrolled
                // row; an odd U (the 3- / 4-attribute K = 1, 2 instances) reads it at run time
                const int e = U % 2 == 0 ? (I0 + t + 1) & 1 : (i + 1) & 1;
                level_emit<NA, FAST, CHAIN>(A, c, gx, e, win[j - 1], u0, u1, w0, w1);
                const int r = rG - K - 2 * j + 1 + i;  // output row
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    if (RED) accum(acc[j - 1][a], r >= rA && r < rB, c, w0[a], w1[a]);
                    if (j == K) {
                        // row r of out (base rA); a shifted segment's row rA - 1 is dropped
                        const int ro = r - rA;
                        store_row<NT>(ro < 0 ? none : B.out[a], soff + (unsigned)(ro < 0 ? 0 : ro) * rowb,
                                      w0[a], w1[a]);
                    } else {
                        pend0[j - 1][a] = w0[a];
                        pend1[j - 1][a] = w1[a];
                    }
                }
#if MM_LEVEL_BARRIER
                // at most two levels in flight: bounds the live registers (occupancy)
                if ((K - j) % MM_LEVEL_BARRIER == MM_LEVEL_BARRIER - 1) __builtin_amdgcn_sched_barrier(0);
#endif
            }
#if MM_ROW_BARRIER
            if (t % MM_ROW_BARRIER == MM_ROW_BARRIER - 1 || t == U - 1) __builtin_amdgcn_sched_barrier(0);
#endif
        }
    }
}

// SEGMENT schedule: R = rB - rA rows (run time). Iterations 0 .. 3K-2 fill the levels
// (compile-time); from iteration I0 = 3K-1 on every level emits, level K writes row
// rA + (i - I0), and the loop runs R iterations (rounded up to U; the extra ones read
// zeros past the input rows and their stores fall past the output rows).
// A wave of an interior strip whose segment touches the grid's first or last rows runs
// the general body only for the iterations that read those rows and the branch-free body
// in between (the general body's per-row branches keep the K levels from interleaving).
// Rows are paired from an even global row (level_emit): a segment whose first input row
// gx0 + rA - K is odd starts one row higher (rG = rA - 1) -- an extra first input row that
// loads as 0 (row -1 of the input descriptor: its offset wraps past num_records) and an
// extra first output row that is not stored or summed (its value depends on that 0 row;
// the rows below it do not).
template <int K, int U, bool RED, int NT, bool FAST, int NA, bool CHAIN>
__device__ __forceinline__ void passk_segment(const PassArgs& A, const Lane& c, long long wid,
                                              int lane, int rA, int rB, unsigned voff,
                                              unsigned soff) {
    constexpr int I0 = 3 * K - 1;
    const int sh = (int)((c.gx0 + rA - K) & 1);
    const int rG = rA - sh;
    const int R = rB - rG;
    double acc[K][NA];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int a = 0; a < NA; ++a) acc[j][a] = 0.0;
    const unsigned rowb = (unsigned)(A.pitch * 8);
    const Bufs<K, NA> B(A, rA, rB);
    voff -= (unsigned)sh * rowb;  // input row k of the segment: row k - sh of B.in
    dv2 raw[U][NA];
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
        for (int a = 0; a < NA; ++a) raw[k][a] = load_row(B.in[a], voff + k * rowb);
    Win win[K][NA];
    double pend0[K][NA], pend1[K][NA];

    // prologue: level j takes part from iteration 3(j-1); nothing is stored yet
#pragma unroll
    for (int i = 0; i < I0; ++i) {
#pragma unroll
        for (int j = K; j >= 1; --j) {
            const int m = i - 3 * (j - 1);
            if (m < 0) continue;  // compile-time
            double u0[NA], u1[NA];
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                if (j == 1) {
                    u0[a] = raw[i % U][a].x;
                    u1[a] = raw[i % U][a].y;
                    raw[i % U][a] = load_row(B.in[a], voff + (i + U) * rowb);
                } else {
                    u0[a] = pend0[j - 2][a];
                    u1[a] = pend1[j - 2][a];
                }
            }
            const long long gx = c.gx0 + rG - K + (j - 1) + m;
            if (m < 2) {
                level_fill<NA, FAST, CHAIN>(A, c, gx, m, j & 1, win[j - 1], u0, u1);
                continue;
            }
            double w0[NA], w1[NA];
            level_emit<NA, FAST, CHAIN>(A, c, gx, (j + m) & 1, win[j - 1], u0, u1, w0, w1);
            const int r = rG - K - 2 * j + 1 + i;  // output row
#pragma unroll
            for (int a = 0; a < NA; ++a) {
                if (RED) accum(acc[j - 1][a], r >= rA && r < rB, c, w0[a], w1[a]);
                pend0[j - 1][a] = w0[a];  // j < K here: level K's m <= 1 in the prologue
                pend1[j - 1][a] = w1[a];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    const int end = I0 + (R + U - 1) / U * U;
    if (FAST) {
        seg_steady<K, U, RED, NT, true, NA, CHAIN>(A, c, B, rG, rA, rB, voff, soff, rowb, I0, end,
                                                   raw, win, pend0, pend1, acc);
    } else {
        int f0 = end, f1 = end;  // iterations [f0, f1) read interior rows only
        if (c.fast_cols) {
            // iteration i: the levels read global rows g - 2(K-1) .. g, g = gx0 + rG - K + i,
            // and emit the rows before them, whose own-weight coefficient the FAST body
            // takes as the interior's (-9): every row read >= 2
            const long long g0 = c.gx0 + rG - K;
            const long long lo = 2 + 2 * (K - 1) - g0;  // first i with every row >= 2
            const long long hi = c.H - 1 - g0;          // first i with a row > H-2
            const long long a0 = lo <= I0 ? I0 : I0 + (lo - I0 + U - 1) / U * U;
            const long long a1 = hi <= I0 ? I0 : I0 + (hi - I0) / U * U;
            f0 = (int)min((long long)end, a0);
            f1 = (int)max((long long)f0, min((long long)end, a1));
        }
        seg_steady<K, U, RED, NT, false, NA, CHAIN>(A, c, B, rG, rA, rB, voff, soff, rowb, I0,
                                                    f0, raw, win, pend0, pend1, acc);
        seg_steady<K, U, RED, NT, true, NA, CHAIN>(A, c, B, rG, rA, rB, voff, soff, rowb, f0, f1,
                                                   raw, win, pend0, pend1, acc);
        seg_steady<K, U, RED, NT, false, NA, CHAIN>(A, c, B, rG, rA, rB, voff, soff, rowb, f1,
                                                    end, raw, win, pend0, pend1, acc);
    }
    if (RED) write_sums<K, NA>(A, wid, lane, acc);
}

// Segment wave -> (strip, rows) inside one row range [lo, hi): the two edge strips come
// first, in segments of re rows; then the other strips in segments of r rows, strips
// fastest, the top and bottom segments (rows next to the grid's first / last row) first.
// Slow work is cut shorter and dispatched first, so the waves of a launch end together.
__device__ __forceinline__ void seg_map(long long w, int lo, int hi, int ns, int r, int re,
                                        int& strip, int& rA, int& rB) {
    const int n = hi - lo;
    int rb, rows;
    if (ns < 3) {
        strip = (int)(w % ns);
        rb = (int)(w / ns);
        rows = re;
    } else {
        const int nbe = (n + re - 1) / re;
        if (w < 2LL * nbe) {
            strip = w < nbe ? 0 : ns - 1;
            rb = (int)(w % nbe);
            rows = re;
        } else {
            const long long t = w - 2LL * nbe;
            const int nb = (n + r - 1) / r;
            strip = 1 + (int)(t % (ns - 2));
            const int q = (int)(t / (ns - 2));
            rb = q == 0 ? 0 : (q == 1 ? nb - 1 : q - 1);
            rows = r;
        }
    }
    rA = lo + rb * rows;
    rB = min(rA + rows, hi);
}

// K steps of the one-pass flow program per launch, NA attributes, transfer chains when
// CHAIN. MODE: kSeg = segment schedule (A.th / A.th_edge rows per wave), else the block
// schedule with MODE rows per wave. U input rows prefetched. RED: per-level sums of the
// owned cells into partials[((partial_base + wave) * K + level) * NA + attribute].
// NT & 1: non-temporal stores.
template <int K, int MODE, int U, bool RED, int NT, int NA, bool CHAIN>
__global__ __launch_bounds__(kBlock, MM_PASSK_MIN_WAVES) void mm_passk_kernel(const PassArgs A) {
    constexpr int L = (K + 1) / 2;          // halo lanes per side
    constexpr int OC = kStripCols - 4 * L;  // output columns per strip
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // optional XCD-aware block order: hardware block b runs on XCD b % 8; logical block
    // (b % 8) * per + b / 8 gives every XCD a contiguous run of tiles
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
    int strip, rA, rB;
    if (MODE == kSeg) {
        seg_map(w, rlo, rhi, A.nstrips, A.th, A.th_edge, strip, rA, rB);
    } else {
        strip = (int)(w % A.nstrips);
        rA = rlo + (int)(w / A.nstrips) * MODE;
        rB = min(rA + MODE, rhi);
    }

    const long long W = A.W;
    const long long c0 = (long long)strip * OC - 2 * L;  // first loaded column (even)
    const long long y0 = c0 + 2 * lane;
    const bool in_row = y0 >= 0 && y0 < A.pitch;  // y0 even, pitch a multiple of 128
    const unsigned voff = in_row ? (unsigned)(y0 * 8) : kOOBk;
    const bool store_lane = lane >= L && lane < 64 - L && y0 < W;
    // columns past W inside the pitch are padding: writing them is harmless
    const unsigned soff = store_lane ? (unsigned)(y0 * 8) : kOOBk;
    Lane c;
    c.H = A.H;
    c.gx0 = A.x_init;
    c.sy0 = span3k(W, y0);
    c.sy1 = span3k(W, y0 + 1);
    c.fast_cols = c0 >= 1 && c0 + kStripCols <= W - 1;  // loaded cols in [1, W-2]
    c.own0 = store_lane;
    c.own1 = store_lane && y0 + 1 < W;
    c.from_lower = ((lane + 63) & 63) * 4;
    c.from_upper = ((lane + 1) & 63) * 4;

    // a wave whose input rows and loaded columns are all interior (cnt == 8 everywhere)
    // runs the branch-free body; edge waves run the general one
#if defined(MM_TEST_BODY) && MM_TEST_BODY == 1
    const bool fast = true;
#elif defined(MM_TEST_BODY) && MM_TEST_BODY == 2
    const bool fast = false;
#else
    const bool fast = c.fast_cols && c.gx0 + rA - K >= 1 && c.gx0 + rB + K - 1 <= A.H - 2;
#endif
    if constexpr (MODE == kSeg) {
        if (fast)
            passk_segment<K, U, RED, NT, true, NA, CHAIN>(A, c, wid, lane, rA, rB, voff, soff);
        else
            passk_segment<K, U, RED, NT, false, NA, CHAIN>(A, c, wid, lane, rA, rB, voff, soff);
    } else {
        // the block's rows' parities are compile-time per parity of its first input row
        const bool gp = ((c.gx0 + rA - K) & 1) != 0;
        if (fast && gp)
            passk_block<K, MODE, U, RED, NT, true, NA, CHAIN, 1>(A, c, wid, lane, rA, rB, voff, soff);
        else if (fast)
            passk_block<K, MODE, U, RED, NT, true, NA, CHAIN, 0>(A, c, wid, lane, rA, rB, voff, soff);
        else if (gp)
            passk_block<K, MODE, U, RED, NT, false, NA, CHAIN, 1>(A, c, wid, lane, rA, rB, voff,
                                                                 soff);
        else
            passk_block<K, MODE, U, RED, NT, false, NA, CHAIN, 0>(A, c, wid, lane, rA, rB, voff,
                                                                 soff);
    }
}

template <int K, int MODE, int U, int NT, int NA, bool CHAIN>
hipError_t launch_k3(bool red, const PassArgs& a, hipStream_t s) {
    // at least one block: a dispatch with no work (mm_prepare) still reaches the queue
    long long blocks = std::max<long long>(1, (a.waves_total + kWavesPerBlock - 1) / kWavesPerBlock);
    if (a.xcd_remap) blocks = (blocks + 7) / 8 * 8;
    const dim3 g((unsigned)blocks), b(kBlock);
    (void)hipGetLastError();  // the status below is this launch's, not an earlier call's
    if (red)
        hipLaunchKernelGGL((mm_passk_kernel<K, MODE, U, true, NT, NA, CHAIN>), g, b, 0, s, a);
    else
        hipLaunchKernelGGL((mm_passk_kernel<K, MODE, U, false, NT, NA, CHAIN>), g, b, 0, s, a);
    return hipGetLastError();
}

// a.seg: segment schedule (variant bit 0: non-temporal stores); else 4-row blocks.
template <int K, int NA, bool CHAIN>
hipError_t launch_k2(bool red, const PassArgs& a, hipStream_t s, int v) {
    constexpr int U = seg_prefetch<NA>();
    if (!a.seg) {
        if (a.th != kBorderRows) return hipErrorInvalidValue;
        return launch_k3<K, kBorderRows, (U < 4 ? U : 4), 0, NA, CHAIN>(red, a, s);
    }
    return (v & 1) ? launch_k3<K, kSeg, U, 1, NA, CHAIN>(red, a, s)
                   : launch_k3<K, kSeg, U, 0, NA, CHAIN>(red, a, s);
}

// Resident blocks per CU of the segment kernel, from its register count: gfx950 gives each
// SIMD lane 512 registers (VGPRs and AGPRs together, allocated in granules of 8), at most
// 8 waves per SIMD, 4 SIMDs per CU (MI355X_MICROARCH.md). The runtime's occupancy query is
// not used: after `import torch` it answers for this kernel with half the true occupancy
// (profiles/r02/occupancy_probe.log), which would halve the waves of every plan.
template <int K, int NA, bool CHAIN, bool RED, int NT>
int seg_blocks_per_cu_v() {
    hipFuncAttributes fa;
    const hipError_t e = hipFuncGetAttributes(
        &fa, reinterpret_cast<const void*>(mm_passk_kernel<K, kSeg, seg_prefetch<NA>(), RED, NT, NA, CHAIN>));
    if (e != hipSuccess) {
        (void)hipGetLastError();  // a failed query must not surface at the next launch
        return 0;
    }
    const int regs = (fa.numRegs + 7) / 8 * 8;
    const int waves_per_simd = regs > 0 ? std::min(8, 512 / regs) : 8;
    return waves_per_simd * 4 / kWavesPerBlock;
}

template <int K, int NA, bool CHAIN>
int seg_blocks_per_cu(bool red, int nt) {
    if (red)
        return nt ? seg_blocks_per_cu_v<K, NA, CHAIN, true, 1>()
                  : seg_blocks_per_cu_v<K, NA, CHAIN, true, 0>();
    return nt ? seg_blocks_per_cu_v<K, NA, CHAIN, false, 1>()
              : seg_blocks_per_cu_v<K, NA, CHAIN, false, 0>();
}

}  // namespace

}  // namespace mm
