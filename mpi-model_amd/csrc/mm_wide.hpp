// mm_wide.hpp -- the level-split K-step kernel (one attribute, one whole-grid Exponencial
// flow): K fused steps per HBM pass, the K levels spread over the P waves of a workgroup.
//
// The step is the generalisation of src/Model.hpp:176-235 + src/Exponencial.hpp:18-20 to
// every cell (oracle/mm_oracle.h): per cell out = r*u, s = out/cnt, d = u - out and
// v' = d + ((c3(y-1) + c3(y+1)) + p), p = s(x-1) + s(x+1), c3 = p + s(x). Every level below
// is that single step, so K fused levels are bit-identical to K single steps.
//
// Why split the levels. A K-level pipeline keeps, per level and column, the shares of two
// rows and the kept value of one (three doubles) plus the row handed to the next level.
// With all K levels in one wave (mm_passk.hpp) the register file caps a lane at 2 columns:
// then 4 of the 18 VALU instructions of a level-row are DPP moves (the +-1 column
// neighbours) and, at K = 10, 20 of the 128 loaded columns are halo whose results are
// thrown away. Here a workgroup of P waves shares ONE strip: wave p runs levels
// p*KW+1 .. (p+1)*KW and hands its last level's rows to wave p+1 through a double-buffered
// LDS row (2 KiB), one workgroup barrier per row. Each wave holds only KW levels, so a lane
// holds 4 columns (one strip = 256 loaded columns, two 16-B loads per lane and row): the
// DPP moves per cell halve, and the halo -- ceil(K/4) lanes per side -- is 12 / 256
// columns per side at K = 12 instead of 10 / 128 at K = 10.
//
// Pipeline (the skew of mm_passk.hpp, across waves): level j's m-th input row arrives at
// iteration m + 3(j-1) and it emits one row per input from its third input on; level j's
// output of iteration i is level j+1's input at iteration i+1 -- in registers inside a
// wave, through LDS between waves. Wave p's levels start at iteration 3*p*KW; before that
// it only joins the barriers, so every wave passes the same number of barriers. Wave 0
// streams the input rows from HBM (U rows prefetched); wave P-1 stores level K's rows.
//
// Columns: lane l holds columns c0+4l .. c0+4l+3. DPP wave_shr / wave_shl give the
// neighbour column of the lanes' first / last column; at the wave's edges that brings
// garbage, which moves one column inward per level and stays inside the halo lanes.
// Strips that touch the grid's first or last column (or run past it) fix up the lanes
// whose columns have 5 (edge), 3 (corner) or 0 (outside) neighbours; segments touching
// the grid's first / last rows run the general body for the iterations that read them.
#pragma once

#include "mm_passk.hpp"

namespace mm {

// per-K entry points (mm_wide_k*.hip)
#define MM_WIDE_DECL(K)                                                                    \
    hipError_t wide_launch_k##K(bool red, const PassArgs& a, hipStream_t s, int v);       \
    int wide_blocks_k##K(bool red, int nt);
MM_WIDE_DECL(4)
MM_WIDE_DECL(8)
MM_WIDE_DECL(12)
MM_WIDE_DECL(16)
MM_WIDE_DECL(20)
#undef MM_WIDE_DECL

namespace {

constexpr int kWideCols = 4;                // columns per lane
constexpr int kWideStrip = 64 * kWideCols;  // loaded columns per strip

#ifndef MM_WIDE_U
#define MM_WIDE_U 4  // input rows prefetched by the first wave (divides MM_WIDE_B)
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 4  // rows per barrier group
#endif
#ifndef MM_WIDE_LEVEL_BARRIER
#define MM_WIDE_LEVEL_BARRIER 0  // scheduling barrier after every this many levels (0: none)
#endif
#ifndef MM_WIDE_MIN_WAVES
#define MM_WIDE_MIN_WAVES 2  // __launch_bounds__ waves per SIMD (caps VGPRs)
#endif

enum { kBodyFast = 0, kBodyEdge = 1, kBodyGen = 2 };

// What every level of a wave needs besides its windows.
struct WLane {
    long long H;
    int sy[4];      // column spans of this lane's four columns
    int cnt[4];     // neighbour counts of the four columns in an interior row (8 / 5 / 0 ...)
    bool special;   // some column of this lane has cnt != 8 (edge strips only)
    bool own[4];    // output cells of this workgroup
};

// One level's window, per column: shares of the row above (sp), shares and u - out of the
// current row (sc, dc).
struct Win4 {
    double sp[4], sc[4], dc[4];
};

// s and d of this lane's four columns of row gx (oracle/mm_oracle.c emit). FAST: interior
// row of an interior strip (cnt == 8: s = u*(r/8), d = fma(s, -8, u)). EDGE: interior row;
// the lanes holding an edge / outside column redo those columns with their true count.
// GEN: any row (the row class is wave-uniform).
template <int BODY>
__device__ __forceinline__ void proc4(const WLane& c, double r, double r8, long long gx,
                                      const double (&u)[4], double (&s)[4], double (&d)[4]) {
    const int sx = BODY == kBodyGen ? span3k(c.H, gx) : 3;
    if (sx == 3) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[k] = u[k] * r8;
            d[k] = __builtin_fma(s[k], -8.0, u[k]);
        }
        if (BODY != kBodyFast && c.special) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (c.cnt[k] != 8) emit_k(r, u[k], c.cnt[k], s[k], d[k]);
        }
    } else if (sx == 0) {  // row outside the grid: emits nothing
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[k] = 0.0;
            d[k] = u[k];
        }
    } else {  // the grid's first / last row: 5 / 3 neighbours
#pragma unroll
        for (int k = 0; k < 4; ++k) emit_k(r, u[k], c.sy[k] ? sx * c.sy[k] - 1 : 0, s[k], d[k]);
    }
}

// Level input m = 0 / 1 (row gx): fill the window.
template <int BODY>
__device__ __forceinline__ void wfill(const WLane& c, double r, double r8, long long gx, int m,
                                      Win4& w, const double (&u)[4]) {
    double s[4], d[4];
    proc4<BODY>(c, r, r8, gx, u, s, d);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (m == 0) {
            w.sp[k] = s[k];
        } else {
            w.sc[k] = s[k];
            w.dc[k] = d[k];
        }
    }
}

// Level input m >= 2 (row gx): emit the window's current row, slide the window.
template <int BODY>
__device__ __forceinline__ void wemit(const WLane& c, double r, double r8, long long gx, Win4& w,
                                      const double (&u)[4], double (&o)[4]) {
    double sn[4], dn[4];
    proc4<BODY>(c, r, r8, gx, u, sn, dn);
    double p[4], c3[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        p[k] = w.sp[k] + sn[k];
        c3[k] = p[k] + w.sc[k];
    }
    const double left = dpp_lower(c3[3]);   // c3 of column y0-1 (lane-1's last column)
    const double right = dpp_upper(c3[0]);  // c3 of column y0+4 (lane+1's first column)
    o[0] = w.dc[0] + ((left + c3[1]) + p[0]);
    o[1] = w.dc[1] + ((c3[0] + c3[2]) + p[1]);
    o[2] = w.dc[2] + ((c3[1] + c3[3]) + p[2]);
    o[3] = w.dc[3] + ((c3[2] + right) + p[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        w.sp[k] = w.sc[k];
        w.sc[k] = sn[k];
        w.dc[k] = dn[k];
    }
}

__device__ __forceinline__ void accum4(double& acc, bool row_own, const WLane& c,
                                       const double (&o)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = acc + ((row_own && c.own[k]) ? o[k] : 0.0);
    asm volatile("" : "+v"(acc));
}

// workgroup barrier ordering LDS only: s_waitcnt lgkmcnt(0); s_barrier -- the prefetched
// HBM rows stay in flight
__device__ __forceinline__ void wg_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Wave roles: the first wave streams the input rows from HBM, the last stores level K's
// rows, the middle ones read and write LDS; with P = 1 one wave does both ends. Each role
// is its own instantiation, so no iteration branches on the role (a branch would split the
// loop body and keep the scheduler from interleaving the levels).
enum { kRoleFirst = 0, kRoleMid = 1, kRoleLast = 2, kRoleOnly = 3 };

// Schedule constants. Rows are exchanged in groups of B iterations with one barrier
// per group. Wave p starts at iteration p*D, D = S0 + B: its first level's m-th input is
// the row wave p-1's last level emitted B iterations earlier, always in the previous
// group; LDS holds RL = 2B rows per stage (a row is overwritten two groups later).
template <int KW, int P, int GB>
struct WGeom {
    static constexpr int K = KW * P;
    static constexpr int B = GB;
    static constexpr int S0 = 3 * KW - 1;  // local iterations before the wave's last level emits
    static constexpr int D = S0 + B;
    static constexpr int RL = 2 * B;
    static constexpr int T0 = (S0 + B - 1) / B * B;  // wave 0: compile-time iterations
};

// Per-wave constants of one block.
struct WCtx {
    WLane c;
    int p, lane, rA, rB;
    int start;            // first iteration of this wave (p * D)
    long long g0;         // global row of input row 0 (rA - K)
    double r, r8;
    unsigned voff, soff, rowb;
    __amdgpu_buffer_rsrc_t in, out;
    dv2* lds_in;          // stage p-1 (RL row slots of 128 dv2)
    dv2* lds_out;         // stage p
    double* partials;
    long long pbase;
};

template <int KW, int U>
struct WState {
    Win4 win[KW];
    double pend[KW][4];  // pend[q]: level q's row of the previous iteration (q < KW-1)
    dv2 raw[U][2];       // first wave: prefetched input rows
    double acc[KW];
};

// One iteration i of a wave (local iteration t = i - start): input row -> its KW levels
// (descending, so pend[q-1] is read before level q-1 refills it) -> level KW-1's row to
// LDS or HBM. PRO: t is a prologue iteration known at compile time (level q takes part from
// t = 3q and emits from t = 3q + 2); otherwise every level emits. slot: ring slot (first
// wave, compile time after unrolling).
template <int KW, int P, int U, int B, bool RED, int NT, int BODY, int ROLE, bool PRO>
__device__ __forceinline__ void wave_iter(const WCtx& x, WState<KW, U>& st, int i, int t,
                                          int slot) {
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    constexpr bool kIn = ROLE == kRoleFirst || ROLE == kRoleOnly;   // input from HBM
    constexpr bool kOut = ROLE == kRoleLast || ROLE == kRoleOnly;  // output to HBM
    double uin[4];
    if (kIn) {
#if MM_LOAD_COPY
        uin[0] = vcopy(st.raw[slot][0].x);
        uin[1] = vcopy(st.raw[slot][0].y);
        uin[2] = vcopy(st.raw[slot][1].x);
        uin[3] = vcopy(st.raw[slot][1].y);
#else
        uin[0] = st.raw[slot][0].x;
        uin[1] = st.raw[slot][0].y;
        uin[2] = st.raw[slot][1].x;
        uin[3] = st.raw[slot][1].y;
#endif
        const unsigned o = x.voff + (unsigned)(i + U) * x.rowb;
        st.raw[slot][0] = load_row(x.in, o);
        st.raw[slot][1] = load_row(x.in, o + 16);
    } else {
        const dv2* src = x.lds_in + ((i - G::B) % G::RL) * 128;  // i >= start >= D > B
        const dv2 a = src[x.lane], b = src[64 + x.lane];
        uin[0] = a.x;
        uin[1] = a.y;
        uin[2] = b.x;
        uin[3] = b.y;
    }
    if (!PRO) t = i - x.start;
#pragma unroll
    for (int q = KW - 1; q >= 0; --q) {
        const int m = t - 3 * q;  // this level's input index
        if (PRO && m < 0) continue;  // compile time
        const int j = x.p * KW + q + 1;  // global level, 1-based
        const long long gx = x.g0 + (j - 1) + m;
        double u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = q == 0 ? uin[k] : st.pend[q - 1][k];
        if (PRO && m < 2) {
            wfill<BODY>(x.c, x.r, x.r8, gx, m, st.win[q], u);
            continue;
        }
        double o[4];
        wemit<BODY>(x.c, x.r, x.r8, gx, st.win[q], u, o);
        if (RED) {
            const int r = x.rA - K + m + j - 2;  // output row of level j
            accum4(st.acc[q], r >= x.rA && r < x.rB, x.c, o);
        }
        if (q == KW - 1) {
            if (kOut) {  // level K: output row m - 2 of the segment
                const unsigned so = x.soff + (unsigned)(m - 2) * x.rowb;
                store_row<NT>(x.out, so, o[0], o[1]);
                store_row<NT>(x.out, so + 16, o[2], o[3]);
            } else {
                dv2* dst = x.lds_out + (i % G::RL) * 128;
                dv2 a, b;
                a.x = o[0];
                a.y = o[1];
                b.x = o[2];
                b.y = o[3];
                dst[x.lane] = a;
                dst[64 + x.lane] = b;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) st.pend[q][k] = o[k];
        }
#if MM_WIDE_LEVEL_BARRIER
        // at most MM_WIDE_LEVEL_BARRIER levels in flight: bounds the live registers
        if (q > 0 && (KW - q) % MM_WIDE_LEVEL_BARRIER == 0) __builtin_amdgcn_sched_barrier(0);
#endif
    }
}

// the barrier that closes iteration i when it ends a group
template <int P, int B>
__device__ __forceinline__ void group_end(int i) {
    if (P > 1 && (i + 1) % B == 0) wg_sync();
}

// Steady groups [b0, b1) (multiples of B) of one wave, B iterations per loop trip (ring
// slot i mod U: U divides B).
template <int KW, int P, int U, int B, bool RED, int NT, int BODY, int ROLE>
__device__ __forceinline__ void wave_groups(const WCtx& x, WState<KW, U>& st, int b0, int b1) {
    for (int base = b0; base < b1; base += B) {
#pragma unroll
        for (int tt = 0; tt < B; ++tt)
            wave_iter<KW, P, U, B, RED, NT, BODY, ROLE, false>(x, st, base + tt, 0, tt % U);
        if (P > 1) wg_sync();
    }
}

// The whole schedule of one wave. MID: body of the groups whose rows are all interior.
template <int KW, int P, int U, int B, bool RED, int NT, int ROLE, int MID>
__device__ __forceinline__ void wave_run(const WCtx& x, long long wid, int iend) {
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    static_assert(B % U == 0, "ring slots repeat within a group");
    constexpr bool kIn = ROLE == kRoleFirst || ROLE == kRoleOnly;
    WState<KW, U> st;
#pragma unroll
    for (int q = 0; q < KW; ++q) st.acc[q] = 0.0;
    int s;  // first iteration of the group loop
    if (kIn) {
        // start = 0: the prologue and the iterations up to the first group boundary are
        // unrolled (compile-time ring slots)
#pragma unroll
        for (int k = 0; k < U; ++k) {
            st.raw[k][0] = load_row(x.in, x.voff + k * x.rowb);
            st.raw[k][1] = load_row(x.in, x.voff + 16 + k * x.rowb);
        }
#pragma unroll
        for (int t = 0; t < G::T0; ++t) {
            if (t < G::S0)
                wave_iter<KW, P, U, B, RED, NT, kBodyGen, ROLE, true>(x, st, t, t, t % U);
            else
                wave_iter<KW, P, U, B, RED, NT, kBodyGen, ROLE, false>(x, st, t, 0, t % U);
            if (P > 1 && (t + 1) % B == 0) wg_sync();
        }
        s = G::T0;
    } else {
        for (int i = 0; i < x.start; ++i) group_end<P, B>(i);
#pragma unroll
        for (int t = 0; t < G::S0; ++t) {
            wave_iter<KW, P, U, B, RED, NT, kBodyGen, ROLE, true>(x, st, x.start + t, t, 0);
            group_end<P, B>(x.start + t);
        }
        s = x.start + G::S0;
        for (; s % B != 0; ++s) {
            wave_iter<KW, P, U, B, RED, NT, kBodyGen, ROLE, false>(x, st, s, 0, 0);
            group_end<P, B>(s);
        }
    }
    // groups whose levels all read interior rows: level j reads row g0 + (j-1) + m,
    // m = i - start - 3q, i.e. rows g0 + p*KW + (i - start) - 2q over q = 0..KW-1
    const long long base = x.g0 + (long long)x.p * KW - x.start;
    const long long lo = 1 + 2 * (KW - 1) - base;  // first i with every row >= 1
    const long long hi = x.c.H - 1 - base;         // first i with a row > H-2
    long long f0 = lo <= s ? s : s + (lo - s + B - 1) / B * B;
    long long f1 = hi <= s ? s : s + (hi - s) / B * B;
    f0 = min(f0, (long long)iend);
    f1 = max(f0, min(f1, (long long)iend));
    wave_groups<KW, P, U, B, RED, NT, kBodyGen, ROLE>(x, st, s, (int)f0);
    wave_groups<KW, P, U, B, RED, NT, MID, ROLE>(x, st, (int)f0, (int)f1);
    wave_groups<KW, P, U, B, RED, NT, kBodyGen, ROLE>(x, st, (int)f1, iend);
    if (RED) {  // partials[partial_base + block][K]: this wave's KW levels
#pragma unroll
        for (int q = 0; q < KW; ++q) {
            const double v = wave_sum_k(st.acc[q]);
            if (x.lane == 0) x.partials[(x.pbase + wid) * K + x.p * KW + q] = v;
        }
    }
}

template <int KW, int P, int U, int B, bool RED, int NT, int MID>
__device__ __forceinline__ void wave_dispatch(const WCtx& x, long long wid, int iend) {
    if (P == 1)
        wave_run<KW, P, U, B, RED, NT, kRoleOnly, MID>(x, wid, iend);
    else if (x.p == 0)
        wave_run<KW, P, U, B, RED, NT, kRoleFirst, MID>(x, wid, iend);
    else if (x.p == P - 1)
        wave_run<KW, P, U, B, RED, NT, kRoleLast, MID>(x, wid, iend);
    else
        wave_run<KW, P, U, B, RED, NT, kRoleMid, MID>(x, wid, iend);
}

// K = KW * P fused steps per launch, one workgroup (P waves) per strip segment. The
// segment map is mm_passk.hpp's seg_map with blocks in place of waves: the two edge strips
// first (A.th_edge rows), then the others (A.th rows). RED: every level's sums of the
// block's output cells into partials[partial_base + block][K]. NT & 1: non-temporal stores.
template <int KW, int P, int U, int B, bool RED, int NT>
__global__ __launch_bounds__(64 * P, MM_WIDE_MIN_WAVES) void mm_wide_kernel(const PassArgs A) {
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    constexpr int LH = (K + kWideCols - 1) / kWideCols;  // halo lanes per side
    constexpr int OC = kWideStrip - 2 * kWideCols * LH;  // output columns per strip
    __shared__ dv2 lds[P > 1 ? P - 1 : 1][G::RL][128];
    const int lane = threadIdx.x & 63;
    const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    long long blk = blockIdx.x;
    if (A.xcd_remap) {
        const long long per = gridDim.x / 8;
        blk = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    if (blk >= A.waves_total) return;  // the whole block: no barrier is left waiting

    int rlo, rhi;
    long long w = blk;
    if (w < A.waves_a) {
        rlo = A.ra0;
        rhi = A.ra1;
    } else {
        w -= A.waves_a;
        rlo = A.rb0;
        rhi = A.rb1;
    }
    WCtx x;
    int strip;
    seg_map(w, rlo, rhi, A.nstrips, A.th, A.th_edge, strip, x.rA, x.rB);
    const long long W = A.W;
    const long long c0 = (long long)strip * OC - kWideCols * LH;  // first loaded column
    const long long y0 = c0 + kWideCols * lane;
    const bool in_row = y0 >= 0 && y0 < A.pitch;  // y0 % 4 == 0, pitch % 128 == 0
    const bool store_lane = lane >= LH && lane < 64 - LH && y0 < W;
    x.voff = in_row ? (unsigned)(y0 * 8) : kOOBk;
    // columns past W inside the pitch are padding: writing them is harmless
    x.soff = store_lane ? (unsigned)(y0 * 8) : kOOBk;
    x.rowb = (unsigned)(A.pitch * 8);
    x.c.H = A.H;
    x.c.special = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        x.c.sy[k] = span3k(W, y0 + k);
        x.c.cnt[k] = x.c.sy[k] ? 3 * x.c.sy[k] - 1 : 0;
        x.c.special = x.c.special || x.c.cnt[k] != 8;
        x.c.own[k] = store_lane && y0 + k < W;
    }
    x.p = p;
    x.lane = lane;
    x.start = p * G::D;
    x.g0 = A.x_init + x.rA - K;
    x.r = A.drate[0];
    x.r8 = x.r * 0.125;
    x.in = rows_rsrc(A.in[0] + (long long)(x.rA - K) * A.pitch, x.rB - x.rA + 2 * K, A.pitch);
    x.out = rows_rsrc(A.out[0] + (long long)x.rA * A.pitch, x.rB - x.rA, A.pitch);
    x.lds_in = p > 0 ? &lds[p - 1][0][0] : &lds[0][0][0];
    x.lds_out = p < P - 1 ? &lds[p][0][0] : &lds[0][0][0];
    x.partials = A.partials;
    x.pbase = A.partial_base;

    // every wave runs to iteration iend (a whole number of groups): the last wave emits
    // the segment's last row at iteration (P-1)*D + S0 + R - 1
    const int need = (P - 1) * G::D + G::S0 + (x.rB - x.rA);
    const int iend = (need + G::B - 1) / G::B * G::B;
    // a strip whose loaded columns include the grid's first / last column or columns past
    // it fixes up the lanes holding them
    const bool edge = !(c0 >= 1 && c0 + kWideStrip <= W - 1);
    if (edge)
        wave_dispatch<KW, P, U, B, RED, NT, kBodyEdge>(x, blk, iend);
    else
        wave_dispatch<KW, P, U, B, RED, NT, kBodyFast>(x, blk, iend);
}

template <int KW, int P, int NT>
hipError_t wide_launch3(bool red, const PassArgs& a, hipStream_t s) {
    constexpr int U = MM_WIDE_U;
    long long blocks = a.waves_total;
    if (a.xcd_remap) blocks = (blocks + 7) / 8 * 8;
    const dim3 g((unsigned)blocks), b(64 * P);
    (void)hipGetLastError();  // the status below is this launch's, not an earlier call's
    if (red)
        hipLaunchKernelGGL((mm_wide_kernel<KW, P, U, MM_WIDE_B, true, NT>), g, b, 0, s, a);
    else
        hipLaunchKernelGGL((mm_wide_kernel<KW, P, U, MM_WIDE_B, false, NT>), g, b, 0, s, a);
    return hipGetLastError();
}

// a.seg must be set (segment schedule); variant bit 0: non-temporal stores.
template <int KW, int P>
hipError_t wide_launch2(bool red, const PassArgs& a, hipStream_t s, int v) {
    if (!a.seg) return hipErrorInvalidValue;
    return (v & 1) ? wide_launch3<KW, P, 1>(red, a, s) : wide_launch3<KW, P, 0>(red, a, s);
}

// Resident workgroups per CU, from the kernel's registers (512 per SIMD lane, granules of
// 8, at most 8 waves per SIMD) and its LDS (160 KiB per CU); see seg_blocks_per_cu_v.
template <int KW, int P, bool RED, int NT>
int wide_blocks_v() {
    hipFuncAttributes fa;
    const hipError_t e = hipFuncGetAttributes(
        &fa, reinterpret_cast<const void*>(mm_wide_kernel<KW, P, MM_WIDE_U, MM_WIDE_B, RED, NT>));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    const int regs = (fa.numRegs + 7) / 8 * 8;
    const int waves_per_simd = regs > 0 ? std::min(8, 512 / regs) : 8;
    int blocks = waves_per_simd * 4 / P;
    if (fa.sharedSizeBytes > 0) blocks = std::min(blocks, (int)(160 * 1024 / fa.sharedSizeBytes));
    return std::max(blocks, 0);
}

template <int KW, int P>
int wide_blocks(bool red, int nt) {
    if (red) return nt ? wide_blocks_v<KW, P, true, 1>() : wide_blocks_v<KW, P, true, 0>();
    return nt ? wide_blocks_v<KW, P, false, 1>() : wide_blocks_v<KW, P, false, 0>();
}

}  // namespace

}  // namespace mm
