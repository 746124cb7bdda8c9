// mm_wide.hpp -- the level-split K-step kernel (one attribute, one whole-grid Exponencial
// flow): K fused steps per HBM pass, the K levels spread over the P waves of a workgroup.
//
// The step is the generalisation of src/Model.hpp:176-235 + src/Exponencial.hpp:18-20 to
// every cell (oracle/mm_oracle.h): per cell the weights w = u * 8/cnt (w = u where cnt = 8,
// 0 outside the grid), the column triple cw of rows x-1..x+1 and the 3 x 3 box sum S of the
// triples of columns y-1..y+1 -- each sum pairing its two rows / columns from an even
// global index, so consecutive rows (a level's consecutive iterations) and consecutive
// columns (a lane's column pairs) share the pair's sum -- and v' = fma(fma(u, m, S), r/8, u),
// m = -(8 + 8/cnt) (-9 inside): the out = r*u, share = out/cnt of every neighbour with r/8
// factored out of the sum. Every level below is that single step, so K fused levels are
// bit-identical to K single steps.
//
// Why split the levels. A K-level pipeline keeps, per level and column, the shares of two
// rows and the kept value of one (three doubles) plus the row handed to the next level.
// With all K levels in one wave (mm_passk.hpp) the register file caps a lane at 2 columns:
// then 4 of the 18 VALU instructions of a level-row are DPP moves (the +-1 column
// neighbours) and, at K = 10, 20 of the 128 loaded columns are halo whose results are
// thrown away. Here a workgroup of P waves shares ONE strip: wave p runs levels
// p*KW+1 .. (p+1)*KW and hands its last level's rows to wave p+1 through a double-buffered
// LDS ring, one workgroup barrier per group of B rows. Each wave holds only KW levels, so a
// lane holds C = 4 columns (one strip = 256 loaded columns, two 16-B loads per lane and
// row): a level-row of a lane is 28 fp64 operations and 4 DPP moves (2 per column at
// C = 2), and the halo -- ceil(K/4) lanes per side -- is 16 / 256 columns per side at
// K = 16 instead of 10 / 128 at K = 10.
//
// Several attributes (config C5: four, with same-cell transfer chains before / after the
// diffusions) hold NA windows per level: C = 2 columns per lane keeps the state of a level
// near a one-attribute level's at C = 4 (NA * C doubles per cell row).
//
// C = 8 columns per lane, column waves, an LDS-DMA input ring, role rotation and
// non-temporal loads were built, measured and dropped (git history).
//
// Pipeline (the skew of mm_passk.hpp, across waves): level j's m-th input row arrives at
// iteration m + 3(j-1) and it emits one row per input from its third input on; level j's
// output of iteration i is level j+1's input at iteration i+1 -- in registers inside a
// wave (MM_WIDE_ASC: at iteration i, skew 2; 0.6 % slower at K = 16), through LDS between
// waves. Wave p's levels start at iteration p*D; before that it only joins the barriers,
// so every wave passes the same number of barriers. Wave 0
// streams the input rows from HBM (U rows prefetched); wave P-1 stores level K's rows.
//
// Columns: lane l holds columns c0+C*l .. c0+C*l+C-1. DPP wave_shr / wave_shl give the
// neighbour column of the lanes' first / last column; at the wave's edges that brings
// garbage, which moves one column inward per level and stays inside the halo lanes.
// Strips that touch the grid's first or last column (or run past it) fix up the lanes
// whose columns have 5 (edge), 3 (corner) or 0 (outside) neighbours; segments touching
// the grid's first / last rows run the general body for the iterations that read them.
#pragma once

#include "mm_passk.hpp"

#ifndef MM_WIDE_GEN_ROW
// GEN body outside the EDGE-impossible strips: row-uniform weight factors (1) or every
// column by its own count (0: fewer registers, which the four-attribute instances need)
#define MM_WIDE_GEN_ROW 1
#endif

namespace mm {

// per-K entry points (mm_wide_k*.hip: one attribute, C = 4)
#define MM_WIDE_DECL(K)                                                                    \
    hipError_t wide_launch_k##K(bool red, const PassArgs& a, hipStream_t s, int v);       \
    int wide_blocks_k##K(bool red, int nt);
MM_WIDE_DECL(4)
MM_WIDE_DECL(8)
MM_WIDE_DECL(12)
MM_WIDE_DECL(16)
MM_WIDE_DECL(20)
#undef MM_WIDE_DECL
int wide_waves_k20();  // waves per workgroup of the K = 20 instance
// four attributes, 2 columns per lane. K = 4 (mm_widea_k4.hip): any pass.
hipError_t widea_launch_k4(int na, bool red, const PassArgs& a, hipStream_t s, int v);
int widea_blocks_k4(int na, bool red, int nt);
// K = 8 (mm_widea_k8.hip, one object per instance): the first N attributes diffuse (the
// engine relabels the attributes so that the diffusing ones come first), with (P = 1) or
// without (P = 0) a post-chain; non-temporal stores.
#define MM_WIDEA8_DECL(N, P)                                                               \
    hipError_t widea8_launch_n##N##_p##P(bool red, const PassArgs& a, hipStream_t s);     \
    int widea8_blocks_n##N##_p##P(bool red);
MM_WIDEA8_DECL(1, 0)
MM_WIDEA8_DECL(2, 0)
MM_WIDEA8_DECL(3, 0)
MM_WIDEA8_DECL(4, 0)
MM_WIDEA8_DECL(1, 1)
MM_WIDEA8_DECL(2, 1)
MM_WIDEA8_DECL(3, 1)
MM_WIDEA8_DECL(4, 1)
#undef MM_WIDEA8_DECL
// four attributes whose pre-chain is the ring t -> t+1 mod 4 (mm_widear_k*.hip)
hipError_t widear_launch_k8(int na, bool red, const PassArgs& a, hipStream_t s, int v);
int widear_blocks_k8(int na, bool red, int nt);
int widear_waves_k8();

namespace {

#ifndef MM_WIDE_U
#define MM_WIDE_U 4  // input rows prefetched by the first wave (divides MM_WIDE_B)
#endif
#ifndef MM_WIDE_B
#define MM_WIDE_B 4  // rows per barrier group
#endif
#ifndef MM_WIDE_MIN_WAVES
#define MM_WIDE_MIN_WAVES 2  // __launch_bounds__ waves per SIMD of the C = 4 instances
#endif
#ifndef MM_WIDE_PRO_MID
#define MM_WIDE_PRO_MID 1  // 0: the pipeline fill of every segment on the GEN body
#endif
#ifndef MM_WIDE_ASC
#define MM_WIDE_ASC 0  // 1: levels in ascending order, each consuming the level below's row
#endif                 // of the same iteration (no pend registers; skew 2 instead of 3)

// Iterations between two consecutive levels' first inputs: 3 with the pend hand-off (level
// q+1 takes level q's row of the previous iteration: the KW level chains of one iteration
// are independent), 2 with MM_WIDE_ASC (level q+1 takes it in the same iteration: C
// registers per level fewer, the scheduler interleaves consecutive iterations instead).
constexpr int kSkew = MM_WIDE_ASC ? 2 : 3;

enum { kBodyFast = 0, kBodyEdge = 1, kBodyGen = 2 };

// What every level of a wave needs besides its windows.
template <int C>
struct WLane {
    long long H;
    int sy[C];      // column spans of this lane's columns (cnt = row span * sy - 1)
    bool eL, eR;    // EDGE body: this lane holds the grid's first column as its column 0 /
                    // its last column as its column C-1
    bool gen;       // (wave-uniform) a strip the EDGE body cannot run: every group GEN
    bool own[C];    // output cells of this workgroup
    double ownw[C]; // own as 1.0 / 0.0 (RED: the weights of the all-rows-owned groups)
};

// One level's window, per column: wa, the weight of the row above (before an even row is
// emitted) or the sum of the weights of the row above and the current row (the pair sum,
// before an odd row), the current row's weights (wm) and values (um). FAST rows hold no
// wm: there w = u, so the window is (wa, um) and wm is rebuilt from um when a FAST run of
// groups ends (wave_run).
template <int C>
struct WinC {
    double wa[C], wm[C], um[C];
};

// 8/cnt for the neighbour counts a cell can have (oracle/mm_oracle.c c8_of): the same
// correctly rounded quotients, no division at run time
__device__ __forceinline__ double c8_of(int cnt) {
    return cnt == 8 ? 1.0
                    : (cnt == 5 ? 8.0 / 5.0
                                : (cnt == 3 ? 8.0 / 3.0
                                            : (cnt == 2 ? 4.0 : (cnt == 1 ? 8.0 : 0.0))));
}

// The weights w of this lane's columns of row gx (oracle/mm_oracle.c w_row). FAST:
// interior row of an interior strip, w = u. EDGE: interior row of a strip holding the
// grid's first (or last) column as a lane's column 0 (C-1), the columns past it in whole
// lanes: the lane holding it scales that column by 8/5 (a multiply every lane issues, a
// select) -- no branch; the columns past the grid keep w = u, and wemit keeps them from
// crossing into the grid. GEN: any row (the row class sx is wave-uniform): the interior
// columns' factor and the first / last column's depend on the row only (scalar selects,
// then EDGE's arithmetic); in a strip the EDGE body cannot run (c.gen) every column by its
// own count, 0 outside the grid.
template <int C, int BODY>
__device__ __forceinline__ void procc(const WLane<C>& c, long long gx, const double (&u)[C],
                                      double (&w)[C]) {
#pragma unroll
    for (int k = 0; k < C; ++k) w[k] = u[k];
    if (BODY == kBodyEdge) {
        constexpr double k85 = 8.0 / 5.0;
        const double w0 = u[0] * k85, w1 = u[C - 1] * k85;
        w[0] = c.eL ? w0 : w[0];
        w[C - 1] = c.eR ? w1 : w[C - 1];
    } else if (BODY == kBodyGen) {
        const int sx = span3k(c.H, gx);
        if (!MM_WIDE_GEN_ROW || c.gen) {
#pragma unroll
            for (int k = 0; k < C; ++k) w[k] = u[k] * c8_of(sx * c.sy[k] - 1);
        } else {
            // 3 * sx - 1 neighbours in an interior column, 2 * sx - 1 in the first / last
            const double fr = c8_of(3 * sx - 1), fe = c8_of(2 * sx - 1);
            const double w0 = u[0] * fe, w1 = u[C - 1] * fe;
#pragma unroll
            for (int k = 0; k < C; ++k) w[k] = u[k] * fr;
            w[0] = c.eL ? w0 : w[0];
            w[C - 1] = c.eR ? w1 : w[C - 1];
        }
    }
}

// Level input m = 0 / 1 (row gx): fill the window. e1: parity of the level's first emitted
// row (the m = 1 row): odd, its window holds the pair sum of rows m = 0, 1. (e1 and wemit's
// e are constants wherever the iteration is unrolled.)
template <int C, int BODY>
__device__ __forceinline__ void wfill(const WLane<C>& c, long long gx, int m, int e1,
                                      WinC<C>& win, const double (&u)[C]) {
    double w[C];
    procc<C, BODY>(c, gx, u, w);
#pragma unroll
    for (int k = 0; k < C; ++k) {
        if (m == 0) {
            win.wa[k] = w[k];
        } else {
            if (e1) win.wa[k] = win.wa[k] + w[k];
            win.wm[k] = w[k];
            win.um[k] = u[k];
        }
    }
}

// Level input m >= 2 (row gx): emit the window's current row (gx - 1), slide the window.
// e: parity of the emitted row. Even: the pair sum of this row and the next, P = wm + wn,
// gives the column triple wa + P and stays in wa for the odd row after it, whose triple is
// P + wn (the rows paired from an even global row, oracle/mm_oracle.h). The
// columns of a lane pair the same way (C even, the lane's first column even): box sums
// cw(y-1) + (cw(y) + cw(y+1)) at even y, (cw(y-1) + cw(y)) + cw(y+1) at odd y.
template <int C, int BODY>
__device__ __forceinline__ void wemit(const WLane<C>& c, double r8, long long gx, int e,
                                      WinC<C>& win, const double (&u)[C], double (&o)[C]) {
    static_assert(C % 2 == 0, "columns paired inside a lane");
    double wn[C];
    procc<C, BODY>(c, gx, u, wn);
    double cw[C], na[C];  // na: the window's next wa
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const double wmk = BODY == kBodyFast ? win.um[k] : win.wm[k];
        const double pr = wmk + wn[k];  // (unused, and dropped, where e == 1)
        const double xk = e ? wn[k] : pr;
        cw[k] = win.wa[k] + xk;
        na[k] = e ? wmk : pr;
    }
    double left = dpp_lower(cw[C - 1]);  // cw of column y0-1 (lane-1's last column)
    double right = dpp_upper(cw[0]);     // cw of column y0+C (lane+1's first column)
    if (BODY != kBodyFast) {
        // outside the grid w = 0, so cw = 0 there: EDGE rows compute anything in the lanes
        // past the grid (procc), and GEN rows of the same strip still hold such weights in
        // their windows from the EDGE rows before them
        left = c.eL ? 0.0 : left;
        right = c.eR ? 0.0 : right;
    }
    // the emitted row's own-weight coefficients: -9 inside; EDGE: the grid's first / last
    // column 8/5 (its interior rows); GEN: by the row's span (row factors) or every column's
    // count -- 0 for a cell without neighbours (a 1 x 1 grid), which keeps its value
    double m[C];
#pragma unroll
    for (int k = 0; k < C; ++k) m[k] = kM8;
    if (BODY == kBodyEdge) {
        m[0] = c.eL ? kM5 : m[0];
        m[C - 1] = c.eR ? kM5 : m[C - 1];
    } else if (BODY == kBodyGen) {
        const int sxm = span3k(c.H, gx - 1);
        if (!MM_WIDE_GEN_ROW || c.gen) {
#pragma unroll
            for (int k = 0; k < C; ++k) m[k] = m8k(sxm * c.sy[k] - 1);
        } else {
            const double mr = m8k(3 * sxm - 1), me = m8k(2 * sxm - 1);
#pragma unroll
            for (int k = 0; k < C; ++k) m[k] = mr;
            m[0] = c.eL ? me : mr;
            m[C - 1] = c.eR ? me : mr;
        }
    }
#pragma unroll
    for (int k = 0; k < C; k += 2) {
        const double cl = k == 0 ? left : cw[k - 1];
        const double cr = k + 1 == C - 1 ? right : cw[k + 2];
        const double pk = cw[k] + cw[k + 1];
        const double s0 = cl + pk, s1 = pk + cr;
        o[k] = __builtin_fma(__builtin_fma(win.um[k], m[k], s0), r8, win.um[k]);
        o[k + 1] = __builtin_fma(__builtin_fma(win.um[k + 1], m[k + 1], s1), r8, win.um[k + 1]);
    }
#pragma unroll
    for (int k = 0; k < C; ++k) {
        win.wa[k] = na[k];
        if (BODY != kBodyFast) win.wm[k] = wn[k];
        win.um[k] = u[k];
    }
}

template <int C>
__device__ __forceinline__ void accumc(double& acc, bool row_own, const WLane<C>& c,
                                       const double (&o)[C]) {
#pragma unroll
    for (int k = 0; k < C; ++k) acc = acc + ((row_own && c.own[k]) ? o[k] : 0.0);
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
    static constexpr int S0 = kSkew * (KW - 1) + 2;  // local iterations before the last level emits
    static constexpr int D = S0 + B;
    static constexpr int RL = 2 * B;
    static constexpr int T0 = (S0 + B - 1) / B * B;  // wave 0: compile-time iterations
};

// Per-wave constants of one block (NA attributes).
template <int C, int NA>
struct WCtx {
    WLane<C> c;
    int p, lane, rA, rB;
    int oA;               // first output row (rA + 1 when the segment is shifted, wide_segment)
    int start;            // first iteration of this wave (p * D)
    int dmask;            // bit a: attribute a diffuses (NA > 1)
    long long g0;         // global row of input row 0 (rA - K)
    double r8[NA];        // rate / 8 of each attribute
    unsigned voff, soff, rowb;
    __amdgpu_buffer_rsrc_t in[NA], out[NA];
    __amdgpu_buffer_rsrc_t none;  // no records: stores through it are dropped
    dv2* lds_in;          // stage p-1 (RL row slots of 32*C*NA dv2)
    dv2* lds_out;         // stage p
    const PassArgs* A;    // transfer chains (NA > 1)
    // MM_CHAIN_ASM: register offsets of the pre / post chains' operands (chain_asm)
    int pia[kMaxChain], pib[kMaxChain], qia[kMaxChain], qib[kMaxChain];
};

template <int C, int NA, int KW, int U>
struct WState {
    WinC<C> win[KW][NA];
    double pend[KW][NA][C];  // pend[q]: level q's row of the previous iteration (q < KW-1)
    dv2 raw[U][NA][C / 2];   // first wave: prefetched input rows
    double acc[KW][NA];
};

// A transfer chain in declared order (oracle/mm_oracle.c, chain_k) on each of this lane's C
// cells: out = r*u_a; u_a -= out; u_b += out (b < 0: the outflow leaves the system); a and
// b are wave-uniform kernel arguments: chain_k's 8-wide register vector indexed with
// s_set_gpr_idx (two moves per operand access). Picking the operands with a scalar branch
// per transfer instead was 2.6x slower for C5 (profiles/r03/r3k: the branches cut the loop
// body into blocks the scheduler cannot interleave).
#ifndef MM_CHAIN_RING
#define MM_CHAIN_RING 0  // 1: pre-chains are the ring a = t, b = t+1 mod NA (engine-checked)
#endif
#ifndef MM_CHAIN_ASM
#define MM_CHAIN_ASM 0  // 1: any chain, operands indexed in the VGPR file (chain_asm)
#endif
#ifndef MM_ND
#define MM_ND 0  // N > 0: attributes 0..N-1 diffuse, the others pass through (engine-checked:
#endif           // it relabels the attributes); 0: the pass's diffuse_mask at run time
#ifndef MM_CHAIN_PRE
#define MM_CHAIN_PRE 1  // MM_CHAIN_ASM: 0 = the instance for programs without a pre-chain
#endif
#ifndef MM_CHAIN_POST
#define MM_CHAIN_POST 1  // MM_CHAIN_ASM: 0 = the instance for programs without a post-chain
#endif

typedef double dv4 __attribute__((ext_vector_type(4)));

// Run-time operands at compile-time cost (four attributes, C = 2 columns per lane): each
// column's four values sit in four consecutive register pairs, pinned to v[200:207] and
// v[210:217] (v[208:209] / v[218:219]: a pad slot that takes outflows leaving the system
// and the unused transfer slots), and the s_set_gpr_idx mode adds the wave-uniform
// register offset of u_a / u_b to the fp64 instructions themselves: per transfer and
// column the ring's 3 operations (out = r*u_a, u_a - out, u_b + out) and no moves, where
// LLVM's own indexing moves every operand through a temporary (2 v_mov_b32 each way). The
// first n transfer slots run. ia / ib: 2 * the attribute (register offset), 8 for the pad. The mode is switched off before the
// block ends; M0 (which holds the offset) is not used by the rest of the kernel.
template <int C, int NA>
__device__ __forceinline__ void chain_asm(double (&u)[NA][C], int n, const int (&ia)[kMaxChain],
                                          const int (&ib)[kMaxChain], const double* tr) {
    static_assert(NA == 4 && C == 2 && kMaxChain == 4, "four attributes, two columns");
    dv4 x = {u[0][0], u[1][0], u[2][0], u[3][0]};
    dv4 y = {u[0][1], u[1][1], u[2][1], u[3][1]};
    double px, py, o0, o1;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"  // M0: no other use in these kernels (asm checked)
#define MM_TR(T)                                                                   \
    "s_set_gpr_idx_on %[ia" #T "], gpr_idx(SRC0)\n\t"                              \
    "v_mul_f64 %[o0], v[200:201], %[r" #T "]\n\t"                                  \
    "v_mul_f64 %[o1], v[210:211], %[r" #T "]\n\t"                                  \
    "s_set_gpr_idx_off\n\t"                                                        \
    "s_set_gpr_idx_on %[ia" #T "], gpr_idx(SRC0,DST)\n\t"                          \
    "v_add_f64 v[200:201], v[200:201], -%[o0]\n\t"                                 \
    "v_add_f64 v[210:211], v[210:211], -%[o1]\n\t"                                 \
    "s_set_gpr_idx_off\n\t"                                                        \
    "s_set_gpr_idx_on %[ib" #T "], gpr_idx(SRC0,DST)\n\t"                          \
    "v_add_f64 v[200:201], v[200:201], %[o0]\n\t"                                  \
    "v_add_f64 v[210:211], v[210:211], %[o1]\n\t"                                  \
    "s_set_gpr_idx_off\n\t"
    // a chain of n < 4 transfers leaves the block after its last one: a scalar branch
    // inside the asm, so the compiler's view stays one straight-line block
#define MM_SKIP(T)                                                                 \
    "s_cmp_le_u32 %[n], " #T "\n\t"                                               \
    "s_cbranch_scc1 .Lmm_chain_end%=\n\t"
    asm volatile(MM_SKIP(0) MM_TR(0) MM_SKIP(1) MM_TR(1) MM_SKIP(2) MM_TR(2) MM_SKIP(3)
                 MM_TR(3) ".Lmm_chain_end%=:"
                 : "+{v[200:207]}"(x), "={v[208:209]}"(px), "+{v[210:217]}"(y),
                   "={v[218:219]}"(py), [o0] "=&v"(o0), [o1] "=&v"(o1)
                 : [n] "s"(n), [ia0] "s"(ia[0]), [ib0] "s"(ib[0]), [r0] "s"(tr[0]),
                   [ia1] "s"(ia[1]), [ib1] "s"(ib[1]), [r1] "s"(tr[1]),
                   [ia2] "s"(ia[2]), [ib2] "s"(ib[2]), [r2] "s"(tr[2]),
                   [ia3] "s"(ia[3]), [ib3] "s"(ib[3]), [r3] "s"(tr[3])
                 : "m0", "scc");
#undef MM_SKIP
#undef MM_TR
#pragma clang diagnostic pop
    (void)px;
    (void)py;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        u[a][0] = x[a];
        u[a][1] = y[a];
    }
}

template <int C, int NA>
__device__ __forceinline__ void chain_cols(double (&u)[NA][C], int n, const signed char* ta,
                                           const signed char* tb, const double* tr) {
#if MM_CHAIN_RING
    // the ring of transfers t -> t+1 mod NA (C5's chain): compile-time operands, 3 fp64
    // operations per transfer and cell (the engine sends only such chains here)
    (void)n;
    (void)ta;
    (void)tb;
#pragma unroll
    for (int t = 0; t < NA; ++t) {
        const double r = tr[t];
#pragma unroll
        for (int k = 0; k < C; ++k) {
            const double out = r * u[t][k];
            u[t][k] = u[t][k] - out;
            u[(t + 1) % NA][k] = u[(t + 1) % NA][k] + out;
        }
    }
#else
#pragma unroll
    for (int k = 0; k < C; ++k) {
        double v[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) v[a] = u[a][k];
        chain_k<NA>(v, n, ta, tb, tr);
#pragma unroll
        for (int a = 0; a < NA; ++a) u[a][k] = v[a];
    }
#endif
}

// The pass's pre-chain on a level's input row (NA > 1): MM_CHAIN_ASM runs the chain's
// first npre slots and leaves the asm block through a scalar branch after the last one
// (one straight-line block for the compiler; a transfer whose outflow leaves the system
// adds it to the pad pair), the other instances only when the pass has a pre-chain.
template <int C, int NA>
__device__ __forceinline__ void pre_chain(const WCtx<C, NA>& x, double (&u)[NA][C]) {
    if constexpr (NA > 1 && MM_CHAIN_ASM) {
        if (MM_CHAIN_PRE) chain_asm<C, NA>(u, x.A->npre, x.pia, x.pib, x.A->pre_r);
    } else if (NA > 1 && x.A->npre) {
        chain_cols<C, NA>(u, x.A->npre, x.A->pre_a, x.A->pre_b, x.A->pre_r);
    }
}

// One level, input m = 0 / 1: the pre-chain (NA > 1), then every attribute's window; an
// attribute that does not diffuse in this pass emits nothing (s = 0, d = u).
template <int C, int NA, int BODY>
__device__ __forceinline__ void lfill(const WCtx<C, NA>& x, long long gx, int m, int e1,
                                      WinC<C> (&w)[NA], double (&u)[NA][C]) {
    pre_chain<C, NA>(x, u);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        if (NA > 1 && !((x.dmask >> a) & 1)) {
#pragma unroll
            for (int k = 0; k < C; ++k) {
                if (m == 0) {
                    w[a].wa[k] = 0.0;
                } else {
                    w[a].wm[k] = 0.0;
                    w[a].um[k] = u[a][k];
                }
            }
        } else {
            wfill<C, BODY>(x.c, gx, m, e1, w[a], u[a]);
        }
    }
}

// One level, input m >= 2: the pre-chain, every attribute's emitted row, the post-chain
// (oracle/mm_oracle.c or_program_step's order within a pass).
template <int C, int NA, int BODY>
__device__ __forceinline__ void lemit(const WCtx<C, NA>& x, long long gx, int e, WinC<C> (&w)[NA],
                                      double (&u)[NA][C], double (&o)[NA][C]) {
    pre_chain<C, NA>(x, u);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        if (NA > 1 && !((x.dmask >> a) & 1)) {
#pragma unroll
            for (int k = 0; k < C; ++k) {
                o[a][k] = w[a].um[k];
                w[a].wa[k] = 0.0;
                w[a].wm[k] = 0.0;
                w[a].um[k] = u[a][k];
            }
        } else {
            wemit<C, BODY>(x.c, x.r8[a], gx, e, w[a], u[a], o[a]);
        }
    }
    if constexpr (NA > 1 && MM_CHAIN_ASM) {
        if (MM_CHAIN_POST) chain_asm<C, NA>(o, x.A->npost, x.qia, x.qib, x.A->post_r);
    } else if (NA > 1 && !MM_CHAIN_RING && x.A->npost) {
        chain_cols<C, NA>(o, x.A->npost, x.A->post_a, x.A->post_b, x.A->post_r);
    }
}

// One iteration i of a wave (local iteration t = i - start): input row -> its KW levels
// (descending, so pend[q-1] is read before level q-1 refills it; ascending with
// MM_WIDE_ASC) -> level KW-1's row to LDS or HBM. PRO: t is a prologue iteration known at
// compile time (level q takes part from t = kSkew*q and emits from t = kSkew*q + 2);
// otherwise every level emits. slot: ring slot (first wave, compile time after unrolling).
// PP: parity of the wave's p; tp: parity of t. With g0 even (wide_segment) they give every
// level's row parities -- level q's input m = t - kSkew*q is global row g0 + p*KW + q + m,
// its emitted row the one before -- as constants wherever the iteration is unrolled (the
// steady groups, the prologue); elsewhere e / e1 are wave-uniform branches.
template <int C, int NA, int KW, int P, int U, int B, bool RED, int NT, int BODY, int ROLE,
          bool PRO, int PP, bool OWNED = false>
__device__ __forceinline__ void wave_iter(const WCtx<C, NA>& x, WState<C, NA, KW, U>& st, int i,
                                          int t, int slot, int tp) {
    constexpr int PK = (PP * KW) & 1;
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    constexpr int H2 = C / 2;       // 16-B pieces per lane, row and attribute
    constexpr int RW = 32 * C * NA; // dv2 per LDS row
    constexpr bool kIn = ROLE == kRoleFirst || ROLE == kRoleOnly;   // input from HBM
    constexpr bool kOut = ROLE == kRoleLast || ROLE == kRoleOnly;  // output to HBM
    double cur[NA][C];  // the row level q consumes
    if (kIn) {
#pragma unroll
        for (int a = 0; a < NA; ++a) {
#pragma unroll
            for (int h = 0; h < H2; ++h) {
#if MM_LOAD_COPY
                cur[a][2 * h] = vcopy(st.raw[slot][a][h].x);
                cur[a][2 * h + 1] = vcopy(st.raw[slot][a][h].y);
#else
                cur[a][2 * h] = st.raw[slot][a][h].x;
                cur[a][2 * h + 1] = st.raw[slot][a][h].y;
#endif
            }
        }
        if (BODY == kBodyGen) {
            // the GEN body weights every column by its own count, 0 outside the grid
            // (w = u * 0): a column past the grid enters as 0, whatever the pitch padding
            // holds, as the OOB loads left of the grid do (EDGE / FAST rows keep such
            // columns out of the grid at the DPP hand-off instead)
#pragma unroll
            for (int a = 0; a < NA; ++a) {
#pragma unroll
                for (int k = 0; k < C; ++k) cur[a][k] = x.c.sy[k] == 0 ? 0.0 : cur[a][k];
            }
        }
        const unsigned o = x.voff + (unsigned)(i + U) * x.rowb;  // x.voff: row -shift
#pragma unroll
        for (int a = 0; a < NA; ++a) {
#pragma unroll
            for (int h = 0; h < H2; ++h) st.raw[slot][a][h] = load_row(x.in[a], o + 16 * h);
        }
    } else {
        const dv2* src = x.lds_in + ((i - G::B) % G::RL) * RW;  // i >= start >= D > B
#pragma unroll
        for (int a = 0; a < NA; ++a) {
#pragma unroll
            for (int h = 0; h < H2; ++h) {
                const dv2 v = src[64 * (a * H2 + h) + x.lane];
                cur[a][2 * h] = v.x;
                cur[a][2 * h + 1] = v.y;
            }
        }
    }
    if (!PRO) t = i - x.start;
    double uin[NA][C];  // descending order: level 0's input
#pragma unroll
    for (int a = 0; a < NA; ++a) {
#pragma unroll
        for (int k = 0; k < C; ++k) uin[a][k] = cur[a][k];
    }
#pragma unroll
    for (int qq = 0; qq < KW; ++qq) {
        const int q = kSkew == 2 ? qq : KW - 1 - qq;
        const int m = t - kSkew * q;  // this level's input index
        if (PRO && m < 0) continue;  // compile time
        const int j = x.p * KW + q + 1;  // global level, 1-based
        const long long gx = x.g0 + (j - 1) + m;
        double u[NA][C];
#pragma unroll
        for (int a = 0; a < NA; ++a) {
#pragma unroll
            for (int k = 0; k < C; ++k)
                u[a][k] = kSkew == 2 ? cur[a][k] : (q == 0 ? uin[a][k] : st.pend[q - 1][a][k]);
        }
        // row parities (constants once the level loop is unrolled): e1 of row g0 + j, the
        // level's first emitted row; e of the row emitted now, gx - 1 = g0 + j + m - 2
        const int e1 = (PK + q + 1) & 1;
        const int e = (PK + q + 1 + tp - kSkew * q) & 1;
        if (PRO && m < 2) {
            lfill<C, NA, BODY>(x, gx, m, e1, st.win[q], u);
            continue;
        }
        double o[NA][C];
        lemit<C, NA, BODY>(x, gx, e, st.win[q], u, o);
        if (RED) {
            if constexpr (OWNED) {
                // every level's row of this iteration is an output row: the lane's fixed
                // column weights (1 owned, 0 not), one fma per column -- fma(o, 1, acc) is
                // acc + o, fma(o, 0, acc) is acc -- instead of a select and an add
#pragma unroll
                for (int a = 0; a < NA; ++a) {
#pragma unroll
                    for (int k = 0; k < C; ++k)
                        st.acc[q][a] = __builtin_fma(o[a][k], x.c.ownw[k], st.acc[q][a]);
                    asm volatile("" : "+v"(st.acc[q][a]));
                }
            } else {
                const int r = x.rA - K + m + j - 2;  // output row of level j
#pragma unroll
                for (int a = 0; a < NA; ++a) accumc<C>(st.acc[q][a], r >= x.oA && r < x.rB, x.c, o[a]);
            }
        }
        if (q == KW - 1) {
            if (kOut) {  // level K: output row m - 2 of the segment, row m - 2 - shift of out
                const int ro = m - 2 - (x.oA - x.rA);
                const unsigned so = x.soff + (unsigned)(ro < 0 ? 0 : ro) * x.rowb;
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    // a shifted segment's first row (above its rows, wide_segment) is dropped
                    // through a descriptor of no records (a scalar select)
                    const __amdgpu_buffer_rsrc_t rs = ro < 0 ? x.none : x.out[a];
#pragma unroll
                    for (int h = 0; h < H2; ++h)
                        store_row<NT>(rs, so + 16 * h, o[a][2 * h], o[a][2 * h + 1]);
                }
            } else {
                dv2* dst = x.lds_out + (i % G::RL) * RW;
#pragma unroll
                for (int a = 0; a < NA; ++a) {
#pragma unroll
                    for (int h = 0; h < H2; ++h) {
                        dv2 v;
                        v.x = o[a][2 * h];
                        v.y = o[a][2 * h + 1];
                        dst[64 * (a * H2 + h) + x.lane] = v;
                    }
                }
            }
        } else {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
#pragma unroll
                for (int k = 0; k < C; ++k) {
                    if (kSkew == 2)
                        cur[a][k] = o[a][k];
                    else
                        st.pend[q][a][k] = o[a][k];
                }
            }
        }
    }
}

// the barrier that closes iteration i when it ends a group
template <int P, int B>
__device__ __forceinline__ void group_end(int i) {
    if (P > 1 && (i + 1) % B == 0) wg_sync();
}

// Steady groups [b0, b1) (multiples of B) of one wave, B iterations per loop trip (ring
// slot i mod U: U divides B). B is even, so iteration base + tt has t = i - p*D of parity
// tt + p*D: a constant per unrolled iteration.
template <int C, int NA, int KW, int P, int U, int B, bool RED, int NT, int BODY, int ROLE,
          int PP, bool OWNED = false>
__device__ __forceinline__ void wave_groups(const WCtx<C, NA>& x, WState<C, NA, KW, U>& st,
                                            int b0, int b1) {
    static_assert(B % 2 == 0, "row pairs: an even number of iterations per group");
    constexpr int PD = (PP * WGeom<KW, P, B>::D) & 1;
    for (int base = b0; base < b1; base += B) {
#pragma unroll
        for (int tt = 0; tt < B; ++tt)
            wave_iter<C, NA, KW, P, U, B, RED, NT, BODY, ROLE, false, PP, OWNED>(
                x, st, base + tt, 0, tt % U, (tt + PD) & 1);
        if (P > 1) wg_sync();
    }
}

// The pipeline fill of one wave (its first input rows, every level joining in turn) up to
// its first group boundary, on the BODY rows' code; returns the first iteration of the
// group loop. The first wave loads U rows ahead and starts at iteration 0 (its ring slots
// compile-time); the others join the barriers until their start.
template <int C, int NA, int KW, int P, int U, int B, bool RED, int NT, int ROLE, int BODY,
          int PP>
__device__ __forceinline__ int wave_prologue(const WCtx<C, NA>& x, WState<C, NA, KW, U>& st) {
    using G = WGeom<KW, P, B>;
    constexpr bool kIn = ROLE == kRoleFirst || ROLE == kRoleOnly;
    if (kIn) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
#pragma unroll
                for (int h = 0; h < C / 2; ++h)
                    st.raw[k][a][h] = load_row(x.in[a], x.voff + 16 * h + k * x.rowb);
            }
        }
#pragma unroll
        for (int t = 0; t < G::T0; ++t) {
            if (t < G::S0)
                wave_iter<C, NA, KW, P, U, B, RED, NT, BODY, ROLE, true, PP>(x, st, t, t, t % U,
                                                                             t & 1);
            else
                wave_iter<C, NA, KW, P, U, B, RED, NT, BODY, ROLE, false, PP>(x, st, t, 0, t % U,
                                                                              t & 1);
            if (P > 1 && (t + 1) % B == 0) wg_sync();
        }
        return G::T0;
    }
    for (int i = 0; i < x.start; ++i) group_end<P, B>(i);
#pragma unroll
    for (int t = 0; t < G::S0; ++t) {
        wave_iter<C, NA, KW, P, U, B, RED, NT, BODY, ROLE, true, PP>(x, st, x.start + t, t, 0,
                                                                     t & 1);
        group_end<P, B>(x.start + t);
    }
    // up to the next group boundary (fewer than B iterations; the row parities are
    // wave-uniform values here, selects instead of constants)
    int s = x.start + G::S0;
    for (; s % B != 0; ++s) {
        wave_iter<C, NA, KW, P, U, B, RED, NT, BODY, ROLE, false, PP>(x, st, s, 0, 0,
                                                                      (s - x.start) & 1);
        group_end<P, B>(s);
    }
    return s;
}

// The whole schedule of one wave. MID: body of the groups whose rows are all interior.
// RED: every level's sum of this wave's owned cells is added to carry[level][attribute]
// (wave-uniform), so a workgroup that runs several segments sums them all.
template <int C, int NA, int KW, int P, int U, int B, bool RED, int NT, int ROLE, int MID,
          int PP>
__device__ __forceinline__ void wave_run(const WCtx<C, NA>& x, int iend,
                                         double (&carry)[KW][NA]) {
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    static_assert(B % U == 0, "ring slots repeat within a group");
    WState<C, NA, KW, U> st;
#pragma unroll
    for (int q = 0; q < KW; ++q) {
#pragma unroll
        for (int a = 0; a < NA; ++a) st.acc[q][a] = 0.0;
    }
    // the pipeline fill on the MID body where the segment's first input rows are interior
    // rows (every segment but the grid's first and its thin last ones): on the GEN body it
    // cost ~4 % of a 2541-row K = 20 segment's time
    const bool pro_mid =
        MM_WIDE_PRO_MID && !(MID == kBodyEdge && x.c.gen) && x.g0 >= 2 &&
        x.g0 + (long long)(G::T0 + (P - 1) * G::D + 2 * K + 2 * B) < x.c.H - 1;
    const int s = pro_mid ? wave_prologue<C, NA, KW, P, U, B, RED, NT, ROLE, MID, PP>(x, st)
                          : wave_prologue<C, NA, KW, P, U, B, RED, NT, ROLE, kBodyGen, PP>(x, st);
    if (MID == kBodyFast && pro_mid) {  // FAST rows hold no wm (w = u): GEN groups may follow
#pragma unroll
        for (int q = 0; q < KW; ++q) {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
#pragma unroll
                for (int k = 0; k < C; ++k) st.win[q][a].wm[k] = st.win[q][a].um[k];
            }
        }
    }
    // groups whose levels all read interior rows and emit from interior rows: level j
    // reads row g0 + (j-1) + m, m = i - start - kSkew*q, i.e. rows g0 + p*KW + (i - start) -
    // (kSkew-1)q, q < KW, and emits the row before it (FAST takes its w = u)
    const long long base = x.g0 + (long long)x.p * KW - x.start;
    const long long lo = 2 + (kSkew - 1) * (KW - 1) - base;  // first i with every row >= 2
    const long long hi = x.c.H - 1 - base;         // first i with a row > H-2
    long long f0 = lo <= s ? s : s + (lo - s + B - 1) / B * B;
    long long f1 = hi <= s ? s : s + (hi - s) / B * B;
    f0 = min(f0, (long long)iend);
    f1 = max(f0, min(f1, (long long)iend));
    if (MID == kBodyEdge && x.c.gen) f0 = f1 = iend;  // a strip the EDGE body cannot run
    wave_groups<C, NA, KW, P, U, B, RED, NT, kBodyGen, ROLE, PP>(x, st, s, (int)f0);
    if (RED) {
        // inside the interior groups, those whose every level's output row lies in
        // [rA, rB) (level q's row: rA - K - 1 + (i - start) + p*KW - (kSkew-1) q) sum with
        // the lanes' fixed weights (wave_iter OWNED)
        const long long r0 = x.start + K + 1 - (long long)x.p * KW + (kSkew - 1) * (KW - 1) +
                             (x.oA - x.rA);
        const long long r1 = x.start + (x.rB - x.rA) + K + 1 - (long long)x.p * KW;
        long long m0 = (r0 + B - 1) / B * B, m1 = r1 / B * B;
        m0 = min(max(m0, f0), f1);
        m1 = max(m0, min(m1, f1));
        wave_groups<C, NA, KW, P, U, B, RED, NT, MID, ROLE, PP>(x, st, (int)f0, (int)m0);
        wave_groups<C, NA, KW, P, U, B, RED, NT, MID, ROLE, PP, true>(x, st, (int)m0, (int)m1);
        wave_groups<C, NA, KW, P, U, B, RED, NT, MID, ROLE, PP>(x, st, (int)m1, (int)f1);
    } else {
        wave_groups<C, NA, KW, P, U, B, RED, NT, MID, ROLE, PP>(x, st, (int)f0, (int)f1);
    }
    if (MID == kBodyFast && f1 > f0) {  // FAST rows hold no wm (w = u there): rebuild it
#pragma unroll
        for (int q = 0; q < KW; ++q) {
#pragma unroll
            for (int a = 0; a < NA; ++a) {
#pragma unroll
                for (int k = 0; k < C; ++k) st.win[q][a].wm[k] = st.win[q][a].um[k];
            }
        }
    }
    wave_groups<C, NA, KW, P, U, B, RED, NT, kBodyGen, ROLE, PP>(x, st, (int)f1, iend);
    if (RED) {
        // the OWNED groups add fma(o, 0, acc) in the columns a lane does not own: lanes that
        // own none (halo lanes, lanes past the grid, which read the pitch padding) leave the
        // sum here, so no value they hold can reach it. The padding columns inside the
        // grid's last lane (W % C != 0) hold only what this kernel stored there: zero at
        // creation (mm_engine_create), host copies write W columns.
        const bool lane_owns = x.c.own[0];
#pragma unroll
        for (int q = 0; q < KW; ++q) {
#pragma unroll
            for (int a = 0; a < NA; ++a)
                carry[q][a] = carry[q][a] + wave_sum_k(lane_owns ? st.acc[q][a] : 0.0);
        }
    }
}

template <int C, int NA, int KW, int P, int U, int B, bool RED, int NT, int MID>
__device__ __forceinline__ void wave_dispatch(const WCtx<C, NA>& x, int iend,
                                              double (&carry)[KW][NA]) {
    // the parity of p fixes the rows' parities of each role's code (wave_iter); the middle
    // waves run one instance per parity when it matters (KW or D odd)
    constexpr bool kMidPar = ((KW | WGeom<KW, P, B>::D) & 1) != 0;
    if (P == 1)
        wave_run<C, NA, KW, P, U, B, RED, NT, kRoleOnly, MID, 0>(x, iend, carry);
    else if (x.p == 0)
        wave_run<C, NA, KW, P, U, B, RED, NT, kRoleFirst, MID, 0>(x, iend, carry);
    else if (x.p == P - 1)
        wave_run<C, NA, KW, P, U, B, RED, NT, kRoleLast, MID, (P - 1) & 1>(x, iend, carry);
    else if (kMidPar && (x.p & 1))
        wave_run<C, NA, KW, P, U, B, RED, NT, kRoleMid, MID, 1>(x, iend, carry);
    else
        wave_run<C, NA, KW, P, U, B, RED, NT, kRoleMid, MID, 0>(x, iend, carry);
}

// One strip segment [rA, rB) (local rows) of strip `strip`: this wave's part of it (level
// group p), adding the level sums to carry (RED).
template <int C, int NA, int KW, int P, int U, int B, bool RED, int NT>
__device__ __forceinline__ void wide_segment(const PassArgs& A, dv2* lds, int p, int lane,
                                             int strip, int rA, int rB,
                                             double (&carry)[KW][NA]) {
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    constexpr int LH = (K + C - 1) / C;       // halo lanes per side
    constexpr int OC = 64 * C - 2 * C * LH;   // output columns per strip
    constexpr int RW = 32 * C * NA;           // dv2 per LDS row
    WCtx<C, NA> x;
    // Rows are paired from an even global row (wemit), and the row parities of each role's
    // code are constants for an even g0, the segment's first input row: a segment whose g0
    // is odd starts one row higher -- an extra first input row that loads as 0 and an extra
    // first output row that no level-K store writes and no sum counts (its value depends
    // on that 0 row; the rows below it do not).
    const int sh = (int)((A.x_init + rA - K) & 1);
    x.rA = rA - sh;
    x.oA = rA;
    x.rB = rB;
    const long long W = A.W;
    // first loaded column: the strip's span starts C * LH columns before its first output
    // column
    const long long c0 = (long long)strip * OC - C * LH;
    const long long y0 = c0 + C * lane;
    const bool in_row = y0 >= 0 && y0 < A.pitch;  // y0 % C == 0, pitch % 128 == 0
    const bool store_lane = lane >= LH && lane < 64 - LH && y0 < W;
    x.rowb = (unsigned)(A.pitch * 8);
    // input row k of the segment is row k - sh of the descriptor (base row rA - K): row -1
    // wraps past num_records (loads 0) in every lane that loads inside the pitch
    x.voff = (in_row ? (unsigned)(y0 * 8) : kOOBk) - (unsigned)sh * x.rowb;
    // columns past W inside the pitch are padding: writing them is harmless
    x.soff = store_lane ? (unsigned)(y0 * 8) : kOOBk;
    x.c.H = A.H;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        x.c.sy[k] = span3k(W, y0 + k);
        x.c.own[k] = store_lane && y0 + k < W;
        x.c.ownw[k] = x.c.own[k] ? 1.0 : 0.0;
    }
    x.p = p;
    x.lane = lane;
    x.start = p * G::D;
    // MM_ND: the diffusion mask at compile time -- the per-attribute pass-through branch of
    // lfill / lemit folds away (C5: 262 -> 290 GCUPS with run-time chain operands, 294 ->
    // 312 with the ring's, profiles/r04/r4e)
    x.dmask = MM_ND ? (1 << MM_ND) - 1 : A.diffuse_mask;
    x.g0 = A.x_init + x.rA - K;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        x.r8[a] = A.drate[a] * 0.125;
        x.in[a] = rows_rsrc(A.in[a] + (long long)(rA - K) * A.pitch, rB - rA + 2 * K, A.pitch);
        x.out[a] = rows_rsrc(A.out[a] + (long long)rA * A.pitch, rB - rA, A.pitch);
    }
    x.none = rows_rsrc(A.out[0], 0, A.pitch);
    x.lds_in = p > 0 ? lds + (p - 1) * G::RL * RW : lds;
    x.lds_out = p < P - 1 ? lds + p * G::RL * RW : lds;
    x.A = &A;
    if (MM_CHAIN_ASM) {  // register offsets of the chains' operands: 2 * attribute, 8 = pad
#pragma unroll
        for (int t = 0; t < kMaxChain; ++t) {
            const bool pu = t < A.npre, qu = t < A.npost;
            x.pia[t] = pu ? 2 * A.pre_a[t] : 8;
            x.pib[t] = pu && A.pre_b[t] >= 0 ? 2 * A.pre_b[t] : 8;
            x.qia[t] = qu ? 2 * A.post_a[t] : 8;
            x.qib[t] = qu && A.post_b[t] >= 0 ? 2 * A.post_b[t] : 8;
        }
    }
    // every wave runs to iteration iend (a whole number of groups): the last wave emits
    // the segment's last row at iteration (P-1)*D + S0 + R - 1
    const int need = (P - 1) * G::D + G::S0 + (x.rB - x.rA);
    const int iend = (need + G::B - 1) / G::B * G::B;
    // a strip whose loaded columns include the grid's first / last column or columns past
    // it: EDGE when it holds one of the two as a lane's column 0 / C-1 (the first column
    // always is: c0 % C == 0; the last one when W % C == 0), GEN otherwise
    const bool hasL = c0 < 1, hasR = c0 + 64 * C - 1 >= W - 1;
    x.c.eL = hasL && y0 == 0;
    x.c.eR = hasR && y0 + C - 1 == W - 1;
    // (both, or the last column inside a lane: GEN for every group, the old fix-up)
    x.c.gen = (hasL && hasR) || (hasR && (W - 1 - c0) % C != C - 1);
    if (!hasL && !hasR)
        wave_dispatch<C, NA, KW, P, U, B, RED, NT, kBodyFast>(x, iend, carry);
    else
        wave_dispatch<C, NA, KW, P, U, B, RED, NT, kBodyEdge>(x, iend, carry);
}

// K = KW * P fused steps per launch of an NA-attribute one-pass program (NA = 1: one
// diffusion; NA > 1: pre-chain, diffusions of the attributes in diffuse_mask, post-chain),
// C columns per lane, MW waves per SIMD, P waves per workgroup, one workgroup per strip
// segment by mm_passk.hpp's seg_map with blocks in place of waves -- the two edge strips
// first (A.th_edge rows), then the others (A.th rows). RED: every level's sums of the
// workgroup's output cells into partials[partial_base + block][K][NA]. NT & 1:
// non-temporal stores.
template <int C, int NA, int KW, int P, int MW, int U, int B, bool RED, int NT>
__global__ __launch_bounds__(64 * P, MW) void mm_wide_kernel(const PassArgs A) {
    using G = WGeom<KW, P, B>;
    constexpr int K = G::K;
    constexpr int RW = 32 * C * NA;  // dv2 per LDS row
    __shared__ dv2 lds[(P > 1 ? P - 1 : 1) * G::RL * RW];
    const int lane = threadIdx.x & 63;
    const int p = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // level group
    const long long blk = blockIdx.x;
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
    int strip, rA, rB;
    seg_map(w, rlo, rhi, A.nstrips, A.th, A.th_edge, strip, rA, rB);
    double carry[KW][NA];
#pragma unroll
    for (int q = 0; q < KW; ++q) {
#pragma unroll
        for (int a = 0; a < NA; ++a) carry[q][a] = 0.0;
    }
    wide_segment<C, NA, KW, P, U, B, RED, NT>(A, lds, p, lane, strip, rA, rB, carry);
    if (RED && lane == 0) {  // partials[partial_base + block][K][NA]: this wave's KW levels
#pragma unroll
        for (int q = 0; q < KW; ++q) {
#pragma unroll
            for (int a = 0; a < NA; ++a)
                A.partials[((A.partial_base + blk) * K + p * KW + q) * NA + a] = carry[q][a];
        }
    }
}

template <int C, int NA, int KW, int P, int MW, int NT>
hipError_t wide_launch3(bool red, const PassArgs& a, hipStream_t s) {
    constexpr int U = MM_WIDE_U;
    // at least one workgroup: a dispatch with no work (mm_prepare) still reaches the queue
    const dim3 g((unsigned)std::max<long long>(a.waves_total, 1)), b(64 * P);
    (void)hipGetLastError();  // the status below is this launch's, not an earlier call's
    if (red)
        hipLaunchKernelGGL((mm_wide_kernel<C, NA, KW, P, MW, U, MM_WIDE_B, true, NT>), g, b, 0, s, a);
    else
        hipLaunchKernelGGL((mm_wide_kernel<C, NA, KW, P, MW, U, MM_WIDE_B, false, NT>), g, b, 0, s, a);
    return hipGetLastError();
}

// one instance (a translation unit per instance builds in parallel: mm_wide_k20.hip)
template <int C, int NA, int KW, int P, int MW, bool RED, int NT>
hipError_t wide_launch4(const PassArgs& a, hipStream_t s) {
    if (!a.seg) return hipErrorInvalidValue;
    // at least one workgroup: a dispatch with no work (mm_prepare) still reaches the queue
    const dim3 g((unsigned)std::max<long long>(a.waves_total, 1)), b(64 * P);
    (void)hipGetLastError();  // the status below is this launch's, not an earlier call's
    hipLaunchKernelGGL((mm_wide_kernel<C, NA, KW, P, MW, MM_WIDE_U, MM_WIDE_B, RED, NT>), g, b, 0,
                       s, a);
    return hipGetLastError();
}

// a.seg must be set (segment schedule); variant bit 0: non-temporal stores.
template <int C, int NA, int KW, int P, int MW>
hipError_t wide_launch2(bool red, const PassArgs& a, hipStream_t s, int v) {
    if (!a.seg) return hipErrorInvalidValue;
    return (v & 1) ? wide_launch3<C, NA, KW, P, MW, 1>(red, a, s)
                   : wide_launch3<C, NA, KW, P, MW, 0>(red, a, s);
}

// Resident workgroups per CU, from the kernel's registers (512 per SIMD lane, granules of
// 8, at most 8 waves per SIMD) and its LDS (160 KiB per CU); see seg_blocks_per_cu_v.
template <int C, int NA, int KW, int P, int MW, bool RED, int NT>
int wide_blocks_v() {
    hipFuncAttributes fa;
    const hipError_t e = hipFuncGetAttributes(
        &fa, reinterpret_cast<const void*>(
                 mm_wide_kernel<C, NA, KW, P, MW, MM_WIDE_U, MM_WIDE_B, RED, NT>));
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

template <int C, int NA, int KW, int P, int MW>
int wide_blocks(bool red, int nt) {
    if (red)
        return nt ? wide_blocks_v<C, NA, KW, P, MW, true, 1>()
                  : wide_blocks_v<C, NA, KW, P, MW, true, 0>();
    return nt ? wide_blocks_v<C, NA, KW, P, MW, false, 1>()
              : wide_blocks_v<C, NA, KW, P, MW, false, 0>();
}

}  // namespace

}  // namespace mm
