// mm_kernels.hip -- gfx950 kernels for the MPI-Model flow step.
//
// Hot path: mm_pass_kernel, the whole-grid Exponencial step (the
// generalisation of src/Model.hpp:176-235 + src/Exponencial.hpp:18-20 to every
// cell and every step). It is HBM-bound (about 11 fp64 flop per 16 B), so the
// design is all about streaming:
//   * one wave owns a strip of 128 columns x th rows; lane l holds columns
//     2l, 2l+1 and moves them as one 16-B double2 (1 KiB per wave-instruction,
//     fully coalesced row-major loads and stores);
//   * the wave slides DOWN its strip keeping three rows of shares s in
//     registers, so the x-1 / x+1 neighbours cost no memory traffic;
//   * the y-1 / y+1 neighbours come from the adjacent lanes through DPP
//     wave_shr:1 / wave_shl:1 (no LDS, no barrier); lanes 0 and 63 additionally
//     load the one column left / right of the strip;
//   * rows are prefetched U at a time so every wave keeps U KiB in flight.
// The K-step temporal-blocking kernel (the single-attribute hot path) lives in
// mm_passk.hpp; this one-step kernel runs flow programs that need more than one pass
// per step, and every program when MM_PASSK=0.
// Layout: every buffer pointer points at owned row 0 of the slab; rows -kGhost..-1 and
// h..h+kGhost-1 are ghost rows (global row = x_init + local row).
// Arithmetic order is the contract in oracle/mm_oracle.h; the .so is built with
// -ffp-contract=off so no multiply/add pair is fused.
#include "mm_internal.hpp"

namespace mm {

namespace {

__device__ __forceinline__ double dpp_from_lower_lane(double src, double old) {
    // lane i <- lane i-1 (wave_shr:1); lane 0 keeps `old`
    const long long s = __double_as_longlong(src), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), 0x138, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double dpp_from_upper_lane(double src, double old) {
    // lane i <- lane i+1 (wave_shl:1); lane 63 keeps `old`
    const long long s = __double_as_longlong(src), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)s, 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(s >> 32), 0x130, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1 + (i > 0) + (i < n-1) inside [0, n), 0 outside: cnt = span(x)*span(y) - 1
__device__ __forceinline__ int span3(long long n, long long i) {
    return (i >= 0 && i < n) ? 1 + (i > 0) + (i < n - 1) : 0;
}

// share of one emitter of the reference's single-source flow (src/Model.hpp:199); cnt ==
// 8 as the exact *0.125
__device__ __forceinline__ double share_of(double out, int cnt) {
    return cnt == 8 ? out * 0.125 : (cnt > 0 ? out / (double)cnt : 0.0);
}

// A neighbour's weight in the whole-grid step (oracle/mm_oracle.c c8_of): w = u * 8/cnt,
// u itself for cnt == 8, 0 outside the grid -- each neighbour's share out/cnt is (r/8) * w.
__device__ __forceinline__ double c8_one(int cnt) {
    return cnt == 8 ? 1.0
                    : (cnt == 5 ? 8.0 / 5.0
                                : (cnt == 3 ? 8.0 / 3.0
                                            : (cnt == 2 ? 4.0 : (cnt == 1 ? 8.0 : 0.0))));
}

// The own-weight coefficient of the box sum (oracle/mm_oracle.c m_of): -(8 + 8/cnt), 0 for a
// cell without neighbours (it keeps its value) or outside the grid.
__device__ __forceinline__ double m8_one(int cnt) {
    return cnt == 8 ? -9.0
                    : (cnt == 5 ? -(8.0 + 8.0 / 5.0)
                                : (cnt == 3 ? -(8.0 + 8.0 / 3.0)
                                            : (cnt == 2 ? -12.0 : (cnt == 1 ? -16.0 : 0.0))));
}

// Chain entries are read with compile-time indices only, so they are scalar loads of
// the kernel arguments that the compiler hoists out of the row loop (a runtime index
// into the by-value PassArgs turns into per-row global loads and vmcnt(0) waits that
// drain the row prefetch). The attribute values sit in one 8-element register vector for
// the chain, indexed by the wave-uniform a / b with s_set_gpr_idx (mm_passk.hpp chain_k);
// a pad slot takes the outflows that leave the system.
template <int NA>
__device__ __forceinline__ void apply_chain(double (&u)[NA], int n, const signed char* ta,
                                            const signed char* tb, const double* tr) {
    static_assert(NA < 8, "one pad slot");
    typedef double dv8 __attribute__((ext_vector_type(8)));
    dv8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = k < NA ? u[k] : 0.0;
#pragma unroll
    for (int t = 0; t < kMaxChain; ++t) {
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

// Raw values of one row as this lane sees them: its two columns + its edge column.
template <int NA>
struct RawRow {
    double v0[NA], v1[NA], ve[NA];
};

// Processed row: weights (three columns), values and the own-weight coefficient
// -(8 + 8/cnt) of the box sum (0 for a cell without neighbours) of the two own columns.
template <int NA>
struct ProcRow {
    double w0[NA], w1[NA], we[NA];
    double u0[NA], u1[NA];
    double m0, m1;
};

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr unsigned kOOB = 0x80000000u;  // voffset past any num_records: loads 0, stores dropped

// Buffer descriptor of local row r of one attribute buffer. Rows outside [0, rmax] get
// num_records = 0: their loads return 0 and their stores are dropped with no memory
// traffic, so every loop iteration issues the same memory instructions (the compiler
// can then keep counted vmcnt waits across the loop instead of draining it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double* buf, int r, int rmax,
                                                           long long pitch) {
    const bool ok = r <= rmax;
    const double* p = buf + (long long)(ok ? r : 0) * pitch;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0,
                                             ok ? (int)(pitch * 8) : 0, 0x00020000);
}

// NT bit 1: non-temporal loads; bit 0: non-temporal stores
template <int NA, int NT>
__device__ __forceinline__ void load_row(const PassArgs& A, int r, int rmax, unsigned voff,
                                         unsigned eoff, RawRow<NA>& o) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        const __amdgpu_buffer_rsrc_t rs = row_rsrc(A.in[a], r, rmax, A.pitch);
        const dv2 p = __builtin_bit_cast(
            dv2, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, (NT & 2) ? 2 : 0));
        o.v0[a] = p.x;
        o.v1[a] = p.y;
        o.ve[a] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, eoff, 0, 0));
    }
}

template <int NA, bool CHAIN>
__device__ __forceinline__ void process_row(const PassArgs& A, int r, const RawRow<NA>& raw,
                                            bool fast_cols, int sy0, int sy1, int sye,
                                            ProcRow<NA>& o) {
    const long long gx = A.x_init + r;
    const int sx = span3(A.H, gx);
    double u0[NA], u1[NA], ue[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        u0[a] = raw.v0[a];
        u1[a] = raw.v1[a];
        ue[a] = raw.ve[a];
    }
    if (CHAIN && A.npre) {
        apply_chain<NA>(u0, A.npre, A.pre_a, A.pre_b, A.pre_r);
        apply_chain<NA>(u1, A.npre, A.pre_a, A.pre_b, A.pre_r);
        apply_chain<NA>(ue, A.npre, A.pre_a, A.pre_b, A.pre_r);
    }
    o.m0 = m8_one(sx * sy0 - 1);
    o.m1 = m8_one(sx * sy1 - 1);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        o.u0[a] = u0[a];
        o.u1[a] = u1[a];
    }
    if (sx == 3 && fast_cols) {  // interior rows and columns: cnt == 8 everywhere, w = u
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const bool dif = A.diffuse_mask & (1 << a);
            o.w0[a] = dif ? u0[a] : 0.0;
            o.w1[a] = dif ? u1[a] : 0.0;
            o.we[a] = dif ? ue[a] : 0.0;
        }
        return;
    }
    // (sx == 0: a row outside the global grid weighs 0; a column outside it -- the pitch
    // padding -- weighs 0 by select, so no value it holds reaches a cell)
    const double c0 = c8_one(sx * sy0 - 1), c1 = c8_one(sx * sy1 - 1), ce = c8_one(sx * sye - 1);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        const bool dif = A.diffuse_mask & (1 << a);
        o.w0[a] = (dif && sy0) ? u0[a] * c0 : 0.0;
        o.w1[a] = (dif && sy1) ? u1[a] * c1 : 0.0;
        o.we[a] = (dif && sye) ? ue[a] * ce : 0.0;
    }
}

template <int NA, bool REDUCE, int NT, bool CHAIN>
__device__ __forceinline__ void emit_row(const PassArgs& A, int r, int rmax, unsigned voff,
                                         bool st2, bool st1, const ProcRow<NA>& P,
                                         const ProcRow<NA>& C, const ProcRow<NA>& N,
                                         double (&acc)[NA]) {
    double w0[NA], w1[NA];
    // the column triples pair the rows from an even global row: row x even
    // w(x-1) + (w(x) + w(x+1)), odd (w(x-1) + w(x)) + w(x+1) (wave-uniform branch)
    const bool even = ((A.x_init + r) & 1) == 0;
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        if (A.diffuse_mask & (1 << a)) {
            double c0, c1, ce;
            if (even) {
                c0 = P.w0[a] + (C.w0[a] + N.w0[a]);
                c1 = P.w1[a] + (C.w1[a] + N.w1[a]);
                ce = P.we[a] + (C.we[a] + N.we[a]);
            } else {
                c0 = (P.w0[a] + C.w0[a]) + N.w0[a];
                c1 = (P.w1[a] + C.w1[a]) + N.w1[a];
                ce = (P.we[a] + C.we[a]) + N.we[a];
            }
            const double left = dpp_from_lower_lane(c1, ce);   // cw at column y0-1
            const double right = dpp_from_upper_lane(c0, ce);  // cw at column y0+2
            const double r8 = A.drate[a] * 0.125;
            // the box sums of the lane's even and odd column (columns paired from y0)
            const double pk = c0 + c1;
            w0[a] = __builtin_fma(__builtin_fma(C.u0[a], C.m0, left + pk), r8, C.u0[a]);
            w1[a] = __builtin_fma(__builtin_fma(C.u1[a], C.m1, pk + right), r8, C.u1[a]);
        } else {
            w0[a] = C.u0[a];
            w1[a] = C.u1[a];
        }
    }
    if (CHAIN && A.npost) {
        apply_chain<NA>(w0, A.npost, A.post_a, A.post_b, A.post_r);
        apply_chain<NA>(w1, A.npost, A.post_a, A.post_b, A.post_r);
    }
    const bool live = r <= rmax;  // wave-uniform
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        dv2 v;
        v.x = w0[a];
        v.y = w1[a];
        // lanes past W write the row's padding columns (never read as cells)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v),
                                               row_rsrc(A.out[a], r, rmax, A.pitch), voff, 0,
                                               (NT & 1) ? 2 : 0);
        if (REDUCE) {
            acc[a] = acc[a] + ((live && st1) ? w0[a] : 0.0);
            acc[a] = acc[a] + ((live && st2) ? w1[a] : 0.0);
        }
    }
}

template <int NA>
__device__ __forceinline__ void copy_row(ProcRow<NA>& d, const ProcRow<NA>& s) {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        d.w0[a] = s.w0[a];
        d.w1[a] = s.w1[a];
        d.we[a] = s.we[a];
        d.u0[a] = s.u0[a];
        d.u1[a] = s.u1[a];
    }
    d.m0 = s.m0;
    d.m1 = s.m1;
}

__device__ __forceinline__ double wave_sum(double v) {
    // fixed butterfly: every lane ends with the same, order-independent-of-timing value
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = v + __shfl_xor(v, m, 64);
    return v;
}

// TH output rows per wave, fully unrolled (no loop back edge, so the compiler keeps
// counted vmcnt waits for every row instead of draining at a loop header).
template <int NA, int TH, int U, bool REDUCE, int NT, bool CHAIN>
__global__ __launch_bounds__(kBlock) void mm_pass_kernel(const PassArgs A) {
    static_assert(U <= TH, "prefetch deeper than the row block");
    const int lane = threadIdx.x & 63;
    // wave-uniform, and provably so for the compiler (scalar descriptors, no waterfalls)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long wid = (long long)blockIdx.x * kWavesPerBlock + wave;
    if (wid >= A.waves_total) return;

    // wave -> (row range, row block, column strip); strips vary fastest so the 4 waves of
    // a block are side by side and share their edge columns in L1/L2.
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
    const int rB = min(rA + TH, rhi);  // output rows [rA, rB); input rows [rA-1, rB]

    const long long base = (long long)strip * kStripCols;
    const long long y0 = base + 2 * lane;
    const long long W = A.W;
    // lane 0 carries the column left of the strip, lane 63 the one right of it
    const long long ye = lane == 0 ? base - 1 : (lane == 63 ? base + kStripCols : -1);
    const bool edge_ok = ye >= 0 && ye < W;
    const int sy0 = span3(W, y0), sy1 = span3(W, y0 + 1), sye = edge_ok ? span3(W, ye) : 0;
    const bool fast_cols = base >= 2 && base + kStripCols <= W - 2;  // wave-uniform
    const bool st1 = y0 < W, st2 = y0 + 1 < W;
    const unsigned voff = (unsigned)(y0 * 8);
    const unsigned eoff = edge_ok ? (unsigned)(ye * 8) : kOOB;

    double acc[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) acc[a] = 0.0;

    // Input row rA-1+i is "input i". Inputs 0 and 1 prime the window; input i >= 2
    // lives in raw[(i-2) % U] and is refilled with input i+U as soon as it is consumed,
    // so U row loads stay in flight down the strip. Rows past rB load as zeros without
    // traffic and output rows past rB-1 are dropped (descriptors with num_records 0).
    RawRow<NA> first, second, raw[U];
    load_row<NA, NT>(A, rA - 1, rB, voff, eoff, first);
    load_row<NA, NT>(A, rA, rB, voff, eoff, second);
#pragma unroll
    for (int k = 0; k < U; ++k) load_row<NA, NT>(A, rA + 1 + k, rB, voff, eoff, raw[k]);
    ProcRow<NA> P, C, N;
    process_row<NA, CHAIN>(A, rA - 1, first, fast_cols, sy0, sy1, sye, P);
    process_row<NA, CHAIN>(A, rA, second, fast_cols, sy0, sy1, sye, C);
#pragma unroll
    for (int k = 0; k < TH; ++k) {
        process_row<NA, CHAIN>(A, rA + 1 + k, raw[k % U], fast_cols, sy0, sy1, sye, N);
        if (k + U < TH)  // input k+2+U is still inside this row block
            load_row<NA, NT>(A, rA + 1 + k + U, rB, voff, eoff, raw[k % U]);
        emit_row<NA, REDUCE, NT, CHAIN>(A, rA + k, rB - 1, voff, st2, st1, P, C, N, acc);
        copy_row<NA>(P, C);
        copy_row<NA>(C, N);
    }

    if (REDUCE) {
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            const double t = wave_sum(acc[a]);
            if (lane == 0) A.partials[(A.partial_base + wid) * NA + a] = t;
        }
    }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// src/Model.hpp:154-157 (value 1.0) or the synthetic input of SURVEY.md 8(d);
// owned rows and the ghost rows that lie inside the grid.
__global__ __launch_bounds__(256) void mm_fill_kernel(double* buf, long long pitch, long long H,
                                                      long long W, long long x_init, long long h,
                                                      int mode, double value,
                                                      unsigned long long seed) {
    const long long n = (h + 2 * kGhost) * W;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const long long r = i / W - kGhost, y = i % W;
        const long long gx = x_init + r;
        if (gx < 0 || gx >= H) continue;
        double v = value;
        if (mode == 1) {
            const unsigned long long z = splitmix64(seed ^ (unsigned long long)(gx * W + y));
            v = 1.0 + (double)(z >> 11) * 0x1.0p-53;
        }
        buf[r * pitch + y] = v;
    }
}

// src/Model.hpp:176-235 on the cells of this slab (one thread per 3x3 cell).
__global__ void mm_point_kernel(double* buf, long long pitch, long long H, long long W,
                                long long x_init, long long h, long long sx, long long sy,
                                double captured, double rate) {
    const int t = threadIdx.x;
    if (t >= 9) return;
    const int cnt = (span3(H, sx) && span3(W, sy)) ? span3(H, sx) * span3(W, sy) - 1 : 0;
    if (cnt <= 0) return;
    const long long x = sx + t / 3 - 1, y = sy + t % 3 - 1;
    if (x < 0 || y < 0 || x >= H || y >= W || x < x_init || x >= x_init + h) return;
    const double out = rate * captured;        // src/Exponencial.hpp:15
    const double share = share_of(out, cnt);   // src/Model.hpp:199
    double* p = buf + (x - x_init) * pitch + y;
    if (t == 4)
        *p = *p - out;    // src/Model.hpp:211
    else
        *p = *p + share;  // src/Model.hpp:206-209,234
}

// Fixed-order sum of n partial rows (na doubles each) -> hist[slot*na ...], the slot from
// a device counter advanced by `entries` (na = entries * attributes).
__global__ __launch_bounds__(256) void mm_finalize_kernel(const double* partials, long long n,
                                                          int na, double* hist,
                                                          unsigned long long* hist_n,
                                                          long long cap, int entries) {
    __shared__ double red[256];
    __shared__ unsigned long long slot;
    if (threadIdx.x == 0) slot = *hist_n;
    __syncthreads();
    for (int a = 0; a < na; ++a) {
        double s = 0.0;
        for (long long i = threadIdx.x; i < n; i += 256) s = s + partials[i * na + a];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int m = 128; m >= 1; m >>= 1) {
            if ((int)threadIdx.x < m) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + m];
            __syncthreads();
        }
        const int per = na / entries;
        const long long idx = (long long)slot + a / per;
        if (threadIdx.x == 0 && idx < cap) hist[idx * per + a % per] = red[0];
        __syncthreads();
    }
    if (threadIdx.x == 0) *hist_n = slot + entries;
}

// Sum of the owned rows of one buffer: block b sums rows b, b+nblocks, ...
__global__ __launch_bounds__(256) void mm_slab_sum_kernel(const double* buf, long long pitch,
                                                          long long W, long long h,
                                                          double* partials) {
    __shared__ double red[256];
    double s = 0.0;
    for (long long r = blockIdx.x; r < h; r += gridDim.x) {
        const double* row = buf + r * pitch;
        for (long long y = threadIdx.x; y < W; y += 256) s = s + row[y];
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int m = 128; m >= 1; m >>= 1) {
        if ((int)threadIdx.x < m) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + m];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

__global__ void mm_sum_partials_kernel(const double* partials, long long n, double* out) {
    __shared__ double red[256];
    double s = 0.0;
    for (long long i = threadIdx.x; i < n; i += 256) s = s + partials[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int m = 128; m >= 1; m >>= 1) {
        if ((int)threadIdx.x < m) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + m];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

template <int NA, int TH, int U, int NT, bool CHAIN>
hipError_t launch_c(bool reduce, const PassArgs& a, hipStream_t s) {
    const long long blocks = (a.waves_total + kWavesPerBlock - 1) / kWavesPerBlock;
    if (reduce)
        hipLaunchKernelGGL((mm_pass_kernel<NA, TH, U, true, NT, CHAIN>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((mm_pass_kernel<NA, TH, U, false, NT, CHAIN>), dim3((unsigned)blocks),
                           dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

// One attribute, no transfers: the headline Exponencial step. Row block TH in
// {8, 16, 32} (a.th), non-temporal policy from the tuning variant (0 none, 1 stores,
// 3 loads+stores).
template <int TH>
hipError_t launch_one(bool reduce, const PassArgs& a, hipStream_t s, int variant) {
    switch (variant) {
        case 1: return launch_c<1, TH, 8, 1, false>(reduce, a, s);
        case 3: return launch_c<1, TH, 8, 3, false>(reduce, a, s);
        default: return launch_c<1, TH, 8, 0, false>(reduce, a, s);
    }
}

// rows kept in flight per wave: 8 KiB at one attribute, fewer rows as the attributes
// (and the registers per row) grow
template <int NA>
constexpr int prefetch_rows() {
    return NA == 1 ? 8 : (NA == 2 ? 4 : 2);
}

template <int NA>
hipError_t launch_pass_na(bool reduce, const PassArgs& a, hipStream_t s, int variant) {
    (void)variant;
    constexpr int U = prefetch_rows<NA>();
    if (a.th != 8) return hipErrorInvalidValue;
    if (a.npre || a.npost) return launch_c<NA, 8, U, 0, true>(reduce, a, s);
    return launch_c<NA, 8, U, 0, false>(reduce, a, s);
}

template <>
hipError_t launch_pass_na<1>(bool reduce, const PassArgs& a, hipStream_t s, int variant) {
    if (a.npre || a.npost) {
        if (a.th != 8) return hipErrorInvalidValue;
        return launch_c<1, 8, 8, 0, true>(reduce, a, s);
    }
    switch (a.th) {
        case 1: return launch_c<1, 1, 1, 0, false>(reduce, a, s);  // border row of a split pass
        case 8: return launch_one<8>(reduce, a, s, variant);
        case 16: return launch_one<16>(reduce, a, s, variant);
        case 32: return launch_one<32>(reduce, a, s, variant);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_pass(int na, bool reduce, const PassArgs& a, hipStream_t s, int variant) {
    if (a.waves_total <= 0) return hipSuccess;
    switch (na) {
        case 1: return launch_pass_na<1>(reduce, a, s, variant);
        case 2: return launch_pass_na<2>(reduce, a, s, variant);
        case 3: return launch_pass_na<3>(reduce, a, s, variant);
        case 4: return launch_pass_na<4>(reduce, a, s, variant);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_fill(double* buf, long long pitch, long long H, long long W, long long x_init,
                       long long h, int mode, double value, unsigned long long seed,
                       hipStream_t s) {
    const long long n = (h + 2 * kGhost) * W;
    long long blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(mm_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, buf, pitch, H, W,
                       x_init, h, mode, value, seed);
    return hipGetLastError();
}

hipError_t launch_point(double* buf, long long pitch, long long H, long long W, long long x_init,
                        long long h, long long sx, long long sy, double captured, double rate,
                        hipStream_t s) {
    hipLaunchKernelGGL(mm_point_kernel, dim3(1), dim3(64), 0, s, buf, pitch, H, W, x_init, h, sx,
                       sy, captured, rate);
    return hipGetLastError();
}

hipError_t launch_finalize(const double* partials, long long n, int na, double* hist,
                           unsigned long long* hist_n, long long cap, hipStream_t s, int entries) {
    hipLaunchKernelGGL(mm_finalize_kernel, dim3(1), dim3(256), 0, s, partials, n, na * entries,
                       hist, hist_n, cap, entries);
    return hipGetLastError();
}

hipError_t launch_slab_sum(const double* buf, long long pitch, long long W, long long h,
                           double* partials, long long nblocks, double* out_sum, hipStream_t s) {
    hipLaunchKernelGGL(mm_slab_sum_kernel, dim3((unsigned)nblocks), dim3(256), 0, s, buf, pitch, W,
                       h, partials);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(mm_sum_partials_kernel, dim3(1), dim3(256), 0, s, partials, nblocks,
                       out_sum);
    return hipGetLastError();
}

}  // namespace mm
