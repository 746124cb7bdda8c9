// mm_internal.hpp -- shared between the gfx950 kernels (mm_kernels.hip) and the
// engine / C ABI (mm_engine.hip). Not part of the public boundary.
#pragma once

#include <hip/hip_runtime.h>

namespace mm {

constexpr int kMaxAttr = 4;     // SoA attributes per fused pass (config C5: 4)
constexpr int kMaxChain = 4;    // elementwise transfers before / after a pass's diffusion
                                // (a longer chain starts a new pass; 4 holds config C5's
                                // chain and, against 8, frees kernel-argument SGPRs: C5 -8 %)
constexpr int kStripCols = 128; // columns per wave: 64 lanes x double2 (16 B per lane)
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = 64 * kWavesPerBlock;
constexpr int kMaxSteps = 10;    // fused steps per pass of mm_passk_kernel (one attribute)
constexpr int kMaxWide = 20;     // fused steps per pass of mm_wide_kernel (one attribute)
constexpr int kGhost = kMaxWide;  // ghost rows above and below a slab (K fused steps need K)
constexpr int kBorderRows = 4;     // rows per wave of the K-step kernel's border launches

// One fused Jacobi pass over a row slab. Every buffer pointer points at owned row 0;
// rows -kGhost..-1 and h..h+kGhost-1 are ghost rows; local row r is global x_init+r.
//   u  = pre-chain transfers applied to the loaded cell values
//   per diffusing attribute a: out = rate_a*u, s = out/cnt, w = (u - out) + nb(s)
//   w  = post-chain transfers applied to w;  store w
// Rows [ra0, ra1) and [rb0, rb1) (local, half-open) are computed; the second
// range lets one launch cover both border rows of a halo-split step.
struct PassArgs {
    const double* in[kMaxAttr];
    double* out[kMaxAttr];
    long long H, W, x_init, pitch;
    int ra0, ra1, rb0, rb1;
    int th;                 // rows per wave
    int nstrips;            // column strips of 128 per row
    long long waves_a;      // waves covering range a
    long long waves_total;  // waves covering both ranges
    int diffuse_mask;       // bit a: attribute a diffuses in this pass
    int npre, npost;
    double drate[kMaxAttr];
    signed char pre_a[kMaxChain], pre_b[kMaxChain];
    signed char post_a[kMaxChain], post_b[kMaxChain];
    double pre_r[kMaxChain], post_r[kMaxChain];
    double* partials;       // REDUCE: [partial_base + wave][NA] (mm_passk_kernel: [..][K])
    long long partial_base;
    int xcd_remap;          // mm_passk_kernel: XCD-contiguous block order (grid padded to 8)
    int seg;                // mm_passk_kernel: segment schedule (th / th_edge rows per wave)
    int th_edge;            // mm_passk_kernel segments: rows per wave of the two edge strips
};

// Launchers (mm_kernels.hip). All enqueue on `s` and return the launch status.
hipError_t launch_pass(int na, bool reduce, const PassArgs& a, hipStream_t s, int variant);
// K fused steps of a one-pass flow program (NA = 1: K 1..10, one diffusion; NA 2..4:
// K 1..2, diffusions and transfer chains) on overlapped strips (mm_passk_kernel,
// mm_kernels_k.hip). a.seg: segment schedule, a.th / a.th_edge rows per wave; else 4-row
// blocks (a.th = 4). a.nstrips = ceil(W / passk_out_cols(k)). red: every level's sums into
// partials[wave][k][na]. variant bit 0: non-temporal stores.
hipError_t launch_passk(int k, int na, bool red, const PassArgs& a, hipStream_t s, int variant);
int passk_out_cols(int k);
int passk_max_steps(int na);
// largest segment (rows) whose buffer offsets stay below 2^31 at this pitch
long long passk_max_rows(int k, long long pitch);
// resident waves per CU of the segment kernel (occupancy API), 0 if unknown
int passk_waves_per_cu(int k, int na, bool red, int nt);
// Level-split K-step kernel (mm_wide_kernel) of a one-pass program with na attributes and
// c columns per lane: na = 1 (one diffusion) with c = 4 for K in {4, 8, 12, 16, 20}; na = 4 (transfer chains + diffusions, config C5) with c = 2 for K in
// {4, 8}. One workgroup of wide_waves_per_block(k, c, na) waves per strip segment, segment
// schedule only (a.seg; a.th / a.th_edge rows per block, a.waves_a / a.waves_total count
// BLOCKS), a.nstrips = ceil(W / wide_out_cols(k, c)). red: every level's sums into
// partials[block][k][na]. variant (and nt) bit 0: non-temporal stores (the four-attribute
// K = 8 instances store non-temporal whatever bit 0 says: only those are built); bit 1: four
// attributes whose pre-chain is the ring t -> t+1 mod 4 and no post-chain (K = 8: the
// compile-time-chain instance); bit 2: the pass has a post-chain (K = 8: the instance
// that runs one); bits 4-6: K = 8, four attributes: the pass's attributes 0..N-1 diffuse,
// the others do not (the engine relabels them so; the instance has N at compile time).
bool wide_has(int k, int c, int na);
int wide_out_cols(int k, int c, int na);
int wide_waves_per_block(int k, int c, int na, bool ring);
int wide_blocks_per_cu(int k, int c, int na, bool red, int nt);
hipError_t launch_wide(int k, int c, int na, bool red, const PassArgs& a, hipStream_t s,
                       int variant);
// Append the levels of `mask` (bit j: step j of a K-step pass) of partials[n][k][na],
// each summed in a fixed order, to the history (na sums per entry).
// perm: partials slot i holds attribute (perm >> 2i) & 3 (relabelled passes).
hipError_t launch_finalize_levels(const double* partials, long long n, int k, int na, int mask,
                                  double* hist, unsigned long long* hist_n, long long cap,
                                  hipStream_t s, int perm);
hipError_t launch_fill(double* buf, long long pitch, long long H, long long W, long long x_init,
                       long long h, int mode, double value, unsigned long long seed, hipStream_t s);
hipError_t launch_point(double* buf, long long pitch, long long H, long long W, long long x_init,
                        long long h, long long sx, long long sy, double captured, double rate,
                        hipStream_t s);
// Sum partials[n][na] in a fixed order into hist[k][na], k = (*hist_n)++ (device
// counter, so the launch is graph-replayable); entries beyond cap are dropped.
hipError_t launch_finalize(const double* partials, long long n, int na, double* hist,
                           unsigned long long* hist_n, long long cap, hipStream_t s,
                           int entries = 1);
// Per-attribute sum of the owned rows of one buffer (no pass), into out[0].
hipError_t launch_slab_sum(const double* buf, long long pitch, long long W, long long h,
                           double* partials, long long nblocks, double* out_sum, hipStream_t s);

}  // namespace mm
