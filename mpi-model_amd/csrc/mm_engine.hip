// mm_engine.hip -- the host engine behind include/mpimodel.h (C ABI).
//
// One engine = one row slab of the global grid on one GPU:
//   * device memory: per attribute two (h + 2*kGhost) x pitch fp64 buffers (Jacobi
//     ping-pong) with kGhost ghost rows above and below, pitch a multiple of 128;
//   * a one-pass flow program runs K steps per kernel pass (mm_passk_kernel, temporal
//     blocking: 16/K B of HBM traffic per cell-update); other programs run one step
//     per pass (mm_pass_kernel);
//   * a compute stream and a comm stream; with a halo (RCCL or host transport) each pass
//     runs the interior rows on the compute stream while the `depth` border rows wait
//     for the exchange on the comm stream (RCCL: ncclSend/ncclRecv of `depth` rows to
//     both neighbours; host: the caller imported them before mm_run);
//   * steps are captured once into a hipGraph (one ping-pong cycle, RCCL calls
//     included) and replayed; a refused capture is reported by mm_engine_info;
//   * per-step sums (MPI_Report) are reduced on the device into a growable history.
// The reference's per-worker body this replaces is src/Model.hpp:135-261.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/mpimodel.h"
#include "mm_internal.hpp"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define MM_HIP(expr)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(MM_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));     \
    } while (0)

#define MM_NCCL(expr)                                                                     \
    do {                                                                                  \
        ncclResult_t r_ = (expr);                                                         \
        if (r_ != ncclSuccess)                                                            \
            return fail(MM_ERR_RCCL, std::string(#expr ": ") + ncclGetErrorString(r_));   \
    } while (0)

#define MM_TRY(expr)             \
    do {                         \
        int rc_ = (expr);        \
        if (rc_ != MM_OK) return rc_; \
    } while (0)

long long span_rows(long long n, long long i) { return (i >= 0 && i < n) ? 1 + (i > 0) + (i < n - 1) : 0; }

struct Transfer {
    int a, b;
    double rate;
};

// A fused pass: pre-chain transfers, at most one diffusion per attribute, post-chain.
struct Pass {
    std::vector<Transfer> pre, post;
    int diffuse_mask = 0;
    double drate[mm::kMaxAttr] = {0, 0, 0, 0};
};

struct FlowDesc {
    int kind, a, b;
    double rate;
};

}  // namespace

struct mm_engine {
    mm_desc d{};
    int na = 1;
    long long pitch = 0;
    long long rows_alloc = 0;  // h + 2 * kGhost
    long long min_rows = 0;    // thinnest slab of the chain: bounds the halo depth
    double* base = nullptr;
    size_t bytes = 0;
    double* buf[2][mm::kMaxAttr] = {};
    int cur = 0;
    hipStream_t s_comp = nullptr, s_comm = nullptr;
    hipEvent_t ev_ready = nullptr, ev_halo = nullptr;
    hipEvent_t ev_comp_mark = nullptr, ev_comm_done = nullptr;
    bool comm_live = false;  // border work of this run is pending on the comm stream
    ncclComm_t comm = nullptr;
    bool split = false;  // interior / border split (RCCL or host halo)

    std::vector<FlowDesc> flows;
    std::vector<Pass> passes;

    int th = 8;              // rows per wave, one-step kernel
    bool passk = true;       // mm_passk_kernel for one-pass programs (MM_PASSK=0: one step per pass)
    int wide = -1;           // mm_wide_kernel for one-diffusion programs where K allows
                             // (MM_WIDE=0/1; -1 auto: slabs of >= kWideCells cells)
    int kpass = 0;           // steps per pass, one attribute (MM_STEPS_PER_PASS, 1..kMaxSteps,
                             // with MM_WIDE also the wide kernel's K; 0: auto)
    int kpass_multi = 2;     // steps per pass, several attributes (MM_STEPS_PER_PASS, 1..2)
    bool plan = true;        // pass-length planner (MM_PASS_PLAN=0: balanced passes of K)
    double seg_waves = 0.0;  // segment waves per resident wave slot (MM_SEG_WAVES; 0: auto)
    double seg_edge = 0.0;   // edge-strip segment length / interior length (MM_SEG_EDGE; 0: auto)
    bool border_segments = true;  // wide split passes: full-length border segments (MM_BORDER_SEGMENTS)
    int xcd = 0;             // XCD-contiguous block order (MM_XCD_REMAP, mm_passk_kernel)
    int ncu = 0;             // compute units of the device
    int wpc[2][2][mm::kMaxAttr + 1][mm::kMaxSteps + 1] = {};  // segment kernel waves/CU cache
    std::map<long long, int> bpc;  // wide kernel blocks/CU cache: (variant, red, k)
    bool ring_ok = true;     // the ring instance for C5-shaped chains (MM_CHAIN_RING=0: off)
    bool self_halo = false;  // test mode: one RCCL rank exchanges border rows with itself
    int variant = 0;  // kernel tuning variant (MM_KERNEL_VARIANT), 0 = default
    int nstrips = 0;
    double* partials = nullptr;
    long long partials_cap = 0;
    double* hist = nullptr;
    unsigned long long* hist_n = nullptr;  // [0] history entries, [1] level-sum workgroups done
    long long hist_cap = 0;
    long long hist_host = 0;    // entries the enqueued work appends (host-side count)
    double* sum_tmp = nullptr;  // mm_sums scratch: nblocks partials + 1 result per attribute
    long long sum_blocks = 0;

    long long steps_done = 0;

    // graph cache: key = (parity, length, reduce_every, reduction phase); value = the
    // executable and whether one replay flips the ping-pong buffers
    std::map<std::tuple<int, long long, long long, long long>, std::pair<hipGraphExec_t, int>> graphs;

    bool graphs_ok = true;      // MM_GRAPH=0 (or a refused capture) runs steps eagerly
    long long graph_min = 16;   // steps a replayed graph holds at least (MM_GRAPH_MIN_STEPS)
    long long graph_max = 128;  // step kernels a graph holds at most (MM_GRAPH_MAX_LAUNCHES)
    int graph_state = 0;        // 0 none yet, 1 replaying, -1 capture refused
    long long graph_launches = 0;
    int graph_count = 0;
    std::string graph_note;

    bool timing = false;
    // mm_synchronize polls its streams (hipStreamQuery) before the blocking wait
    // (MM_SYNC_SPIN=0: the blocking wait alone)
    bool sync_spin = true;
    std::vector<hipEvent_t> ev_pool;
    std::vector<double> ev_bytes;  // algorithmic bytes of each timed launch (pairs of events)
    size_t ev_used = 0;
    long long timed_launches = 0;
    double timed_ms = 0.0;
    double timed_bytes = 0.0;
};

namespace {

int set_device(mm_engine* e) {
    MM_HIP(hipSetDevice(e->d.device));
    return MM_OK;
}

void drop_graphs(mm_engine* e) {
    for (auto& kv : e->graphs) (void)hipGraphExecDestroy(kv.second.first);
    e->graphs.clear();
}

int compile_passes(mm_engine* e) {
    e->passes.clear();
    Pass cur;
    bool open = false;
    for (const FlowDesc& f : e->flows) {
        if (f.kind == MM_FLOW_TRANSFER) {
            if (!open) {
                cur = Pass();
                open = true;
            }
            std::vector<Transfer>& chain = cur.diffuse_mask ? cur.post : cur.pre;
            if ((int)chain.size() >= mm::kMaxChain) {
                e->passes.push_back(cur);
                cur = Pass();
                cur.pre.push_back({f.a, f.b, f.rate});
            } else {
                chain.push_back({f.a, f.b, f.rate});
            }
        } else {  // MM_FLOW_DIFFUSE
            if (!open) {
                cur = Pass();
                open = true;
            }
            if ((cur.diffuse_mask & (1 << f.a)) || !cur.post.empty()) {
                e->passes.push_back(cur);
                cur = Pass();
            }
            cur.diffuse_mask |= 1 << f.a;
            cur.drate[f.a] = f.rate;
        }
    }
    if (open) e->passes.push_back(cur);
    return MM_OK;
}

// Waves for a row range of n rows at th rows per wave (nstrips column strips).
long long waves_for(long long nstrips, long long n, int th) {
    if (n <= 0) return 0;
    return nstrips * ((n + th - 1) / th);
}
long long waves_for(const mm_engine* e, long long n, int th) { return waves_for(e->nstrips, n, th); }
long long waves_for(const mm_engine* e, long long n) { return waves_for(e, n, e->th); }

void fill_args(const mm_engine* e, const Pass& p, mm::PassArgs& A) {
    std::memset(&A, 0, sizeof A);
    for (int a = 0; a < e->na; ++a) {
        A.in[a] = e->buf[e->cur][a];
        A.out[a] = e->buf[e->cur ^ 1][a];
    }
    A.H = e->d.H;
    A.W = e->d.W;
    A.x_init = e->d.x_init;
    A.pitch = e->pitch;
    A.th = e->th;
    A.nstrips = e->nstrips;
    A.diffuse_mask = p.diffuse_mask;
    for (int a = 0; a < mm::kMaxAttr; ++a) A.drate[a] = p.drate[a];
    A.npre = (int)p.pre.size();
    A.npost = (int)p.post.size();
    for (size_t i = 0; i < p.pre.size(); ++i) {
        A.pre_a[i] = (signed char)p.pre[i].a;
        A.pre_b[i] = (signed char)p.pre[i].b;
        A.pre_r[i] = p.pre[i].rate;
    }
    for (size_t i = 0; i < p.post.size(); ++i) {
        A.post_a[i] = (signed char)p.post[i].a;
        A.post_b[i] = (signed char)p.post[i].b;
        A.post_r[i] = p.post[i].rate;
    }
    A.partials = e->partials;
}

hipEvent_t next_event(mm_engine* e) {
    if (e->ev_used == e->ev_pool.size()) {
        hipEvent_t ev;
        if (hipEventCreate(&ev) != hipSuccess) return nullptr;
        e->ev_pool.push_back(ev);
    }
    return e->ev_pool[e->ev_used++];
}

// Columns per lane of the wide kernel: 4 for one attribute, 2 for several.
int wcols(const mm_engine* e, int) { return e->na > 1 ? 2 : 4; }

// Variant bit 1 of a wide launch: a one-pass program of four attributes whose pre-chain
// is the ring of transfers t -> t+1 mod 4 in that order, without a post-chain (config C5's
// topology), runs the instance with the chain's operands fixed at compile time.
int wring(const mm_engine* e) {
    if (!e->ring_ok || e->na != 4 || e->passes.size() != 1) return 0;
    const Pass& p = e->passes[0];
    if ((int)p.pre.size() != e->na || !p.post.empty() || p.diffuse_mask != 15) return 0;
    for (int t = 0; t < e->na; ++t)
        if (p.pre[t].a != t || p.pre[t].b != (t + 1) % e->na) return 0;
    return 2;
}

// Variant bits of a wide launch beyond bit 0 (mm_internal.hpp): the ring instance (2), a
// post-chain (4), the number of diffusing attributes (bits 4-6; relabel puts them first).
int wvar(const mm_engine* e) {
    if (e->na == 1 || e->passes.size() != 1) return 0;
    const Pass& p = e->passes[0];
    return wring(e) | (p.post.empty() ? 0 : 4) | (__builtin_popcount((unsigned)p.diffuse_mask) << 4);
}

// Identity attribute permutation, packed 2 bits per slot (launch_finalize_levels).
constexpr int kPermIdentity = 0 | 1 << 2 | 2 << 4 | 3 << 6;

// A four-attribute wide pass runs an instance with its diffusing attributes first: the
// pass's arguments are relabelled so that physical slot i holds logical attribute perm[i]
// -- the diffusing attributes in order, then the others -- its buffers, rates and chain
// operands with them. Returns the permutation packed like kPermIdentity, for the step
// sums (partials come out in physical order; the history is logical).
int relabel(const mm_engine* e, mm::PassArgs& A) {
    if (e->na == 1) return kPermIdentity;
    const Pass& p = e->passes[0];
    int perm[mm::kMaxAttr], inv[mm::kMaxAttr], n = 0;
    for (int a = 0; a < e->na; ++a)
        if ((p.diffuse_mask >> a) & 1) perm[n++] = a;
    const int nd = n;
    for (int a = 0; a < e->na; ++a)
        if (!((p.diffuse_mask >> a) & 1)) perm[n++] = a;
    int code = 0;
    for (int i = 0; i < e->na; ++i) {
        inv[perm[i]] = i;
        code |= perm[i] << (2 * i);
        A.in[i] = e->buf[e->cur][perm[i]];
        A.out[i] = e->buf[e->cur ^ 1][perm[i]];
        A.drate[i] = p.drate[perm[i]];
    }
    A.diffuse_mask = (1 << nd) - 1;
    for (size_t t = 0; t < p.pre.size(); ++t) {
        A.pre_a[t] = (signed char)inv[p.pre[t].a];
        A.pre_b[t] = (signed char)(p.pre[t].b < 0 ? -1 : inv[p.pre[t].b]);
    }
    for (size_t t = 0; t < p.post.size(); ++t) {
        A.post_a[t] = (signed char)inv[p.post[t].a];
        A.post_b[t] = (signed char)(p.post[t].b < 0 ? -1 : inv[p.post[t].b]);
    }
    return code;
}

// Launch a one-step pass (kpass == 0), a K-step pass (kpass = K > 0: mm_passk_kernel;
// kpass = -K: mm_wide_kernel) covering `rows`
// rows on the compute stream, with an event pair around it when timing. Algorithmic
// bytes: every cell of those rows read once and written once per attribute.
int launch_timed(mm_engine* e, bool red, const mm::PassArgs& A, long long rows, bool time_it,
                 int kpass) {
    hipEvent_t a = nullptr, b = nullptr;
    if (time_it) {
        a = next_event(e);
        b = next_event(e);
        if (!a || !b) return fail(MM_ERR_HIP, "hipEventCreate failed");
        e->ev_bytes.resize(e->ev_used / 2);
        e->ev_bytes.back() = 16.0 * (double)rows * (double)e->d.W * e->na;
        MM_HIP(hipEventRecord(a, e->s_comp));
    }
    if (kpass > 0)
        MM_HIP(mm::launch_passk(kpass, e->na, red, A, e->s_comp, e->variant));
    else if (kpass < 0)
        MM_HIP(mm::launch_wide(-kpass, wcols(e, -kpass), e->na, red, A, e->s_comp,
                               (e->variant & 1) | wvar(e)));
    else
        MM_HIP(mm::launch_pass(e->na, red, A, e->s_comp, e->variant));
    if (time_it) MM_HIP(hipEventRecord(b, e->s_comp));
    return MM_OK;
}

long long nstrips_k(const mm_engine* e, int k) {
    const int oc = mm::passk_out_cols(k);
    return (e->d.W + oc - 1) / oc;
}

// Border-row exchange with both neighbours in one RCCL group: the first / last `depth`
// owned rows go to rank-1 / rank+1, their rows land in the ghost rows. Rows are
// contiguous (pitch doubles each), so every message is one contiguous block. The
// engine keeps depth <= min_rows, so the sent rows are always owned rows.
int halo_rccl(mm_engine* e, int depth) {
    const int r = e->d.rank, n = e->d.nranks;
    const long long P = e->pitch, h = e->d.h;
    const size_t cnt = (size_t)(depth * P);
    MM_NCCL(ncclGroupStart());
    for (int a = 0; a < e->na; ++a) {
        double* b = e->buf[e->cur][a];
        if (e->self_halo) {
            // one rank, both neighbours itself: the first rows land in the bottom ghost
            // rows and the last rows in the top ghost rows. Those ghost rows lie outside
            // the grid, so the kernels never read them as cells: the exchange exercises
            // the RCCL path without changing the result.
            MM_NCCL(ncclSend(b, cnt, ncclDouble, 0, e->comm, e->s_comm));
            MM_NCCL(ncclSend(b + (h - depth) * P, cnt, ncclDouble, 0, e->comm, e->s_comm));
            MM_NCCL(ncclRecv(b + h * P, cnt, ncclDouble, 0, e->comm, e->s_comm));
            MM_NCCL(ncclRecv(b - depth * P, cnt, ncclDouble, 0, e->comm, e->s_comm));
            continue;
        }
        if (r > 0) {
            MM_NCCL(ncclSend(b, cnt, ncclDouble, r - 1, e->comm, e->s_comm));
            MM_NCCL(ncclRecv(b - depth * P, cnt, ncclDouble, r - 1, e->comm, e->s_comm));
        }
        if (r < n - 1) {
            MM_NCCL(ncclSend(b + (h - depth) * P, cnt, ncclDouble, r + 1, e->comm, e->s_comm));
            MM_NCCL(ncclRecv(b + h * P, cnt, ncclDouble, r + 1, e->comm, e->s_comm));
        }
    }
    MM_NCCL(ncclGroupEnd());
    return MM_OK;
}

bool rccl_halo(const mm_engine* e) { return e->comm != nullptr; }

// Rows [lo, hi) of the slab as range a, optional [lo2, hi2) as range b (A.th set).
void set_ranges(mm::PassArgs& A, long long lo, long long hi, long long lo2, long long hi2) {
    A.ra0 = (int)lo;
    A.ra1 = (int)hi;
    A.rb0 = (int)lo2;
    A.rb1 = (int)hi2;
    A.waves_a = waves_for(A.nstrips, hi - lo, A.th);
    A.waves_total = A.waves_a + waves_for(A.nstrips, hi2 - lo2, A.th);
}

// Start of a split pass. Two streams per pass, joined by events:
//   comm:    [RCCL exchange k (right after border k-1)] -> [after interior k-1] border k
//   compute: [after border k-1] interior k
// so the exchange and the border rows run beside the interior kernels. Interior k reads
// rows border k-1 wrote; border k reads rows interior k-1 wrote and writes rows interior
// k-1 read; ghost rows are only touched on comm; the rows an exchange sends were written
// by the border kernel before it. With the host transport the caller has already put the
// neighbours' rows into the ghost rows, and the same schedule runs without the exchange.
// A split pass in two halves, the compute stream's first: the interior rows need only the
// previous border rows, not this pass's exchange, so their launch goes ahead of the
// exchange's host-side enqueue (an RCCL group call took 64 us before the interior's launch
// in profiles/r06/trace20).
int split_comp(mm_engine* e) {
    // interior k reads the rows border k-1 wrote
    if (e->comm_live) MM_HIP(hipStreamWaitEvent(e->s_comp, e->ev_comm_done, 0));
    // everything the compute stream ran before interior k: interior k-1, the fills
    MM_HIP(hipEventRecord(e->ev_comp_mark, e->s_comp));
    return MM_OK;
}

int split_comm(mm_engine* e, int depth) {
    // first split pass of the run: the exchange follows all earlier compute work
    if (!e->comm_live) MM_HIP(hipStreamWaitEvent(e->s_comm, e->ev_comp_mark, 0));
    if (rccl_halo(e)) MM_TRY(halo_rccl(e, depth));  // needs only border k-1 (same stream)
    // border k reads rows interior k-1 wrote (and reuses the partials finalize k-1 read)
    MM_HIP(hipStreamWaitEvent(e->s_comm, e->ev_comp_mark, 0));
    return MM_OK;
}

// Slab too thin to split: exchange first, then one launch on the compute stream.
int unsplit_halo(mm_engine* e, int depth) {
    if (!rccl_halo(e)) return MM_OK;
    MM_HIP(hipEventRecord(e->ev_ready, e->s_comp));
    MM_HIP(hipStreamWaitEvent(e->s_comm, e->ev_ready, 0));
    MM_TRY(halo_rccl(e, depth));
    MM_HIP(hipEventRecord(e->ev_halo, e->s_comm));
    MM_HIP(hipStreamWaitEvent(e->s_comp, e->ev_halo, 0));
    return MM_OK;
}

// One single-step kernel pass over the slab (1-row halo). With a halo the interior rows
// run while the rows are in flight, then the border row on each side. One history entry
// of n_attr sums is appended when red.
int enqueue_pass(mm_engine* e, const Pass& p, bool red, bool time_it) {
    const long long h = e->d.h;
    const int depth = 1;
    mm::PassArgs A;
    fill_args(e, p, A);
    long long total_waves = 0;
    if (e->split && h >= 2 * depth + 1) {
        MM_TRY(split_comp(e));
        set_ranges(A, depth, h - depth, 0, 0);
        const long long interior_waves = A.waves_total;
        mm::PassArgs B = A;
        A.partial_base = 0;
        MM_TRY(launch_timed(e, red, A, h - 2 * depth, time_it, 0));
        MM_TRY(split_comm(e, depth));
        B.th = 1;  // border: short row blocks, the launch is latency-bound
        set_ranges(B, 0, depth, h - depth, h);
        B.partial_base = interior_waves;
        MM_HIP(mm::launch_pass(e->na, red, B, e->s_comm, e->variant));
        MM_HIP(hipEventRecord(e->ev_comm_done, e->s_comm));
        e->comm_live = true;
        total_waves = interior_waves + B.waves_total;
        if (red) MM_HIP(hipStreamWaitEvent(e->s_comp, e->ev_comm_done, 0));
    } else {
        if (e->split) MM_TRY(unsplit_halo(e, depth));
        set_ranges(A, 0, h, 0, 0);
        A.partial_base = 0;
        MM_TRY(launch_timed(e, red, A, h, time_it, 0));
        total_waves = A.waves_total;
    }
    if (red)
        MM_HIP(mm::launch_finalize(e->partials, total_waves, e->na, e->hist, e->hist_n,
                                   e->hist_cap, e->s_comp, 1));
    e->cur ^= 1;
    return MM_OK;
}

// Waves of a segment-scheduled range of n rows over ns strips (mm_passk.hpp seg_map).
long long seg_wave_count(long long n, long long ns, long long r, long long re) {
    if (n <= 0) return 0;
    if (ns < 3) return ns * ((n + re - 1) / re);
    return 2 * ((n + re - 1) / re) + (ns - 2) * ((n + r - 1) / r);
}

// Edge-strip segment length / interior segment length of a k-step pass. The two edge
// strips run the general body, several times slower per row than the branch-free one,
// and at K >= 8 it spills; their segments are cut shorter so they end with the rest
// (profiles/r02b/k9k10/edge_*: K = 10 at 0.5 takes 1.5x the pass time of 0.1;
// profiles/r02_end/edge/sweep_*: on slabs of >= 2^26 cells K = 6..8 at 0.3 are 1-3 %
// faster than at 0.5 at 16384^2 and within 0.2 % at 32768^2; the short segments of
// smaller slabs keep 0.5).
double seg_edge_of(const mm_engine* e, int k) {
    if (e->seg_edge > 0.0) return e->seg_edge;
    if (k >= 10) return 0.1;
    if (k == 9) return 0.2;
    return (double)e->d.h * (double)e->d.W >= 67108864.0 ? 0.3 : 0.5;
}

// Segment plan of rows [lo, hi) of a k-step pass: r rows per interior-strip segment, re
// per edge-strip segment (seg_edge x r: the edge strips run the slower general body),
// the smallest r for which every wave fits seg_waves x the chip's resident wave slots
// (the kernel's occupancy x CUs). Auto: 4 waves per slot while segments stay >= 256 rows
// (large slabs: the waves that finish last are shorter), else 2 (short segments pay 2K
// extra input rows each) -- profiles/r02b/segwaves: 32768^2 K = 7/8 and 16384^2 K = 6..8
// run 3-5 % faster at 4 than at 2, 4096^2 K = 7 12 % slower.
void seg_range(mm_engine* e, int k, bool red, mm::PassArgs& A, long long lo, long long hi) {
    const int nt = e->variant & 1;
    int& wpc = e->wpc[red ? 1 : 0][nt][e->na][k];
    if (!wpc) wpc = std::max(1, mm::passk_waves_per_cu(k, e->na, red, nt));
    const long long n = hi - lo, ns = A.nstrips;
    const long long maxr = std::max<long long>(16, mm::passk_max_rows(k, e->pitch));
    const double edge = seg_edge_of(e, k);
    const double units = ns < 3 ? (double)ns / edge : (double)(ns - 2) + 2.0 / edge;
    // even segment lengths: with an even first row (x_init and lo even, as every bench
    // slab) no segment pays the odd-start shift of the row-paired kernels (one extra row)
    auto even_rows = [&](long long rr) { return std::min(maxr & ~1LL, rr + (rr & 1)); };
    auto re_of = [&](long long rr) {
        return even_rows(std::min(maxr, std::max<long long>(8, (long long)((double)rr * edge))));
    };
    auto plan = [&](double sw) {
        const long long want = std::max<long long>(1, (long long)(sw * e->ncu * wpc));
        long long r = (long long)std::ceil((double)std::max<long long>(n, 1) * units / (double)want);
        r = std::min(std::max<long long>(r, 16), maxr);
        while (r < maxr && seg_wave_count(n, ns, r, re_of(r)) > want) r += std::max<long long>(1, r / 64);
        return even_rows(std::min(r, maxr));
    };
    long long r;
    if (e->seg_waves > 0.0) {
        r = plan(e->seg_waves);
    } else {
        r = plan(4.0);
        if (r < 256) r = plan(2.0);
    }
    A.seg = 1;
    A.th = (int)r;
    A.th_edge = (int)re_of(r);
    A.ra0 = (int)lo;
    A.ra1 = (int)hi;
    A.rb0 = A.rb1 = 0;
    A.waves_a = A.waves_total = seg_wave_count(n, ns, r, A.th_edge);
}

bool passk_ok(const mm_engine* e);

// The level-split kernel runs this pass: one attribute, one diffusion, K one of its
// instances, MM_WIDE on.
constexpr double kWideCells = 268435456.0;  // 2^28: 16384^2, 8192 x 32768 and up
// Below 2^25 cells (4096^2 and down) one K = 8 pass of the level-split kernel beats
// mm_passk_kernel's K = 7 / 8: its 4 waves share a segment's pipeline fill, so segments
// are 2.7x longer for the same number of resident waves (1000 steps of 4096^2: 1513-1585
// vs 1410-1443 GCUPS; one pass per step at 1024^2 / 2048^2: 4.54 / 6.39 vs 6.22 / 6.69 us,
// profiles/r03/c2graph); 8192^2 favours mm_passk_kernel K = 7 (32.4 vs 35.0 us).
constexpr double kWideSmallCells = 33554432.0;
constexpr int kWideSmallAuto = 8;

double slab_cells(const mm_engine* e) { return (double)e->min_rows * (double)e->d.W; }

// the K = 20 planner's slabs (forced MM_WIDE=1 plans every slab that way)
// Slabs of 2^27 - 2^28 cells (the 4096 x 32768 slabs of an 8-GPU c3 run) also take the
// K = 20 planner. Round 4 kept mm_passk_kernel there without a halo (2050 vs ~1920 GCUPS,
// profiles/r04/midslab); since the box-sum step the level-split kernel runs the split
// 4096 x 32768 slab at 2532 GCUPS against 1194-1272 for mm_passk_kernel's 7 + 7 + 6 without
// one (20 steps, profiles/r06/self20, profiles/r06/selfhalo).
constexpr double kWideSplitCells = 134217728.0;  // 2^27

bool wide_big(const mm_engine* e) {
    return e->wide > 0 || slab_cells(e) >= kWideCells ||
           (e->wide < 0 && e->na == 1 && slab_cells(e) >= kWideSplitCells);
}

bool wide_on(const mm_engine* e) {
    // auto: several attributes always (K = 8 instead of mm_passk_kernel's 2); one attribute
    // on slabs of >= kWideCells or < kWideSmallCells cells, or >= kWideSplitCells with a
    // halo, sized by the chain's thinnest slab (rank-invariant, like every plan input)
    return e->wide > 0 ||
           (e->wide < 0 && (e->na > 1 || wide_big(e) || slab_cells(e) < kWideSmallCells));
}

bool use_wide(const mm_engine* e, int k) {
    // four attributes: a pass with at least one diffusion (the instances diffuse 1..4)
    return wide_on(e) && passk_ok(e) && mm::wide_has(k, wcols(e, k), e->na) &&
           (e->na == 1 || e->passes[0].diffuse_mask != 0);
}

long long nstrips_wide(const mm_engine* e, int k) {
    const int oc = mm::wide_out_cols(k, wcols(e, k), e->na);
    return (e->d.W + oc - 1) / oc;
}

// Segment plan of rows [lo, hi) for the wide kernel: one workgroup per strip segment, r
// rows per interior-strip segment and re per edge-strip segment, the smallest r for which
// the blocks fit seg_waves x the chip's resident blocks. Auto: 4 per resident slot, fewer
// (down to 1) while segments are shorter than 20 K rows -- a segment pays 3K - 1 pipeline
// iterations and 2K extra input rows, 15 % of a 318-row segment at K = 16 (4096 x 32768,
// profiles/r03/kernel_table).
void wide_range(mm_engine* e, int k, bool red, mm::PassArgs& A, long long lo, long long hi) {
    const int nt = (e->variant & 1) | wvar(e);
    const int c = wcols(e, k);
    int& bpc = e->bpc[((long long)nt << 8) | (red ? 128 : 0) | k];
    if (!bpc) bpc = std::max(1, mm::wide_blocks_per_cu(k, c, e->na, red, nt));
    const long long n = hi - lo, ns = A.nstrips;
    const long long maxr = std::max<long long>(16, mm::passk_max_rows(k, e->pitch));
    // edge strips: full-length segments for one attribute (the EDGE / GEN bodies cost
    // little more than the interior's since round 5: c2 / c3 +0.5-1.5 %, c4 and the split
    // slabs within +-1 %), half length for four (their per-column GEN body: C5 -10 % at
    // full length; profiles/r05/edge)
    const double edge = e->seg_edge > 0.0 ? e->seg_edge : (e->na == 1 ? 1.0 : 0.5);
    const double units = ns < 3 ? (double)ns / edge : (double)(ns - 2) + 2.0 / edge;
    // even segment lengths: with an even first row (x_init and lo even, as every bench
    // slab) no segment pays the odd-start shift of the row-paired kernels (one extra row)
    auto even_rows = [&](long long rr) { return std::min(maxr & ~1LL, rr + (rr & 1)); };
    auto re_of = [&](long long rr) {
        return even_rows(std::min(maxr, std::max<long long>(8, (long long)((double)rr * edge))));
    };
    auto plan = [&](double sw) {
        const long long want = std::max<long long>(1, (long long)(sw * e->ncu * bpc));
        long long r = (long long)std::ceil((double)std::max<long long>(n, 1) * units / (double)want);
        r = std::min(std::max<long long>(r, 16), maxr);
        while (r < maxr && seg_wave_count(n, ns, r, re_of(r)) > want) r += std::max<long long>(1, r / 64);
        return even_rows(std::min(r, maxr));
    };
    long long r;
    if (e->seg_waves > 0.0) {
        r = plan(e->seg_waves);
    } else {
        // 4, 3, 2, 1 segment waves per slot while segments are shorter than 20 K rows: the
        // 4096 x 32768 split slab of an 8-GPU c3 run takes 3 (460-row segments; 2 gave 683:
        // kernel 1000-1022 vs 1069-1082 us, 200 steps +2.9 %, profiles/r05/sw3); the other
        // bench shapes keep their plans (c2 ends at 1, 32768^2 / 16384^2 / 8192-row slabs at 4)
        double sw = 4.0;
        r = plan(sw);
        while (sw > 1.0 && r < 20LL * k) {
            sw -= 1.0;
            r = plan(sw);
        }
    }
    A.seg = 1;
    A.th = (int)r;
    A.th_edge = (int)re_of(r);
    A.ra0 = (int)lo;
    A.ra1 = (int)hi;
    A.rb0 = A.rb1 = 0;
    A.waves_a = A.waves_total = seg_wave_count(n, ns, r, A.th_edge);
}

// A k-step pass on the level-split kernel: enqueue_passk's two-stream structure; the border
// rows are one `depth`-row segment per strip and side (ranges a and b of one launch).
int enqueue_wide(mm_engine* e, int k, int mask, bool time_it) {
    const long long h = e->d.h;
    const int depth = k;
    const bool red = mask != 0;
    mm::PassArgs A;
    fill_args(e, e->passes[0], A);
    const int perm = relabel(e, A);
    A.nstrips = (int)nstrips_wide(e, k);
    long long total_blocks = 0;  // partials units: one per workgroup
    if (e->split && h >= 2 * depth + 1) {
        MM_TRY(split_comp(e));
        // The rows that read the exchanged ghost rows, [0, K) and [h-K, h), run on the comm
        // stream after the exchange. By default as the top and bottom segments of every
        // strip at the slab plan's full segment length T (what the unsplit plan would run
        // there), the rest of the plan now: a K-row border segment paid the K = 20 pipeline
        // fill (~94 iterations) for 20 rows beside the interior (MM_BORDER_SEGMENTS=0).
        long long T = depth;
        if (e->border_segments) {
            mm::PassArgs P = A;
            wide_range(e, k, red, P, 0, h);
            T = std::min<long long>(std::max<long long>(P.th, depth), h / 2);
        }
        wide_range(e, k, red, A, T, h - T);
        const long long interior = A.waves_total;
        mm::PassArgs B = A;
        A.partial_base = 0;
        MM_TRY(launch_timed(e, red, A, h - 2 * T, time_it, -k));
        MM_TRY(split_comm(e, depth));
        B.th = B.th_edge = (int)T;
        B.ra0 = 0;
        B.ra1 = (int)T;
        B.rb0 = (int)(h - T);
        B.rb1 = (int)h;
        B.waves_a = seg_wave_count(T, B.nstrips, T, T);
        B.waves_total = 2 * B.waves_a;
        B.partial_base = interior;
        MM_HIP(mm::launch_wide(k, wcols(e, k), e->na, red, B, e->s_comm, wvar(e)));
        MM_HIP(hipEventRecord(e->ev_comm_done, e->s_comm));
        e->comm_live = true;
        total_blocks = interior + B.waves_total;
        if (red) MM_HIP(hipStreamWaitEvent(e->s_comp, e->ev_comm_done, 0));
    } else {
        if (e->split) MM_TRY(unsplit_halo(e, depth));
        wide_range(e, k, red, A, 0, h);
        A.partial_base = 0;
        MM_TRY(launch_timed(e, red, A, h, time_it, -k));
        total_blocks = A.waves_total;
    }
    if (red)
        MM_HIP(mm::launch_finalize_levels(e->partials, total_blocks, k, e->na, mask, e->hist,
                                          e->hist_n, e->hist_cap, e->s_comp, perm));
    e->cur ^= 1;
    return MM_OK;
}

// k fused steps of the one-pass program in one mm_passk_kernel pass; bit j of `mask`:
// append the sums after step j+1 of the pass to the history. Same two-stream structure as
// enqueue_pass, with a k-row halo (every k steps): the interior rows run as segments
// beside the exchange, the border rows as 4-row blocks after it.
int enqueue_passk(mm_engine* e, int k, int mask, bool time_it) {
    if (use_wide(e, k)) return enqueue_wide(e, k, mask, time_it);
    const long long h = e->d.h;
    const int depth = k;
    const bool red = mask != 0;
    mm::PassArgs A;
    fill_args(e, e->passes[0], A);
    A.nstrips = (int)nstrips_k(e, k);
    A.xcd_remap = e->xcd;
    long long total_waves = 0;
    if (e->split && h >= 2 * depth + 1) {
        MM_TRY(split_comp(e));
        seg_range(e, k, red, A, depth, h - depth);
        const long long interior_waves = A.waves_total;
        mm::PassArgs B = A;
        A.partial_base = 0;
        MM_TRY(launch_timed(e, red, A, h - 2 * depth, time_it, k));
        MM_TRY(split_comm(e, depth));
        B.seg = 0;
        B.th = mm::kBorderRows;  // border: short row blocks, the launch is latency-bound
        B.xcd_remap = 0;
        set_ranges(B, 0, depth, h - depth, h);
        B.partial_base = interior_waves;
        MM_HIP(mm::launch_passk(k, e->na, red, B, e->s_comm, 0));
        MM_HIP(hipEventRecord(e->ev_comm_done, e->s_comm));
        e->comm_live = true;
        total_waves = interior_waves + B.waves_total;
        if (red) MM_HIP(hipStreamWaitEvent(e->s_comp, e->ev_comm_done, 0));
    } else {
        if (e->split) MM_TRY(unsplit_halo(e, depth));
        seg_range(e, k, red, A, 0, h);
        A.partial_base = 0;
        MM_TRY(launch_timed(e, red, A, h, time_it, k));
        total_waves = A.waves_total;
    }
    if (red)
        MM_HIP(mm::launch_finalize_levels(e->partials, total_waves, k, e->na, mask, e->hist,
                                          e->hist_n, e->hist_cap, e->s_comp, kPermIdentity));
    e->cur ^= 1;
    return MM_OK;
}

// One step (all passes); reduce: append the per-attribute sums to the history.
int enqueue_step(mm_engine* e, bool reduce, bool time_it) {
    const int np = (int)e->passes.size();
    for (int pi = 0; pi < np; ++pi)
        MM_TRY(enqueue_pass(e, e->passes[pi], reduce && pi == np - 1, time_it));
    return MM_OK;
}

// Can the program run on mm_passk_kernel? One pass per step (one attribute: a single
// diffusion; several: diffusions and transfer chains) and buffer offsets below 2^31.
bool passk_ok(const mm_engine* e) {
    if (!e->passk || e->passes.size() != 1) return false;
    if (mm::passk_max_rows(mm::kMaxSteps, e->pitch) < 64) return false;
    const Pass& p = e->passes[0];
    if (e->na == 1) return p.diffuse_mask == 1 && p.pre.empty() && p.post.empty();
    return true;
}

constexpr int kWideAuto = 20;      // auto steps per pass of the wide kernel, one attribute
constexpr int kWideAutoMulti = 8;  // several attributes

// Steps per K-step pass: the configured K, capped so that a depth-K halo never reaches
// past the thinnest slab of the chain (every rank sends K owned rows each way).
int passk_steps(const mm_engine* e) {
    // one attribute, auto: K = 8 on slabs of >= 2^27 cells, else 7 -- the fastest K per
    // step of the round-2 sweeps (profiles/r02/sweep_k_*.log, profiles/r02c/sweep_*x32768:
    // 32768^2, 16384^2 and the 8192- and 4096-row slabs of 32768 columns favour 8, 4096^2
    // with its short segments 7; K <= 4 leaves the VALU idle behind the HBM stream)
    // (sized by the chain's thinnest slab, the same on every rank: every rank of a halo
    // chain must run the same passes, or the K-row exchanges would not pair up)
    // wide (mm_wide_kernel): auto K = kWideAuto
    // (wide on a small slab: kWideSmallAuto passes, no planner)
    const int kauto = (wide_on(e) && e->na == 1)
                          ? (wide_big(e) ? kWideAuto : kWideSmallAuto)
                          : (slab_cells(e) >= 134217728.0 ? 8 : 7);
    int k1 = e->kpass > 0 ? e->kpass : kauto;
    if (!(wide_on(e) && e->na == 1)) k1 = std::min(k1, mm::kMaxSteps);  // mm_passk_kernel's K
    int k = e->na == 1 ? k1 : std::min(e->kpass_multi, mm::passk_max_steps(e->na));
    // several attributes, wide kernel: its K (auto kWideAutoMulti), or mm_passk_kernel's
    if (e->na > 1 && wide_on(e) && passk_ok(e)) {
        k = e->kpass > 0 ? e->kpass : kWideAutoMulti;
        if (!mm::wide_has(k, 2, e->na)) k = std::min(k, mm::passk_max_steps(e->na));
    }
    if (e->d.nranks > 1) k = (int)std::min<long long>(k, e->min_rows);
    return std::max(1, k);
}

// Steps one kernel pass advances: K with the K-step kernel, 1 otherwise.
int steps_per_launch(const mm_engine* e) { return passk_ok(e) ? passk_steps(e) : 1; }

// Ghost rows one exchange must fill (host transport: mm_halo_export_rows / _import_rows).
int halo_depth(const mm_engine* e) { return steps_per_launch(e); }

// Modelled time of one K-step pass of a large one-attribute slab, relative to the K = 8
// pass: the HBM stream of the grid (`kStream`: the K <= 7 passes, which the stream
// bounds), or the VALU work of K levels over the strips' 128 - 4*ceil(K/2) output
// columns, whichever is longer (K >= 8 are VALU-bound: 32768^2 on one box, K = 8 / 9 /
// 10: 3437 / 3884 / 4326 us, profiles/r02b/k9k10/edge_*; K = 7 0.93 of K = 8,
// profiles/r02b/segwaves).
double pass_cost(int k) {
    constexpr double kStream = 0.93;
    constexpr double kValuPerLevel = 112.0 / (8.0 * 128.0);  // K = 8 -> 1.0
    const double useful = (double)mm::passk_out_cols(k) / (double)mm::kStripCols;
    return std::max(kStream, kValuPerLevel * (double)k / useful);
}

// Steps of the next K-step pass when n steps remain: ceil(n / K) passes of balanced
// length (20 steps at K = 8: 7 + 7 + 6, not 8 + 8 + 4), where K is the auto or configured
// steps per pass. On a large one-attribute slab with K auto, the planner also considers
// fewer, longer passes (up to kMaxSteps, capped by the chain's thinnest slab) and takes
// the plan of least modelled time: 20 steps run as 10 + 10, a long run stays at K = 8
// (1000 steps: 125 passes).
// A pass of k steps has a kernel: the wide one (use_wide) or mm_passk_kernel (k <= 10).
bool pass_len_ok(const mm_engine* e, long long k) {
    return k >= 1 && (k <= mm::passk_max_steps(e->na) || use_wide(e, (int)k));
}

// Modelled time of one k-step pass on a large slab with the wide kernel on, in ms at
// 32768^2: mm_passk_kernel K <= 7 stream-bound at ~3.5 ms, K = 8 / 9 / 10 at 3.66 / 4.14 /
// 4.62 (profiles/r02b); mm_wide_kernel K = 4 / 8 at 3.69 / 3.68 (profiles/r03/kernel_table)
// and K = 12 / 16 / 20 at 0.778 / 1 / 1.236 of the K = 16 pass (one box,
// profiles/r03/xcd2/kernel_table.log: 5120 / 6578 / 8128 us; K = 20 with ascending levels).
double wide_plan_cost(const mm_engine* e, int k) {
    if (use_wide(e, k)) {
        switch (k) {
            case 4: return 3.69;
            case 8: return 3.68;
            case 12: return 4.84;
            case 16: return 6.22;
            default: return 7.69;
        }
    }
    if (k <= 7) return 3.50;
    return k == 8 ? 3.66 : (k == 9 ? 4.14 : 4.62);
}

// Steps of the first pass of the cheapest plan of n steps (wide on, K auto): a dynamic
// program over the pass lengths both kernels have (capped by the chain's thinnest slab).
// Runs longer than kDpMax steps start with a pass of the best per-step length (K = 20).
int wide_plan_first(const mm_engine* e, long long n, int kcap) {
    constexpr int kDpMax = 256;
    if (n > kDpMax) return std::min(kWideAuto, kcap);
    std::vector<double> best((size_t)n + 1, 1e300);
    std::vector<int> first((size_t)n + 1, 1);
    best[0] = 0.0;
    for (long long m = 1; m <= n; ++m)
        for (int k = 1; k <= std::min<long long>(m, kcap); ++k) {
            if (!pass_len_ok(e, k)) continue;
            const double c = wide_plan_cost(e, k) + best[(size_t)(m - k)];
            if (c < best[(size_t)m] * (1.0 - 1e-9)) {
                best[(size_t)m] = c;
                first[(size_t)m] = k;
            }
        }
    return first[(size_t)n];
}

int next_pass_len(const mm_engine* e, long long n) {
    const int kp = passk_steps(e);
    if (e->na > 1 && wide_on(e)) {  // passes of K while n >= K, then the longest that fit
        long long k = std::min<long long>(n, kp);
        while (k > 1 && !pass_len_ok(e, k)) --k;
        return (int)std::max<long long>(1, k);
    }
    if (wide_on(e) && e->na == 1) {
        if (e->kpass == 0 && e->plan && wide_big(e)) {
            int cap = mm::kMaxWide;
            if (e->d.nranks > 1) cap = (int)std::min<long long>(cap, e->min_rows);
            return wide_plan_first(e, n, cap);
        }
        // configured K: passes of K while n >= K, a shorter run in one pass when a kernel
        // has that length, else the longest length a kernel has
        long long k = std::min<long long>(n, kp);
        while (k > 1 && !pass_len_ok(e, k)) --k;
        return (int)std::max<long long>(1, k);
    }
    long long best_p = (n + kp - 1) / kp;
    // the planner's slabs: >= 2^28 cells in >= 256 strips. With fewer strips the two edge
    // strips (the general body, which spills at K >= 9) weigh more and deep passes lose:
    // 16384^2, 20 steps: 10 + 10 2.85 ms vs 7 + 7 + 6 2.61 ms; 32768 columns at 8192 and
    // 32768 rows: 10 + 10 wins by 7 % (profiles/r02_end/k10tune, profiles/r02c).
    const bool big = (double)e->min_rows * (double)e->d.W >= 268435456.0 &&  // rank-invariant
                     nstrips_k(e, mm::kMaxSteps) >= 256;
    if (e->plan && e->kpass == 0 && e->na == 1 && big && n > kp) {
        long long kx = mm::passk_max_steps(1);
        if (e->d.nranks > 1) kx = std::min<long long>(kx, e->min_rows);
        double best = 1e300;
        const long long p_max = best_p;
        for (long long p = (n + kx - 1) / kx; p <= p_max; ++p) {
            const long long q = n / p, r = n % p;  // r passes of q + 1 steps, p - r of q
            const double t = (double)r * pass_cost((int)q + 1) + (double)(p - r) * pass_cost((int)q);
            if (t < best * (1.0 - 1e-9)) {
                best = t;
                best_p = p;
            }
        }
    }
    return (int)((n + best_p - 1) / best_p);
}

// Enqueue steps [first, first+n) of a run (1-based step numbers decide the reductions).
int enqueue_steps(mm_engine* e, long long first, long long n, long long reduce_every,
                  bool time_it) {
    long long s = first;
    const long long end = first + n;
    auto red = [&](long long step) { return reduce_every > 0 && step % reduce_every == 0; };
    if (passk_ok(e)) {
        while (s < end) {
            const int k = next_pass_len(e, end - s);
            int mask = 0;
            for (int j = 0; j < k; ++j)
                if (red(s + j)) mask |= 1 << j;
            MM_TRY(enqueue_passk(e, k, mask, time_it));
            s += k;
        }
    } else {
        for (; s < end; ++s) MM_TRY(enqueue_step(e, red(s), time_it));
    }
    // the compute stream is the tail of every run (and of every captured graph)
    if (e->comm_live) {
        MM_HIP(hipStreamWaitEvent(e->s_comp, e->ev_comm_done, 0));
        e->comm_live = false;
    }
    return MM_OK;
}

long long gcd_ll(long long a, long long b) {
    while (b) {
        long long t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// Every rank of an RCCL chain must run the same passes, or the K-row exchanges would not
// pair up: a graph replays the passes of its length, the eager fallback plans the rest of
// the run. So whether a capture worked is agreed over the chain (one all-reduce of a flag,
// at the first capture of each graph: every rank captures the same keys at the same call,
// which needs the same MM_GRAPH setting, timing mode and run lengths on every rank --
// include/mpimodel.h). The all-reduce shares the communicator with the halo send / recv
// of earlier runs, which may still be replaying on the compute stream: both streams are
// drained first, so no two RCCL operations of this communicator are in flight at once.
int agree_capture(mm_engine* e, bool ok) {
    if (!e->comm || e->d.nranks <= 1) return ok ? MM_OK : MM_ERR_HIP;
    int v = ok ? 1 : 0;
    int* dv = reinterpret_cast<int*>(e->sum_tmp);
    if (hipStreamSynchronize(e->s_comp) != hipSuccess ||
        hipStreamSynchronize(e->s_comm) != hipSuccess ||
        hipMemcpy(dv, &v, sizeof v, hipMemcpyHostToDevice) != hipSuccess ||
        ncclAllReduce(dv, dv, 1, ncclInt32, ncclMin, e->comm, e->s_comm) != ncclSuccess ||
        hipStreamSynchronize(e->s_comm) != hipSuccess ||
        hipMemcpy(&v, dv, sizeof v, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(MM_ERR_RCCL, "capture agreement all-reduce failed");
    if (v) return MM_OK;
    return ok ? fail(MM_ERR_HIP, "another rank's stream capture was refused") : MM_ERR_HIP;
}

int capture_graph(mm_engine* e, long long len, long long reduce_every, long long phase,
                  hipGraphExec_t* out, int* flip);

int get_graph(mm_engine* e, long long len, long long reduce_every, long long phase,
              hipGraphExec_t* out, int* flip) {
    auto key = std::make_tuple(e->cur, len, reduce_every, phase);
    auto it = e->graphs.find(key);
    if (it != e->graphs.end()) {
        *out = it->second.first;
        *flip = it->second.second;
        return MM_OK;
    }
    const int rc = capture_graph(e, len, reduce_every, phase, out, flip);
    const std::string why = g_last_error;
    const int ra = agree_capture(e, rc == MM_OK);
    if (rc != MM_OK) g_last_error = why;
    return rc != MM_OK ? rc : ra;
}

int capture_graph(mm_engine* e, long long len, long long reduce_every, long long phase,
                  hipGraphExec_t* out, int* flip) {
    auto key = std::make_tuple(e->cur, len, reduce_every, phase);
    const int cur0 = e->cur;
    MM_HIP(hipStreamBeginCapture(e->s_comp, hipStreamCaptureModeThreadLocal));
    const int rc = enqueue_steps(e, phase + 1, len, reduce_every, false);
    hipGraph_t g = nullptr;
    hipError_t ec = hipStreamEndCapture(e->s_comp, &g);
    const int parity = e->cur ^ cur0;  // the captured passes' buffer flips, mod 2
    e->cur = cur0;  // capture only recorded the work; the state advances at replay
    e->comm_live = false;
    if (rc != MM_OK) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (ec != hipSuccess) return fail(MM_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
    hipGraphExec_t ge = nullptr;
    ec = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ec != hipSuccess) return fail(MM_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ec));
    e->graphs[key] = std::make_pair(ge, parity);
    e->graph_count += 1;
    *out = ge;
    *flip = parity;
    return MM_OK;
}

// Rows per wave of the one-step kernel (a compile-time row block: 8, 16 or 32). Short
// blocks give the most waves in flight, which is what the memory system wants
// (tools/sweep.py, profiles/r01): 8 by default, MM_ROWS_PER_WAVE overrides.
int choose_th(const mm_engine* e) {
    (void)e;
    if (const char* s = std::getenv("MM_ROWS_PER_WAVE")) {
        const int v = std::atoi(s);
        if (v == 8 || v == 16 || v == 32) return v;
    }
    return 8;
}

int ensure_partials(mm_engine* e) {
    // doubles: one-step kernel, 128-column strips x 8-row blocks with kMaxAttr sums per
    // wave (+ 1-row border blocks); mm_passk_kernel, segments of >= 8 rows (edge strips)
    // plus 4-row border blocks (depth <= kGhost rows on each side) with K x NA sums per
    // wave: K <= kMaxSteps for one attribute, K <= 2 for up to kMaxAttr
    long long need = (waves_for(e, e->d.h, 8) + 2 * waves_for(e, 2, 1) + 16) * mm::kMaxAttr;
    const long long ns = nstrips_k(e, mm::kMaxSteps);
    const long long border = 2 * ((mm::kGhost + mm::kBorderRows - 1) / mm::kBorderRows) + 2;
    need = std::max(need, (ns * ((e->d.h + 7) / 8 + border) + 16) *
                              std::max(mm::kMaxWide, 8 * mm::kMaxAttr));
    if (need <= e->partials_cap) return MM_OK;
    if (e->partials) (void)hipFree(e->partials);
    e->partials = nullptr;
    MM_HIP(hipMalloc(&e->partials, sizeof(double) * (size_t)need));
    e->partials_cap = need;
    return MM_OK;
}

// Make room for `more` history entries beyond the ones already enqueued. The history
// pointer is captured by the step graphs, so growing it drops them.
int reserve_history(mm_engine* e, long long more) {
    const long long need = e->hist_host + more;
    if (need <= e->hist_cap) return MM_OK;
    const long long cap = std::max(need, 2 * e->hist_cap);
    double* nh = nullptr;
    MM_HIP(hipStreamSynchronize(e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    MM_HIP(hipMalloc(&nh, sizeof(double) * (size_t)cap * e->na));
    MM_HIP(hipMemcpyAsync(nh, e->hist, sizeof(double) * (size_t)e->hist_cap * e->na,
                          hipMemcpyDeviceToDevice, e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    (void)hipFree(e->hist);
    e->hist = nh;
    e->hist_cap = cap;
    drop_graphs(e);
    return MM_OK;
}

int copy_rows(mm_engine* e, bool to_host, long long row0, int nrows, double* host) {
    const long long W = e->d.W, P = e->pitch;
    for (int a = 0; a < e->na; ++a) {
        double* dev = e->buf[e->cur][a] + row0 * P;
        double* hp = host + (size_t)a * nrows * W;
        if (to_host)
            MM_HIP(hipMemcpy2DAsync(hp, sizeof(double) * W, dev, sizeof(double) * P,
                                    sizeof(double) * W, nrows, hipMemcpyDeviceToHost, e->s_comp));
        else
            MM_HIP(hipMemcpy2DAsync(dev, sizeof(double) * P, hp, sizeof(double) * W,
                                    sizeof(double) * W, nrows, hipMemcpyHostToDevice, e->s_comp));
    }
    return MM_OK;
}

}  // namespace

extern "C" {

int mm_abi_version(void) { return MM_ABI_VERSION; }

const char* mm_last_error(void) { return g_last_error.c_str(); }

long long mm_step_count(double time, double time_step) {
    if (!(time_step > 0.0)) return -1;  // the reference would loop forever
    long long n = 0;
    for (double t = 0; t < time; t = t + time_step) ++n;  // src/Model.hpp:48, same fp64 sequence
    return n;
}

int mm_partition_reference(int H, int W, int P, int k, int* x_init, int* y_init, int* height,
                           int* width) {
    if (H <= 0 || W <= 0 || P <= 0 || k < 1 || k > P || !x_init || !y_init || !height || !width)
        return fail(MM_ERR_INVALID, "mm_partition_reference: bad arguments");
    const int count = (H * W) / P;  // src/Model.hpp:63
    const int offset = (k - 1) * count;
    *x_init = offset / W;  // src/Model.hpp:72
    *y_init = 0;
    *height = H / P;
    *width = W;
    return MM_OK;
}

int mm_owner_reference(int H, int P, int x) {
    if (H <= 0 || P <= 0 || H / P == 0) return -1;
    return x / (H / P) + 1;  // src/Model.hpp:80
}

int mm_partition_rows(long long H, int G, int g, long long* x_init, long long* h) {
    if (H <= 0 || G <= 0 || g < 0 || g >= G || !x_init || !h)
        return fail(MM_ERR_INVALID, "mm_partition_rows: bad arguments");
    const long long a = (g * H) / G, b = ((g + 1) * H) / G;
    *x_init = a;
    *h = b - a;
    return MM_OK;
}

int mm_neighbor_count(long long H, long long W, long long x, long long y) {
    const long long sx = span_rows(H, x), sy = span_rows(W, y);
    return (sx && sy) ? (int)(sx * sy - 1) : 0;
}

int mm_comm_id_size(void) { return (int)sizeof(ncclUniqueId); }

int mm_comm_id_create(void* out, int len) {
    if (!out || len < (int)sizeof(ncclUniqueId)) return fail(MM_ERR_INVALID, "mm_comm_id_create: buffer too small");
    ncclUniqueId id;
    MM_NCCL(ncclGetUniqueId(&id));
    std::memcpy(out, &id, sizeof id);
    return MM_OK;
}

int mm_device_synchronize(int device) {
    MM_HIP(hipSetDevice(device));
    MM_HIP(hipDeviceSynchronize());
    return MM_OK;
}

int mm_device_count(int* n) {
    if (!n) return fail(MM_ERR_INVALID, "mm_device_count: null");
    MM_HIP(hipGetDeviceCount(n));
    return MM_OK;
}

int mm_engine_create(const mm_desc* desc, mm_engine** out) {
    if (!desc || !out) return fail(MM_ERR_INVALID, "mm_engine_create: null argument");
    *out = nullptr;
    const mm_desc& d = *desc;
    if (d.H <= 0 || d.W <= 0 || d.h <= 0 || d.x_init < 0 || d.x_init + d.h > d.H)
        return fail(MM_ERR_INVALID, "mm_engine_create: slab outside the grid");
    if (d.n_attr < 1 || d.n_attr > mm::kMaxAttr)
        return fail(MM_ERR_INVALID, "mm_engine_create: n_attr must be 1..4");
    if (d.nranks < 1 || d.rank < 0 || d.rank >= d.nranks)
        return fail(MM_ERR_INVALID, "mm_engine_create: bad rank/nranks");
    if (d.nranks == 1 && (d.x_init != 0 || d.h != d.H))
        return fail(MM_ERR_INVALID, "mm_engine_create: a single slab must own the whole grid");
    if (d.halo_mode == MM_HALO_RCCL && !d.comm_id)
        return fail(MM_ERR_INVALID, "mm_engine_create: MM_HALO_RCCL needs comm_id");
    if (d.nranks > 1 && d.halo_mode == MM_HALO_NONE)
        return fail(MM_ERR_INVALID, "mm_engine_create: nranks > 1 needs a halo mode");
    if (d.W > (1LL << 30) || d.h > (1LL << 30))
        return fail(MM_ERR_INVALID, "mm_engine_create: slab too large");

    mm_engine* e = new mm_engine();
    e->d = d;
    e->na = d.n_attr;
    e->pitch = (d.W + mm::kStripCols - 1) / mm::kStripCols * mm::kStripCols;
    e->nstrips = (int)(e->pitch / mm::kStripCols);
    e->rows_alloc = d.h + 2 * mm::kGhost;
    // thinnest slab of the chain: mm_partition_rows slabs are at least floor(H/G) rows
    // (RCCL engines replace this with the chain's true minimum below)
    e->min_rows = std::min<long long>(d.h, d.H / d.nranks);
    if (const char* g = std::getenv("MM_GRAPH")) e->graphs_ok = std::atoi(g) != 0;
    if (const char* g = std::getenv("MM_GRAPH_MIN_STEPS")) {
        const long long v = std::atoll(g);
        if (v >= 1 && v <= 256) e->graph_min = v;
    }
    if (const char* g = std::getenv("MM_GRAPH_MAX_LAUNCHES")) {
        const long long v = std::atoll(g);
        if (v >= 1 && v <= 4096) e->graph_max = v;
    }
    e->th = choose_th(e);
    if (const char* f = std::getenv("MM_FUSE")) e->passk = e->passk && std::atoi(f) != 0;
    if (const char* p = std::getenv("MM_PASSK")) e->passk = e->passk && std::atoi(p) != 0;
    if (const char* w = std::getenv("MM_WIDE")) e->wide = std::atoi(w) != 0 ? 1 : 0;
    if (const char* k = std::getenv("MM_STEPS_PER_PASS")) {
        const int v = std::atoi(k);
        if (v >= 1 && (v <= mm::kMaxSteps || (e->wide != 0 && (mm::wide_has(v, 4, 1) || mm::wide_has(v, 2, 4)))))
            e->kpass = v;
        if (v >= 1) e->kpass_multi = std::min(v, 2);
    }
    if (const char* p = std::getenv("MM_PASS_PLAN")) e->plan = std::atoi(p) != 0;
    if (const char* f = std::getenv("MM_SEG_WAVES")) {
        const double v = std::atof(f);
        if (v > 0.0) e->seg_waves = v;
    }
    if (const char* f = std::getenv("MM_SEG_EDGE")) {
        const double v = std::atof(f);
        if (v > 0.0 && v <= 1.0) e->seg_edge = v;
    }
    if (const char* x = std::getenv("MM_XCD_REMAP")) e->xcd = std::atoi(x) != 0;
    if (const char* b = std::getenv("MM_BORDER_SEGMENTS")) e->border_segments = std::atoi(b) != 0;
    if (const char* r = std::getenv("MM_CHAIN_RING")) e->ring_ok = std::atoi(r) != 0;
    if (const char* r = std::getenv("MM_SYNC_SPIN")) e->sync_spin = std::atoi(r) != 0;
    // non-temporal stores pay once the two buffers outgrow the 256 MiB Infinity Cache
    // (profiles/r01 sweeps); MM_KERNEL_VARIANT overrides
    e->variant = 2.0 * 8.0 * (double)e->pitch * (double)d.h * d.n_attr > 256.0 * 1048576.0 ? 1 : 0;
    if (const char* v = std::getenv("MM_KERNEL_VARIANT")) e->variant = std::atoi(v);

    auto cleanup = [&](int rc) {
        mm_engine_destroy(e);
        return rc;
    };
    hipError_t he = hipSetDevice(d.device);
    if (he != hipSuccess) return cleanup(fail(MM_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he)));
    he = hipDeviceGetAttribute(&e->ncu, hipDeviceAttributeMultiprocessorCount, d.device);
    if (he != hipSuccess || e->ncu <= 0) e->ncu = 256;

    const size_t per = (size_t)e->rows_alloc * (size_t)e->pitch;  // doubles per buffer
    const size_t per_al = (per + 31) / 32 * 32;                   // 256-B aligned buffers
    e->bytes = sizeof(double) * per_al * 2 * (size_t)e->na;
    if (hipStreamCreateWithFlags(&e->s_comp, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_comm, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_halo, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_comp_mark, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e->ev_comm_done, hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(MM_ERR_HIP, "stream/event creation failed"));

    he = hipMalloc(&e->base, e->bytes);
    if (he != hipSuccess) return cleanup(fail(MM_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(he)));
    // zeroed on the compute stream: every fill, upload and pass is enqueued there (or, on
    // the comm stream, behind an event recorded there), so they all follow it. A zeroing
    // on the null stream would not be ordered before them -- the engine's streams are
    // non-blocking -- and once did land after a fill on memory another engine had just
    // freed (tests/test_gpu_parity.py::test_fill_after_freed_engine)
    he = hipMemsetAsync(e->base, 0, e->bytes, e->s_comp);
    if (he != hipSuccess) return cleanup(fail(MM_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(he)));
    for (int k = 0; k < 2; ++k)
        for (int a = 0; a < e->na; ++a)
            e->buf[k][a] = e->base + per_al * (size_t)(k * e->na + a) + mm::kGhost * e->pitch;

    int rc = ensure_partials(e);
    if (rc != MM_OK) return cleanup(rc);
    e->hist_cap = 1 << 12;
    if (hipMalloc(&e->hist, sizeof(double) * (size_t)e->hist_cap * e->na) != hipSuccess ||
        hipMalloc(&e->hist_n, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemsetAsync(e->hist_n, 0, 2 * sizeof(unsigned long long), e->s_comp) != hipSuccess)
        return cleanup(fail(MM_ERR_NOMEM, "history allocation failed"));
    e->sum_blocks = std::min<long long>(1024, std::max<long long>(1, d.h));
    if (hipMalloc(&e->sum_tmp, sizeof(double) * (size_t)(e->sum_blocks + mm::kMaxAttr)) != hipSuccess)
        return cleanup(fail(MM_ERR_NOMEM, "sum scratch allocation failed"));
    // the zeroing above is queued on the compute stream; waiting for it here keeps a
    // failure on this call (and costs no other engine anything: only this stream)
    he = hipStreamSynchronize(e->s_comp);
    if (he != hipSuccess) return cleanup(fail(MM_ERR_HIP, std::string("hipStreamSynchronize: ") + hipGetErrorString(he)));

    if (const char* sh = std::getenv("MM_SELF_HALO"))
        e->self_halo = d.nranks == 1 && d.halo_mode == MM_HALO_RCCL && std::atoi(sh) != 0;
    if ((d.nranks > 1 || e->self_halo) && d.halo_mode == MM_HALO_RCCL) {
        // a process that loaded another librccl.so.1 first (PyTorch bundles one) would
        // run this code against a different RCCL: refuse instead of crashing later
        int v = 0;
        if (ncclGetVersion(&v) != ncclSuccess || v != NCCL_VERSION_CODE) {
            char msg[160];
            std::snprintf(msg, sizeof msg,
                          "RCCL %d loaded, engine built against %d: load libmpimodel_hip.so "
                          "before any library that bundles its own librccl (e.g. torch)",
                          v, NCCL_VERSION_CODE);
            return cleanup(fail(MM_ERR_RCCL, msg));
        }
        ncclUniqueId id;
        std::memcpy(&id, d.comm_id, sizeof id);
        ncclResult_t nr = ncclCommInitRank(&e->comm, d.nranks, id, d.rank);
        if (nr != ncclSuccess)
            return cleanup(fail(MM_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(nr)));
        // the chain's thinnest slab (one setup-time collective): a depth-K exchange must
        // never send more rows than any rank owns
        long long hmin = d.h;
        double* dv = e->sum_tmp;
        if (hipMemcpy(dv, &hmin, sizeof hmin, hipMemcpyHostToDevice) != hipSuccess ||
            ncclAllReduce(dv, dv, 1, ncclInt64, ncclMin, e->comm, e->s_comm) != ncclSuccess ||
            hipStreamSynchronize(e->s_comm) != hipSuccess ||
            hipMemcpy(&hmin, dv, sizeof hmin, hipMemcpyDeviceToHost) != hipSuccess)
            return cleanup(fail(MM_ERR_RCCL, "min slab rows all-reduce failed"));
        e->min_rows = hmin;
        e->split = true;
    } else if (d.nranks > 1 && d.halo_mode == MM_HALO_HOST) {
        // the host transport sizes K and the halo depth from the standard partition
        // (min_rows above), so a neighbour of a caller-chosen thinner slab could be asked
        // for rows it does not own: only mm_partition_rows slabs are accepted
        long long x0 = 0, hh = 0;
        if (mm_partition_rows(d.H, d.nranks, d.rank, &x0, &hh) != MM_OK || x0 != d.x_init ||
            hh != d.h)
            return cleanup(fail(MM_ERR_INVALID, "mm_engine_create: MM_HALO_HOST slabs must be "
                                                "mm_partition_rows(H, nranks, rank)"));
        e->split = true;
    }
    // default program: one Exponencial flow on attribute 0 is set by the caller
    *out = e;
    return MM_OK;
}

int mm_engine_destroy(mm_engine* e) {
    if (!e) return MM_OK;
    (void)hipSetDevice(e->d.device);
    if (e->s_comp) (void)hipStreamSynchronize(e->s_comp);
    if (e->s_comm) (void)hipStreamSynchronize(e->s_comm);
    drop_graphs(e);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    for (hipEvent_t ev : e->ev_pool) (void)hipEventDestroy(ev);
    if (e->ev_ready) (void)hipEventDestroy(e->ev_ready);
    if (e->ev_halo) (void)hipEventDestroy(e->ev_halo);
    if (e->ev_comp_mark) (void)hipEventDestroy(e->ev_comp_mark);
    if (e->ev_comm_done) (void)hipEventDestroy(e->ev_comm_done);
    if (e->s_comp) (void)hipStreamDestroy(e->s_comp);
    if (e->s_comm) (void)hipStreamDestroy(e->s_comm);
    if (e->base) (void)hipFree(e->base);
    if (e->partials) (void)hipFree(e->partials);
    if (e->hist) (void)hipFree(e->hist);
    if (e->hist_n) (void)hipFree(e->hist_n);
    if (e->sum_tmp) (void)hipFree(e->sum_tmp);
    (void)hipGetLastError();  // statuses above are ignored on purpose; do not leave them pending
    delete e;
    return MM_OK;
}

int mm_engine_info(mm_engine* e, mm_info* info) {
    if (!e || !info) return fail(MM_ERR_INVALID, "mm_engine_info: null");
    std::memset(info, 0, sizeof *info);
    info->pitch = e->pitch;
    info->bytes_device = (long long)e->bytes;
    info->n_passes = (int)e->passes.size();
    const int spl = steps_per_launch(e);
    if (passk_ok(e) && use_wide(e, spl)) {  // one workgroup of 4 waves per strip segment
        mm::PassArgs A;
        std::memset(&A, 0, sizeof A);
        A.nstrips = (int)nstrips_wide(e, spl);
        wide_range(e, spl, false, A, 0, e->d.h);
        info->rows_per_wave = A.th;
        const int c = wcols(e, spl);
        info->waves_per_pass = A.waves_total * mm::wide_waves_per_block(spl, c, e->na, wring(e) != 0);
        info->kernel = 3;
        if (e->na > 1) info->chain_kernel = (wring(e) && spl == 8) ? MM_CHAIN_RING : MM_CHAIN_RUNTIME;
        info->seg_waves_per_cu =
            e->bpc[((long long)((e->variant & 1) | wvar(e)) << 8) | spl] *
            mm::wide_waves_per_block(spl, c, e->na, wring(e) != 0);
    } else if (passk_ok(e)) {  // the whole-slab segment plan of one pass
        mm::PassArgs A;
        std::memset(&A, 0, sizeof A);
        A.nstrips = (int)nstrips_k(e, spl);
        seg_range(e, spl, false, A, 0, e->d.h);
        info->rows_per_wave = A.th;
        info->waves_per_pass = A.waves_total;
        info->kernel = 2;
        info->seg_waves_per_cu = e->wpc[0][e->variant & 1][e->na][spl];
    } else {
        info->kernel = 0;
        info->rows_per_wave = e->th;
        info->waves_per_pass = waves_for(e, e->d.h);
    }
    info->steps_done = e->steps_done;
    info->fused_attrs = e->na;
    info->steps_per_launch = spl;
    info->halo_depth = halo_depth(e);
    info->graph_state = e->graph_state;
    info->graph_count = e->graph_count;
    info->graph_launches = e->graph_launches;
    info->hist_entries = e->hist_host;
    std::snprintf(info->graph_note, sizeof info->graph_note, "%s", e->graph_note.c_str());
    return MM_OK;
}

int mm_fill(mm_engine* e, int attr, int mode, double value, unsigned long long seed) {
    if (!e || attr < 0 || attr >= e->na || (mode != MM_FILL_UNIFORM && mode != MM_FILL_RANDOM))
        return fail(MM_ERR_INVALID, "mm_fill: bad arguments");
    MM_TRY(set_device(e));
    MM_HIP(mm::launch_fill(e->buf[e->cur][attr], e->pitch, e->d.H, e->d.W, e->d.x_init, e->d.h,
                           mode, value, seed, e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    e->steps_done = 0;
    return MM_OK;
}

int mm_upload(mm_engine* e, int attr, const double* host) {
    if (!e || !host || attr < 0 || attr >= e->na) return fail(MM_ERR_INVALID, "mm_upload: bad arguments");
    MM_TRY(set_device(e));
    MM_HIP(hipMemcpy2DAsync(e->buf[e->cur][attr], sizeof(double) * e->pitch, host,
                            sizeof(double) * e->d.W, sizeof(double) * e->d.W, e->d.h,
                            hipMemcpyHostToDevice, e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    e->steps_done = 0;
    return MM_OK;
}

int mm_download(mm_engine* e, int attr, double* host) {
    if (!e || !host || attr < 0 || attr >= e->na) return fail(MM_ERR_INVALID, "mm_download: bad arguments");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    MM_HIP(hipMemcpy2DAsync(host, sizeof(double) * e->d.W, e->buf[e->cur][attr],
                            sizeof(double) * e->pitch, sizeof(double) * e->d.W, e->d.h,
                            hipMemcpyDeviceToHost, e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    return MM_OK;
}

int mm_clear_flows(mm_engine* e) {
    if (!e) return fail(MM_ERR_INVALID, "mm_clear_flows: null");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    e->flows.clear();
    e->passes.clear();
    drop_graphs(e);
    return MM_OK;
}

int mm_add_flow(mm_engine* e, int kind, int a, int b, double rate) {
    if (!e) return fail(MM_ERR_INVALID, "mm_add_flow: null");
    if (kind != MM_FLOW_DIFFUSE && kind != MM_FLOW_TRANSFER)
        return fail(MM_ERR_INVALID, "mm_add_flow: unknown flow kind");
    if (a < 0 || a >= e->na) return fail(MM_ERR_INVALID, "mm_add_flow: attribute out of range");
    if (kind == MM_FLOW_TRANSFER && b >= e->na)
        return fail(MM_ERR_INVALID, "mm_add_flow: target attribute out of range");
    if (!std::isfinite(rate)) return fail(MM_ERR_INVALID, "mm_add_flow: rate must be finite");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    e->flows.push_back({kind, a, kind == MM_FLOW_TRANSFER ? (b < 0 ? -1 : b) : a, rate});
    drop_graphs(e);
    MM_TRY(compile_passes(e));
    // transfers or several attributes: the generic kernel exists for 8-row blocks only
    bool chains = e->na > 1;
    for (const Pass& p : e->passes) chains = chains || !p.pre.empty() || !p.post.empty();
    if (chains && e->th != 8) {
        e->th = 8;
        MM_TRY(ensure_partials(e));
    }
    return MM_OK;
}

int mm_point_apply(mm_engine* e, int attr, long long sx, long long sy, double captured,
                   double rate) {
    if (!e || attr < 0 || attr >= e->na) return fail(MM_ERR_INVALID, "mm_point_apply: bad arguments");
    if (sx < 0 || sy < 0 || sx >= e->d.H || sy >= e->d.W)
        return fail(MM_ERR_INVALID, "mm_point_apply: source cell outside the grid");
    MM_TRY(set_device(e));
    MM_HIP(mm::launch_point(e->buf[e->cur][attr], e->pitch, e->d.H, e->d.W, e->d.x_init, e->d.h,
                            sx, sy, captured, rate, e->s_comp));
    return MM_OK;
}

int mm_point_apply_strict(mm_engine* e, int attr, long long sx, long long sy, double captured,
                          double rate, int P, int* applied) {
    if (applied) *applied = 0;
    if (!e || e->d.H > INT32_MAX || e->d.W > INT32_MAX)
        return fail(MM_ERR_INVALID, "mm_point_apply_strict: bad arguments");
    const int ok = mm_point_strict_applies((int)e->d.H, (int)e->d.W, P, (int)sx, (int)sy);
    if (ok < 0) return fail(MM_ERR_INVALID, "mm_point_apply_strict: bad source or worker count");
    if (ok == 0) return MM_OK;  // the reference changes no cell here
    if (applied) *applied = 1;
    return mm_point_apply(e, attr, sx, sy, captured, rate);
}

}  // extern "C"

namespace {

// Graph plan of a run of nsteps steps: `per` steps per replayed graph (0: run eagerly).
// A graph holds a whole number of K-step passes, an even number of buffer flips (so the
// captured pointers are valid again) and of reduction periods (so the phase is the same at
// every replay).
long long graph_per(const mm_engine* e, long long nsteps, long long reduce_every,
                    bool any = false) {
    const long long unit = steps_per_launch(e);
    const long long flips = passk_ok(e) ? 1 : (long long)e->passes.size();
    long long len = unit * ((flips % 2) ? 2 : 1);
    if (reduce_every > 0) len = len / gcd_ll(len, reduce_every) * reduce_every;
    if (len > 256 || nsteps < len || (!e->graphs_ok && !any)) return 0;
    long long per = len;
    while (per < e->graph_min && per * 2 <= nsteps) per *= 2;
    // a short run that is not a whole number of graphs becomes one graph (its passes
    // balanced, enqueue_steps), instead of graphs plus an eager tail; keyed by the buffer
    // parity like every graph, so an odd number of flips is fine
    if (nsteps % per != 0 && nsteps <= 64 * unit) per = nsteps;
    // fewer, longer graphs: consecutive graph launches start ~9 us apart on the GPU, the
    // kernels inside one graph back to back (c2, 16-step graphs: 62 such gaps in 1000
    // steps, 5 % of the run, profiles/r04/final/prof_c2_k8). So the longest whole number of
    // base blocks (the pass length and the reduce period, so every graph starts at the
    // same phase) that divides the run, up to graph_max step kernels
    const long long base = reduce_every > 0 ? unit / gcd_ll(unit, reduce_every) * reduce_every : unit;
    if (nsteps % base == 0) {
        const long long m = nsteps / base, per_block = base / unit * flips;  // kernels per block
        for (long long d = std::min(m, e->graph_max / per_block); d * base > per; --d)
            if (m % d == 0) {
                per = d * base;
                break;
            }
    }
    return per;
}

int check_run(mm_engine* e, long long nsteps, long long reduce_every, const char* who) {
    if (!e || nsteps < 0 || reduce_every < 0) return fail(MM_ERR_INVALID, std::string(who) + ": bad arguments");
    if (nsteps == 0) return MM_OK;
    if (e->passes.empty()) return fail(MM_ERR_STATE, std::string(who) + ": no flow added (mm_add_flow)");
    if (e->d.halo_mode == MM_HALO_HOST && e->d.nranks > 1) {
        if (e->passes.size() != 1)
            return fail(MM_ERR_STATE, std::string(who) + ": the host halo transport runs one-pass flow programs only");
        // one pass per call: the pass planner's length for nsteps (<= kGhost rows exchanged)
        if (nsteps > mm::kGhost || (passk_ok(e) ? next_pass_len(e, nsteps) : 1) != nsteps)
            return fail(MM_ERR_STATE, std::string(who) + ": host halo transport: one pass per call "
                                      "(mm_pass_plan's pass lengths; exchange that many rows between calls)");
    }
    return MM_OK;
}

}  // namespace

extern "C" {

int mm_prepare(mm_engine* e, long long nsteps, long long reduce_every) {
    MM_TRY(check_run(e, nsteps, reduce_every, "mm_prepare"));
    if (nsteps == 0) return MM_OK;
    MM_TRY(set_device(e));
    const long long phase = reduce_every > 0 ? e->steps_done % reduce_every : 0;
    // the history the run appends, grown now: growing it inside mm_run would drop (and
    // re-capture) the graph prepared here
    const long long entries =
        reduce_every > 0 ? (phase + nsteps) / reduce_every - phase / reduce_every : 0;
    MM_TRY(reserve_history(e, entries));
    const long long per = e->timing ? 0 : graph_per(e, nsteps, reduce_every);
    long long tail = nsteps;
    if (per > 0) {
        // both buffer parities: untimed warmup steps run after mm_prepare may leave the
        // state at either one (graphs are keyed by the parity they start from)
        const int cur0 = e->cur;
        for (int par = 0; par < 2 && e->graphs_ok; ++par) {
            e->cur = cur0 ^ par;
            hipGraphExec_t g = nullptr;
            int flip = 0;
            if (get_graph(e, per, reduce_every, phase, &g, &flip) != MM_OK) {
                e->graph_note = g_last_error;
                (void)hipGetLastError();
                e->graphs_ok = false;
                e->graph_state = -1;
            } else {
                MM_HIP(hipGraphUpload(g, e->s_comp));  // the first launch then uploads nothing
                tail = nsteps % per;
            }
        }
        e->cur = cur0;
        MM_HIP(hipStreamSynchronize(e->s_comp));
    }
    // the eagerly launched passes: plan them now, which loads their kernels' code objects,
    // and dispatch each planned kernel once with no work (every workgroup leaves at its
    // first instruction: waves_total = 0), so the queue's scratch is sized for it here and
    // not by the first timed pass (the K = 20 kernel keeps a few hundred bytes of scratch
    // per lane in its GEN code: its first dispatch started 172 us after its launch,
    // profiles/r06/hiptrace). No step runs: no buffer is read or written.
    if (passk_ok(e) && tail > 0) {
        const bool red = reduce_every > 0;
        for (long long s = 0, k = 0; s < tail; s += k) {
            k = next_pass_len(e, tail - s);
            mm::PassArgs A;
            std::memset(&A, 0, sizeof A);
            const bool wide = use_wide(e, (int)k);
            if (wide) {
                A.nstrips = (int)nstrips_wide(e, (int)k);
                wide_range(e, (int)k, red, A, 0, e->d.h);
            } else {
                A.nstrips = (int)nstrips_k(e, (int)k);
                seg_range(e, (int)k, red, A, 0, e->d.h);
            }
            A.waves_total = 0;
            A.waves_a = -1;  // the priming mark (mm::launch_passk / launch_wide)
            MM_TRY(launch_timed(e, red, A, 0, false, wide ? -(int)k : (int)k));
            // a split pass also launches its border rows on the comm stream, another queue
            // with its own scratch: unprimed, the first border launch of a 20-step run
            // blocked the host for 1.5 ms (8192 x 32768 self-halo, profiles/r06/trace20)
            if (e->split && e->d.h >= 2 * k + 1) {
                mm::PassArgs B = A;
                if (wide) {
                    MM_HIP(mm::launch_wide((int)k, wcols(e, (int)k), e->na, red, B, e->s_comm,
                                           wvar(e)));
                } else {
                    B.seg = 0;
                    B.th = mm::kBorderRows;
                    MM_HIP(mm::launch_passk((int)k, e->na, red, B, e->s_comm, 0));
                }
            }
        }
        MM_HIP(hipStreamSynchronize(e->s_comp));
        if (e->split) MM_HIP(hipStreamSynchronize(e->s_comm));
    }
    return MM_OK;
}

int mm_pass_plan(mm_engine* e, long long nsteps, int* lens, int cap, int* count) {
    if (!e || nsteps < 0 || cap < 0 || (cap > 0 && !lens) || !count)
        return fail(MM_ERR_INVALID, "mm_pass_plan: bad arguments");
    if (e->passes.empty()) return fail(MM_ERR_STATE, "mm_pass_plan: no flow added (mm_add_flow)");
    int n = 0;
    if (passk_ok(e)) {
        for (long long s = 0, k = 0; s < nsteps; s += k, ++n) {
            k = next_pass_len(e, nsteps - s);
            if (n < cap) lens[n] = (int)k;
        }
    } else {
        for (long long s = 0; s < nsteps; ++s, ++n)
            if (n < cap) lens[n] = 1;
    }
    *count = n;
    return MM_OK;
}

int mm_pass_kernel(mm_engine* e, int k, int* kernel, int* cols_per_lane, long long* strips) {
    if (!e || k < 1 || !kernel || !cols_per_lane || !strips)
        return fail(MM_ERR_INVALID, "mm_pass_kernel: bad arguments");
    if (e->passes.empty()) return fail(MM_ERR_STATE, "mm_pass_kernel: no flow added (mm_add_flow)");
    if (!passk_ok(e)) {  // one mm_pass_kernel launch per pass of the step
        *kernel = 0;
        *cols_per_lane = 1;
        *strips = 0;
    } else if (use_wide(e, k)) {
        *kernel = 3;
        *cols_per_lane = wcols(e, k);
        *strips = nstrips_wide(e, k);
    } else {
        *kernel = 2;
        *cols_per_lane = 2;
        *strips = nstrips_k(e, k);
    }
    return MM_OK;
}

int mm_run(mm_engine* e, long long nsteps, long long reduce_every) {
    MM_TRY(check_run(e, nsteps, reduce_every, "mm_run"));
    if (nsteps == 0) return MM_OK;
    MM_TRY(set_device(e));
    // steps are numbered from the last fill / upload on, so a run split into several
    // calls reduces the same steps as one call
    const long long phase = reduce_every > 0 ? e->steps_done % reduce_every : 0;
    const long long entries =
        reduce_every > 0 ? (phase + nsteps) / reduce_every - phase / reduce_every : 0;
    MM_TRY(reserve_history(e, entries));
    auto finish = [&]() {
        e->steps_done += nsteps;
        e->hist_host += entries;
        return MM_OK;
    };
    // eager launches plan their passes in the graph path's blocks (graph_per ignoring
    // graphs_ok / timing), so a rank whose capture was refused, or that times its
    // kernels, runs the same pass sequence -- the same K-row exchanges -- as the others
    auto eager = [&](bool timed) -> int {
        const long long pp = graph_per(e, nsteps, reduce_every, true);
        long long d = 0;
        if (pp > 0)
            for (; d + pp <= nsteps; d += pp) MM_TRY(enqueue_steps(e, phase + d + 1, pp, reduce_every, timed));
        if (d < nsteps) MM_TRY(enqueue_steps(e, phase + d + 1, nsteps - d, reduce_every, timed));
        return MM_OK;
    };
    if (e->timing) {  // eager launches with an event pair around each step kernel
        MM_TRY(eager(true));
        return finish();
    }
    const long long per = graph_per(e, nsteps, reduce_every);
    if (per == 0) {
        MM_TRY(eager(false));
        return finish();
    }
    hipGraphExec_t g = nullptr;
    int flip = 0;
    if (get_graph(e, per, reduce_every, phase, &g, &flip) != MM_OK) {
        // stream capture refused (e.g. by the RCCL build): run the same steps eagerly and
        // say so in mm_engine_info (graph_state -1, graph_note)
        e->graph_note = g_last_error;
        (void)hipGetLastError();
        e->graphs_ok = false;
        e->graph_state = -1;
        MM_TRY(eager(false));
        return finish();
    }
    e->graph_state = 1;
    long long done = 0;
    for (; done + per <= nsteps; done += per) {
        if (done > 0 && flip) {  // an odd graph replays at the other parity: its own graph
            MM_TRY(get_graph(e, per, reduce_every, phase, &g, &flip));
        }
        MM_HIP(hipGraphLaunch(g, e->s_comp));
        e->graph_launches += 1;
        e->cur ^= flip;
    }
    if (done < nsteps)
        MM_TRY(enqueue_steps(e, phase + done + 1, nsteps - done, reduce_every, false));
    return finish();
}

int mm_synchronize(mm_engine* e) {
    if (!e) return fail(MM_ERR_INVALID, "mm_synchronize: null");
    MM_TRY(set_device(e));
    if (e->sync_spin) {
        // poll the completion signals: the blocking wait returns tens to hundreds of us after
        // the last kernel ends (a sleeping host thread), time the GPU then sits idle in a
        // timed region or before the next launch
        for (hipStream_t s : {e->s_comp, e->s_comm}) {
            hipError_t q;
            while ((q = hipStreamQuery(s)) == hipErrorNotReady) __builtin_ia32_pause();
            if (q != hipSuccess) MM_HIP(q);
        }
    }
    MM_HIP(hipStreamSynchronize(e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    return MM_OK;
}

int mm_sums(mm_engine* e, double* out) {
    if (!e || !out) return fail(MM_ERR_INVALID, "mm_sums: null");
    MM_TRY(set_device(e));
    for (int a = 0; a < e->na; ++a)
        MM_HIP(mm::launch_slab_sum(e->buf[e->cur][a], e->pitch, e->d.W, e->d.h, e->sum_tmp,
                                   e->sum_blocks, e->sum_tmp + e->sum_blocks + a, e->s_comp));
    MM_HIP(hipMemcpyAsync(out, e->sum_tmp + e->sum_blocks, sizeof(double) * e->na,
                          hipMemcpyDeviceToHost, e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    return MM_OK;
}

int mm_sums_history(mm_engine* e, double* out, long long max_entries, long long* n) {
    if (!e || !n || (max_entries > 0 && !out)) return fail(MM_ERR_INVALID, "mm_sums_history: bad arguments");
    MM_TRY(set_device(e));
    unsigned long long cnt = 0;
    MM_HIP(hipStreamSynchronize(e->s_comp));
    MM_HIP(hipMemcpy(&cnt, e->hist_n, sizeof cnt, hipMemcpyDeviceToHost));
    if ((long long)cnt > e->hist_cap)  // reserve_history keeps this from happening
        return fail(MM_ERR_STATE, "mm_sums_history: history overflowed its buffer");
    const long long k = std::min((long long)cnt, max_entries);
    if (k > 0) MM_HIP(hipMemcpy(out, e->hist, sizeof(double) * (size_t)(k * e->na), hipMemcpyDeviceToHost));
    *n = (long long)cnt;
    return MM_OK;
}

int mm_clear_history(mm_engine* e) {
    if (!e) return fail(MM_ERR_INVALID, "mm_clear_history: null");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    MM_HIP(hipMemsetAsync(e->hist_n, 0, sizeof(unsigned long long), e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    e->hist_host = 0;
    return MM_OK;
}

int mm_halo_export_rows(mm_engine* e, int nrows, double* top, double* bottom) {
    if (!e || nrows < 1 || nrows > e->d.h || nrows > mm::kGhost)
        return fail(MM_ERR_INVALID, "mm_halo_export_rows: nrows must be 1..min(h, kGhost)");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    if (top) MM_TRY(copy_rows(e, true, 0, nrows, top));
    if (bottom) MM_TRY(copy_rows(e, true, e->d.h - nrows, nrows, bottom));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    return MM_OK;
}

int mm_halo_import_rows(mm_engine* e, int nrows, const double* top, const double* bottom) {
    if (!e || nrows < 1 || nrows > mm::kGhost)
        return fail(MM_ERR_INVALID, "mm_halo_import_rows: nrows must be 1..kGhost");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    if (top) MM_TRY(copy_rows(e, false, -nrows, nrows, const_cast<double*>(top)));
    if (bottom) MM_TRY(copy_rows(e, false, e->d.h, nrows, const_cast<double*>(bottom)));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    return MM_OK;
}

int mm_halo_export(mm_engine* e, double* top, double* bottom) {
    return mm_halo_export_rows(e, 1, top, bottom);
}

int mm_halo_import(mm_engine* e, const double* top, const double* bottom) {
    return mm_halo_import_rows(e, 1, top, bottom);
}

int mm_debug_read_rows(mm_engine* e, int attr, long long row0, long long nrows, double* host) {
    if (!e || !host || attr < 0 || attr >= e->na || nrows < 0 || row0 < -mm::kGhost ||
        row0 + nrows > e->d.h + mm::kGhost)
        return fail(MM_ERR_INVALID, "mm_debug_read_rows: rows outside the slab + ghost rows");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    MM_HIP(hipMemcpy2DAsync(host, sizeof(double) * e->d.W, e->buf[e->cur][attr] + row0 * e->pitch,
                            sizeof(double) * e->pitch, sizeof(double) * e->d.W, nrows,
                            hipMemcpyDeviceToHost, e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    return MM_OK;
}

int mm_debug_fill_padding(mm_engine* e, double value) {
    if (!e) return fail(MM_ERR_INVALID, "mm_debug_fill_padding: null");
    const long long pad = e->pitch - e->d.W;
    if (pad <= 0) return MM_OK;
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comm));
    std::vector<double> src((size_t)(pad * e->rows_alloc), value);
    for (int k = 0; k < 2; ++k)
        for (int a = 0; a < e->na; ++a)
            MM_HIP(hipMemcpy2DAsync(e->buf[k][a] - mm::kGhost * e->pitch + e->d.W,
                                    sizeof(double) * e->pitch, src.data(), sizeof(double) * pad,
                                    sizeof(double) * pad, e->rows_alloc, hipMemcpyHostToDevice,
                                    e->s_comp));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    return MM_OK;
}

int mm_set_timing(mm_engine* e, int on) {
    if (!e) return fail(MM_ERR_INVALID, "mm_set_timing: null");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    e->timing = on != 0;
    e->ev_used = 0;
    e->ev_bytes.clear();
    e->timed_launches = 0;
    e->timed_ms = 0.0;
    e->timed_bytes = 0.0;
    return MM_OK;
}

int mm_timing(mm_engine* e, long long* n, double* total_ms, double* bytes_per_launch) {
    if (!e) return fail(MM_ERR_INVALID, "mm_timing: null");
    MM_TRY(set_device(e));
    MM_HIP(hipStreamSynchronize(e->s_comp));
    for (size_t i = 0; i + 1 < e->ev_used; i += 2) {
        float ms = 0.f;
        MM_HIP(hipEventElapsedTime(&ms, e->ev_pool[i], e->ev_pool[i + 1]));
        e->timed_ms += ms;
        e->timed_launches += 1;
        e->timed_bytes += e->ev_bytes[i / 2];
    }
    e->ev_used = 0;
    e->ev_bytes.clear();
    if (n) *n = e->timed_launches;
    if (total_ms) *total_ms = e->timed_ms;
    // algorithmic bytes of a timed launch: each cell of its rows read once and written
    // once per attribute (16 B), whether the launch advances one step or K
    if (bytes_per_launch)
        *bytes_per_launch = e->timed_launches ? e->timed_bytes / (double)e->timed_launches : 0.0;
    return MM_OK;
}

}  // extern "C"
