/*
 * mpimodel.h -- C ABI of the MI355X engine for MPI-Model's flow step.
 *
 * This is the drop-in boundary: plain C types, plain pointers and sizes, no
 * torch or HIP types. It is called by
 *   - the C++ API headers (mpi-model_amd/api/Model.hpp & co.), which keep the
 *     reference's Model / CellularSpace / Cell / Attribute / Flow / Exponencial
 *     classes so a Main.cpp-style program builds unchanged, and
 *   - Python through ctypes (mpi-model_amd/mpimodel.py), used by bench.py/tests.
 * Implementation: mpi-model_amd/csrc/ -> libmpimodel_hip.so (gfx950 only).
 *
 * Each entry point names the reference code it replaces (paths relative to the
 * reference repository root). The reference has no C ABI of its own; its
 * boundary is the C++ template API. INTEGRATION.md shows how a
 * reference Model::execute binds to these calls.
 *
 * Errors: every int-returning call returns MM_OK (0) or an MM_ERR_* code and
 * stores a message retrievable with mm_last_error() (thread-local). The C++
 * layer turns non-zero codes into std::runtime_error, as src/MPIImpl.cpp:7-8,13-14
 * does for MPI failures.
 */
#ifndef MPIMODEL_H
#define MPIMODEL_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MM_ABI_VERSION 3

enum mm_status {
    MM_OK = 0,
    MM_ERR_INVALID = 1,     /* bad argument / shape */
    MM_ERR_HIP = 2,         /* HIP runtime failure (no device, launch failure, ...) */
    MM_ERR_RCCL = 3,        /* RCCL failure in the halo exchange */
    MM_ERR_STATE = 4,       /* call not valid in the engine's current state */
    MM_ERR_NOMEM = 5,       /* device allocation failed */
    MM_ERR_UNSUPPORTED = 6
};

/* Flow kinds of the flow program (applied in declared order every step). */
enum mm_flow_kind {
    /* Exponencial from every cell of attribute a to its Moore neighbours:
     * out = rate*v (src/Exponencial.hpp:18-20), share = out/count_neighbors
     * (src/Model.hpp:199), v' = (v - out) + sum of neighbour shares
     * (src/Model.hpp:206-211,234). The generalised whole-grid step. */
    MM_FLOW_DIFFUSE = 1,
    /* Exponencial from attribute a to attribute b of the SAME cell:
     * out = rate*v_a; v_a -= out; v_b += out (b < 0: outflow leaves the system). */
    MM_FLOW_TRANSFER = 2
};

enum mm_fill_mode {
    MM_FILL_UNIFORM = 0,  /* v = value (the reference init is 1.0, src/Model.hpp:155) */
    MM_FILL_RANDOM = 1    /* v = 1 + u(splitmix64(seed ^ (x*W+y))), global index keyed */
};

enum mm_halo_mode {
    MM_HALO_NONE = 0,     /* single slab (nranks == 1) */
    MM_HALO_RCCL = 1,     /* ncclSend/ncclRecv of border rows over xGMI, on a comm stream */
    MM_HALO_HOST = 2      /* caller moves border rows (mm_halo_export / mm_halo_import) */
};

/* Engine description: one engine = one row slab of one grid on one GPU. */
typedef struct mm_desc {
    long long H, W;      /* global grid: DIMX rows x DIMY columns (src/Defines.hpp:5-6) */
    long long x_init;    /* first global row owned by this slab (src/Model.hpp:72) */
    long long h;         /* rows owned (src/Model.hpp:72 height) */
    int n_attr;          /* attributes per cell, 1..4 (SoA fp64 buffers) */
    int device;          /* HIP device ordinal */
    int rank, nranks;    /* position in the 1-D chain of slabs (rank r-1 owns the rows above) */
    int halo_mode;       /* enum mm_halo_mode */
    const void* comm_id; /* MM_HALO_RCCL: mm_comm_id_size() bytes from mm_comm_id_create() on rank 0 */
} mm_desc;

typedef struct mm_engine mm_engine;

/* Engine facts for measurement / debugging. */
typedef struct mm_info {
    long long pitch;           /* row pitch in doubles (>= W, multiple of 128) */
    long long bytes_device;    /* device bytes held by the engine */
    int n_passes;              /* kernel passes per step of the current flow program */
    int rows_per_wave;         /* row block height of the step kernel */
    long long waves_per_pass;  /* waves launched per pass */
    long long steps_done;      /* steps run since the last fill/upload */
    int fused_attrs;           /* attributes carried per fused pass */
    int steps_per_launch;      /* steps fused per kernel pass (temporal blocking): 1..10
                                  (mm_passk_kernel), 4/8/12/16/20 (mm_wide_kernel, 4/8 for
                                  four-attribute programs); mixed plans: mm_pass_plan */
    int kernel;                /* step kernel: 0 mm_pass_kernel (one step per pass),
                                  2 mm_passk_kernel (steps_per_launch steps per pass, all
                                  levels in one wave), 3 mm_wide_kernel (steps_per_launch
                                  steps per pass, the levels split over 4 waves) */
    int halo_depth;            /* ghost rows one border exchange fills (= steps per pass) */
    int graph_state;           /* 0 no graph used yet, 1 steps replayed as hipGraphs,
                                  -1 stream capture refused: steps run eagerly (graph_note) */
    int graph_count;           /* hipGraphs instantiated so far */
    long long graph_launches;  /* hipGraphLaunch calls so far */
    long long hist_entries;    /* step-sum history entries enqueued (MPI_Report) */
    char graph_note[160];      /* why capture was refused ("" otherwise) */
    int seg_waves_per_cu;      /* resident waves per CU the K-step segment plan assumes */
    int chain_kernel;          /* transfer chains of a four-attribute mm_wide_kernel pass
                                  (MM_CHAIN_*): MM_CHAIN_NONE not that kernel,
                                  MM_CHAIN_RING the ring t -> t+1 mod 4 with compile-time
                                  operands, MM_CHAIN_RUNTIME any chain, its operands
                                  indexed at run time in the register file (chain_asm);
                                  the value 1 is not used */
} mm_info;

/* mm_info.chain_kernel */
#define MM_CHAIN_NONE 0
#define MM_CHAIN_RING 2
#define MM_CHAIN_RUNTIME 3

/* ---- host-only helpers (no GPU needed) ---------------------------------- */
int mm_abi_version(void);
const char* mm_last_error(void);

/* src/Model.hpp:47-51 -- number of iterations of for(t=0; t<time; t+=time_step). */
long long mm_step_count(double time, double time_step);

/* src/Model.hpp:60-76 -- reference partition of worker k (1..P) of P = comm_size-1,
 * int arithmetic exactly as the reference (remainder rows are dropped). */
int mm_partition_reference(int H, int W, int P, int k,
                           int* x_init, int* y_init, int* height, int* width);
/* src/Model.hpp:80 -- rank owning global row x under the reference partition. */
int mm_owner_reference(int H, int P, int x);
/* Engine partition: slab g of G owns rows [floor(g*H/G), floor((g+1)*H/G)).
 * Identical to mm_partition_reference(k = g+1) whenever G divides H. */
int mm_partition_rows(long long H, int G, int g, long long* x_init, long long* h);
/* src/Cell.hpp:71-157 -- Moore neighbour count of (x,y): 3 corner, 5 edge, 8 inside. */
int mm_neighbor_count(long long H, long long W, long long x, long long y);

/* src/ModelRectangular.hpp:69-80 -- 2-D block descriptor of worker k (1-based) of the
 * block model: blocks of (H/lines) x (W/columns) cells dealt row-major; the column
 * offset wraps to the next band of rows only when it lands exactly on W (int
 * arithmetic as the reference, which never wraps when columns does not divide W). */
int mm_partition_rect_reference(int H, int W, int lines, int columns, int k,
                                int* x_init, int* y_init, int* height, int* width);
/* src/ModelRectangular.hpp:85 -- owner rank of the source (x,y): (x+y)/space_height + 1
 * (the reference's formula, bug included). */
int mm_owner_rect_reference(int space_height, int x, int y);

/* src/Model.hpp:176-235 -- does the reference's single-source flow change any cell when
 * run by P workers? 1 only for a source with 8 neighbours on the last row of its owner's
 * slab (src/Model.hpp:189-216) whose owner has a successor (the share of the row below
 * goes to owner+1, :202-204); 0 otherwise (the reference does nothing there -- and its
 * owner+1 then waits forever, or it aborts); -1 for bad arguments. */
int mm_point_strict_applies(int H, int W, int P, int x, int y);

/* Control-message wire format (src/Model.hpp:70-86,138-167,
 * src/ModelRectangular.hpp:69-92): the master sends every worker a MM_WIRE_LEN-char
 * partition descriptor "%d|%d:%d|%d" = x_init|y_init:height|width (tag 0, FROM_MASTER)
 * and a flow descriptor "%d|%d:%d|%lf" = owner|x:y|rate (tag 999). Formatting writes
 * the text, NUL-padded to len (MM_ERR_INVALID if it does not fit; the reference's
 * sprintf would overflow its buffer). Parsing follows the reference's strtok/atoi
 * sequence; for the flow it also returns the rate as the reference reads it (atoi, an
 * int) and losslessly (strtod). */
#define MM_WIRE_LEN 23
#define MM_TAG_PARTITION 0
#define MM_TAG_FLOW 999
int mm_wire_format_partition(char* out, int len, int x_init, int y_init, int height, int width);
int mm_wire_format_flow(char* out, int len, int owner, int x, int y, double rate);
int mm_wire_parse_partition(const char* msg, int len, int* x_init, int* y_init, int* height,
                            int* width);
int mm_wire_parse_flow(const char* msg, int len, int* owner, int* x, int* y, int* rate_atoi,
                       double* rate);

/* RCCL bootstrap: rank 0 creates the id, every rank passes it in mm_desc.comm_id.
 * Replaces the master's partition/flow descriptor messages (src/Model.hpp:70-86). */
int mm_comm_id_size(void);
int mm_comm_id_create(void* out, int len);

int mm_device_count(int* n);
/* hipDeviceSynchronize on one device: every stream of every engine on it. */
int mm_device_synchronize(int device);

/* ---- engine ------------------------------------------------------------- */
/* Replaces the per-worker CellularSpace construction (src/Model.hpp:149) and the
 * init loop (src/Model.hpp:154-157): device buffers are (h + 2*kGhost) x pitch fp64 per
 * attribute (kGhost = 20 ghost rows above and below, the deepest K-step pass), two of
 * them (Jacobi ping-pong).
 * With nranks > 1 the steps per kernel pass (and so the halo depth) are capped by the
 * thinnest slab of the chain: RCCL engines all-reduce it at creation; host-transport
 * engines accept mm_partition_rows slabs only (floor(H/nranks) rows at least) and
 * return MM_ERR_INVALID otherwise.
 * Environment: MM_PASSK=0 (or MM_FUSE=0) runs one step per kernel pass, MM_GRAPH=0
 * disables the hipGraph replay (a graph holds MM_GRAPH_MIN_STEPS steps at least and, when
 * that divides the run, the longest run-dividing block of up to MM_GRAPH_MAX_LAUNCHES step
 * kernels, default 128), MM_WIDE=0/1 selects the level-split K-step kernel for
 * one-diffusion programs, MM_STEPS_PER_PASS (1..10, or 4/8/12/16/20 with the wide
 * kernel; fixes K), MM_PASS_PLAN=0
 * (balanced passes of K, no planner), MM_ROWS_PER_WAVE (8/16/32),
 * MM_SEG_WAVES, MM_SEG_EDGE, MM_XCD_REMAP (mm_passk_kernel's block order only; the
 * level-split kernel keeps the hardware order), MM_BORDER_SEGMENTS=0 (the level-split
 * kernel's split passes with K-row border segments instead of full-length top / bottom
 * segments) and MM_KERNEL_VARIANT (non-temporal stores;
 * the four-attribute K = 8 instances always store non-temporal) override tuning;
 * MM_SELF_HALO=1 with MM_HALO_RCCL and nranks == 1 makes the rank
 * exchange border rows with itself (ghost rows outside the grid: exercises the RCCL
 * path, result unchanged).
 * An RCCL chain runs in lockstep: every rank must call mm_prepare / mm_run with the same
 * step counts and reduce_every, with the same MM_GRAPH* settings and the same timing mode
 * (mm_set_timing), so that all ranks run the same K-row exchanges and capture the same
 * graphs at the same call (the first capture of each graph agrees on success with one
 * all-reduce, after draining this engine's streams). */
int mm_engine_create(const mm_desc* desc, mm_engine** out);
int mm_engine_destroy(mm_engine* eng);
int mm_engine_info(mm_engine* eng, mm_info* info);

/* src/Model.hpp:154-157 -- initialise one attribute on the device (owned and ghost rows). */
int mm_fill(mm_engine* eng, int attr, int mode, double value, unsigned long long seed);
/* Host <-> device copies of the OWNED rows (h x W, row-major, contiguous). */
int mm_upload(mm_engine* eng, int attr, const double* host);
int mm_download(mm_engine* eng, int attr, double* host);

/* Flow program. src/Model.hpp:23-27 stores one Flow; the engine keeps an ordered list.
 * One step applies the flows in order; the engine groups them into kernel passes (a
 * diffusion per attribute with up to 4 same-cell transfers before and after it; longer
 * chains start a new pass), which changes no result. */
int mm_clear_flows(mm_engine* eng);
int mm_add_flow(mm_engine* eng, int kind, int a, int b, double rate);

/* src/Model.hpp:176-235 -- the reference's single-source Exponencial application:
 * out = rate*captured (src/Exponencial.hpp:14-16, the Flow's own copy of the
 * source value), share = out/count_neighbors to every in-grid Moore neighbour,
 * source -= out. Applied in place to the cells this slab owns; no message needed
 * (every slab computes the share from the same flow description). */
int mm_point_apply(mm_engine* eng, int attr, long long sx, long long sy,
                   double captured, double rate);
/* Strict-reference point mode (opt-in): the same update, applied only where the
 * reference's P-worker run applies it (mm_point_strict_applies); elsewhere the grid is
 * left unchanged, as the reference leaves it. *applied (may be NULL) reports which. */
int mm_point_apply_strict(mm_engine* eng, int attr, long long sx, long long sy,
                          double captured, double rate, int P, int* applied);

/* Run nsteps steps of the flow program (the commented-out time loop,
 * src/Model.hpp:180-183, made real). Every reduce_every-th step (0 = never; steps
 * counted from the last mm_fill / mm_upload, across mm_run calls) the per-attribute
 * sums of the owned cells are reduced on the device and appended to the engine's
 * history (src/Model.hpp:237-243 per-rank sum; MPI_Report); the history grows as
 * needed. Asynchronous: returns once the work is enqueued. MM_HALO_HOST engines with
 * nranks > 1 run exactly one kernel pass per call: nsteps must be the next length
 * mm_pass_plan returns (at most kGhost = 20); the caller exchanges that many rows
 * (mm_halo_export_rows / mm_halo_import_rows) between calls, and the engine runs the
 * same interior / border split as with RCCL. */
int mm_run(mm_engine* eng, long long nsteps, long long reduce_every);
/* Do the one-time work of a following mm_run(eng, nsteps, reduce_every) now -- capture and
 * instantiate its hipGraph, plan its eager tail passes and dispatch each of their kernels
 * once with no work on every stream the run uses (which loads the kernel and sizes that
 * queue's scratch) -- without running any step: no buffer is read or written. Optional:
 * mm_run does the same work on first use, except the empty dispatches. */
int mm_prepare(mm_engine* eng, long long nsteps, long long reduce_every);
/* The kernel passes mm_run(eng, nsteps, .) launches: *count passes, the steps of the first
 * min(*count, cap) in lens[] (K-step passes; 1 per step for the one-step kernel). Host-only
 * planning, no device work. Replaces nothing in the reference: its time loop
 * (src/Model.hpp:180-183) is commented out. */
int mm_pass_plan(mm_engine* eng, long long nsteps, int* lens, int cap, int* count);
/* The kernel a pass of k steps launches (for rooflines): *kernel 0 = one-step
 * mm_pass_kernel, 2 = mm_passk_kernel, 3 = mm_wide_kernel; *cols_per_lane = columns one
 * lane computes (2 for mm_passk_kernel; 4, or 2 for four-attribute programs, for mm_wide_kernel); *strips = column
 * strips of the slab, counted in 64-lane wave columns (a mm_wide_kernel strip of several
 * column waves counts each; 0 for the one-step kernel). */
int mm_pass_kernel(mm_engine* eng, int k, int* kernel, int* cols_per_lane, long long* strips);
int mm_synchronize(mm_engine* eng);

/* Sums of the owned cells. mm_sums reduces the CURRENT state now (synchronous).
 * mm_sums_history copies up to max_entries recorded reductions (n_attr doubles
 * each, oldest first) and returns the count in *n. */
int mm_sums(mm_engine* eng, double* out_per_attr);
int mm_sums_history(mm_engine* eng, double* out, long long max_entries, long long* n);
int mm_clear_history(mm_engine* eng);

/* MM_HALO_HOST transport: copy this slab's first/last nrows owned rows of every
 * attribute out (top/bottom: n_attr*nrows*W doubles each, [attr][row][col]), and the
 * neighbours' rows into the nrows ghost rows above / below (NULL = no neighbour on
 * that side). nrows is info.halo_depth (1..kGhost = 20). Replaces the scalar halo messages
 * src/Model.hpp:202-204 <-> :228-230 with whole rows. mm_halo_export/import move one
 * row (nrows = 1). */
int mm_halo_export_rows(mm_engine* eng, int nrows, double* top, double* bottom);
int mm_halo_import_rows(mm_engine* eng, int nrows, const double* top, const double* bottom);
int mm_halo_export(mm_engine* eng, double* top, double* bottom);
int mm_halo_import(mm_engine* eng, const double* top, const double* bottom);

/* Test/debug: copy nrows rows starting at local row row0 (owned rows are 0..h-1, ghost
 * rows -kGhost..-1 and h..h+kGhost-1, kGhost = 20) of the current buffer of one attribute to host (W each). */
int mm_debug_read_rows(mm_engine* eng, int attr, long long row0, long long nrows, double* host);
/* Test/debug: write `value` into the pitch padding (columns W..pitch-1 of every row, ghost
 * rows included) of both buffers of every attribute. No result depends on the padding: the
 * tests poison it with NaN and compare cells and step sums bit for bit. */
int mm_debug_fill_padding(mm_engine* eng, double value);

/* Measurement: with timing on, mm_run records a HIP event pair around every
 * step-kernel launch on the stream it is launched on; mm_timing returns the
 * number of timed launches, their summed duration (ms) and the average algorithmic
 * bytes one launch moves: 16 B per cell of its rows per attribute (read once, written
 * once), whether the launch advances one step or K. */
int mm_set_timing(mm_engine* eng, int on);
int mm_timing(mm_engine* eng, long long* n_launches, double* total_ms, double* bytes_per_launch);

#ifdef __cplusplus
}
#endif
#endif
