/*
 * mm_oracle -- CPU restatement of daviidsilvaa/MPI-Model's flow step.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker the HIP path is compared with;
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it. The product (libmpimodel_hip.so, mpi-model_amd/) never links or calls it.
 *
 * Pinning: the single-source application (or_point_apply) is checked bit-exactly
 * against golden grids produced by the reference itself (tests/golden/, made by
 * tests/golden/make_golden.py from oracle/_ref/). The generalised whole-grid,
 * multi-step step (or_field_step*) has no reference implementation (the
 * reference's time loop is commented out, Model.hpp:180-183). It is pinned to the
 * reference's arithmetic through or_field_step_general, which applies the reference's
 * update (Model.hpp:176-235: out = r*v, share = out/cnt, neighbours += share, source -=
 * out) to an arbitrary outflow field and is bit-for-bit the reference's single-source
 * application when the outflow is zero but at the source; with out = r*v everywhere it
 * equals or_field_step within a few ulp per step, and iterated over the bench runs' 20 and
 * 1000 steps within 3.6e-14 relative on edge-dominated grids (tests/test_oracle.py, bound
 * asserted 1e-12 = north_star's), plus invariants (conservation, flip symmetry, uniform
 * fixed point). See DESIGN.md "Oracle".
 *
 * Arithmetic contract of the whole-grid step (shared with the HIP kernels, compiled
 * -ffp-contract=off, the two fma explicit):
 *   w(c)  = v(c) * c8(c),  c8 = 8/cnt(c) rounded (1 for cnt 8: w = v), 0 outside the grid
 *   cw(c) = w(x-1,y) + (w(x,y) + w(x+1,y))   x even   (the column triple; rows paired
 *         = (w(x-1,y) + w(x,y)) + w(x+1,y)   x odd     from an even global row)
 *   S(c)  = cw(x,y-1) + (cw(x,y) + cw(x,y+1))   y even (the 3 x 3 box sum; columns
 *         = (cw(x,y-1) + cw(x,y)) + cw(x,y+1)   y odd   paired from an even column)
 *   v'(c) = fma(fma(v(c), m(c), S(c)), r/8, v(c)),  m = -(8 + c8) rounded (-9 for cnt 8)
 *                                                     (cnt(c) > 0; else v' = v)
 * i.e. v' = v - r*v + sum_nbr r*v_nbr/cnt_nbr (Exponencial.hpp:18-20: out = r*v;
 * Model.hpp:199: share = out/cnt; Model.hpp:206-211,234: neighbours += share, source
 * -= out) with r/8 factored out of the neighbours' sum: an interior cell's neighbours
 * cost no multiply, and a pair of rows (columns) shares the sum of its two middle
 * weights, so a kernel adds 5 fp64 operations per cell. The step commutes with flipping
 * an axis of even length (pairs map onto pairs). cnt is the number of in-grid Moore
 * neighbours (Cell.hpp:71-157 gives 3/5/8 for grids of at least 2x2).
 */
#ifndef MM_ORACLE_H
#define MM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Model.hpp:47-51: for(double t = 0; t < time; t = t + time_step) -- count only. */
long long or_step_count(double time, double time_step);

/* Model.hpp:60-76: worker k (1-based) of P = comm_size-1 workers. int arithmetic,
 * exactly as the reference (remainder rows silently dropped). */
void or_partition_reference(int H, int W, int P, int k,
                            int* x_init, int* y_init, int* height, int* width);
/* Model.hpp:80: owner rank of row x. */
int or_owner_reference(int H, int P, int x);

/* Balanced row partition used by the engine: part g of G gets rows
 * [floor(g*H/G), floor((g+1)*H/G)). Equal to or_partition_reference when G | H. */
void or_partition_rows(long long H, int G, int g, long long* x_init, long long* h);

/* Cell.hpp:71-157 generalised: number of in-grid Moore neighbours of (x,y). */
int or_neighbor_count(long long H, long long W, long long x, long long y);

/* Deterministic synthetic input keyed by GLOBAL cell index:
 * v = 1 + u, u = (splitmix64(seed ^ (x*W+y)) >> 11) * 2^-53. Rows
 * [x_init, x_init+h) into out[h*W]. */
void or_fill_random(long long H, long long W, long long x_init, long long h,
                    uint64_t seed, double* out);

/* Model.hpp:176-235: the single-source application on a full H x W grid, the
 * source's outflow from the Flow's captured value (Exponencial.hpp:14-16). */
void or_point_apply(long long H, long long W, double* v, long long sx, long long sy,
                    double captured, double rate);

/* One generalised step on the full grid (Jacobi, v -> vout). The step functions return 0,
 * or -1 when a row buffer cannot be allocated (vout then unwritten). */
int or_field_step(long long H, long long W, const double* v, double* vout, double rate);

/* One generalised step on a row slab with ghost rows: vg has (h+2) rows of W,
 * row 0 = global row x_init-1, row h+1 = global row x_init+h (ignored when
 * outside the grid). Writes h rows to vout; rows outside the grid are written as 0. */
int or_field_step_slab(long long H, long long W, long long x_init, long long h,
                       const double* vg, double* vout, double rate);

/* The same step with an arbitrary per-cell outflow field outf (instead of
 * r*v): s = outf/cnt, v' = (v - outf) + nb -- the reference's per-emitter update. With
 * outf = r*v it is or_field_step up to the per-receiver rounding (a few ulp per step);
 * with outf zero except r*captured at the source it is or_point_apply bit-for-bit -- the algebraic link between the generalised
 * step and the reference's single-source update (Model.hpp:176-235). */
int or_field_step_general(long long H, long long W, const double* v, const double* outf,
                          double* vout);

/* Multi-attribute flow program (config C5). Each flow is applied in declared
 * order to the whole grid; a step applies all of them once.
 *   kind 1 = DIFFUSE  : Exponencial of attribute a to its Moore neighbours
 *   kind 2 = TRANSFER : out = r*v_a; v_a -= out; v_b += out (b < 0: sink)  */
typedef struct {
    int kind;
    int a;
    int b;
    double rate;
} or_flow;

int or_program_step(long long H, long long W, int n_attr, double* const* v,
                    const or_flow* flows, int n_flows, double* scratch);

/* Rows [lo, hi) of the seeded random grid (or_fill_random) after `steps` whole-grid steps
 * (or_field_step), computed on those rows' dependency cone only: the fill of rows
 * [lo - steps, hi + steps), then step s on the rows still exact after it,
 * [lo - steps + s, hi + steps - s) (clipped to the grid, whose edges are exact). The same
 * operations as or_field_step in the same order -- bit-identical rows -- with the
 * neighbour counts hoisted out of the interior rows and the explicit fma of the cnt == 8
 * cells on the FMA instruction where the CPU has one. For full-size GPU checks
 * (32768^2 x 20+ steps), run over row chunks in threads. Returns 0, or -1 if out of
 * memory. */
int or_field_rows(long long H, long long W, long long lo, long long hi, int steps,
                  double rate, uint64_t seed, double* out);

/* Neumaier-compensated sum (used for quick checks; tests use math.fsum). */
double or_sum(const double* v, size_t n);

#ifdef __cplusplus
}
#endif
#endif
