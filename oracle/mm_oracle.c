/*
 * mm_oracle.c -- CPU restatement of the reference flow step (TEST INFRASTRUCTURE).
 * Contract and citations: mm_oracle.h. Build: make -C oracle oracle
 * (-ffp-contract=off, no fast-math: every operation is one IEEE-754 binary64
 * operation in the order written, the same order the HIP kernels use).
 */
#include "mm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

long long or_step_count(double time, double time_step) {
    /* Model.hpp:48. Guard: a non-positive step never terminates in the reference. */
    if (!(time_step > 0.0)) return -1;
    long long n = 0;
    for (double t = 0; t < time; t = t + time_step) ++n;
    return n;
}

void or_partition_reference(int H, int W, int P, int k,
                            int* x_init, int* y_init, int* height, int* width) {
    /* Model.hpp:63-64,70-75: count = (H*W)/P; worker k gets offset (k-1)*count. */
    int count = (H * W) / P;
    int offset = (k - 1) * count;
    *x_init = offset / W;
    *y_init = 0; /* cellular_space.y_init of the caller's space, 0 in Main.cpp:25 */
    *height = H / P;
    *width = W;
}

int or_owner_reference(int H, int P, int x) {
    return (x / (H / P)) + 1; /* Model.hpp:80 */
}

void or_partition_rows(long long H, int G, int g, long long* x_init, long long* h) {
    long long a = (g * H) / G;
    long long b = ((g + 1) * H) / G;
    *x_init = a;
    *h = b - a;
}

static inline long long span3(long long n, long long i) {
    long long c = 1;
    if (i > 0) ++c;
    if (i < n - 1) ++c;
    return c;
}

int or_neighbor_count(long long H, long long W, long long x, long long y) {
    if (x < 0 || y < 0 || x >= H || y >= W) return 0;
    return (int)(span3(H, x) * span3(W, y) - 1);
}

static inline uint64_t splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void or_fill_random(long long H, long long W, long long x_init, long long h,
                    uint64_t seed, double* out) {
    (void)H;
    for (long long i = 0; i < h; ++i)
        for (long long y = 0; y < W; ++y) {
            uint64_t gidx = (uint64_t)((x_init + i) * W + y);
            uint64_t z = splitmix64(seed ^ gidx);
            double u = (double)(z >> 11) * 0x1.0p-53;
            out[i * W + y] = 1.0 + u;
        }
}

/* share of one emitter: s = out / cnt, cnt == 8 as the exact *0.125 */
static inline double share_of(double out, int cnt) {
    if (cnt == 8) return out * 0.125;
    if (cnt <= 0) return 0.0;
    return out / (double)cnt;
}

void or_point_apply(long long H, long long W, double* v, long long sx, long long sy,
                    double captured, double rate) {
    int cnt = or_neighbor_count(H, W, sx, sy);
    if (cnt <= 0) return;
    double out = rate * captured;          /* Exponencial.hpp:15 */
    double share = share_of(out, cnt);     /* Model.hpp:199 */
    for (long long dx = -1; dx <= 1; ++dx)
        for (long long dy = -1; dy <= 1; ++dy) {
            long long x = sx + dx, y = sy + dy;
            if ((dx == 0 && dy == 0) || x < 0 || y < 0 || x >= H || y >= W) continue;
            v[x * W + y] = v[x * W + y] + share;    /* Model.hpp:206-209,234 */
        }
    v[sx * W + sy] = v[sx * W + sy] - out;          /* Model.hpp:211 */
}

/* The whole-grid step (mm_oracle.h): every emitter's outflow is out = r*v and each of
 * its cnt neighbours receives out/cnt. Written per receiving cell c with the cells'
 * weights w = v * 8/cnt (w = v for cnt == 8, 0 outside the grid) and the 3 x 3 box sum S of
 * the weights (the cell's own weight included):
 *   v'(c) = v - r*v + sum_nbr r*v_nbr/cnt_nbr = v + (r/8) * (S - (8 + c8) v)
 * computed as fma(fma(v, -(8 + c8), S), r/8, v) -- the multiply by r/8 factored out of the
 * sum, so an interior cell's neighbours cost no multiply. The box sum adds the column
 * triples cw of three columns, each triple and the three columns paired from an even
 * global index: cw(x,y) = w(x-1,y) + (w(x,y) + w(x+1,y)) for even x, (w(x-1,y) + w(x,y)) +
 * w(x+1,y) for odd x, S likewise over cw(x,y-1..y+1) by the parity of y -- so two
 * consecutive rows (columns) share the sum of their pair: the kernels add 5 fp64
 * operations per cell where the pairwise-symmetric form took 6. */
static inline double c8_of(int cnt) { return cnt == 8 ? 1.0 : (cnt > 0 ? 8.0 / (double)cnt : 0.0); }

/* the own-weight coefficient -(8 + c8): -9 for an interior cell */
static inline double m_of(int cnt) { return cnt > 0 ? -(8.0 + c8_of(cnt)) : 0.0; }

static inline double update_of(double v, double s9, int cnt, double r8) {
    return cnt > 0 ? fma(fma(v, m_of(cnt), s9), r8, v) : v;
}

/* the box sum of column y from the padded column triples cw[y .. y+2] (columns y-1 .. y+1),
 * paired from an even column */

static inline double box_of(long long y, const double* cw) {
    return (y & 1) == 0 ? cw[y] + (cw[y + 1] + cw[y + 2]) : (cw[y] + cw[y + 1]) + cw[y + 2];
}

/* w row of global row gx (NULL vrow or outside grid -> +0.0) */
static void w_row(long long H, long long W, long long gx, const double* vrow, double* w) {
    if (vrow == NULL || gx < 0 || gx >= H) {
        for (long long y = 0; y < W; ++y) w[y] = 0.0;
        return;
    }
    for (long long y = 0; y < W; ++y) w[y] = vrow[y] * c8_of(or_neighbor_count(H, W, gx, y));
}

/* rows(gx) gives the v row for any global gx in [x_lo-1, x_hi]. */
typedef const double* (*row_fn)(const void* ctx, long long gx);

/* returns 0, or -1 when its row buffers cannot be allocated (nothing written) */
static int step_rows(long long H, long long W, long long x_lo, long long x_hi,
                     row_fn rows, const void* ctx, double* vout, double rate) {
    double* buf = (double*)malloc(sizeof(double) * (size_t)(4 * W + 2));
    if (!buf) return -1;
    double* w_prev = buf;
    double* w_cur = buf + W;
    double* w_next = buf + 2 * W;
    double* cw = buf + 3 * W; /* W+2 entries, cw[y+1] for column y */
    const double r8 = rate * 0.125;
    cw[0] = 0.0;
    cw[W + 1] = 0.0;
    w_row(H, W, x_lo - 1, rows(ctx, x_lo - 1), w_prev);
    w_row(H, W, x_lo, rows(ctx, x_lo), w_cur);
    for (long long x = x_lo; x < x_hi; ++x) {
        w_row(H, W, x + 1, rows(ctx, x + 1), w_next);
        if ((x & 1) == 0) {  /* the column triples, rows paired from an even row */
            for (long long y = 0; y < W; ++y) cw[y + 1] = w_prev[y] + (w_cur[y] + w_next[y]);
        } else {
            for (long long y = 0; y < W; ++y) cw[y + 1] = (w_prev[y] + w_cur[y]) + w_next[y];
        }
        const double* v = rows(ctx, x);
        double* o = vout + (x - x_lo) * W;
        if (v == NULL) {  /* output row outside the grid (or the slab): no cells, zeros */
            for (long long y = 0; y < W; ++y) o[y] = 0.0;
        } else {
            long long y = 0;
            for (; y + 1 < W; y += 2) {  /* box_of of an even column and the odd one after it */
                const double p = cw[y + 1] + cw[y + 2];
                o[y] = update_of(v[y], cw[y] + p, or_neighbor_count(H, W, x, y), r8);
                o[y + 1] = update_of(v[y + 1], p + cw[y + 3], or_neighbor_count(H, W, x, y + 1), r8);
            }
            if (y < W) o[y] = update_of(v[y], box_of(y, cw), or_neighbor_count(H, W, x, y), r8);
        }
        double* t = w_prev;
        w_prev = w_cur;
        w_cur = w_next;
        w_next = t;
    }
    free(buf);
    return 0;
}

typedef struct {
    const double* v;
    long long H, W, base; /* v row 0 is global row `base` */
    long long lo, hi;     /* valid global rows [lo, hi) */
} grid_ctx;

static const double* grid_row(const void* ctx_, long long gx) {
    const grid_ctx* c = (const grid_ctx*)ctx_;
    if (gx < c->lo || gx >= c->hi || gx < 0 || gx >= c->H) return NULL;
    return c->v + (gx - c->base) * c->W;
}

int or_field_step(long long H, long long W, const double* v, double* vout, double rate) {
    grid_ctx c = {v, H, W, 0, 0, H};
    return step_rows(H, W, 0, H, grid_row, &c, vout, rate);
}

int or_field_step_slab(long long H, long long W, long long x_init, long long h,
                       const double* vg, double* vout, double rate) {
    grid_ctx c = {vg, H, W, x_init - 1, x_init - 1, x_init + h + 1};
    return step_rows(H, W, x_init, x_init + h, grid_row, &c, vout, rate);
}

/* step_rows with the counts hoisted: rows strictly inside the grid have cnt == 8 except in
 * their first and last column. Same operations, same order, same results. */
#if defined(__x86_64__)
#define OR_FAST_TARGET __attribute__((target("avx2,fma")))
#else
#define OR_FAST_TARGET
#endif
static OR_FAST_TARGET void w_row_fast(long long H, long long W, long long gx,
                                      const double* vrow, double* w) {
    if (vrow == NULL || gx <= 0 || gx >= H - 1 || W < 3) {
        w_row(H, W, gx, vrow, w);
        return;
    }
    w[0] = vrow[0] * c8_of(or_neighbor_count(H, W, gx, 0));
    for (long long y = 1; y < W - 1; ++y) w[y] = vrow[y];  /* cnt 8: w = v * 1.0 = v */
    w[W - 1] = vrow[W - 1] * c8_of(or_neighbor_count(H, W, gx, W - 1));
}

static OR_FAST_TARGET int step_rows_fast(long long H, long long W, long long x_lo,
                                         long long x_hi, row_fn rows, const void* ctx,
                                         double* vout, double rate) {
    double* buf = (double*)malloc(sizeof(double) * (size_t)(4 * W + 2));
    if (!buf) return -1;
    double* w_prev = buf;
    double* w_cur = buf + W;
    double* w_next = buf + 2 * W;
    double* cw = buf + 3 * W;
    const double r8 = rate * 0.125;
    cw[0] = 0.0;
    cw[W + 1] = 0.0;
    w_row_fast(H, W, x_lo - 1, rows(ctx, x_lo - 1), w_prev);
    w_row_fast(H, W, x_lo, rows(ctx, x_lo), w_cur);
    for (long long x = x_lo; x < x_hi; ++x) {
        w_row_fast(H, W, x + 1, rows(ctx, x + 1), w_next);
        if ((x & 1) == 0) {
            for (long long y = 0; y < W; ++y) cw[y + 1] = w_prev[y] + (w_cur[y] + w_next[y]);
        } else {
            for (long long y = 0; y < W; ++y) cw[y + 1] = (w_prev[y] + w_cur[y]) + w_next[y];
        }
        const double* v = rows(ctx, x);
        double* o = vout + (x - x_lo) * W;
        if (v == NULL) {
            for (long long y = 0; y < W; ++y) o[y] = 0.0;
        } else if (x > 0 && x < H - 1 && W >= 3) {
            for (long long y = 0; y < W; y += W - 1)  /* first and last column */
                o[y] = update_of(v[y], box_of(y, cw), or_neighbor_count(H, W, x, y), r8);
            for (long long y = 1; y < W - 1; y += 2) {  /* cnt == 8: odd y, then even y + 1 */
                o[y] = fma(fma(v[y], -9.0, (cw[y] + cw[y + 1]) + cw[y + 2]), r8, v[y]);
                if (y + 1 < W - 1)
                    o[y + 1] = fma(fma(v[y + 1], -9.0, cw[y + 1] + (cw[y + 2] + cw[y + 3])), r8, v[y + 1]);
            }
        } else {
            for (long long y = 0; y < W; ++y)
                o[y] = update_of(v[y], box_of(y, cw), or_neighbor_count(H, W, x, y), r8);
        }
        double* t = w_prev;
        w_prev = w_cur;
        w_cur = w_next;
        w_next = t;
    }
    free(buf);
    return 0;
}

static int fast_ok(void) {
#if defined(__x86_64__)
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
#else
    return 1;
#endif
}

int or_field_rows(long long H, long long W, long long lo, long long hi, int steps,
                  double rate, uint64_t seed, double* out) {
    if (lo < 0) lo = 0;
    if (hi > H) hi = H;
    if (hi <= lo || W <= 0) return 0;
    if (steps < 0) steps = 0;
    const long long clo = lo - steps > 0 ? lo - steps : 0;
    const long long chi = hi + steps < H ? hi + steps : H;
    const size_t n = (size_t)((chi - clo) * W);
    double* a = (double*)malloc(sizeof(double) * n);
    double* b = (double*)malloc(sizeof(double) * n);
    if (!a || !b) {
        free(a);
        free(b);
        return -1;
    }
    or_fill_random(H, W, clo, chi - clo, seed, a);
    const int fast = fast_ok();
    long long plo = clo, phi = chi;  /* rows of `a` exact after the previous step */
    for (int st = 1; st <= steps; ++st) {
        const long long elo = lo - steps + st > 0 ? lo - steps + st : 0;
        const long long ehi = hi + steps - st < H ? hi + steps - st : H;
        grid_ctx c = {a, H, W, clo, plo, phi};
        const int rc = fast ? step_rows_fast(H, W, elo, ehi, grid_row, &c, b + (elo - clo) * W, rate)
                            : step_rows(H, W, elo, ehi, grid_row, &c, b + (elo - clo) * W, rate);
        if (rc != 0) {  /* out of memory: the caller raises, never compares garbage */
            free(a);
            free(b);
            return -1;
        }
        double* t = a;
        a = b;
        b = t;
        plo = elo;
        phi = ehi;
    }
    memcpy(out, a + (lo - clo) * W, sizeof(double) * (size_t)((hi - lo) * W));
    free(a);
    free(b);
    return 0;
}

int or_field_step_general(long long H, long long W, const double* v, const double* outf,
                          double* vout) {
    double* s = (double*)malloc(sizeof(double) * (size_t)(H * W > 0 ? H * W : 1));
    if (!s) return -1;
    for (long long x = 0; x < H; ++x)
        for (long long y = 0; y < W; ++y)
            s[x * W + y] = share_of(outf[x * W + y], or_neighbor_count(H, W, x, y));
#define S(x, y) (((x) < 0 || (y) < 0 || (x) >= H || (y) >= W) ? 0.0 : s[(x) * W + (y)])
    for (long long x = 0; x < H; ++x)
        for (long long y = 0; y < W; ++y) {
            double p = S(x - 1, y) + S(x + 1, y);
            double c3l = (S(x - 1, y - 1) + S(x + 1, y - 1)) + S(x, y - 1);
            double c3r = (S(x - 1, y + 1) + S(x + 1, y + 1)) + S(x, y + 1);
            double nb = (c3l + c3r) + p;
            vout[x * W + y] = (v[x * W + y] - outf[x * W + y]) + nb;
        }
#undef S
    free(s);
    return 0;
}

int or_program_step(long long H, long long W, int n_attr, double* const* v,
                    const or_flow* flows, int n_flows, double* scratch) {
    const long long n = H * W;
    for (int f = 0; f < n_flows; ++f) {
        const or_flow* fl = &flows[f];
        if (fl->a < 0 || fl->a >= n_attr) continue;
        if (fl->kind == 1) {
            if (or_field_step(H, W, v[fl->a], scratch, fl->rate) != 0) return -1;
            memcpy(v[fl->a], scratch, sizeof(double) * (size_t)n);
        } else if (fl->kind == 2) {
            double* va = v[fl->a];
            double* vb = (fl->b >= 0 && fl->b < n_attr) ? v[fl->b] : NULL;
            for (long long i = 0; i < n; ++i) {
                double out = fl->rate * va[i];
                va[i] = va[i] - out;
                if (vb) vb[i] = vb[i] + out;
            }
        }
    }
    return 0;
}

double or_sum(const double* v, size_t n) {
    double s = 0.0, c = 0.0;
    for (size_t i = 0; i < n; ++i) {
        double x = v[i];
        double t = s + x;
        if (fabs(s) >= fabs(x))
            c += (s - t) + x;
        else
            c += (x - t) + s;
        s = t;
    }
    return s + c;
}
