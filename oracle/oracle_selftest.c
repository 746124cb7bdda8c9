/*
 * oracle_selftest.c -- TEST INFRASTRUCTURE ONLY: the CPU restatement under AddressSanitizer
 * and UndefinedBehaviorSanitizer (the reference itself has stack
 * overflows and uninitialised reads; the checker must have none).
 *
 *   make -C oracle asan   -> oracle/_build/oracle_selftest_asan, run by tests/test_oracle.py
 *
 * Exercises every function of mm_oracle.h on small and degenerate grids (1x1, 1xW, Hx1,
 * 2x2, ragged) and checks the invariants that need no reference: the slab decomposition
 * reproduces the whole-grid step bit for bit, the step conserves the total, the general
 * step with out = r*v is the step to a few ulp, the flow program conserves its attributes' total.
 * Exit status 0 = all checks passed and no sanitizer report.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mm_oracle.h"

static int failures = 0;

#define CHECK(cond, ...)                      \
    do {                                      \
        if (!(cond)) {                        \
            fprintf(stderr, "FAIL: " __VA_ARGS__); \
            fprintf(stderr, "\n");            \
            ++failures;                       \
        }                                     \
    } while (0)

static void grid_case(long long H, long long W) {
    const size_t n = (size_t)(H * W);
    double* v = malloc(n * sizeof *v);
    double* a = malloc(n * sizeof *a);
    double* b = malloc(n * sizeof *b);
    double* outf = malloc(n * sizeof *outf);
    or_fill_random(H, W, 0, H, 0x4D50494DULL, v);
    or_field_step(H, W, v, a, 0.3);
    /* conservation */
    const double s0 = or_sum(v, n), s1 = or_sum(a, n);
    CHECK(fabs(s1 - s0) <= 1e-12 * s0, "conservation %lldx%lld", H, W);
    /* general step with out = r*v for every cell that has neighbours: the step's value up
     * to rounding (the step factors r/8 out of the neighbours' sum) */
    for (long long x = 0; x < H; ++x)
        for (long long y = 0; y < W; ++y)
            outf[x * W + y] = or_neighbor_count(H, W, x, y) > 0 ? 0.3 * v[x * W + y] : 0.0;
    or_field_step_general(H, W, v, outf, b);
    for (size_t i = 0; i < n; ++i)
        CHECK(fabs(a[i] - b[i]) <= 1e-14 * fabs(b[i]), "general %lldx%lld at %zu", H, W, i);
    /* slab decomposition: every G, ghost rows from the neighbours */
    for (int G = 1; G <= 4 && G <= H; ++G) {
        for (int g = 0; g < G; ++g) {
            long long x0, h;
            or_partition_rows(H, G, g, &x0, &h);
            double* vg = calloc((size_t)((h + 2) * W), sizeof *vg);
            double* o = malloc((size_t)(h * W) * sizeof *o);
            for (long long r = -1; r <= h; ++r) {
                const long long gx = x0 + r;
                if (gx >= 0 && gx < H) memcpy(vg + (r + 1) * W, v + gx * W, (size_t)W * sizeof *v);
            }
            or_field_step_slab(H, W, x0, h, vg, o, 0.3);
            for (long long i = 0; i < h * W; ++i)
                CHECK(o[i] == a[x0 * W + i], "slab %lldx%lld G=%d g=%d", H, W, G, g);
            free(vg);
            free(o);
        }
    }
    /* the dependency-cone rows (or_field_rows) after 3 steps: every row range */
    {
        double* c = malloc(n * sizeof *c);
        double* d = malloc(n * sizeof *d);
        memcpy(c, v, n * sizeof *v);
        for (int st = 0; st < 3; ++st) {
            or_field_step(H, W, c, d, 0.3);
            memcpy(c, d, n * sizeof *c);
        }
        for (long long lo = 0; lo < H; ++lo)
            for (long long hi = lo + 1; hi <= H; hi += 2) {
                CHECK(or_field_rows(H, W, lo, hi, 3, 0.3, 0x4D50494DULL, d) == 0, "rows alloc");
                for (long long i = 0; i < (hi - lo) * W; ++i)
                    CHECK(d[i] == c[lo * W + i], "rows %lldx%lld [%lld,%lld)", H, W, lo, hi);
            }
        free(c);
        free(d);
    }
    /* the reference's single-source application on every cell of small grids */
    if (H * W <= 64) {
        for (long long x = 0; x < H; ++x)
            for (long long y = 0; y < W; ++y) {
                for (size_t i = 0; i < n; ++i) b[i] = 1.0;
                or_point_apply(H, W, b, x, y, 2.2, 0.1);
                const double t = or_sum(b, n);
                CHECK(fabs(t - (double)n) <= 1e-12 * (double)n, "point %lld,%lld", x, y);
            }
    }
    /* flow program: 3 attributes, transfers (one to the sink) and diffusions */
    double* f[3];
    for (int k = 0; k < 3; ++k) {
        f[k] = malloc(n * sizeof *f[k]);
        or_fill_random(H, W, 0, H, 0x4D50494DULL + (unsigned)k, f[k]);
    }
    const or_flow flows[] = {{2, 0, 1, 0.05}, {1, 0, 0, 0.1}, {2, 2, 1, 0.2}, {1, 1, 1, 0.3}, {1, 2, 2, 0.05}};
    double t0 = 0.0, t1 = 0.0;
    for (int k = 0; k < 3; ++k) t0 += or_sum(f[k], n);
    or_program_step(H, W, 3, f, flows, 5, b);
    for (int k = 0; k < 3; ++k) t1 += or_sum(f[k], n);
    CHECK(fabs(t1 - t0) <= 1e-12 * t0, "program conservation %lldx%lld", H, W);
    for (int k = 0; k < 3; ++k) free(f[k]);
    free(v);
    free(a);
    free(b);
    free(outf);
}

int main(void) {
    const long long shapes[][2] = {{1, 1}, {1, 7}, {7, 1}, {2, 2}, {3, 5}, {5, 3}, {8, 8}, {13, 29}, {64, 33}};
    for (size_t i = 0; i < sizeof shapes / sizeof shapes[0]; ++i) grid_case(shapes[i][0], shapes[i][1]);
    CHECK(or_step_count(10.0, 0.2) == 51, "step count 51");
    CHECK(or_step_count(1.0, 0.0) == -1, "step count guard");
    int xi, yi, h, w;
    for (int P = 1; P <= 7; ++P)
        for (int k = 1; k <= P; ++k) {
            or_partition_reference(100, 100, P, k, &xi, &yi, &h, &w);
            CHECK(h == 100 / P && w == 100, "partition P=%d", P);
        }
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("oracle selftest ok\n");
    return 0;
}
