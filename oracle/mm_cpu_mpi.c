/*
 * mm_cpu_mpi.c -- CPU baseline of the flow step with the reference's decomposition
 * (TEST INFRASTRUCTURE: bench.py's cpu_baseline leg and tests/ only; never the product).
 *
 * The reference runs one MPI rank per core (worker) on a row block of the grid and moves
 * data between ranks with blocking point-to-point MPI_Send/MPI_Recv: the partition and
 * flow descriptors (src/Model.hpp:70-86,138-167), the halo (src/Model.hpp:202-204 <->
 * :228-230) and the per-rank sums (src/Model.hpp:88-92,243). This program keeps that
 * structure -- 1-D row slabs (or_partition_rows), one ghost row above and below, a
 * blocking MPI_Sendrecv of the border rows before every neighbour-reading flow, sums
 * combined in rank order -- and computes each slab with the oracle's restated step
 * (or_field_step_slab, mm_oracle.c), so its grid is the oracle's grid bit for bit.
 *
 *   mpirun -np P mm_cpu_mpi H W RATE SECONDS [MAXSTEPS] [DUMP]
 *
 * MM_PROGRAM="kind:a:b:rate,..." (environment) runs a multi-attribute flow program
 * instead of the single Exponencial diffusion (config C5, or_program_step's semantics:
 * kind 1 = DIFFUSE a, kind 2 = TRANSFER a -> b, in declared order), with the per-step
 * per-attribute sums gathered to rank 0 and added in rank order every step (MPI_Report).
 *
 * Input v0 = 1 + U[0,1) (or_fill_random, seed 0x4D50494D). Runs untimed steps for a tenth of
 * SECONDS (at least 2), sizes the timed run to about SECONDS from them (at most MAXSTEPS,
 * default 100000; a negative MAXSTEPS means exactly -MAXSTEPS steps), times it between barriers (max over ranks) and
 * prints one JSON line from rank 0: ranks, steps, seconds, GCUPS and the grid total
 * (per-rank or_sum in rank order). DUMP: rank 0 writes the final H x W grid (raw fp64).
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mm_oracle.h"

#define SEED 0x4D50494DULL

#define MAXA 4
#define MAXF 32

typedef struct {
    long long H, W, x0, h;
    int rank, size;
    int na, nflows;
    or_flow flows[MAXF];
    double* vg[MAXA]; /* (h+2) x W with ghost rows 0 and h+1 */
    double* vn;
    double* sums;     /* rank 0: per step, na sums (program mode) */
    double* gath;     /* rank 0: size x na gathered partials */
} slab;

static void exchange(slab* s, double* vg) {
    const int up = s->rank - 1, down = s->rank + 1;
    const int W = (int)s->W;
    /* first owned row -> up, last owned row -> down; ghosts from the neighbours */
    if (up >= 0)
        MPI_Sendrecv(vg + s->W, W, MPI_DOUBLE, up, 0, vg, W, MPI_DOUBLE, up, 1,
                     MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    if (down < s->size)
        MPI_Sendrecv(vg + s->h * s->W, W, MPI_DOUBLE, down, 1, vg + (s->h + 1) * s->W, W,
                     MPI_DOUBLE, down, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
}

/* one diffusion of attribute a (the vn buffer becomes the attribute's buffer) */
static void diffuse(slab* s, int a, double rate) {
    exchange(s, s->vg[a]);
    if (or_field_step_slab(s->H, s->W, s->x0, s->h, s->vg[a], s->vn + s->W, rate) != 0)
        MPI_Abort(MPI_COMM_WORLD, 3);  /* out of memory */
    double* t = s->vg[a];
    s->vg[a] = s->vn;
    s->vn = t;
}

static void step(slab* s, double rate) {
    if (s->nflows == 0) {
        diffuse(s, 0, rate);
        return;
    }
    /* or_program_step's semantics on the slab: flows in declared order */
    const long long n = s->h * s->W;
    for (int f = 0; f < s->nflows; ++f) {
        const or_flow* fl = &s->flows[f];
        if (fl->kind == 1) {
            diffuse(s, fl->a, fl->rate);
        } else {
            double* va = s->vg[fl->a] + s->W;
            double* vb = fl->b >= 0 ? s->vg[fl->b] + s->W : NULL;
            for (long long i = 0; i < n; ++i) {
                const double out = fl->rate * va[i];
                va[i] = va[i] - out;
                if (vb) vb[i] = vb[i] + out;
            }
        }
    }
    /* per-step sums of every attribute (MPI_Report), combined in rank order on rank 0 */
    double mine[MAXA];
    for (int a = 0; a < s->na; ++a) mine[a] = or_sum(s->vg[a] + s->W, (size_t)n);
    MPI_Gather(mine, s->na, MPI_DOUBLE, s->gath, s->na, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    if (s->rank == 0)
        for (int a = 0; a < s->na; ++a) {
            double t = 0.0;
            for (int r = 0; r < s->size; ++r) t = t + s->gath[r * s->na + a];
            s->sums[a] = t;
        }
}

static int parse_program(slab* s, const char* txt) {
    s->nflows = 0;
    s->na = 1;
    const char* p = txt;
    while (*p && s->nflows < MAXF) {
        or_flow f;
        int used = 0;
        if (sscanf(p, "%d:%d:%d:%lf%n", &f.kind, &f.a, &f.b, &f.rate, &used) != 4) return -1;
        if (f.a < 0 || f.a >= MAXA || f.b >= MAXA || (f.kind != 1 && f.kind != 2)) return -1;
        if (f.kind == 1) f.b = f.a;
        s->flows[s->nflows++] = f;
        if (f.a + 1 > s->na) s->na = f.a + 1;
        if (f.b + 1 > s->na) s->na = f.b + 1;
        p += used;
        if (*p == ',') ++p;
    }
    return 0;
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    slab s;
    MPI_Comm_rank(MPI_COMM_WORLD, &s.rank);
    MPI_Comm_size(MPI_COMM_WORLD, &s.size);
    if (argc < 5) {
        if (s.rank == 0) fprintf(stderr, "usage: mm_cpu_mpi H W RATE SECONDS [MAXSTEPS] [DUMP]\n");
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    s.H = atoll(argv[1]);
    s.W = atoll(argv[2]);
    const double rate = atof(argv[3]);
    const double seconds = atof(argv[4]);
    const long long maxsteps = argc > 5 ? atoll(argv[5]) : 100000;
    const char* dump = argc > 6 ? argv[6] : NULL;
    s.nflows = 0;
    s.na = 1;
    const char* prog = getenv("MM_PROGRAM");
    if (prog && *prog && parse_program(&s, prog) != 0) {
        if (s.rank == 0) fprintf(stderr, "bad MM_PROGRAM\n");
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    or_partition_rows(s.H, s.size, s.rank, &s.x0, &s.h);
    const size_t n = (size_t)((s.h + 2) * s.W);
    for (int a = 0; a < s.na; ++a) {
        s.vg[a] = (double*)calloc(n, sizeof(double));
        if (!s.vg[a]) MPI_Abort(MPI_COMM_WORLD, 3);
        /* attribute a: seed + a, as the engine's fills (bench.py) */
        or_fill_random(s.H, s.W, s.x0, s.h, SEED + (uint64_t)a, s.vg[a] + s.W);
    }
    s.vn = (double*)calloc(n, sizeof(double));
    s.sums = (double*)calloc(MAXA, sizeof(double));
    s.gath = (double*)calloc((size_t)s.size * MAXA, sizeof(double));
    if (!s.vn || !s.sums || !s.gath) MPI_Abort(MPI_COMM_WORLD, 3);

    long long steps = maxsteps < 0 ? -maxsteps : 0, warm = 0;
    if (steps == 0) {
        /* untimed calibration: whole steps until a tenth of the sample (>= 2 steps) */
        MPI_Barrier(MPI_COMM_WORLD);
        double t0 = MPI_Wtime(), mx = 0.0;
        do {
            step(&s, rate);
            ++warm;
            double dt = MPI_Wtime() - t0;
            MPI_Allreduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        } while (warm < 2 || (mx < 0.1 * seconds && warm < maxsteps));
        steps = mx > 0.0 ? (long long)(seconds * (double)warm / mx) : maxsteps;
        if (steps < 1) steps = 1;
        if (steps > maxsteps) steps = maxsteps;
    }
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = MPI_Wtime();
    for (long long i = 0; i < steps; ++i) step(&s, rate);
    double el = MPI_Wtime() - t0, mx = 0.0;
    MPI_Allreduce(&el, &mx, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);

    double mine = 0.0;
    for (int a = 0; a < s.na; ++a) mine = mine + or_sum(s.vg[a] + s.W, (size_t)(s.h * s.W));
    double* all = s.rank == 0 ? (double*)malloc(sizeof(double) * (size_t)s.size) : NULL;
    MPI_Gather(&mine, 1, MPI_DOUBLE, all, 1, MPI_DOUBLE, 0, MPI_COMM_WORLD);

    if (dump) {
        int* counts = NULL;
        int* displs = NULL;
        double* grid = NULL;
        if (s.rank == 0) {
            counts = (int*)malloc(sizeof(int) * (size_t)s.size);
            displs = (int*)malloc(sizeof(int) * (size_t)s.size);
            for (int r = 0; r < s.size; ++r) {
                long long a, h;
                or_partition_rows(s.H, s.size, r, &a, &h);
                counts[r] = (int)(h * s.W);
                displs[r] = (int)(a * s.W);
            }
            grid = (double*)malloc(sizeof(double) * (size_t)(s.H * s.W));
        }
        MPI_Gatherv(s.vg[0] + s.W, (int)(s.h * s.W), MPI_DOUBLE, grid, counts, displs, MPI_DOUBLE, 0,
                    MPI_COMM_WORLD);
        if (s.rank == 0) {
            FILE* f = fopen(dump, "wb");
            if (!f || fwrite(grid, sizeof(double), (size_t)(s.H * s.W), f) != (size_t)(s.H * s.W))
                MPI_Abort(MPI_COMM_WORLD, 4);
            fclose(f);
            free(grid);
            free(counts);
            free(displs);
        }
    }
    if (s.rank == 0) {
        double total = 0.0;
        for (int r = 0; r < s.size; ++r) total = total + all[r];
        printf("{\"ranks\": %d, \"H\": %lld, \"W\": %lld, \"n_attr\": %d, \"n_flows\": %d, "
               "\"steps\": %lld, \"warmup_steps\": %lld, "
               "\"seconds\": %.6f, \"GCUPS\": %.6f, \"total\": %.17g}\n",
               s.size, s.H, s.W, s.na, s.nflows, steps, warm, mx,
               (double)s.H * (double)s.W * (double)steps / mx / 1e9, total);
        fflush(stdout);
        free(all);
    }
    for (int a = 0; a < s.na; ++a) free(s.vg[a]);
    free(s.vn);
    free(s.sums);
    free(s.gath);
    MPI_Finalize();
    return 0;
}
