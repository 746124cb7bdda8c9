/*
 * mm_cpu_mpi.c -- CPU baseline of the flow step with the reference's decomposition
 * (TEST INFRASTRUCTURE: bench.py's cpu_baseline leg and tests/ only; never the product).
 *
 * The reference runs one MPI rank per core on row blocks and moves border rows with
 * blocking MPI_Send/MPI_Recv (src/MPIImpl.cpp:21-79 comm_send/comm_recv, called from
 * src/Model.hpp:90-121 and 154-238). This program keeps that structure -- 1-D row slabs
 * (or_partition_rows), one ghost row above and below, a blocking MPI_Sendrecv of the border
 * rows every step -- and computes each slab with the oracle's restated step
 * (or_field_step_slab, mm_oracle.c), so its grid is the oracle's grid bit for bit.
 *
 *   mpirun -np P mm_cpu_mpi H W RATE SECONDS [MAXSTEPS] [DUMP]
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

typedef struct {
    long long H, W, x0, h;
    int rank, size;
    double *vg, *vn; /* (h+2) x W with ghost rows 0 and h+1 */
} slab;

static void exchange(slab* s) {
    const int up = s->rank - 1, down = s->rank + 1;
    const int W = (int)s->W;
    /* first owned row -> up, last owned row -> down; ghosts from the neighbours */
    if (up >= 0)
        MPI_Sendrecv(s->vg + s->W, W, MPI_DOUBLE, up, 0, s->vg, W, MPI_DOUBLE, up, 1,
                     MPI_COMM_WORLD, MPI_STATUS_IGNORE);
    if (down < s->size)
        MPI_Sendrecv(s->vg + s->h * s->W, W, MPI_DOUBLE, down, 1, s->vg + (s->h + 1) * s->W, W,
                     MPI_DOUBLE, down, 0, MPI_COMM_WORLD, MPI_STATUS_IGNORE);
}

static void step(slab* s, double rate) {
    exchange(s);
    or_field_step_slab(s->H, s->W, s->x0, s->h, s->vg, s->vn + s->W, rate);
    double* t = s->vg;
    s->vg = s->vn;
    s->vn = t;
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
    or_partition_rows(s.H, s.size, s.rank, &s.x0, &s.h);
    const size_t n = (size_t)((s.h + 2) * s.W);
    s.vg = (double*)calloc(n, sizeof(double));
    s.vn = (double*)calloc(n, sizeof(double));
    if (!s.vg || !s.vn) MPI_Abort(MPI_COMM_WORLD, 3);
    or_fill_random(s.H, s.W, s.x0, s.h, SEED, s.vg + s.W);

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

    double mine = or_sum(s.vg + s.W, (size_t)(s.h * s.W));
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
        MPI_Gatherv(s.vg + s.W, (int)(s.h * s.W), MPI_DOUBLE, grid, counts, displs, MPI_DOUBLE, 0,
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
        printf("{\"ranks\": %d, \"H\": %lld, \"W\": %lld, \"steps\": %lld, \"warmup_steps\": %lld, "
               "\"seconds\": %.6f, \"GCUPS\": %.6f, \"total\": %.17g}\n",
               s.size, s.H, s.W, steps, warm, mx, (double)s.H * (double)s.W * (double)steps / mx / 1e9,
               total);
        fflush(stdout);
        free(all);
    }
    free(s.vg);
    free(s.vn);
    MPI_Finalize();
    return 0;
}
