// grid_flow_main.cpp -- the generalised model through the drop-in API: every cell of
// an H x W space is an Exponencial source (Exponencial(rate)), for step_count(time,
// time_step) steps (src/Model.hpp:47-51 loop semantics), on one GPU per worker.
//   mpirun -np 3 ./grid_flow_main [H W time time_step rate]
// The master prints MPI_Report as one JSON line: steps, per-step global sums, GCUPS.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "CellularSpace.hpp"
#include "Exponencial.hpp"
#include "Model.hpp"

int main(int argc, char* argv[]) {
    MPI_Init(&argc, &argv);
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    const int H = argc > 1 ? std::atoi(argv[1]) : 1000;
    const int W = argc > 2 ? std::atoi(argv[2]) : 1000;
    const double time = argc > 3 ? std::atof(argv[3]) : 10.0;
    const double dt = argc > 4 ? std::atof(argv[4]) : 0.2;
    const double rate = argc > 5 ? std::atof(argv[5]) : 0.1;

    CellularSpace<double> space(H, W);
    Model<Exponencial<double> > model(Exponencial<double>(rate), time, dt);
    model.execute<double>(MPI_COMM_WORLD, space);

    if (rank == 0) {
        const MPI_Report& r = model.report;
        std::printf("{\"comm_size\": %d, \"steps\": %lld, \"initial_sum\": %.17g, \"final_sum\": %.17g, "
                    "\"seconds\": %.6f, \"gcups\": %.3f, \"halo_mode\": %d, \"sums\": [",
                    r.comm_size, r.steps, r.initial_sum,
                    r.step_sums.empty() ? r.initial_sum : r.step_sums.back(), r.seconds, r.gcups,
                    r.halo_mode);
        for (size_t i = 0; i < r.step_sums.size(); ++i)
            std::printf("%s\"%a\"", i ? ", " : "", r.step_sums[i]);
        std::printf("]}\n");
    }
    MPI_Finalize();
    return 0;
}
