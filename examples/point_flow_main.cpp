// point_flow_main.cpp -- the reference's single-source Exponencial flow (src/Main.cpp:33,
// src/Model.hpp:176-235) through the drop-in API on a run-time grid:
//   mpirun -np P+1 ./point_flow_main H W src_x src_y value rate
// The master prints MPI_Report as one JSON line (owner, final sum, block descriptors).
// Large grids with 10+ workers give descriptors longer than the reference's 23-byte
// control messages; the run must still complete (mm_driver.hpp wire_limit_warning).
#include <mpi.h>

#include <cstdio>
#include <cstdlib>

#include "CellularSpace.hpp"
#include "Exponencial.hpp"
#include "Model.hpp"

int main(int argc, char* argv[]) {
    MPI_Init(&argc, &argv);
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    const int H = argc > 1 ? std::atoi(argv[1]) : 100;
    const int W = argc > 2 ? std::atoi(argv[2]) : 100;
    const int sx = argc > 3 ? std::atoi(argv[3]) : 19;
    const int sy = argc > 4 ? std::atoi(argv[4]) : 3;
    const double value = argc > 5 ? std::atof(argv[5]) : 2.2;
    const double rate = argc > 6 ? std::atof(argv[6]) : 0.1;

    CellularSpace<double> space(H, W);
    Model<Exponencial<double> > model(
        Exponencial<double>(Cell<double>(sx, sy, Attribute<double>(99, value)), rate), 10.0, 0.2);
    model.execute<double>(MPI_COMM_WORLD, space);

    if (rank == 0) {
        const MPI_Report& r = model.report;
        std::printf("{\"comm_size\": %d, \"owner\": %d, \"final_sum\": \"%a\", \"initial_sum\": \"%a\", "
                    "\"blocks\": [",
                    r.comm_size, r.owner, r.final_sum, r.initial_sum);
        for (size_t i = 0; i < r.blocks.size(); i += 4)
            std::printf("%s[%d, %d, %d, %d]", i ? ", " : "", r.blocks[i], r.blocks[i + 1],
                        r.blocks[i + 2], r.blocks[i + 3]);
        std::printf("]}\n");
    }
    MPI_Finalize();
    return 0;
}
