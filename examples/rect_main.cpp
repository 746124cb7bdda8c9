// rect_main.cpp -- the reference's ModelRectangular use, as in the commented-out block of
// its Main.cpp (src/Main.cpp:37-47), through the drop-in API: a 2-D block model of the
// DIMX_REC x DIMY_REC grid (DefinesRectangular.hpp) on LINES_REC x COLUMNS_REC workers.
//   mpirun -np 7 ./rect_main            (source (18,19), value 2.2, rate 0.1)
//   mpirun -np 7 ./rect_main grid 0.1   (whole-grid Exponencial(rate), step_count(10, 0.2) steps)
// The master prints the flow descriptor line as the reference does, then MPI_Report as one
// JSON line: the block descriptors sent to the workers, the owner, the global sum.
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "CellularSpaceRectangular.hpp"
#include "Exponencial.hpp"
#include "ModelRectangular.hpp"

int main(int argc, char* argv[]) {
    MPI_Init(&argc, &argv);
    int rank = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    const bool grid = argc > 1 && std::strcmp(argv[1], "grid") == 0;

    CellularSpaceRectangular<double> cs2 = CellularSpaceRectangular<double>(PROC_DIMX_REC, PROC_DIMY_REC);
    if (rank == 0) std::cout << cs2.height << "\t" << cs2.width << std::endl;
    if (rank == 0) std::cout << "\t(ModelRectangular)m2.execute()" << std::endl;

    ModelRectangular<Exponencial<double> > m2 =
        grid ? ModelRectangular<Exponencial<double> >(
                   Exponencial<double>(argc > 2 ? std::atof(argv[2]) : 0.1), 10.0, 0.2)
             : ModelRectangular<Exponencial<double> >(
                   Exponencial<double>(Cell<double>(18, 19, Attribute<double>(99, 2.2)), 0.1), 10.0, 0.2);
    m2.execute<double>(MPI_COMM_WORLD, cs2);

    if (rank == 0) {
        const MPI_Report& r = m2.report;
        std::printf("{\"comm_size\": %d, \"owner\": %d, \"steps\": %lld, \"final_sum\": \"%a\", \"blocks\": [",
                    r.comm_size, r.owner, r.steps, r.final_sum);
        for (size_t i = 0; i < r.blocks.size(); i += 4)
            std::printf("%s[%d, %d, %d, %d]", i ? ", " : "", r.blocks[i], r.blocks[i + 1],
                        r.blocks[i + 2], r.blocks[i + 3]);
        std::printf("]}\n");
    }
    MPI_Finalize();
    return 0;
}
