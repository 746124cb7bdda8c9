/*
 * TEST INFRASTRUCTURE ONLY (oracle pinning). Never linked into the product.
 *
 * Records the reference's own MPI traffic. This driver of ours runs the UNMODIFIED
 * reference headers (compiled where they lie, -I/root/reference/src) and interposes the
 * C binding MPI_Send through the MPI profiling interface: every message is logged to
 * stderr, then passed on to PMPI_Send. That captures, byte for byte, what the reference
 * puts on the wire:
 *   - the 23-char partition descriptors "%d|%d:%d|%d" (src/Model.hpp:70-76,
 *     src/ModelRectangular.hpp:69-80) and flow descriptors "%d|%d:%d|%lf"
 *     (src/Model.hpp:80-86, src/ModelRectangular.hpp:85-92), tag FROM_MASTER / 999;
 *   - the scalar halo messages, the per-rank sums and the file-name messages of
 *     src/Model.hpp:202-204,243,260.
 * The 2-D block bookkeeping of ModelRectangular (which changes no cell)
 * is pinned by exactly these descriptors.
 *
 * argv: mode(row|rect) src_x src_y captured_value rate [space_height space_width]
 *   row : Model<Exponencial<double>>::execute on CellularSpace(DIMX, DIMY) (Main.cpp:25-35)
 *   rect: ModelRectangular<Exponencial<double>>::execute on
 *         CellularSpaceRectangular(space_height, space_width), default
 *         (PROC_DIMX_REC, PROC_DIMY_REC) as the commented-out block of Main.cpp:37-47.
 * The interposer is oracle/mpi_send_log.cpp (linked in; log format there).
 */
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

// the reference's own include order (src/Main.cpp:4-13): MPIImpl.hpp first
#include "MPIImpl.hpp"
#include "Attribute.hpp"
#include "Cell.hpp"
#include "CellularSpace.hpp"
#include "CellularSpaceRectangular.hpp"
#include "Exponencial.hpp"
#include "Model.hpp"
#include "ModelRectangular.hpp"

int main(int argc, char* argv[]) {
    MPI_Init(&argc, &argv);
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s row|rect src_x src_y value rate [h w]\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    const std::string mode = argv[1];
    const int sx = std::atoi(argv[2]);
    const int sy = std::atoi(argv[3]);
    const double value = std::strtod(argv[4], nullptr);
    const double rate = std::strtod(argv[5], nullptr);
    Exponencial<double> flow(Cell<double>(sx, sy, Attribute<double>(99, value)), rate);
    if (mode == "row") {
        CellularSpace<double> cs = CellularSpace<double>(DIMX, DIMY);
        Model<Exponencial<double> > m(flow, 10.0, 0.2);
        m.execute<double>(MPI_COMM_WORLD, cs);
    } else {
        const int h = argc > 6 ? std::atoi(argv[6]) : PROC_DIMX_REC;
        const int w = argc > 7 ? std::atoi(argv[7]) : PROC_DIMY_REC;
        CellularSpaceRectangular<double> cs = CellularSpaceRectangular<double>(h, w);
        ModelRectangular<Exponencial<double> > m(flow, 10.0, 0.2);
        m.execute<double>(MPI_COMM_WORLD, cs);
    }
    MPI_Finalize();
    return 0;
}
