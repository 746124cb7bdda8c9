// drop_in_main.cpp -- a Main.cpp-style user program for the drop-in API: the same
// includes, classes and calls a reference user writes (reference: src/Main.cpp:17-52),
// built against mpi-model_amd/api/ instead of the reference headers.
//   mpirun -np 6 ./drop_in_main      (5 GPU workers + the master, as the reference)
#include <mpi.h>
#include <stdio.h>
#include <iostream>
#include "MPIImpl.hpp"
#include "Attribute.hpp"
#include "Cell.hpp"
#include "CellularSpace.hpp"
#include "CellularSpaceRectangular.hpp"
#include "Exponencial.hpp"
#include "Model.hpp"
#include "ModelRectangular.hpp"
#include "Defines.hpp"
#include "DefinesRectangular.hpp"

int main(int argc, char* argv[]) {
    int rank = 0, size = 1;
    MPI_Init(&argc, &argv);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);

    CellularSpace<double> space(DIMX, DIMY);
    if (rank == 0) std::cout << space.height << "\t" << space.width << std::endl;
    if (rank == 0) std::cout << "\t(Model)m1.execute()" << std::endl;

    // one Exponencial flow out of cell (19, 3) whose captured value is 2.2, rate 0.1
    Cell<double> source(19, 3, Attribute<double>(99, 2.2));
    Model<Exponencial<double> > model(Exponencial<double>(source, 0.1), 10.0, 0.2);
    model.execute<double>(MPI_COMM_WORLD, space);

    MPI_Finalize();
    return 0;
}
