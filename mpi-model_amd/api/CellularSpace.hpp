// CellularSpace.hpp -- a rectangular space or one rank's row slab of it
// (reference: src/CellularSpace.hpp:8-34). The reference embeds a static
// Cell[PROC_DIMX*PROC_DIMY] array (96 B per cell, on the stack); here the space is a
// descriptor and the cell values live on the GPU as fp64 arrays owned by the engine
// (Model::execute). `memoria` stays empty: results reach the caller as the reference's
// output files and through MPI_Report, so host memory stays O(1).
#ifndef CELLULARSPACE_HPP
#define CELLULARSPACE_HPP

#include <vector>

#include "mpi.h"
#include "Cell.hpp"
#include "Defines.hpp"
#include "mm_engine.hpp"

template <class T>
class CellularSpace {
public:
    int x_init;
    int y_init;
    int width;
    int height;
    mutable std::vector<Cell<T> > memoria;

    CellularSpace() : x_init(0), y_init(0), width(0), height(0) {}
    CellularSpace(const int& height_, const int& width_)
        : x_init(0), y_init(0), width(width_), height(height_) {}
    CellularSpace(const int& x_init_, const int& y_init_, const int& height_, const int& width_)
        : x_init(x_init_), y_init(y_init_), width(width_), height(height_) {}

    // The reference's Scatter (CellularSpace.hpp:36-79) builds a slab and drops it.
    // Here it turns this space into the calling worker's slab of the reference
    // partition (src/Model.hpp:60-76); rank 0 (the master) keeps the whole space.
    void Scatter(const MPI_Comm& comm) {
        int size = 1, rank = 0;
        MPI_Comm_size(comm, &size);
        MPI_Comm_rank(comm, &rank);
        if (rank == 0 || size < 2) return;
        int xi, yi, h, w;
        mm::check(mm_partition_reference(height, width, size - 1, rank, &xi, &yi, &h, &w));
        x_init = xi;
        y_init = yi;
        height = h;
        width = w;
    }
};

#endif
