// CellularSpaceRectangular.hpp -- space of the 2-D block model
// (reference: src/CellularSpaceRectangular.hpp:8-32). Descriptor only, as CellularSpace.
#ifndef CELLULARSPACERECTANGULAR_HPP
#define CELLULARSPACERECTANGULAR_HPP

#include <vector>

#include "mpi.h"
#include "Cell.hpp"
#include "DefinesRectangular.hpp"

template <class T>
class CellularSpaceRectangular {
public:
    int x_init;
    int y_init;
    int width;
    int height;
    mutable std::vector<Cell<T> > memoria;

    CellularSpaceRectangular() : x_init(0), y_init(0), width(0), height(0) {}
    CellularSpaceRectangular(const int& height_, const int& width_)
        : x_init(0), y_init(0), width(width_), height(height_) {}
    CellularSpaceRectangular(const int& x_init_, const int& y_init_, const int& height_,
                             const int& width_)
        : x_init(x_init_), y_init(y_init_), width(width_), height(height_) {}
};

#endif
