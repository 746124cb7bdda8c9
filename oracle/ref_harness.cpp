/*
 * TEST INFRASTRUCTURE ONLY (oracle pinning). Never linked into the product.
 *
 * A driver of our own for the UNMODIFIED reference headers, compiled where
 * they lie (-I/root/reference/src). It replaces the reference's Main.cpp
 * (/root/reference/src/Main.cpp:17-52) only to make three things run-time /
 * build-time parameters instead of literals:
 *   - the geometry (DIMX, DIMY, NWORKERS) -> oracle/ref_defines.h
 *   - the flow's source cell, captured value and rate (Main.cpp:33) -> argv
 *   - the text precision of the per-rank dump (Model.hpp:252-255, default
 *     ostream precision 6) -> the cell value type R prints itself as a C99
 *     hex float, so the golden grids are exact.
 * R = RefExactDouble is a one-double wrapper; every arithmetic operation the
 * reference performs on R (Model.hpp:88-91,155,199,206-211,234,238-240) is
 * forwarded to plain double arithmetic, and MPI moves it as MPI_DOUBLE through
 * the reference's own getAbstractionDataType<> hook (Abstraction.hpp:23-26).
 *
 * argv: src_x src_y captured_value rate     (values parsed with strtod, hex ok)
 * Output: the reference's own ../output/comm_rank%d.txt files (cwd-relative).
 */
#include <mpi.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include "MPIImpl.hpp"
#include "Attribute.hpp"
#include "Cell.hpp"
#include "CellularSpace.hpp"
#include "Exponencial.hpp"
#include "Model.hpp"

struct RefExactDouble {
    double v;
    RefExactDouble() {}
    RefExactDouble(double x) : v(x) {}
    operator double() const { return v; }
    RefExactDouble& operator+=(const RefExactDouble& o) { v += o.v; return *this; }
    RefExactDouble& operator-=(double o) { v -= o; return *this; }
};

template <>
inline Abstraction::DataType getAbstractionDataType<RefExactDouble>() {
    return Abstraction::type_double;
}

static std::ostream& operator<<(std::ostream& os, const RefExactDouble& d) {
    char buf[64];
    std::snprintf(buf, sizeof buf, "%a", d.v);
    return os << buf;
}

int main(int argc, char* argv[]) {
    MPI_Init(&argc, &argv);
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s src_x src_y value rate\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    const int sx = std::atoi(argv[1]);
    const int sy = std::atoi(argv[2]);
    const double value = std::strtod(argv[3], nullptr);
    const double rate = std::strtod(argv[4], nullptr);

    CellularSpace<RefExactDouble> cs1 = CellularSpace<RefExactDouble>(DIMX, DIMY);
    Model<Exponencial<double> > m1 = Model<Exponencial<double> >(
        Exponencial<double>(Cell<double>(sx, sy, Attribute<double>(99, value)), rate), 10.0, 0.2);
    m1.execute<RefExactDouble>(MPI_COMM_WORLD, cs1);

    MPI_Finalize();
    return 0;
}
