// ModelRectangular.hpp -- the 2-D block variant of Model
// (reference: src/ModelRectangular.hpp:13-273). The reference cuts a DIMX_REC x DIMY_REC
// grid into LINES_REC x COLUMNS_REC blocks (:69-80) but changes no cell (its owner and
// index arithmetic miss the source). Here the block descriptors are
// computed with the same integer bookkeeping (rect_block) and the flow itself is run
// by the row-slab engine, which is the better decomposition on one node of GPUs
// (contiguous border rows, one exchange partner per side).
#ifndef MODELRECTANGULAR_HPP
#define MODELRECTANGULAR_HPP

#include "CellularSpaceRectangular.hpp"
#include "DefinesRectangular.hpp"
#include "Flow.hpp"
#include "MPIImpl.hpp"
#include "MPI_Report.hpp"
#include "mm_driver.hpp"

namespace mm {
// src/ModelRectangular.hpp:69-80: descriptor of worker k (1-based): blocks are dealt
// row-major, PROC_DIMY_REC columns at a time, wrapping to the next band of rows.
inline void rect_block(int k, int* x_init, int* y_init, int* height, int* width) {
    int ox = 0, oy = 0;
    for (int dest = 1; dest < k; ++dest) {
        oy += PROC_DIMY_REC;
        if (oy == DIMY_REC) {
            ox += PROC_DIMX_REC;
            oy = 0;
        }
    }
    *x_init = ox;
    *y_init = oy;
    *height = PROC_DIMX_REC;
    *width = PROC_DIMY_REC;
}
}  // namespace mm

template <class T>
class ModelRectangular {
public:
    T flow;
    double time;
    double time_step;
    MPI_Report report;

    ModelRectangular() : time(0.0), time_step(0.0) {}
    ModelRectangular(const T& flow_, const double& time_, const double& time_step_)
        : flow(flow_), time(time_), time_step(time_step_) {}
    ModelRectangular(const ModelRectangular<T>& o)
        : flow(o.flow), time(o.time), time_step(o.time_step), report(o.report) {}
    ModelRectangular<T>& operator=(const ModelRectangular<T>& o) {
        flow = o.flow;
        time = o.time;
        time_step = o.time_step;
        report = o.report;
        return *this;
    }
    ~ModelRectangular() {}

    double execute() {
        const long long n = mm_step_count(time, time_step);
        for (long long i = 0; i < n; ++i) flow.last_execute = flow.execute();
        return flow.last_execute;
    }

    template <class R>
    void execute(const MPI_Comm& mpi_comm, const CellularSpaceRectangular<R>& cellular_space) {
        mm::FlowSpec f;
        f.whole_grid = flow.whole_grid;
        f.src_x = flow.source.x;
        f.src_y = flow.source.y;
        f.captured = flow.source.attribute.value;
        f.rate = flow.flow_rate;
        f.attribute = flow.attribute;
        if (!f.whole_grid) flow.last_execute = flow.execute();
        mm::run_model<R>(mpi_comm, f, time, time_step, cellular_space.height,
                         cellular_space.width, report);
    }
};

#endif
