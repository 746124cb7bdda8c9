// ModelRectangular.hpp -- the 2-D block variant of Model
// (reference: src/ModelRectangular.hpp:13-273). The reference cuts the DIMX_REC x DIMY_REC
// grid of DefinesRectangular.hpp into LINES_REC x COLUMNS_REC blocks, sends each worker its
// block descriptor and the flow descriptor (:69-92), but changes no cell (its owner and
// index arithmetic miss the source) and writes no result (:94-129,236-270
// are commented out). Here the master sends the same descriptors (mm_partition_rect_reference,
// mm_owner_rect_reference, mm_wire_*: byte-identical to the reference's,
// tests/golden/wire_rect_*.json) and reports them in MPI_Report::blocks / owner; the flow
// itself is run on the grid by the row-slab engine (the better decomposition on one node of
// GPUs: contiguous border rows, one exchange partner per side). As the reference, no
// result files are written unless MM_WRITE_OUTPUT=1.
#ifndef MODELRECTANGULAR_HPP
#define MODELRECTANGULAR_HPP

#include "CellularSpaceRectangular.hpp"
#include "DefinesRectangular.hpp"
#include "Flow.hpp"
#include "MPIImpl.hpp"
#include "MPI_Report.hpp"
#include "mm_driver.hpp"

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
        if (!f.whole_grid) flow.last_execute = flow.execute();  // src/ModelRectangular.hpp:179
        mm::Layout L;
        L.rect = true;
        L.lines = LINES_REC;
        L.columns = COLUMNS_REC;
        L.space_height = cellular_space.height;  // the owner formula's divisor (:85)
        mm::run_model<R>(mpi_comm, f, time, time_step, DIMX_REC, DIMY_REC, report, L);
    }
};

#endif
