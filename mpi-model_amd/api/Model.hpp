// Model.hpp -- a flow applied to a cellular space (reference: src/Model.hpp:14-263).
// Same class, constructor and execute signatures; execute(comm, space) runs on the
// GPUs through mm_driver.hpp (master/worker layout kept, one GPU slab per worker).
#ifndef MODEL_HPP
#define MODEL_HPP

#include "CellularSpace.hpp"
#include "Flow.hpp"
#include "MPIImpl.hpp"
#include "MPI_Report.hpp"
#include "mm_driver.hpp"

template <class T>
class Model {
public:
    T flow;
    double time;
    double time_step;
    MPI_Report report;  // filled on the master by execute(comm, space)

    Model() : time(0.0), time_step(0.0) {}
    Model(const T& flow_, const double& time_, const double& time_step_)
        : flow(flow_), time(time_), time_step(time_step_) {}
    Model(const Model<T>& o) : flow(o.flow), time(o.time), time_step(o.time_step), report(o.report) {}
    Model<T>& operator=(const Model<T>& o) {
        flow = o.flow;
        time = o.time;
        time_step = o.time_step;
        report = o.report;
        return *this;
    }
    ~Model() {}

    // src/Model.hpp:47-51: the flow evaluated once per time step, no space. The
    // reference falls off the end without a return; here the last outflow is returned.
    double execute() {
        const long long n = mm_step_count(time, time_step);
        for (long long i = 0; i < n; ++i) flow.last_execute = flow.execute();
        return flow.last_execute;
    }

    // src/Model.hpp:53-262. A source-cell flow (Exponencial(cell, rate)) is applied once,
    // as in the reference; a whole-grid flow (Exponencial(rate)) runs
    // step_count(time, time_step) steps.
    template <class R>
    void execute(const MPI_Comm& mpi_comm, const CellularSpace<R>& cellular_space) {
        mm::FlowSpec f;
        f.whole_grid = flow.whole_grid;
        f.src_x = flow.source.x;
        f.src_y = flow.source.y;
        f.captured = flow.source.attribute.value;
        f.rate = flow.flow_rate;
        f.attribute = flow.attribute;
        if (!f.whole_grid) flow.last_execute = flow.execute();  // src/Model.hpp:181
        mm::run_model<R>(mpi_comm, f, time, time_step, cellular_space.height,
                         cellular_space.width, report);
    }
};

#endif
