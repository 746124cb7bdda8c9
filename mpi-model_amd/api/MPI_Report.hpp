// MPI_Report.hpp -- run report (reference: src/MPI_Report.hpp:5-20, where it holds only
// {comm_size, rank_id} and is never filled). Here Model::execute fills it on the master
// with what BASELINE.json asks of it: the per-step global sums of the attribute (the
// reference's conservation reduction, src/Model.hpp:88-95, done every step) and timing.
#ifndef MPI_REPORT_HPP
#define MPI_REPORT_HPP

#include <vector>

class MPI_Report {
public:
    int comm_size;
    int rank_id;
    long long steps = 0;                 // steps run (src/Model.hpp:47-51 loop count)
    std::vector<double> step_sums;       // global sum after every step, workers in rank order
    double initial_sum = 0.0;            // global sum before the first step
    double final_sum = 0.0;              // global sum at the end: the workers' slab sums added
                                         // in rank order (src/Model.hpp:88-92)
    double seconds = 0.0;                // slowest worker's device time for the steps
    double gcups = 0.0;                  // cell updates per second / 1e9
    int devices = 0;                     // GPUs used by the workers
    int halo_mode = 0;                   // enum mm_halo_mode of the run
    int owner = 0;                       // worker the flow descriptor names (src/Model.hpp:80,
                                         // src/ModelRectangular.hpp:85; 0 for a whole-grid flow)
    std::vector<int> blocks;             // x_init, y_init, height, width of every worker's
                                         // descriptor as sent on the wire (rank 0 only)

    MPI_Report() : comm_size(0), rank_id(0) {}
    MPI_Report(const MPI_Report& o) = default;
    MPI_Report& operator=(const MPI_Report& o) = default;
    MPI_Report(const int& comm_size_, const int& rank_id_)
        : comm_size(comm_size_), rank_id(rank_id_) {}
    ~MPI_Report() {}
};

#endif
