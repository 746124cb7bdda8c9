// mm_driver.hpp -- the MPI master/worker driver behind Model::execute (drop-in API).
//
// Keeps the reference's process layout (src/Model.hpp:53-262): rank 0 is the master
// (no cells: it reduces the workers' sums, checks conservation, merges the result
// files), ranks 1..P are workers, each owning one row slab. What changed is what a
// worker is: a GPU engine (include/mpimodel.h) instead of a stack array of 96-B cells.
//   * partition descriptors and the flow descriptor are computed on every rank
//     (identical integer bookkeeping, src/Model.hpp:60-86) instead of being sent as
//     23-char strings;
//   * the single-source flow (reference form) is applied by every slab to the cells it
//     owns, so the scalar halo messages src/Model.hpp:202-204 / :228-230 disappear;
//   * a whole-grid flow (Exponencial(rate)) runs step_count(time, time_step) steps
//     (the commented-out loop, src/Model.hpp:180-183) with border rows exchanged over
//     RCCL (workers on distinct GPUs) or through MPI (workers sharing a GPU);
//   * the per-rank text dump and the master's merge keep the reference's format
//     (src/Model.hpp:97-131,245-260).
// Environment: MM_OUTPUT_DIR (default "../output", as the reference),
//              MM_WRITE_OUTPUT=0 disables the text files (large grids).
#ifndef MM_DRIVER_HPP
#define MM_DRIVER_HPP

#include <cassert>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "mpi.h"
#include "MPI_Report.hpp"
#include "mm_engine.hpp"

namespace mm {

struct FlowSpec {
    bool whole_grid;
    long long src_x, src_y;
    double captured;  // the Flow's own copy of the source value (src/Flow.hpp:19)
    double rate;
    int attribute;
};

inline std::string output_dir() {
    const char* d = std::getenv("MM_OUTPUT_DIR");
    return d ? std::string(d) : std::string("../output");
}

inline bool write_output() {
    const char* w = std::getenv("MM_WRITE_OUTPUT");
    return !(w && std::strcmp(w, "0") == 0);
}

// Workers' communicator and device placement.
struct WorkerComm {
    MPI_Comm wcomm = MPI_COMM_NULL;
    int wrank = 0, wsize = 1;
    int device = 0, ndev = 1;
    bool distinct_devices = true;
};

inline WorkerComm make_worker_comm(const MPI_Comm& comm, bool is_worker) {
    WorkerComm w;
    MPI_Comm_split(comm, is_worker ? 1 : MPI_UNDEFINED, 0, &w.wcomm);
    if (!is_worker) return w;
    MPI_Comm_rank(w.wcomm, &w.wrank);
    MPI_Comm_size(w.wcomm, &w.wsize);
    MPI_Comm node;
    MPI_Comm_split_type(w.wcomm, MPI_COMM_TYPE_SHARED, w.wrank, MPI_INFO_NULL, &node);
    int lr = 0, ls = 1;
    MPI_Comm_rank(node, &lr);
    MPI_Comm_size(node, &ls);
    MPI_Comm_free(&node);
    check(mm_device_count(&w.ndev));
    w.device = lr % w.ndev;
    int max_ls = ls;
    MPI_Allreduce(&ls, &max_ls, 1, MPI_INT, MPI_MAX, w.wcomm);
    w.distinct_devices = max_ls <= w.ndev;
    return w;
}

// One step of the MPI host transport: first/last owned rows to the neighbours,
// their rows into the ghost rows (whole rows; replaces src/Model.hpp:202-204,228-230).
inline void host_halo(Engine& e, const WorkerComm& w, std::vector<double>& top,
                      std::vector<double>& bot, std::vector<double>& gtop,
                      std::vector<double>& gbot) {
    const int up = w.wrank > 0 ? w.wrank - 1 : MPI_PROC_NULL;
    const int down = w.wrank < w.wsize - 1 ? w.wrank + 1 : MPI_PROC_NULL;
    const int n = (int)top.size();
    e.halo_export(top.data(), bot.data());
    MPI_Sendrecv(top.data(), n, MPI_DOUBLE, up, 71, gbot.data(), n, MPI_DOUBLE, down, 71,
                 w.wcomm, MPI_STATUS_IGNORE);
    MPI_Sendrecv(bot.data(), n, MPI_DOUBLE, down, 72, gtop.data(), n, MPI_DOUBLE, up, 72,
                 w.wcomm, MPI_STATUS_IGNORE);
    e.halo_import(up == MPI_PROC_NULL ? nullptr : gtop.data(),
                  down == MPI_PROC_NULL ? nullptr : gbot.data());
}

template <class R>
std::string write_rank_file(int rank, long long x_init, long long h, long long W,
                            const std::vector<double>& v) {
    char name[512];
    std::snprintf(name, sizeof name, "%s/comm_rank%d.txt", output_dir().c_str(), rank);
    std::ofstream f(name, std::ios::out | std::ios::trunc);
    if (!f.is_open()) {
        std::cerr << "mpimodel: cannot write " << name << std::endl;
        return std::string(name);
    }
    for (long long i = 0; i < h * W; ++i)  // src/Model.hpp:252-255 line format
        f << (x_init + i / W) << "\t" << (i % W) << "\t" << static_cast<R>(v[(size_t)i]) << std::endl;
    return std::string(name);
}

inline void merge_files(const std::vector<std::string>& names) {
    // src/Model.hpp:100-131: "<dir>/output <__TIMESTAMP__>.txt", rank files in order
    std::string out = output_dir() + "/output " + __TIMESTAMP__ + ".txt";
    std::ofstream o(out.c_str(), std::ios::out | std::ios::ate);
    if (!o.is_open()) {
        std::cerr << "mpimodel: cannot write " << out << std::endl;
        return;
    }
    for (const std::string& n : names) {
        std::ifstream in(n.c_str());
        std::string line;
        while (std::getline(in, line)) o << line << "\n";
    }
}

// The worker body: one slab on one GPU. Returns the slab sum (src/Model.hpp:237-240).
template <class R>
double worker(const WorkerComm& w, int rank, int P, const FlowSpec& f, double time,
              double time_step, long long H, long long W, std::vector<double>& hist,
              double& seconds, int& halo_mode, std::string& file) {
    mm_desc d;
    std::memset(&d, 0, sizeof d);
    d.H = H;
    d.W = W;
    check(mm_partition_rows(H, P, rank - 1, &d.x_init, &d.h));
    d.n_attr = 1;
    d.device = w.device;
    d.rank = rank - 1;
    d.nranks = P;
    d.halo_mode = P == 1 ? MM_HALO_NONE
                         : ((f.whole_grid && w.distinct_devices) ? MM_HALO_RCCL : MM_HALO_HOST);
    halo_mode = d.halo_mode;
    std::vector<char> id;
    if (d.halo_mode == MM_HALO_RCCL) {
        id.resize((size_t)mm_comm_id_size());
        if (w.wrank == 0) check(mm_comm_id_create(id.data(), (int)id.size()));
        MPI_Bcast(id.data(), (int)id.size(), MPI_BYTE, 0, w.wcomm);
        d.comm_id = id.data();
    }
    Engine e(d);
    e.fill_uniform(0, 1.0);  // src/Model.hpp:155: Attribute(i, 1)
    seconds = 0.0;
    if (!f.whole_grid) {
        // src/Model.hpp:176-182: the owner reports the source cell and the outflow
        const int owner = mm_owner_reference((int)H, P, (int)f.src_x);
        if (rank == owner) {
            std::cout << f.src_x << " " << f.src_y << " "
                      << mm_neighbor_count(H, W, f.src_x, f.src_y) << std::endl;
            std::cout << rank << ": " << f.rate * f.captured << std::endl;
        }
        e.point_apply(0, f.src_x, f.src_y, f.captured, f.rate);
        e.synchronize();
    } else {
        e.add_flow(MM_FLOW_DIFFUSE, 0, 0, f.rate);
        const long long n = mm_step_count(time, time_step);
        MPI_Barrier(w.wcomm);
        const auto t0 = std::chrono::steady_clock::now();
        if (d.halo_mode == MM_HALO_HOST) {
            std::vector<double> top((size_t)W), bot((size_t)W), gtop((size_t)W), gbot((size_t)W);
            for (long long s = 0; s < n; ++s) {
                host_halo(e, w, top, bot, gtop, gbot);
                e.run(1, 1);
            }
        } else {
            e.run(n, 1);
        }
        e.synchronize();
        seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        hist = e.history();
    }
    const double local = e.sums()[0];
    if (write_output()) {
        std::vector<double> v = e.download(0);
        file = write_rank_file<R>(rank, d.x_init, d.h, W, v);
    }
    return local;
}

template <class R>
void run_model(const MPI_Comm& comm, const FlowSpec& f, double time, double time_step,
               long long H, long long W, MPI_Report& rep) {
    int size = 1, rank = 0;
    MPI_Comm_size(comm, &size);
    MPI_Comm_rank(comm, &rank);
    const bool single = size == 1;  // one process: master and the only worker
    const int P = single ? 1 : size - 1;
    rep.comm_size = size;
    rep.rank_id = rank;
    rep.initial_sum = (double)H * (double)W;  // every cell starts at 1.0

    if (rank == 0 && !f.whole_grid) {
        // src/Model.hpp:80-82: the flow descriptor line the reference master prints
        char line[64];
        std::snprintf(line, sizeof line, "%d|%lld:%lld|%lf", mm_owner_reference((int)H, P, (int)f.src_x),
                      f.src_x, f.src_y, f.rate);
        std::cout << line << std::endl;
    }
    const bool is_worker = single || rank != 0;
    WorkerComm w = make_worker_comm(comm, is_worker);
    std::vector<double> hist;
    double seconds = 0.0, local = 0.0;
    int halo_mode = 0;
    std::string file;
    if (is_worker)
        local = worker<R>(w, single ? 1 : rank, P, f, time, time_step, H, W, hist, seconds,
                          halo_mode, file);

    long long n = f.whole_grid ? mm_step_count(time, time_step) : 0;
    if (single) {
        rep.step_sums = hist;
        rep.seconds = seconds;
        rep.halo_mode = halo_mode;
        rep.devices = 1;
        rep.steps = n;
        rep.gcups = seconds > 0 ? (double)H * W * n / seconds / 1e9 : 0.0;
        assert(std::fabs(local - rep.initial_sum) <= 1e-9 * rep.initial_sum);
        if (write_output()) merge_files(std::vector<std::string>(1, file));
    } else if (rank == 0) {
        // src/Model.hpp:88-95: per-worker sums, received in rank order
        double acc = 0.0;
        for (int k = 1; k <= P; ++k) {
            double t = 0.0;
            MPI_Recv(&t, 1, MPI_DOUBLE, k, k, comm, MPI_STATUS_IGNORE);
            acc += t;
        }
        rep.step_sums.assign((size_t)n, 0.0);
        std::vector<double> h((size_t)n);
        for (int k = 1; k <= P && n > 0; ++k) {
            double sec = 0.0;
            MPI_Recv(h.data(), (int)n, MPI_DOUBLE, k, 1000 + k, comm, MPI_STATUS_IGNORE);
            MPI_Recv(&sec, 1, MPI_DOUBLE, k, 2000 + k, comm, MPI_STATUS_IGNORE);
            for (long long s = 0; s < n; ++s) rep.step_sums[(size_t)s] += h[(size_t)s];
            if (sec > rep.seconds) rep.seconds = sec;
        }
        MPI_Recv(&rep.devices, 1, MPI_INT, 1, 3001, comm, MPI_STATUS_IGNORE);
        MPI_Recv(&rep.halo_mode, 1, MPI_INT, 1, 3002, comm, MPI_STATUS_IGNORE);
        rep.steps = n;
        rep.gcups = rep.seconds > 0 ? (double)H * W * n / rep.seconds / 1e9 : 0.0;
        // the reference's check, made two-sided and size-aware (src/Model.hpp:95)
        assert(std::fabs(acc - rep.initial_sum) <= 1e-9 * rep.initial_sum);
        if (write_output()) {
            std::vector<std::string> names;
            for (int k = 1; k <= P; ++k) {
                char buf[512];
                MPI_Recv(buf, (int)sizeof buf, MPI_CHAR, k, 4000 + k, comm, MPI_STATUS_IGNORE);
                names.push_back(std::string(buf));
            }
            merge_files(names);
        }
    } else {
        MPI_Send(&local, 1, MPI_DOUBLE, 0, rank, comm);  // src/Model.hpp:243
        if (n > 0) {
            hist.resize((size_t)n, 0.0);
            MPI_Send(hist.data(), (int)n, MPI_DOUBLE, 0, 1000 + rank, comm);
            MPI_Send(&seconds, 1, MPI_DOUBLE, 0, 2000 + rank, comm);
        }
        if (rank == 1) {
            int devs = std::min(w.wsize, w.ndev);
            MPI_Send(&devs, 1, MPI_INT, 0, 3001, comm);
            MPI_Send(&halo_mode, 1, MPI_INT, 0, 3002, comm);
        }
        if (write_output()) {
            char buf[512];
            std::memset(buf, 0, sizeof buf);
            std::strncpy(buf, file.c_str(), sizeof buf - 1);
            MPI_Send(buf, (int)sizeof buf, MPI_CHAR, 0, 4000 + rank, comm);  // src/Model.hpp:260
        }
    }
    if (w.wcomm != MPI_COMM_NULL) MPI_Comm_free(&w.wcomm);
}

}  // namespace mm

#endif
