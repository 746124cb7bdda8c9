// mm_driver.hpp -- the MPI master/worker driver behind Model::execute and
// ModelRectangular::execute (drop-in API).
//
// Keeps the reference's process layout and control plane (src/Model.hpp:53-262,
// src/ModelRectangular.hpp:52-272): rank 0 is the master (no cells), ranks 1..P are
// workers. The master sends every worker the reference's 23-char partition descriptor
// ("%d|%d:%d|%d", tag 0) and flow descriptor ("%d|%d:%d|%lf", tag 999) -- the same bytes
// (tests/golden/wire_*.json), formatted and parsed by the C ABI (mm_wire_*); it then
// reduces the workers' sums in rank order, checks conservation and merges the result
// files. What changed is what a worker is: a GPU engine (include/mpimodel.h) instead of
// a stack array of 96-B cells.
//   * Model: row slabs. A worker owns rows mm_partition_rows(H, P, k-1), which are the
//     descriptor's rows whenever P divides H (the only layout the reference itself
//     completes); when it does not, the reference drops the
//     remainder rows while the engine slabs cover them.
//   * ModelRectangular: the DIMX_REC x DIMY_REC grid of DefinesRectangular.hpp, 2-D block
//     descriptors (mm_partition_rect_reference) and owner formula (mm_owner_rect_reference)
//     as the reference; the cells are computed on row slabs (the better decomposition for
//     GPUs on one node), and, as the reference, no result files by default.
//   * the single-source flow (reference form) is applied by every slab to the cells it
//     owns, so the scalar halo messages src/Model.hpp:202-204 / :228-230 disappear;
//   * a whole-grid flow (Exponencial(rate)) runs step_count(time, time_step) steps
//     (the commented-out loop, src/Model.hpp:180-183) with border rows exchanged over
//     RCCL (workers on distinct GPUs) or through MPI (workers sharing a GPU: before each
//     K-step pass of the engine's plan, K rows per exchange);
//   * the per-rank text dump and the master's merge keep the reference's format
//     (src/Model.hpp:97-131,245-260).
// Environment: MM_OUTPUT_DIR (default "../output", as the reference),
//              MM_WRITE_OUTPUT=0/1 disables / enables the text files (large grids),
//              MM_STRICT_REFERENCE=1 applies a single-source flow only where the
//              reference's P-worker run does (mm_point_apply_strict; elsewhere, e.g. an
//              edge source, the grid is left as the reference leaves it).
#ifndef MM_DRIVER_HPP
#define MM_DRIVER_HPP

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <stdexcept>
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

// Which reference model drives the run.
struct Layout {
    bool rect = false;      // ModelRectangular: 2-D block descriptors
    int lines = 1, columns = 1;
    int space_height = 0;   // the caller's space height (ModelRectangular owner formula)
};

inline std::string output_dir() {
    const char* d = std::getenv("MM_OUTPUT_DIR");
    return d ? std::string(d) : std::string("../output");
}

inline bool write_output(bool dflt) {
    const char* w = std::getenv("MM_WRITE_OUTPUT");
    if (!w) return dflt;
    return std::strcmp(w, "0") != 0;
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

// One exchange of the MPI host transport: the first / last `rows` owned rows to the
// neighbours, theirs into the ghost rows (whole rows, `rows` deep; replaces
// src/Model.hpp:202-204,228-230).
inline void host_halo(Engine& e, const WorkerComm& w, int rows, std::vector<double>& top,
                      std::vector<double>& bot, std::vector<double>& gtop,
                      std::vector<double>& gbot) {
    const int up = w.wrank > 0 ? w.wrank - 1 : MPI_PROC_NULL;
    const int down = w.wrank < w.wsize - 1 ? w.wrank + 1 : MPI_PROC_NULL;
    const int n = (int)(rows * e.desc().W);
    e.halo_export(rows, top.data(), bot.data());
    MPI_Sendrecv(top.data(), n, MPI_DOUBLE, up, 71, gbot.data(), n, MPI_DOUBLE, down, 71,
                 w.wcomm, MPI_STATUS_IGNORE);
    MPI_Sendrecv(bot.data(), n, MPI_DOUBLE, down, 72, gtop.data(), n, MPI_DOUBLE, up, 72,
                 w.wcomm, MPI_STATUS_IGNORE);
    e.halo_import(rows, up == MPI_PROC_NULL ? nullptr : gtop.data(),
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

// The control messages of worker k (1-based): what the reference's master sends, and the
// numbers they carry (computed here on every rank, so nothing depends on the bytes).
struct Descriptors {
    char partition[MM_WIRE_LEN];
    char flow[MM_WIRE_LEN];
    int owner;
    int x0, y0, h, w;
    bool fits;  // both messages fit the reference's 23 bytes (with the NUL)
};

// A descriptor past the reference's 23-char buffer (e.g. "10|10000:10000|0.100000", or a
// large rate through %lf) cannot go on the reference's wire. It is a limit of the wire
// format, not of the run: the message goes out as 23 NUL bytes, every rank uses the numbers
// it computed itself, and rank 0 says so once on stderr.
inline void wire_limit_warning(bool fits, int rank) {
    static bool said = false;
    if (fits || said || rank != 0) return;
    said = true;
    std::cerr << "mpimodel: a control descriptor does not fit the reference's " << MM_WIRE_LEN
              << "-byte message (src/Model.hpp:71,81); sending NUL bytes, every rank uses its "
                 "own partition and owner" << std::endl;
}

inline Descriptors make_descriptors(const Layout& L, const FlowSpec& f, int H, int W, int P,
                                    int k) {
    Descriptors d;
    if (L.rect)
        check(mm_partition_rect_reference(H, W, L.lines, L.columns, k, &d.x0, &d.y0, &d.h, &d.w));
    else
        check(mm_partition_reference(H, W, P, k, &d.x0, &d.y0, &d.h, &d.w));
    // mm_wire_format_* leave an all-NUL buffer when the text does not fit
    d.fits = mm_wire_format_partition(d.partition, MM_WIRE_LEN, d.x0, d.y0, d.h, d.w) == MM_OK;
    if (f.whole_grid) {  // extension: every cell is a source; no owner, no source cell
        d.owner = 0;
        d.fits = mm_wire_format_flow(d.flow, MM_WIRE_LEN, 0, -1, -1, f.rate) == MM_OK && d.fits;
    } else {
        d.owner = L.rect ? mm_owner_rect_reference(L.space_height, (int)f.src_x, (int)f.src_y)
                         : mm_owner_reference(H, P, (int)f.src_x);
        d.fits = mm_wire_format_flow(d.flow, MM_WIRE_LEN, d.owner, (int)f.src_x, (int)f.src_y,
                                     f.rate) == MM_OK && d.fits;
    }
    return d;
}

// The reference's conservation check (src/Model.hpp:95), two-sided and size-aware, as a
// check that survives NDEBUG: a violation throws std::runtime_error like the reference's
// MPI failures (src/MPIImpl.cpp:7-8).
inline void check_conservation(double sum, double initial) {
    if (!(std::fabs(sum - initial) <= 1e-9 * initial)) {
        char msg[160];
        std::snprintf(msg, sizeof msg, "mpimodel: conservation violated: sum %.17g, initial %.17g",
                      sum, initial);
        throw std::runtime_error(msg);
    }
}

// The worker body: one slab on one GPU. Returns the slab sum (src/Model.hpp:237-240).
template <class R>
double worker(const WorkerComm& w, int rank, int P, const FlowSpec& f, int owner, double time,
              double time_step, long long H, long long W, bool files, std::vector<double>& hist,
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
        if (rank == owner) {
            std::cout << f.src_x << " " << f.src_y << " "
                      << mm_neighbor_count(H, W, f.src_x, f.src_y) << std::endl;
            std::cout << rank << ": " << f.rate * f.captured << std::endl;
        }
        const char* strict = std::getenv("MM_STRICT_REFERENCE");
        if (f.src_x < H && f.src_y < W) {
            if (strict && std::strcmp(strict, "0") != 0)
                e.point_apply_strict(0, f.src_x, f.src_y, f.captured, f.rate, P);
            else
                e.point_apply(0, f.src_x, f.src_y, f.captured, f.rate);
        }
        e.synchronize();
    } else {
        e.add_flow(MM_FLOW_DIFFUSE, 0, 0, f.rate);
        const long long n = mm_step_count(time, time_step);
        MPI_Barrier(w.wcomm);
        const auto t0 = std::chrono::steady_clock::now();
        if (d.halo_mode == MM_HALO_HOST) {
            // workers sharing a GPU: before each K-step pass of the engine's plan (the same
            // on every worker: it is sized by the thinnest slab) that pass's K border rows
            // go through MPI, then the pass runs
            const std::vector<int> plan = e.pass_plan(n);
            const int depth = plan.empty() ? 1 : *std::max_element(plan.begin(), plan.end());
            const size_t sz = (size_t)depth * (size_t)W;
            std::vector<double> top(sz), bot(sz), gtop(sz), gbot(sz);
            for (const int k : plan) {
                host_halo(e, w, k, top, bot, gtop, gbot);
                e.run(k, 1);
            }
        } else {
            e.run(n, 1);
        }
        e.synchronize();
        seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        hist = e.history();
    }
    const double local = e.sums()[0];
    if (files) {
        std::vector<double> v = e.download(0);
        file = write_rank_file<R>(rank, d.x_init, d.h, W, v);
    }
    return local;
}

template <class R>
void run_model(const MPI_Comm& comm, const FlowSpec& f, double time, double time_step,
               long long H, long long W, MPI_Report& rep, const Layout& L = Layout()) {
    int size = 1, rank = 0;
    MPI_Comm_size(comm, &size);
    MPI_Comm_rank(comm, &rank);
    const bool single = size == 1;  // one process: master and the only worker
    const int P = single ? 1 : size - 1;
    const bool files = write_output(!L.rect);  // ModelRectangular writes none (as the reference)
    rep.comm_size = size;
    rep.rank_id = rank;
    rep.initial_sum = (double)H * (double)W;  // every cell starts at 1.0

    // control plane: the reference's descriptors, master -> every worker
    Descriptors mine = make_descriptors(L, f, (int)H, (int)W, P, single ? 1 : (rank ? rank : 1));
    rep.owner = mine.owner;
    if (rank == 0) {
        rep.blocks.clear();
        for (int k = 1; k <= P; ++k) {
            const Descriptors dk = make_descriptors(L, f, (int)H, (int)W, P, k);
            wire_limit_warning(dk.fits, rank);
            int x0 = dk.x0, y0 = dk.y0, h = dk.h, w = dk.w;
            if (dk.fits)  // what a worker reads back (src/Model.hpp:139-146)
                check(mm_wire_parse_partition(dk.partition, MM_WIRE_LEN, &x0, &y0, &h, &w));
            rep.blocks.insert(rep.blocks.end(), {x0, y0, h, w});
            if (!single) MPI_Send(dk.partition, MM_WIRE_LEN, MPI_CHAR, k, MM_TAG_PARTITION, comm);
        }
        if (!f.whole_grid) {
            // src/Model.hpp:82 (ModelRectangular.hpp:88 appends the owner)
            if (L.rect)
                std::cout << mine.flow << " " << mine.owner << std::endl;
            else
                std::cout << mine.flow << std::endl;
        }
        if (!single)
            for (int k = 1; k <= P; ++k)
                MPI_Send(mine.flow, MM_WIRE_LEN, MPI_CHAR, k, MM_TAG_FLOW, comm);
    }
    int owner = mine.owner;
    if (!single && rank != 0) {
        // src/Model.hpp:138-167: the worker's receive and strtok/atoi parse
        char part[MM_WIRE_LEN + 1] = {0}, flow[MM_WIRE_LEN + 1] = {0};
        MPI_Recv(part, MM_WIRE_LEN, MPI_CHAR, 0, MM_TAG_PARTITION, comm, MPI_STATUS_IGNORE);
        MPI_Recv(flow, MM_WIRE_LEN, MPI_CHAR, 0, MM_TAG_FLOW, comm, MPI_STATUS_IGNORE);
        int x0, y0, h, w, fx, fy, rate_atoi, parsed_owner;
        double rate;
        // a descriptor past the wire's 23 bytes arrives as NUL bytes: keep the local numbers
        if (mm_wire_parse_partition(part, MM_WIRE_LEN, &x0, &y0, &h, &w) == MM_OK &&
            mm_wire_parse_flow(flow, MM_WIRE_LEN, &parsed_owner, &fx, &fy, &rate_atoi, &rate) == MM_OK)
            owner = parsed_owner;
        if (L.rect) std::cout << flow << std::endl;  // src/ModelRectangular.hpp:158
    }

    const bool is_worker = single || rank != 0;
    WorkerComm w = make_worker_comm(comm, is_worker);
    std::vector<double> hist;
    double seconds = 0.0, local = 0.0;
    int halo_mode = 0;
    std::string file;
    if (is_worker)
        local = worker<R>(w, single ? 1 : rank, P, f, owner, time, time_step, H, W, files, hist,
                          seconds, halo_mode, file);

    long long n = f.whole_grid ? mm_step_count(time, time_step) : 0;
    if (single) {
        rep.step_sums = hist;
        rep.seconds = seconds;
        rep.halo_mode = halo_mode;
        rep.devices = 1;
        rep.steps = n;
        rep.gcups = seconds > 0 ? (double)H * W * n / seconds / 1e9 : 0.0;
        rep.final_sum = local;
        check_conservation(local, rep.initial_sum);
        if (files) merge_files(std::vector<std::string>(1, file));
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
        rep.final_sum = acc;
        check_conservation(acc, rep.initial_sum);
        if (files) {
            // src/Model.hpp:110-111: file names in rank order, tag = rank
            std::vector<std::string> names;
            for (int k = 1; k <= P; ++k) {
                char buf[512];
                std::memset(buf, 0, sizeof buf);
                MPI_Recv(buf, (int)sizeof buf - 1, MPI_CHAR, k, k, comm, MPI_STATUS_IGNORE);
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
        if (files) {
            // src/Model.hpp:260: the file name, 30 chars as the reference when it fits
            char buf[512];
            std::memset(buf, 0, sizeof buf);
            std::strncpy(buf, file.c_str(), sizeof buf - 1);
            const int len = file.size() < 30 ? 30 : (int)file.size() + 1;
            MPI_Send(buf, len, MPI_CHAR, 0, rank, comm);
        }
    }
    if (w.wcomm != MPI_COMM_NULL) MPI_Comm_free(&w.wcomm);
}

}  // namespace mm

#endif
