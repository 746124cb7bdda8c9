// mm_engine.hpp -- C++ RAII face of the C ABI (include/mpimodel.h) for the drop-in
// headers. Non-zero status codes become std::runtime_error, the reference's error
// convention (src/MPIImpl.cpp:7-8,13-14).
#ifndef MM_ENGINE_HPP
#define MM_ENGINE_HPP

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "mpimodel.h"

namespace mm {

inline void check(int rc) {
    if (rc != MM_OK) throw std::runtime_error(std::string("mpimodel: ") + mm_last_error());
}

class Engine {
public:
    explicit Engine(const mm_desc& d) : e_(nullptr), d_(d) { check(mm_engine_create(&d, &e_)); }
    ~Engine() { mm_engine_destroy(e_); }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    const mm_desc& desc() const { return d_; }
    void fill_uniform(int attr, double v) { check(mm_fill(e_, attr, MM_FILL_UNIFORM, v, 0)); }
    void fill_random(int attr, unsigned long long seed) {
        check(mm_fill(e_, attr, MM_FILL_RANDOM, 0.0, seed));
    }
    void add_flow(int kind, int a, int b, double rate) { check(mm_add_flow(e_, kind, a, b, rate)); }
    void point_apply(int attr, long long sx, long long sy, double captured, double rate) {
        check(mm_point_apply(e_, attr, sx, sy, captured, rate));
    }
    bool point_apply_strict(int attr, long long sx, long long sy, double captured, double rate,
                            int workers) {
        int applied = 0;
        check(mm_point_apply_strict(e_, attr, sx, sy, captured, rate, workers, &applied));
        return applied != 0;
    }
    void run(long long steps, long long reduce_every) { check(mm_run(e_, steps, reduce_every)); }
    // the K-step passes a run of `steps` steps launches (the engine's pass planner)
    std::vector<int> pass_plan(long long steps) {
        int n = 0;
        check(mm_pass_plan(e_, steps, nullptr, 0, &n));
        std::vector<int> lens((size_t)n);
        if (n) check(mm_pass_plan(e_, steps, lens.data(), n, &n));
        return lens;
    }
    void synchronize() { check(mm_synchronize(e_)); }
    std::vector<double> sums() {
        std::vector<double> s(d_.n_attr);
        check(mm_sums(e_, s.data()));
        return s;
    }
    std::vector<double> history() {
        long long n = 0;
        check(mm_sums_history(e_, nullptr, 0, &n));
        std::vector<double> h((size_t)n * d_.n_attr);
        long long got = n;
        if (n) check(mm_sums_history(e_, h.data(), n, &got));
        h.resize((size_t)std::min(n, got) * d_.n_attr);
        return h;
    }
    std::vector<double> download(int attr) {
        std::vector<double> v((size_t)(d_.h * d_.W));
        check(mm_download(e_, attr, v.data()));
        return v;
    }
    mm_info info() {
        mm_info i;
        check(mm_engine_info(e_, &i));
        return i;
    }
    // first / last nrows owned rows of every attribute, [attr][row][col]
    void halo_export(int nrows, double* top, double* bottom) {
        check(mm_halo_export_rows(e_, nrows, top, bottom));
    }
    void halo_import(int nrows, const double* top, const double* bottom) {
        check(mm_halo_import_rows(e_, nrows, top, bottom));
    }

private:
    mm_engine* e_;
    mm_desc d_;
};

}  // namespace mm

#endif
