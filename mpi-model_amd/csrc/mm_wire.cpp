// mm_wire.cpp -- host-only bookkeeping of the reference's control plane (C ABI,
// include/mpimodel.h): the 2-D block partition and owner formula of ModelRectangular and
// the 23-char control messages both models send from the master to every worker.
// Pinned against the reference's own MPI traffic (tests/golden/wire_*.json, recorded by
// oracle/ref_wire_harness.cpp) in tests/test_abi.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/mpimodel.h"

namespace {

// strtok-style tokenizer over a private, NUL-terminated copy (the reference runs strtok
// on its receive buffer, src/Model.hpp:139-142,160-163): a token is the next maximal run
// of characters not in `delim`, after skipping leading delimiters.
struct Tokens {
    std::string buf;
    size_t pos = 0;
    Tokens(const char* msg, int len) {
        size_t n = 0;
        while ((int)n < len && msg[n]) ++n;
        buf.assign(msg, n);
    }
    bool next(const char* delim, std::string& tok) {
        while (pos < buf.size() && std::strchr(delim, buf[pos])) ++pos;
        if (pos >= buf.size()) return false;
        const size_t start = pos;
        while (pos < buf.size() && !std::strchr(delim, buf[pos])) ++pos;
        tok = buf.substr(start, pos - start);
        if (pos < buf.size()) ++pos;  // strtok overwrites the delimiter that ended the token
        return true;
    }
};

int fit(char* out, int len, int n) {
    if (n < 0 || n >= len) {
        if (out && len > 0) std::memset(out, 0, (size_t)len);
        return MM_ERR_INVALID;
    }
    std::memset(out + n, 0, (size_t)(len - n));  // the reference sends stack garbage here
    return MM_OK;
}

}  // namespace

extern "C" {

int mm_partition_rect_reference(int H, int W, int lines, int columns, int k, int* x_init,
                                int* y_init, int* height, int* width) {
    if (H <= 0 || W <= 0 || lines <= 0 || columns <= 0 || k < 1 || !x_init || !y_init ||
        !height || !width)
        return MM_ERR_INVALID;
    // src/ModelRectangular.hpp:69-80: offsets advance PROC_DIMY_REC = W / columns per
    // worker and wrap to the next band of PROC_DIMX_REC = H / lines rows only when the
    // column offset lands exactly on W (never, if columns does not divide W)
    const int ph = H / lines, pw = W / columns;
    int ox = 0, oy = 0;
    for (int dest = 1; dest < k; ++dest) {
        oy = oy + pw;
        if (oy == W) {
            ox = ox + ph;
            oy = 0;
        }
    }
    *x_init = ox;
    *y_init = oy;
    *height = ph;
    *width = pw;
    return MM_OK;
}

int mm_owner_rect_reference(int space_height, int x, int y) {
    if (space_height <= 0) return -1;
    return (x + y) / space_height + 1;  // src/ModelRectangular.hpp:85
}

int mm_point_strict_applies(int H, int W, int P, int x, int y) {
    if (H <= 0 || W <= 0 || P <= 0 || x < 0 || y < 0 || x >= H || y >= W || H / P == 0) return -1;
    // src/Model.hpp:80: the owner; rows past P*(H/P) (dropped remainder rows) have none
    const int owner = x / (H / P) + 1;
    if (owner > P) return 0;
    // src/Model.hpp:189: only a source on its slab's last row (PROC_DIMX-1) emits ...
    int x0, y0, h, w;
    if (mm_partition_reference(H, W, P, owner, &x0, &y0, &h, &w) != MM_OK) return -1;
    if (x - x0 != h - 1) return 0;
    // ... and only with 8 neighbours (:190-216: cases 3 and 5 print a line and do nothing)
    if (mm_neighbor_count(H, W, x, y) != 8) return 0;
    // :202-204 sends the lower row's share to owner+1; without that worker the reference
    // aborts in MPI_Send, so nothing is applied
    if (owner + 1 > P) return 0;
    return 1;
}

int mm_wire_format_partition(char* out, int len, int x_init, int y_init, int height, int width) {
    if (!out || len <= 0) return MM_ERR_INVALID;
    // src/Model.hpp:71-72, src/ModelRectangular.hpp:70-71
    return fit(out, len, std::snprintf(out, (size_t)len, "%d|%d:%d|%d", x_init, y_init, height, width));
}

int mm_wire_format_flow(char* out, int len, int owner, int x, int y, double rate) {
    if (!out || len <= 0) return MM_ERR_INVALID;
    // src/Model.hpp:81, src/ModelRectangular.hpp:87
    return fit(out, len, std::snprintf(out, (size_t)len, "%d|%d:%d|%lf", owner, x, y, rate));
}

int mm_wire_parse_partition(const char* msg, int len, int* x_init, int* y_init, int* height,
                            int* width) {
    if (!msg || len <= 0 || !x_init || !y_init || !height || !width) return MM_ERR_INVALID;
    // src/Model.hpp:139-146: strtok "|", ":", "|", ":" and atoi
    Tokens t(msg, len);
    std::string a, b, c, d;
    if (!t.next("|", a) || !t.next(":", b) || !t.next("|", c) || !t.next(":", d))
        return MM_ERR_INVALID;
    *x_init = std::atoi(a.c_str());
    *y_init = std::atoi(b.c_str());
    *height = std::atoi(c.c_str());
    *width = std::atoi(d.c_str());
    return MM_OK;
}

int mm_wire_parse_flow(const char* msg, int len, int* owner, int* x, int* y, int* rate_atoi,
                       double* rate) {
    if (!msg || len <= 0 || !owner || !x || !y) return MM_ERR_INVALID;
    // src/Model.hpp:160-167: strtok "|:", ":", "|", "|:" and atoi -- the reference reads
    // the rate back as an int (0 for any rate below 1) and never uses it; *rate is the
    // lossless strtod of the same token
    Tokens t(msg, len);
    std::string a, b, c, d;
    if (!t.next("|:", a) || !t.next(":", b) || !t.next("|", c) || !t.next("|:", d))
        return MM_ERR_INVALID;
    *owner = std::atoi(a.c_str());
    *x = std::atoi(b.c_str());
    *y = std::atoi(c.c_str());
    if (rate_atoi) *rate_atoi = std::atoi(d.c_str());
    if (rate) *rate = std::strtod(d.c_str(), nullptr);
    return MM_OK;
}

}  // extern "C"
