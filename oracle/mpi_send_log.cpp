/*
 * TEST INFRASTRUCTURE ONLY. Never linked into the product.
 *
 * MPI_Send interposer (MPI profiling interface): linked into a test executable, it logs
 * every message to stderr and passes it on to PMPI_Send. Used to record the reference's
 * traffic (oracle/ref_wire_harness.cpp -> tests/golden/wire_*.json) and to compare the
 * drop-in driver's control messages with it (oracle/_build/dropin_wire_main, the drop-in
 * example program examples/drop_in_main.cpp linked with this file).
 * Log line: MPISEND src=<rank> dest=<d> tag=<t> type=<char|int|double|other> count=<n>
 *           data=<chars up to the first NUL | values>
 */
#include <mpi.h>

#include <cstdio>
#include <string>

extern "C" int MPI_Send(const void* buf, int count, MPI_Datatype dt, int dest, int tag,
                        MPI_Comm comm) {
    int rank = -1;
    PMPI_Comm_rank(MPI_COMM_WORLD, &rank);
    std::string data;
    const char* type = "other";
    char tmp[64];
    if (dt == MPI_CHAR) {
        type = "char";
        const char* c = static_cast<const char*>(buf);
        for (int i = 0; i < count && c[i]; ++i) {
            const unsigned char u = (unsigned char)c[i];
            if (u >= 32 && u < 127 && u != '\\') {
                data += c[i];
            } else {
                std::snprintf(tmp, sizeof tmp, "\\x%02x", u);
                data += tmp;
            }
        }
    } else if (dt == MPI_INT) {
        type = "int";
        for (int i = 0; i < count; ++i) {
            std::snprintf(tmp, sizeof tmp, "%s%d", i ? "," : "", static_cast<const int*>(buf)[i]);
            data += tmp;
        }
    } else if (dt == MPI_DOUBLE) {
        type = "double";
        for (int i = 0; i < count; ++i) {
            std::snprintf(tmp, sizeof tmp, "%s%a", i ? "," : "", static_cast<const double*>(buf)[i]);
            data += tmp;
        }
    }
    std::fprintf(stderr, "MPISEND src=%d dest=%d tag=%d type=%s count=%d data=%s\n", rank, dest,
                 tag, type, count, data.c_str());
    std::fflush(stderr);
    return PMPI_Send(buf, count, dt, dest, tag, comm);
}

