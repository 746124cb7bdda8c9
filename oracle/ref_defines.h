/*
 * TEST INFRASTRUCTURE ONLY (oracle pinning). Never linked into the product.
 *
 * Pre-included (g++ -include) ahead of the reference headers so that the
 * reference's own include guard (DEFINES_HPP, /root/reference/src/Defines.hpp:2-3)
 * is already taken and its hard-coded geometry (Defines.hpp:5-13) is replaced
 * by the values given on the command line. The macro spellings below mirror
 * the reference exactly, including the unparenthesised PROC_DIMX, because the
 * reference's arithmetic depends on that expansion (Model.hpp:189,252).
 *
 * Usage: g++ -include oracle/ref_defines.h -DREF_DIMX=40 -DREF_DIMY=64 -DREF_NWORKERS=4 ...
 */
#ifndef DEFINES_HPP
#define DEFINES_HPP

#ifndef REF_DIMX
#define REF_DIMX 100
#endif
#ifndef REF_DIMY
#define REF_DIMY 100
#endif
#ifndef REF_NWORKERS
#define REF_NWORKERS 5
#endif

#define DIMX REF_DIMX
#define DIMY REF_DIMY
#define NWORKERS REF_NWORKERS
#define PROC_DIMX DIMX/NWORKERS
#define PROC_DIMY DIMY
#define MASTER 0
#define FROM_MASTER 0
#define FROM_WORKER 1
#define NEIGHBORS 8

#endif
