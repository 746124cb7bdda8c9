// Defines.hpp -- compile-time geometry of the drop-in API (reference: src/Defines.hpp:5-13).
// Same macro names and meanings; unlike the reference every value can be overridden
// with -D (the reference has no #ifndef guards). PROC_DIMX keeps the reference's
// unparenthesised expansion, which user code may rely on.
#ifndef DEFINES_HPP
#define DEFINES_HPP

#ifndef DIMX
#define DIMX 100
#endif
#ifndef DIMY
#define DIMY 100
#endif
#ifndef NWORKERS
#define NWORKERS 5
#endif
#ifndef PROC_DIMX
#define PROC_DIMX DIMX/NWORKERS
#endif
#ifndef PROC_DIMY
#define PROC_DIMY DIMY
#endif
#define MASTER 0
#define FROM_MASTER 0
#define FROM_WORKER 1
#define NEIGHBORS 8

#endif
