/*
 * TEST INFRASTRUCTURE ONLY (oracle pinning). Never linked into the product.
 *
 * Pre-included (g++ -include) ahead of the reference headers, like ref_defines.h: takes
 * the reference's own include guard (DEFINESRECTANGULAR_HPP,
 * /root/reference/src/DefinesRectangular.hpp:2-3) and replaces its hard-coded 2-D block
 * geometry (DefinesRectangular.hpp:5-11) with values from the command line. The macro
 * spellings mirror the reference, unparenthesised divisions included
 * (ModelRectangular.hpp:71,74,77 expand them).
 *
 * Usage: g++ -include oracle/ref_defines_rect.h -DREF_DIMX_REC=20 -DREF_DIMY_REC=60 \
 *            -DREF_LINES_REC=2 -DREF_COLUMNS_REC=3 ...
 */
#ifndef DEFINESRECTANGULAR_HPP
#define DEFINESRECTANGULAR_HPP

#ifndef REF_DIMX_REC
#define REF_DIMX_REC 20
#endif
#ifndef REF_DIMY_REC
#define REF_DIMY_REC 60
#endif
#ifndef REF_LINES_REC
#define REF_LINES_REC 2
#endif
#ifndef REF_COLUMNS_REC
#define REF_COLUMNS_REC 3
#endif

#define DIMX_REC REF_DIMX_REC
#define DIMY_REC REF_DIMY_REC
#define LINES_REC REF_LINES_REC
#define COLUMNS_REC REF_COLUMNS_REC
#define NWORKERS_REC LINES_REC*COLUMNS_REC
#define PROC_DIMX_REC DIMX_REC/LINES_REC
#define PROC_DIMY_REC DIMY_REC/COLUMNS_REC

#endif
