// DefinesRectangular.hpp -- 2-D block geometry (reference: src/DefinesRectangular.hpp:5-11).
#ifndef DEFINESRECTANGULAR_HPP
#define DEFINESRECTANGULAR_HPP

#ifndef DIMX_REC
#define DIMX_REC 20
#endif
#ifndef DIMY_REC
#define DIMY_REC 60
#endif
#ifndef LINES_REC
#define LINES_REC 2
#endif
#ifndef COLUMNS_REC
#define COLUMNS_REC 3
#endif
#define NWORKERS_REC LINES_REC*COLUMNS_REC
#define PROC_DIMX_REC DIMX_REC/LINES_REC
#define PROC_DIMY_REC DIMY_REC/COLUMNS_REC

#endif
