#!/bin/bash
# SQ wave-cycle split of the K = 8 pass (32-step run: 4 x 8) and the K = 10 pass (the
# driver's 20-step run: 10 + 10), c3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-sq}
PSTEPS=32 OUT=$O/pmc_sq_c3_k8 WL=c3 bash scripts/gpu_pmc_sq.sh > $O.k8.log 2>&1 || { echo "sq k8 failed"; tail -20 $O.k8.log; exit 3; }
cat $O/pmc_sq_c3_k8/summary.json
PSTEPS=20 OUT=$O/pmc_sq_c3_k10 WL=c3 bash scripts/gpu_pmc_sq.sh > $O.k10.log 2>&1 || { echo "sq k10 failed"; tail -20 $O.k10.log; exit 3; }
cat $O/pmc_sq_c3_k10/summary.json
