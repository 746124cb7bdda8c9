#!/bin/bash
# Pass time per K on the slabs the driver's c3 scaling runs give each GPU (32768 columns,
# 8192 rows at N = 4, 4096 rows at N = 8): is K = 10 as good per step as on the full grid?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-slabk}
mkdir -p $O
C='[{"MM_STEPS_PER_PASS":7},{"MM_STEPS_PER_PASS":8},{"MM_STEPS_PER_PASS":9},{"MM_STEPS_PER_PASS":10},{"MM_STEPS_PER_PASS":6}]'
for R in 8192 4096; do
  timeout -k 10 300 python3 -u tools/sweep.py --rows $R --size 32768 --steps 360 --rounds 3 --configs "$C" > $O/sweep_${R}x32768.log 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_${R}x32768.log; exit 3; }
  echo "== $R x 32768"; cut -c1-230 $O/sweep_${R}x32768.log
done
