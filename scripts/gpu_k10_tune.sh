#!/bin/bash
# K = 10 (the driver's 20-step passes) tuning at 32768^2: prefetched rows (var/k10u*) and
# segment waves per slot (MM_SEG_WAVES), bit-exact checked.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-k10tune}
mkdir -p $O
timeout -k 10 400 python3 -u tools/libsweep.py --size 32768 --steps 30 --rounds 3 --env '{"MM_STEPS_PER_PASS": 10}' var/*/libmpimodel_hip.so > $O/libsweep_k10_u.log 2>&1 || { echo "libsweep failed"; tail $O/libsweep_k10_u.log; exit 3; }
grep variant $O/libsweep_k10_u.log
C='[{"MM_STEPS_PER_PASS":10},{"MM_STEPS_PER_PASS":10,"MM_SEG_WAVES":2},{"MM_STEPS_PER_PASS":10,"MM_SEG_WAVES":3},{"MM_STEPS_PER_PASS":10,"MM_SEG_WAVES":6},{"MM_STEPS_PER_PASS":10,"MM_SEG_EDGE":0.15}]'
timeout -k 10 300 python3 -u tools/sweep.py --size 32768 --steps 360 --rounds 3 --configs "$C" > $O/sweep_k10.log 2>&1 || { echo "sweep failed"; tail $O/sweep_k10.log; exit 3; }
cut -c1-230 $O/sweep_k10.log
