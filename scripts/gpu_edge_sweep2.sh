#!/bin/bash
# Edge-strip segment length for the K <= 7 passes (20-step runs split 7 + 7 + 6; c2 runs K = 7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-edgesw2}
mkdir -p $O
for S in 16384 4096; do for K in 7 6; do
  C="[{\"MM_STEPS_PER_PASS\":$K},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.3},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.2},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.1}]"
  ST=$((K*12)); [ $S -eq 4096 ] && ST=$((K*60))
  timeout -k 10 300 python3 -u tools/sweep.py --size $S --steps $ST --rounds 3 --configs "$C" > $O/sweep_${S}_k$K.log 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_${S}_k$K.log; exit 3; }
  echo "== $S K=$K"; cut -c1-200 $O/sweep_${S}_k$K.log
done; done
