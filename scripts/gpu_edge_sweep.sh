#!/bin/bash
# Edge-strip segment length (MM_SEG_EDGE) at 16384^2 and 32768^2, K = 8 and 10.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-edgesw}
mkdir -p $O
for S in 16384 32768; do for K in 8 10; do
  C="[{\"MM_STEPS_PER_PASS\":$K},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.5},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.3},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.2},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.1},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.05}]"
  timeout -k 10 300 python3 -u tools/sweep.py --size $S --steps $((K*12)) --rounds 3 --configs "$C" > $O/sweep_${S}_k$K.log 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_${S}_k$K.log; exit 3; }
  echo "== $S K=$K"; cut -c1-200 $O/sweep_${S}_k$K.log
done; done
