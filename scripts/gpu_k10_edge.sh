#!/bin/bash
# K = 9 / 10 passes with shorter edge-strip segments (MM_SEG_EDGE): is the slow general
# body of the two edge strips what holds the deep passes back? 32768^2, tools/sweep.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-k10e}
mkdir -p $O
for K in 10 9; do
  C="[{\"MM_STEPS_PER_PASS\":8},{\"MM_STEPS_PER_PASS\":$K},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.2},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.1},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.05},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_EDGE\":0.02}]"
  timeout -k 10 300 python3 -u tools/sweep.py --size 32768 --steps 360 --rounds 2 --configs "$C" > $O/sweep_32768_k$K.log 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_32768_k$K.log; exit 3; }
  echo "== K=$K"; cut -c1-230 $O/sweep_32768_k$K.log
done
