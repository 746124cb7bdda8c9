#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${SIZES:-4096 16384 32768}; do
  steps=100; [ $n -ge 16384 ] && steps=20; [ $n -ge 32768 ] && steps=8
  timeout -k 10 300 python -u tools/sweep.py --size $n --steps $steps --rounds 2 > gpurun_out/sweep_$n.log 2>&1 || { echo "sweep $n rc=$?"; tail gpurun_out/sweep_$n.log; exit 3; }
  echo "== $n"; head -9 gpurun_out/sweep_$n.log
done
