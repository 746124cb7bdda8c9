#!/bin/bash
# Kernel tuning sweeps (tools/sweep.py) at the bench grid sizes, each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${SIZES:-4096 16384 32768}; do
  steps=96; [ $n -ge 16384 ] && steps=24; [ $n -ge 32768 ] && steps=12
  timeout -k 10 400 python -u tools/sweep.py --size $n --steps $steps --rounds ${ROUNDS:-2} --preset ${PRESET:-seg} > gpurun_out/sweep_$n.log 2>&1 || { echo "sweep $n rc=$?"; tail gpurun_out/sweep_$n.log; exit 3; }
  echo "== $n"; head -${TOP:-12} gpurun_out/sweep_$n.log
done
