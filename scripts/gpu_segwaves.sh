#!/bin/bash
# Segment waves per resident wave slot (MM_SEG_WAVES) for the K the engine uses on the
# bench grids: K = 6, 7, 8 at 32768^2 and 16384^2, K = 7 at 4096^2 (tools/sweep.py,
# bit-exact across configurations of one K).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-segw}
mkdir -p $O
for N in 32768 16384; do
  for K in 8 7 6; do
    C="[{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_WAVES\":2},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_WAVES\":2.5},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_WAVES\":3},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_WAVES\":4},{\"MM_STEPS_PER_PASS\":$K,\"MM_SEG_WAVES\":6}]"
    timeout -k 10 300 python3 -u tools/sweep.py --size $N --steps $((K*6)) --rounds 3 --configs "$C" > $O/sweep_${N}_k$K.log 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_${N}_k$K.log; exit 3; }
    echo "== $N K=$K"; cut -c1-220 $O/sweep_${N}_k$K.log
  done
done
C='[{"MM_STEPS_PER_PASS":7,"MM_SEG_WAVES":2},{"MM_STEPS_PER_PASS":7,"MM_SEG_WAVES":3},{"MM_STEPS_PER_PASS":7,"MM_SEG_WAVES":4},{"MM_STEPS_PER_PASS":7,"MM_SEG_WAVES":1.5}]'
timeout -k 10 300 python3 -u tools/sweep.py --size 4096 --steps 210 --rounds 3 --configs "$C" > $O/sweep_4096_k7.log 2>&1 || { echo "sweep failed"; exit 3; }
echo "== 4096 K=7"; cut -c1-220 $O/sweep_4096_k7.log
# C5 (4 attributes): K = 2 vs K = 1 passes and the segment plan size
for E in '{}' '{"MM_STEPS_PER_PASS":1}' '{"MM_SEG_WAVES":1}' '{"MM_SEG_WAVES":4}' '{"MM_STEPS_PER_PASS":1,"MM_SEG_WAVES":1}' '{"MM_STEPS_PER_PASS":1,"MM_SEG_WAVES":4}'; do
  timeout -k 10 200 python3 -u tools/libsweep.py --program c5 --size 4096 --steps 8 --rounds 3 --env "$E" mpi-model_amd/libmpimodel_hip.so > $O/c5.tmp 2>&1 || { echo "c5 sweep failed"; tail $O/c5.tmp; exit 3; }
  echo "$E $(grep variant $O/c5.tmp)" | tee -a $O/c5_sweep.log
done
