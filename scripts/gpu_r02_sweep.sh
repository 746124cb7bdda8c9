#!/bin/bash
# Round-2 K sweep: GPU tests, then steps-per-pass K = 4..8 at the C2/C4/C3 sizes
# (tools/sweep.py, one process), then prefetch-depth variants at K = 7 / 8 (tools/libsweep.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_all.log; exit 3; }
tail -2 gpurun_out/pytest_all.log
CFG='[{"MM_STEPS_PER_PASS":4},{"MM_STEPS_PER_PASS":5},{"MM_STEPS_PER_PASS":6},{"MM_STEPS_PER_PASS":7},{"MM_STEPS_PER_PASS":8}]'
for n in ${SIZES:-32768 16384 4096}; do
  timeout -k 10 300 python -u tools/sweep.py --size $n --steps 840 --rounds 2 --configs "$CFG" > gpurun_out/sweep_k_$n.log 2>&1 || { echo "sweep $n failed"; tail gpurun_out/sweep_k_$n.log; exit 3; }
  echo "== $n"; cat gpurun_out/sweep_k_$n.log
done
for k in 7 8; do
  timeout -k 10 300 python -u tools/libsweep.py --size 32768 --steps 840 --rounds 2 --env "{\"MM_STEPS_PER_PASS\": \"$k\"}" var/*/libmpimodel_hip.so > gpurun_out/libsweep_u_k$k.log 2>&1 || { echo "libsweep failed"; tail gpurun_out/libsweep_u_k$k.log; exit 3; }
  echo "== K=$k"; grep -A4 summary gpurun_out/libsweep_u_k$k.log
done
