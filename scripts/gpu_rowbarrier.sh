#!/bin/bash
# Steady-loop scheduling barrier every 1 / 2 rows / none (var/rb*), K = 8 and 10, 32768^2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-rowbar}
mkdir -p $O
for K in 10 8; do
  timeout -k 10 300 python3 -u tools/libsweep.py --size 32768 --steps $((K*4)) --rounds 3 --env "{\"MM_STEPS_PER_PASS\": $K}" var/*/libmpimodel_hip.so > $O/ls_k$K.log 2>&1 || { echo "failed"; tail $O/ls_k$K.log; exit 3; }
  echo "== K=$K"; grep variant $O/ls_k$K.log | cut -c1-200
done
