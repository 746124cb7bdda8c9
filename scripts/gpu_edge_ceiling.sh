#!/bin/bash
# Ceiling of the edge-strip work: every wave on the branch-free body (-DMM_TEST_BODY=1,
# wrong numbers on the grid's edge cells) vs the real kernel, K = 8 and 10.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-edgeceil}
mkdir -p $O
for S in 32768 16384; do for K in 8 10; do
  timeout -k 10 300 python3 -u tools/libsweep.py --size $S --steps $((K*3)) --rounds 3 --env "{\"MM_STEPS_PER_PASS\": $K}" var/*/libmpimodel_hip.so > $O/ls_${S}_k$K.log 2>&1 || { echo "failed"; tail $O/ls_${S}_k$K.log; exit 3; }
  echo "== $S K=$K"; grep variant $O/ls_${S}_k$K.log | cut -c1-200
done; done
