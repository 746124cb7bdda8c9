#!/bin/bash
# C5 (4 attributes, chained transfers): the select-based chain (in-tree library) vs the
# vector-indexed chain (var/chainv8), K = 2 and K = 1 passes, bit-exact checked.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c5chain}
mkdir -p $O
for E in '{}' '{"MM_STEPS_PER_PASS":1}'; do
  timeout -k 10 300 python3 -u tools/libsweep.py --program c5 --size 4096 --steps 8 --rounds 3 --env "$E" mpi-model_amd/libmpimodel_hip.so var/chainv8/libmpimodel_hip.so > $O/c5.tmp 2>&1 || { echo "c5 sweep failed"; tail $O/c5.tmp; exit 3; }
  echo "$E"; grep variant $O/c5.tmp | tee -a $O/c5_chain.log
done
