#!/bin/bash
# C5 tuning variants of the K = 2 unit (tools/build_variants.sh): chain capacity,
# prefetched rows, occupancy; bit-exact checked (tools/libsweep.py --program c5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-c5var}
mkdir -p $O
timeout -k 10 400 python3 -u tools/libsweep.py --program c5 --size 4096 --steps 8 --rounds 3 var/*/libmpimodel_hip.so > $O/c5_var.log 2>&1 || { echo "c5 sweep failed"; tail $O/c5_var.log; exit 3; }
grep variant $O/c5_var.log
