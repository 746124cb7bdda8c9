#!/bin/bash
# Round-6 evidence on the committed tree, part A (FINAL_PART=a): GPU suite + smoke, every
# bench line with its CPU baseline, C5 with run-time chain operands, the standalone
# 4096 x 32768 slab; part B (FINAL_PART=b): rocprofv3 kernel traces + PMC traffic of each
# line's own plan and length, SQ wave-cycle splits, L2 hit / miss of the K = 20 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6final}
mkdir -p "$D"
if [ "${FINAL_PART:-a}" = a ]; then
    D=$D bash tools/gpu.sh test || exit 3
    D=$D bash tools/gpu.sh lines || exit 3
    MM_CHAIN_RING=0 TAG=runtime_chain D=$D bash tools/gpu.sh bench c5 1000 50 || exit 3
    TAG=4096x32768 D=$D bash tools/gpu.sh bench c3 20 5 --grid 4096 32768 --no-cpu-baseline || exit 3
else
    D=$D bash tools/gpu.sh prof c3_k20 c3 20 5 || exit 3
    D=$D bash tools/gpu.sh prof c4_k20 c4 1000 50 || exit 3
    D=$D bash tools/gpu.sh prof c2_k8 c2 1000 50 || exit 3
    D=$D bash tools/gpu.sh prof c5_k8 c5 1000 50 || exit 3
    D=$D bash tools/gpu.sh sq c3_k20 c3 20 5 || exit 3
    D=$D bash tools/gpu.sh sq c2 c2 1000 50 || exit 3
    D=$D bash tools/gpu.sh sq c5_k8 c5 1000 50 || exit 3
    D=$D bash tools/gpu.sh pmc c3tcc c3 20 5 "TCC_HIT_sum TCC_MISS_sum" || exit 3
fi
