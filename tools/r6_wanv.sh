#!/bin/bash
# C5 with run-time chain operands: chain_asm without `volatile` (abx/wanv) against the tree;
# then a HIP-runtime trace of a 20-step split pass after priming (8192 x 32768 self-halo).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6l}
mkdir -p "$D"
N=mpi-model_amd/libmpimodel_hip.so
D=$D bash tools/gpu.sh ab wanv c5 1000 2 "MM_LIB_PATH=$N MM_CHAIN_RING=0" "MM_LIB_PATH=abx/wanv/libmpimodel_hip.so MM_CHAIN_RING=0" || exit 3
D=$D bash tools/r6_trace20.sh || exit 3
