#!/bin/bash
# Round-6 tuning A/B: C2 with 4-row barrier groups (abx/k8b4, abx/k8b4u4) against the tree;
# the 4096 x 32768 split slab's segment plan (waves per slot, K) on the box-sum kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6k}
mkdir -p "$D"
N=mpi-model_amd/libmpimodel_hip.so
D=$D bash tools/gpu.sh ab k8b4 c2 1000 3 "MM_LIB_PATH=$N" "MM_LIB_PATH=abx/k8b4/libmpimodel_hip.so" || exit 3
D=$D bash tools/gpu.sh ab k8b4u4 c2 1000 2 "MM_LIB_PATH=$N" "MM_LIB_PATH=abx/k8b4u4/libmpimodel_hip.so" || exit 3
THIN_STEPS=200 THIN_SW="2 3 4" THIN_K="16" D=$D bash tools/gpu.sh thin || exit 3
