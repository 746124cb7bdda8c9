cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
D=gpurun_out/r6e
mkdir -p $D
N=mpi-model_amd/libmpimodel_hip.so
D=$D bash tools/gpu.sh ab k8asc c2 1000 3 "MM_LIB_PATH=$N" "MM_LIB_PATH=abx/k8asc/libmpimodel_hip.so" || exit 3
D=$D bash tools/gpu.sh ab c5ring0 c5 1000 2 "MM_LIB_PATH=$N MM_CHAIN_RING=0" "MM_LIB_PATH=abx/c5ascu2/libmpimodel_hip.so MM_CHAIN_RING=0" || exit 3
