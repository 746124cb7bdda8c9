#!/bin/bash
# Round-6 working call: padding tests, GPU suite, a HIP-runtime trace of the driver's
# command, and the K = 8 variant A/B (tools/build_variants.sh OUT=abx). Every GPU step
# runs under its own limit; a failing test run ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6c}
mkdir -p "$D"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_padding.py -x -q --timeout 120 \
    --timeout-method thread > "$D/pytest_padding.log" 2>&1 || { tail -30 "$D/pytest_padding.log"; exit 3; }
tail -2 "$D/pytest_padding.log"
D=$D bash tools/gpu.sh test || exit 3
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$D/hiptrace" -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$D/hiptrace.log" 2>&1 || exit 3
B=mpi-model_amd/libmpimodel_hip.so
D=$D bash tools/gpu.sh ab k8asc c2 1000 4 "MM_LIB_PATH=$B" "MM_LIB_PATH=abx/k8asc/libmpimodel_hip.so"
D=$D bash tools/gpu.sh ab k8asc4 c2 1000 4 "MM_LIB_PATH=$B" "MM_LIB_PATH=abx/k8asc4/libmpimodel_hip.so"
