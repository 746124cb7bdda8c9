#!/bin/bash
# Round-6 working call: the GPU suite on the box-sum step (ascending-level K = 8 and
# four-attribute instances, primed kernels), the bench lines (+ C5 with the run-time-operand
# chain), a HIP-runtime trace of the driver's command, and the A/B of the driver's command
# against the round-5 library (abx/base). Every GPU step runs under its own limit; a failing
# step ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6f}
mkdir -p "$D"
D=$D bash tools/gpu.sh test || exit 3
D=$D bash tools/gpu.sh lines || exit 3
MM_CHAIN_RING=0 TAG=runtime_chain D=$D bash tools/gpu.sh bench c5 1000 50 --no-cpu-baseline || exit 3
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$D/hiptrace" -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$D/hiptrace.log" 2>&1 || exit 3
python3 tools/launch_latency.py "$D/hiptrace" > "$D/launch_latency.txt" 2>&1; cat "$D/launch_latency.txt"
B=abx/base/libmpimodel_hip.so
N=mpi-model_amd/libmpimodel_hip.so
D=$D bash tools/gpu.sh ab c3_20 c3 20 3 "MM_LIB_PATH=$B" "MM_LIB_PATH=$N" || exit 3
