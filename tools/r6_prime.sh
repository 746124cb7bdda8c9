#!/bin/bash
# Priming check: the tests that call mm_prepare, a HIP-runtime trace of the driver's command
# (launch-to-start latency of the first timed K = 20 dispatch), the driver's command 3 times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6g}
mkdir -p "$D"
timeout -k 10 600 python3 -u -m pytest $(grep -l "prepare" tests/test_gpu*.py) -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$D/pytest_prepare.log" 2>&1 || { tail -30 "$D/pytest_prepare.log"; exit 3; }
tail -2 "$D/pytest_prepare.log"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$D/hiptrace" -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$D/hiptrace.log" 2>&1 || exit 3
python3 tools/launch_latency.py "$D/hiptrace" > "$D/launch_latency.txt" 2>&1; cat "$D/launch_latency.txt"
for r in 0 1 2; do
    TAG=rep$r D=$D bash tools/gpu.sh bench c3 20 5 --no-cpu-baseline | cut -c1-140 || exit 3
done
