#!/bin/bash
# HIP-runtime + kernel trace of a 20-step split-schedule run (self-halo) on one slab shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6i}
mkdir -p "$D"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$D/hiptrace" -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --grid 8192 32768 --self-halo > "$D/hiptrace.log" 2>&1 || exit 3
python3 tools/launch_latency.py "$D/hiptrace" > "$D/launch_latency.txt" 2>&1; cat "$D/launch_latency.txt"
grep '^{' "$D/hiptrace.log" | cut -c1-120
