#!/bin/bash
# The split schedule's price at the driver's 20 steps after priming both streams: every
# scaling slab plain and self-halo, then the driver's command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6j}
mkdir -p "$D"
for g in "32768 32768" "16384 32768" "8192 32768" "4096 32768" "16384 16384"; do
    set -- $g
    TAG="${1}x${2}_plain" D=$D bash tools/gpu.sh bench c3 20 5 --grid $1 $2 --no-cpu-baseline | cut -c1-110 || exit 3
    TAG="${1}x${2}_self" D=$D bash tools/gpu.sh bench c3 20 5 --grid $1 $2 --no-cpu-baseline --self-halo | cut -c1-110 || exit 3
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "prepare or graph" > "$D/pytest_prepare.log" 2>&1 || { tail -30 "$D/pytest_prepare.log"; exit 3; }
tail -1 "$D/pytest_prepare.log"
