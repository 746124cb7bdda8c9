#!/bin/bash
# Split passes with the interior launched ahead of the exchange: the halo / split / bench
# GPU tests, then every scaling slab plain and split at the driver's 20 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6m}
mkdir -p "$D"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_halo.py tests/test_gpu_fullsize.py tests/test_bench_multi.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > "$D/pytest_split.log" 2>&1 || { tail -30 "$D/pytest_split.log"; exit 3; }
tail -1 "$D/pytest_split.log"
for g in "32768 32768" "16384 32768" "8192 32768" "4096 32768" "16384 16384"; do
    set -- $g
    TAG="${1}x${2}_plain" D=$D bash tools/gpu.sh bench c3 20 5 --grid $1 $2 --no-cpu-baseline | cut -c1-100 || exit 3
    TAG="${1}x${2}_self" D=$D bash tools/gpu.sh bench c3 20 5 --grid $1 $2 --no-cpu-baseline --self-halo | cut -c1-100 || exit 3
done
