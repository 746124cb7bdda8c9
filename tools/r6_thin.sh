#!/bin/bash
# Thin slabs and the split schedule on the box-sum kernels: bench.py --self-halo beside the
# plain run on every scaling slab (20 and 200 steps), then kernel traces of the thin split
# slabs decomposed per pass (tools/thin_trace.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6h}
mkdir -p "$D"
D=$D bash tools/gpu.sh selfhalo || exit 3
D=$D bash tools/gpu.sh thintrace || exit 3
