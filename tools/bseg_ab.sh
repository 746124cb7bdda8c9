#!/bin/bash
# Wide split passes, full-length border segments (default) against K-row border segments
# (MM_BORDER_SEGMENTS=0): 20-step self-halo lines on every scaling slab, A B A B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
D=${D:-gpurun_out/r6r}
mkdir -p $D
for g in "32768 32768" "16384 32768" "8192 32768" "4096 32768" "16384 16384"; do
  set -- $g
  for r in 0 1 2; do
    for b in 0 1; do
      v=$(MM_BORDER_SEGMENTS=$b TAG="${1}x${2}_b${b}_$r" D=$D bash tools/gpu.sh bench c3 20 5 --grid $1 $2 --no-cpu-baseline --self-halo | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])") || exit 3
      echo "$1x$2 steps=20 border_segments=$b rep=$r $v"
    done
  done
done
