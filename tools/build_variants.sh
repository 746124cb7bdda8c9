#!/bin/bash
# Build tuning variants of libmpimodel_hip.so that differ only in the compile-time
# flags of the K-step kernel units (UNITS, default mm_passk_k4). Each variant lands in
# $OUT/<name>/libmpimodel_hip.so (OUT default var, which stays on this machine; OUT=abx
# travels to the GPU box for A/B runs through MM_LIB_PATH) with its kernel resource usage
# (VGPRs, SGPRs, occupancy) next to it. Usage:
#   tools/build_variants.sh "w1u8:-DMM_PASSK_MIN_WAVES=1 -DMM_SEG_U1=8" "w3u6:..." ...
# The other objects come from the regular build (make -C mpi-model_amd first).
set -e
cd "$(dirname "$0")/../mpi-model_amd"
ROCM=${ROCM:-/opt/rocm}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -mllvm -pragma-unroll-threshold=200000 -I$ROCM/include -I../include"
UNITS=${UNITS:-"mm_passk_k4"}
build_one() {
  local name=${1%%:*} extra=${1#*:}
  local out=../${OUT:-var}/$name
  mkdir -p "$out"
  local objs=""
  for o in build/*.o; do
    local b=$(basename "$o" .o)
    if [[ " $UNITS " == *" $b "* ]]; then
      $ROCM/bin/hipcc $FLAGS $extra -c csrc/$b.hip -o $out/$b.o \
        -Rpass-analysis=kernel-resource-usage 2> $out/$b.res
      objs="$objs $out/$b.o"
    else
      objs="$objs $o"
    fi
  done
  $ROCM/bin/hipcc --offload-arch=gfx950 $objs -shared -L$ROCM/lib -Wl,-rpath,$ROCM/lib -Wl,-z,now -lrccl -o $out/libmpimodel_hip.so
  echo "$extra" > $out/flags.txt
  for u in $UNITS; do
    python3 ../tools/res_summary.py $out/$u.res > $out/$u.res.txt
  done
  echo "built $name ($extra)"
}
for v in "$@"; do build_one "$v" & done
wait
