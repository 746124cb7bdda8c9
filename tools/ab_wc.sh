# The K = 20 instance with two column waves per level group (MM_WIDE_WC=2, a variant
# library from tools/build_variants.sh under varx/) against the default: parity of the
# variant (every K-step test, the driver configuration at full size), then interleaved
# c3 lines (the driver's 20 steps, and 200).
export D=${D:-gpurun_out/wc}
mkdir -p $D
V=$PWD/varx/k20wc2/libmpimodel_hip.so
MM_LIB_PATH=$V timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -x -q -m gpu \
  -k "fused_steps or driver_config or c4_production or rccl_halo or planner" --timeout 300 --timeout-method thread \
  > $D/pytest_wc2.log 2>&1 || { tail -40 $D/pytest_wc2.log; exit 3; }
tail -2 $D/pytest_wc2.log
for rep in 1 2; do
  TAG=base_$rep bash tools/gpu.sh bench c3 20 5 --no-cpu-baseline || exit 3
  MM_LIB_PATH=$V TAG=wc2_$rep bash tools/gpu.sh bench c3 20 5 --no-cpu-baseline || exit 3
  TAG=base_$rep bash tools/gpu.sh bench c3 200 5 --no-cpu-baseline || exit 3
  MM_LIB_PATH=$V TAG=wc2_$rep bash tools/gpu.sh bench c3 200 5 --no-cpu-baseline || exit 3
done
