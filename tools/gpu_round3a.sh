# round 3: kernel table per size, then the GPU test suite (wide variants included)
set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 400 python3 -u tools/kernel_table.py > gpurun_out/r3a/kernel_table.log 2>&1 || exit 1
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r3a/pytest_gpu.log 2>&1
echo "pytest rc=$?"
