# round 3: 8-column wide instances vs the 4-column ones (kernel table), then the GPU suite
# and the driver bench command. Every GPU step has its own time limit; a failure ends it.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3d}
mkdir -p $D
timeout -k 10 300 python3 -u tools/kernel_table.py --sizes 32768x32768 --old 8 --wide 16,20 \
    --wide8 8,12,16 > $D/kernel_table_32768.log 2>&1 || { tail -20 $D/kernel_table_32768.log; exit 1; }
cat $D/kernel_table_32768.log
timeout -k 10 300 python3 -u tools/kernel_table.py --sizes 16384x16384,4096x4096 --old 7,8 \
    --wide 16 --wide8 8,12,16 > $D/kernel_table_small.log 2>&1 || { tail -20 $D/kernel_table_small.log; exit 1; }
cat $D/kernel_table_small.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
