# round 3: GPU suite, driver bench command, kernel table with the wide segment plan
set -o pipefail
D=gpurun_out/r3b
mkdir -p $D
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -3 $D/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || exit 1
tail -1 $D/bench_driver_cmd.log
timeout -k 10 300 python3 -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline > $D/bench_c3_1000.log 2>&1 || exit 1
tail -1 $D/bench_c3_1000.log
timeout -k 10 400 python3 -u tools/kernel_table.py --old 8 --wide 8,12,16,20 > $D/kernel_table.log 2>&1 || exit 1
cat $D/kernel_table.log
