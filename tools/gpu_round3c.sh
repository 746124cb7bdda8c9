# round 3 (re-entry): GPU suite, the driver bench command, a long run, rocprof of the
# driver command's kernels. Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3c}
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
timeout -k 10 300 python3 -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline > $D/bench_c3_1000.log 2>&1 || { tail -20 $D/bench_c3_1000.log; exit 1; }
tail -1 $D/bench_c3_1000.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_c3_driver -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/prof_c3_driver.log 2>&1 || { echo "prof rc=$?"; tail -20 $D/prof_c3_driver.log; exit 1; }
echo prof ok
