# round 3: small slabs (< 2^25 cells) on mm_wide_kernel K = 8 by default -- the whole GPU
# suite, then C2 at 1000 steps and the driver command.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3p}
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 200 python3 -u bench.py --workload c2 --steps 1000 --warmup 20 > $D/bench_c2.log 2>&1 || { tail -20 $D/bench_c2.log; exit 1; }
tail -1 $D/bench_c2.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
