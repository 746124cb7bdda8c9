# round 3: rest of the GPU suite (from test_gpu_parity), C5 benches, driver command.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3k}
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu_parity.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu_parity.log; exit 1; }
tail -2 $D/pytest_gpu_parity.log
for k in 4 8; do
MM_STEPS_PER_PASS=$k timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 --no-cpu-baseline \
    > $D/bench_c5_k$k.log 2>&1 || { tail -20 $D/bench_c5_k$k.log; exit 1; }
tail -1 $D/bench_c5_k$k.log | cut -c1-1200
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
