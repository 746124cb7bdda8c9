# round 3: four-attribute programs on the level-split kernel (C5), then the whole GPU suite
# and the driver bench command (warmup now right before the timed region).
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3f}
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "flow_program" > $D/pytest_flow.log 2>&1 \
    || { echo "flow rc=$?"; tail -40 $D/pytest_flow.log; exit 1; }
tail -2 $D/pytest_flow.log
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 --no-cpu-baseline \
    > $D/bench_c5.log 2>&1 || { tail -20 $D/bench_c5.log; exit 1; }
tail -1 $D/bench_c5.log
MM_WIDE=0 timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 \
    --no-cpu-baseline > $D/bench_c5_passk.log 2>&1 || { tail -20 $D/bench_c5_passk.log; exit 1; }
tail -1 $D/bench_c5_passk.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
