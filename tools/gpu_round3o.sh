# round 3: parity after removing the branch-chain path (XCD-chunk block orders included),
# then the whole GPU suite. Every GPU step has its own time limit; a failure ends it.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3o}
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
