# round 3: warmup scenarios of the 20-step timed run; C5 on the retuned multi-attribute
# instances; the halo + flow-program GPU tests.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3g}
mkdir -p $D
timeout -k 10 200 python3 -u tools/timed_gap2.py > $D/timed_gap2.log 2>&1 || { tail -20 $D/timed_gap2.log; exit 1; }
cat $D/timed_gap2.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "flow_program or chain" > $D/pytest_flow.log 2>&1 \
    || { echo "flow rc=$?"; tail -40 $D/pytest_flow.log; exit 1; }
tail -2 $D/pytest_flow.log
for k in 8 4; do
MM_STEPS_PER_PASS=$k timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 --no-cpu-baseline \
    > $D/bench_c5_k$k.log 2>&1 || { tail -20 $D/bench_c5_k$k.log; exit 1; }
tail -1 $D/bench_c5_k$k.log | cut -c1-900
done
