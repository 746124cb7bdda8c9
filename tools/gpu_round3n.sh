# round 3: barrier-group size B for the K = 16 / 20 wide passes (probe, one box), then the
# C5 ring-chain instance: flow-program tests and the c5 bench line.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r3n
mkdir -p $D
for m in 16 164 20 204 16 164 20 204; do timeout -k 10 100 tools/wide8_probe $m 3 >> $D/probe_B.log 2>&1 || { tail $D/probe_B.log; exit 1; }; done
cat $D/probe_B.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "flow_program or chain" > $D/pytest_flow.log 2>&1 \
    || { echo "flow rc=$?"; tail -30 $D/pytest_flow.log; exit 1; }
tail -1 $D/pytest_flow.log
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 > $D/bench_c5.log 2>&1 || { tail -20 $D/bench_c5.log; exit 1; }
tail -1 $D/bench_c5.log | cut -c1-1500
