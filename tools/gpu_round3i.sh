set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r3i
mkdir -p $D
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_halo.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "deep_halo_chain_bit_exact" > $D/halo_alone.log 2>&1; echo "alone rc=$?"; tail -3 $D/halo_alone.log
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_halo.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "flow_program_wide_kernel or deep_halo_chain_bit_exact" > $D/halo_after_wide.log 2>&1; echo "after rc=$?"; tail -3 $D/halo_after_wide.log
for k in 4 8; do
MM_STEPS_PER_PASS=$k timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 --no-cpu-baseline \
    > $D/bench_c5_k$k.log 2>&1 || { tail -20 $D/bench_c5_k$k.log; exit 1; }
tail -1 $D/bench_c5_k$k.log | cut -c1-1200
done
timeout -k 10 200 python3 -u tools/timed_gap2.py > $D/timed_gap2.log 2>&1 || { tail -20 $D/timed_gap2.log; exit 1; }
cat $D/timed_gap2.log
