set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r3h
mkdir -p $D
timeout -k 10 120 python3 -u tools/dbg_chain.py > $D/dbg_chain.log 2>&1 || { tail -20 $D/dbg_chain.log; exit 1; }
cat $D/dbg_chain.log
for k in 4 8; do
MM_STEPS_PER_PASS=$k timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 --no-cpu-baseline \
    > $D/bench_c5_k$k.log 2>&1 || { tail -20 $D/bench_c5_k$k.log; exit 1; }
tail -1 $D/bench_c5_k$k.log | cut -c1-1200
done
timeout -k 10 200 python3 -u tools/timed_gap2.py > $D/timed_gap2.log 2>&1 || { tail -20 $D/timed_gap2.log; exit 1; }
cat $D/timed_gap2.log
