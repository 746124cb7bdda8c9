# round 3: GPU suite, smoke, the driver command and every workload's bench line.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3l}
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
for wl in c3 c4 c2 c5; do
timeout -k 10 300 python3 -u bench.py --workload $wl --steps 1000 --warmup 20 > $D/bench_${wl}_1000.log 2>&1 || { tail -20 $D/bench_${wl}_1000.log; exit 1; }
tail -1 $D/bench_${wl}_1000.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('valu',{}).get('frac'), d['config']['path'], d.get('cpu_baseline',{}).get('value'))"
done
