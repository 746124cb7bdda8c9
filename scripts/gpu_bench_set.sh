#!/bin/bash
# GPU tests, then the driver's bench command and 1000-step c3 / c4 lines (no CPU leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-bset}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { echo "bench failed"; tail $O/bench_driver_cmd.log; exit 3; }
tail -1 $O/bench_driver_cmd.log
for wl in ${WLS:-c3 c4}; do
  timeout -k 10 400 python3 -u bench.py --workload $wl --steps 1000 --warmup 50 --no-cpu-baseline > $O/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail $O/bench_$wl.log; exit 3; }
  python3 -c "import json; d=json.loads(open('$O/bench_$wl.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['config']['rows_per_wave'])"
done
