#!/bin/bash
# Round-2 evidence run on one MI355X: GPU tests, the bench lines (c3 = the driver's default,
# then c2/c4/c5), rocprofv3 kernel trace + FETCH/WRITE per workload, SQ split for c3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r02/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/r02/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/r02/smoke.log; exit 3; }
cat gpurun_out/r02/smoke.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r02/bench_driver_cmd.log 2>&1 || { echo "bench failed"; tail gpurun_out/r02/bench_driver_cmd.log; exit 3; }
for wl in c3 c2 c4 c5; do
  timeout -k 10 400 python3 -u bench.py --workload $wl --steps 1000 --warmup 50 > gpurun_out/r02/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail gpurun_out/r02/bench_$wl.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r02/bench_$wl.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], d['cpu_baseline']['value'])"
done
for wl in c3 c4 c2 c5; do
  OUT=gpurun_out/r02/prof_$wl WL=$wl bash scripts/gpu_profile.sh > gpurun_out/r02/prof_$wl.log 2>&1 || { echo "profile $wl failed"; tail -30 gpurun_out/r02/prof_$wl.log; exit 3; }
  grep -h '"avg_us"\|hbm_bytes_per_launch' gpurun_out/r02/prof_$wl/summary.json
done
OUT=gpurun_out/r02/pmc_sq_c3 WL=c3 bash scripts/gpu_pmc_sq.sh > gpurun_out/r02/pmc_sq_c3.log 2>&1 || { echo "pmc sq failed"; tail -20 gpurun_out/r02/pmc_sq_c3.log; exit 3; }
grep -h 'frac_\|clock' gpurun_out/r02/pmc_sq_c3/summary.json
