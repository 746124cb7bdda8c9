#!/bin/bash
# Round-2 closing evidence on the committed tree: GPU tests, smoke, the driver's bench
# command, 1000-step lines for c3 / c4 / c2 / c5, rocprofv3 trace + FETCH/WRITE for the c3
# K = 10 pass (the driver's 20-step run) and the K = 8 pass (long runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r02end}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 3; }
cat $O/smoke.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { echo "bench failed"; tail $O/bench_driver_cmd.log; exit 3; }
tail -1 $O/bench_driver_cmd.log
for wl in c3 c4 c2 c5; do
  timeout -k 10 400 python3 -u bench.py --workload $wl --steps 1000 --warmup 50 > $O/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail $O/bench_$wl.log; exit 3; }
  python3 -c "import json; d=json.loads(open('$O/bench_$wl.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], r['kernel_avg_us'], r['frac'], r.get('valu', {}).get('frac'), d['cpu_baseline']['value'], d['config']['path'])"
done
PSTEPS=20 PMCSTEPS=20 OUT=$O/prof_c3_k10 WL=c3 bash scripts/gpu_profile.sh > $O/prof_c3_k10.log 2>&1 || { echo "profile k10 failed"; tail -30 $O/prof_c3_k10.log; exit 3; }
grep -h '"kernel_name"\|"avg_us"\|hbm_bytes_per_launch' $O/prof_c3_k10/summary.json
OUT=$O/prof_c3_k8 WL=c3 bash scripts/gpu_profile.sh > $O/prof_c3_k8.log 2>&1 || { echo "profile k8 failed"; tail -30 $O/prof_c3_k8.log; exit 3; }
grep -h '"kernel_name"\|"avg_us"\|hbm_bytes_per_launch' $O/prof_c3_k8/summary.json
OUT=$O/prof_c5 WL=c5 bash scripts/gpu_profile.sh > $O/prof_c5.log 2>&1 || { echo "profile c5 failed"; tail -30 $O/prof_c5.log; exit 3; }
grep -h '"kernel_name"\|"avg_us"\|hbm_bytes_per_launch' $O/prof_c5/summary.json
