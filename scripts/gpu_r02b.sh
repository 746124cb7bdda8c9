#!/bin/bash
# Round-2 (second session) evidence on the committed tree: GPU tests, smoke, the driver's
# bench command (default c3), a 1000-step c3 line and the c3 rocprofv3 trace + FETCH/WRITE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r02b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 3; }
cat $O/smoke.log
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { echo "bench failed"; tail $O/bench_driver_cmd.log; exit 3; }
tail -1 $O/bench_driver_cmd.log
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 1000 --warmup 50 > $O/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail $O/bench_c3.log; exit 3; }
tail -1 $O/bench_c3.log
OUT=$O/prof_c3 WL=c3 bash scripts/gpu_profile.sh > $O/prof_c3.log 2>&1 || { echo "profile c3 failed"; tail -30 $O/prof_c3.log; exit 3; }
cat $O/prof_c3/summary.json
