#!/bin/bash
# Round-2 measurement: the driver's default bench line (c3, N=1) with its CPU baseline,
# the other workloads' lines, and rocprofv3 kernel trace + FETCH/WRITE passes per workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02
timeout -k 10 400 python3 -u bench.py --steps 1000 --warmup 50 > gpurun_out/r02/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail gpurun_out/r02/bench_c3.log; exit 3; }
tail -1 gpurun_out/r02/bench_c3.log
for wl in c2 c4 c5; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --steps 1000 --warmup 50 > gpurun_out/r02/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail gpurun_out/r02/bench_$wl.log; exit 3; }
  tail -1 gpurun_out/r02/bench_$wl.log
done
for wl in c3 c4 c2 c5; do
  OUT=gpurun_out/r02/prof_$wl WL=$wl bash scripts/gpu_profile.sh > gpurun_out/r02/prof_$wl.log 2>&1 || { echo "profile $wl failed"; tail -30 gpurun_out/r02/prof_$wl.log; exit 3; }
  tail -3 gpurun_out/r02/prof_$wl.log
done
