#!/bin/bash
# rocprofv3 trace + FETCH/WRITE for the c3 K = 10 pass (the driver's 20-step run) and the
# K = 8 pass (long runs), committed tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-profc3}
mkdir -p $O
PSTEPS=20 PMCSTEPS=20 OUT=$O/prof_c3_k10 WL=c3 bash scripts/gpu_profile.sh > $O/prof_c3_k10.log 2>&1 || { echo "profile k10 failed"; tail -30 $O/prof_c3_k10.log; exit 3; }
grep -h '"kernel_name"\|"calls"\|"avg_us"\|hbm_bytes_per_launch' $O/prof_c3_k10/summary.json
OUT=$O/prof_c3_k8 WL=c3 bash scripts/gpu_profile.sh > $O/prof_c3_k8.log 2>&1 || { echo "profile k8 failed"; tail -30 $O/prof_c3_k8.log; exit 3; }
grep -h '"kernel_name"\|"calls"\|"avg_us"\|hbm_bytes_per_launch' $O/prof_c3_k8/summary.json
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { echo "bench failed"; exit 3; }
tail -1 $O/bench_driver_cmd.log
