#!/bin/bash
# The planner on other grids: 20-step runs with and without it (c4 16384^2, c3 32768^2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-planc4}
mkdir -p $O
for wl in c4 c3; do
  for p in 1 0 1 0; do
    MM_PASS_PLAN=$p timeout -k 10 200 python3 -u bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit 3
    python3 -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$wl plan=$p', d['value'], round(d['ms_per_step']*d['steps'],3), r['kernel_avg_us'], d['config']['path'])" | tee -a $O/plan.log
  done
done
