#!/bin/bash
# The driver's 20-step timed run after a 5-step warmup: hipGraph replay vs eager launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/gap2
for g in 1 0 1 0; do
  MM_GRAPH=$g timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gap2/b.log 2>&1 || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/gap2/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('graph=$g', d['value'], d['ms_per_step']*d['steps'], r['kernel_avg_us'], d['config']['path'])"
done
