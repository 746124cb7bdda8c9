#!/bin/bash
# Border rows of a split pass as depth-row segments (default) vs 4-row blocks
# (MM_BORDER_SEG=0): GPU tests, then the RCCL self-halo bench (the split schedule on one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-border}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
for st in 20 200; do for b in 1 0 1 0; do
  MM_BORDER_SEG=$b timeout -k 10 200 python3 -u bench.py --self-halo --steps $st --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit 3
  python3 -c "import json; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print('steps=$st border_seg=$b', d['value'], round(d['ms_per_step']*d['steps'],3), d['roofline']['kernel_avg_us'])" | tee -a $O/border.log
done; done
