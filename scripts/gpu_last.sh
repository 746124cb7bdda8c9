#!/bin/bash
# Last check of the committed tree: GPU tests, smoke, the driver's bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-last}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 3; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 3; }
cat $O/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || { echo "bench failed"; tail $O/bench_driver_cmd.log; exit 3; }
tail -1 $O/bench_driver_cmd.log
