#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script
# (exit codes other than 0 = ok and 1 = ordinary test failure).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-all}
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    echo "=== $name" | tee -a gpurun_out/steps.log
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
rocm-smi --showproductname > gpurun_out/rocm-smi.log 2>&1 || true
if [[ $STEPS == all || $STEPS == *tests* ]]; then
  step pytest_gpu 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  step smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  step bench 400 python -u bench.py ${BENCH_ARGS:-}
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-}
fi
echo done
