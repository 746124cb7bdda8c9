#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box):
#   1. --kernel-trace --stats of a bench run (per-kernel average duration)
#   2. two PMC passes, FETCH_SIZE and WRITE_SIZE (they do not fit one pass on gfx950)
# Each step under its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
WL=${WL:-c3}
ARGS="--workload $WL --steps ${PSTEPS:-96} --warmup 16 --no-cpu-baseline"
mkdir -p $OUT
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -20 $OUT/trace.log; exit 3; }
echo trace ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS --steps ${PMCSTEPS:-32} > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -20 $OUT/fetch.log; exit 3; }
echo fetch ok
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS --steps ${PMCSTEPS:-32} > $OUT/write.log 2>&1 || { echo "write rc=$?"; tail -20 $OUT/write.log; exit 3; }
echo write ok
python3 tools/prof_summary.py $OUT $WL > $OUT/summary.json && cat $OUT/summary.json
