#!/bin/bash
# rocprofv3 evidence for round 3: per workload a --kernel-trace --stats run of bench.py and
# two PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs on gfx950), summarised by
# tools/prof_summary.py. Each step under its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${R:-gpurun_out/prof_r3}
set -o pipefail
run() {  # name workload steps warmup
  local OUT=$R/$1 ARGS="--workload $2 --steps $3 --warmup $4 --no-cpu-baseline"
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "$1 trace rc=$?"; tail -20 $OUT/trace.log; return 3; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "$1 fetch rc=$?"; tail -20 $OUT/fetch.log; return 3; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "$1 write rc=$?"; tail -20 $OUT/write.log; return 3; }
  python3 tools/prof_summary.py $OUT $2 > $OUT/summary.json && cat $OUT/summary.json
}
for spec in ${SPECS:-"c3_k20:c3:20:5" "c3_k16:c3:96:16" "c4_k16:c4:96:16" "c5_k8:c5:96:16" "c2:c2:96:16"}; do
  IFS=: read name wl steps warm <<< "$spec"
  run $name $wl $steps $warm || exit 3
done
