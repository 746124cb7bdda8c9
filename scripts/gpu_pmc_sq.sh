#!/bin/bash
# SQ wave-cycle split and effective clock of the dominant step kernel (one --pmc pass:
# 6 SQ + 1 GRBM counters fit gfx950's slots), with the kernel-trace average from the same
# bench command for the clock estimate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c3}
OUT=${OUT:-gpurun_out/pmc_sq_$WL}
ARGS="--workload $WL --steps ${PSTEPS:-32} --warmup 16 --no-cpu-baseline"
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail $OUT/trace.log; exit 3; }
AVG=$(python3 -c "
import csv,glob
r=[x for f in glob.glob('$OUT/trace/**/*kernel_stats.csv',recursive=True) for x in csv.DictReader(open(f)) if ('mm_pass' in x['Name'] or 'mm_wide' in x['Name'])]
r.sort(key=lambda x: float(x['TotalDurationNs']), reverse=True); print(float(r[0]['AverageNs'])/1e3)")
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 bench.py $ARGS > $OUT/pmc.log 2>&1 || { echo "pmc rc=$?"; tail $OUT/pmc.log; exit 3; }
python3 tools/pmc_sq_summary.py $OUT/pmc $AVG > $OUT/summary.json && cat $OUT/summary.json
