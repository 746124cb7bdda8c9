# C2 (4096^2, 1000 steps): steps per replayed hipGraph (MM_GRAPH_MIN_STEPS) on the default
# plan and the wide K = 8 plan; then the one-pass kernel table at the sizes between C2 and
# the wide kernel's 2^28-cell threshold.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/c2graph}
mkdir -p $D
for rep in 1 2; do
  for g in 16 64 256; do
    for v in default wide8; do
      case $v in
        default) envs="MM_GRAPH_MIN_STEPS=$g" ;;
        wide8) envs="MM_GRAPH_MIN_STEPS=$g MM_WIDE=1 MM_STEPS_PER_PASS=8" ;;
      esac
      env $envs timeout -k 10 120 python3 -u bench.py --workload c2 --steps 1000 --warmup 20 \
          --no-cpu-baseline > $D/$v.g$g.$rep.log 2>&1 || { tail -20 $D/$v.g$g.$rep.log; exit 1; }
      python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], l['value'], l['roofline']['kernel_avg_us'], l['config']['path'])" $D/$v.g$g.$rep.log "$v g$g"
    done
  done
done
timeout -k 10 300 python3 -u tools/kernel_table.py --sizes 1024x1024,2048x2048,8192x8192,4096x32768,16384x16384 \
    --old 7,8 --wide 8 --reps 10 > $D/table.log 2>&1 || { tail -20 $D/table.log; exit 1; }
cat $D/table.log
