# C2 (4096^2, 1000 steps): the default plan (mm_passk_kernel K = 7) against K = 8 on both
# kernels, alternating, twice -- is a wide K = 8 plan worth switching C2 to.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/c2bench}
mkdir -p $D
for rep in 1 2; do
  for v in default passk8 wide8 wide8sw1; do
    case $v in
      default) envs="" ;;
      passk8) envs="MM_STEPS_PER_PASS=8" ;;
      wide8) envs="MM_WIDE=1 MM_STEPS_PER_PASS=8" ;;
      wide8sw1) envs="MM_WIDE=1 MM_STEPS_PER_PASS=8 MM_SEG_WAVES=1" ;;
    esac
    env $envs timeout -k 10 120 python3 -u bench.py --workload c2 --steps 1000 --warmup 20 \
        --no-cpu-baseline > $D/$v.$rep.log 2>&1 || { tail -20 $D/$v.$rep.log; exit 1; }
    python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], l['value'], l['roofline']['kernel_avg_us'], l['config']['path'])" $D/$v.$rep.log $v
  done
done
