# round 3, final tree: GPU suite, smoke, every bench line, rocprof + PMC of every workload.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3final}
mkdir -p $D
D=$D bash tools/gpu_round3l.sh || exit 1
R=${R:-gpurun_out/prof_r3c} bash tools/gpu_prof_r3.sh > $D/prof.log 2>&1 || { tail -30 $D/prof.log; exit 1; }
grep -E '"(workload|kernel_name|avg_us|hbm_bytes_per_launch)"' $D/prof.log
timeout -k 10 200 python3 -u tools/power_probe.py > $D/power_probe.log 2>&1 || { tail -20 $D/power_probe.log; exit 1; }
cat $D/power_probe.log
