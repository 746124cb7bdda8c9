# round 3: the C5 ring instance on two levels per wave (4 waves) -- whole GPU suite, the C5
# bench line, its rocprofv3 + PMC passes, then the driver command.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3q}
mkdir -p $D
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $D/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 1000 --warmup 20 > $D/bench_c5_1000.log 2>&1 || { tail -20 $D/bench_c5_1000.log; exit 1; }
tail -1 $D/bench_c5_1000.log
R=gpurun_out/prof_c5q SPECS="c5_k8:c5:96:16" bash tools/gpu_prof_r3.sh > $D/prof.log 2>&1 || { tail -30 $D/prof.log; exit 1; }
cat $D/prof.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $D/bench_driver_cmd.log 2>&1 || { tail -20 $D/bench_driver_cmd.log; exit 1; }
tail -1 $D/bench_driver_cmd.log
