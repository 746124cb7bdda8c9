# round 3: bench.py at N > 1 on the one GPU with the host halo (gloo), c3 strong and c4 weak;
# then the rocprof evidence of the final kernels (tools/gpu_prof_r3.sh)
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/r3m}
mkdir -p $D
for spec in "c3:2:20:5" "c3:4:20:5" "c4:2:100:20" "c5:2:100:20"; do
  IFS=: read wl n steps warm <<< "$spec"
  timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n --halo host --workload $wl --steps $steps --warmup $warm \
      > $D/bench_${wl}_n${n}_host.log 2>&1 || { tail -30 $D/bench_${wl}_n${n}_host.log; exit 1; }
  grep '^{"metric"' $D/bench_${wl}_n${n}_host.log | tail -1 | cut -c1-900
done
R=gpurun_out/prof_r3b bash tools/gpu_prof_r3.sh > $D/prof.log 2>&1 || { tail -30 $D/prof.log; exit 1; }
grep -E '"(workload|kernel_name|avg_us|hbm_bytes_per_launch|hbm_read_bytes_per_launch|hbm_write_bytes_per_launch)"' $D/prof.log
