cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp
for s in 96 1000 3000 96; do
  timeout -k 10 200 python3 -u bench.py --steps $s --warmup 16 --no-cpu-baseline > gpurun_out/exp/b_$s.log 2>&1 || exit 3
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/exp/b_$s.log').read().strip().splitlines()[-1]); print($s, d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
rocm-smi --showclocks --showpower --showtemp > gpurun_out/exp/smi.log 2>&1; grep -E "sclk|Power|Temp" gpurun_out/exp/smi.log | head
