cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/gap
for a in "--steps 20 --warmup 5" "--steps 20 --warmup 20" "--steps 20 --warmup 5" "--steps 40 --warmup 5" "--steps 20 --warmup 25"; do
  timeout -k 10 200 python3 -u bench.py $a --no-cpu-baseline > gpurun_out/gap/b.log 2>&1 || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/gap/b.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$a', d['value'], d['ms_per_step']*d['steps'], r['kernel_avg_us'], d['config']['path'])"
done
