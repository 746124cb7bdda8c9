set -o pipefail
mkdir -p gpurun_out
for k in 16 20; do
  timeout -k 10 400 python3 -u tools/libsweep.py --size 32768 --steps $((k*2)) --rounds 2 --timeout 150 --check-steps $((2*k+3)) --env "{\"MM_WIDE\": 1, \"MM_STEPS_PER_PASS\": $k}" var/*/libmpimodel_hip.so > gpurun_out/sweep_w$k.log 2>&1 || exit 1
done
