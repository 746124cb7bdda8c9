set -o pipefail
D=gpurun_out/var_k20
mkdir -p $D
timeout -k 10 500 python3 -u tools/libsweep.py --size 32768 --steps 40 --rounds 3 --timeout 150 \
    --check-steps 43 --env '{"MM_WIDE": 1, "MM_STEPS_PER_PASS": 20}' \
    var/*/libmpimodel_hip.so > $D/sweep_k20.log 2>&1 || { tail -20 $D/sweep_k20.log; exit 1; }
grep -A20 summary $D/sweep_k20.log
