# Compare variant builds (tools/build_variants.sh -> var/*/libmpimodel_hip.so) of the wide
# kernel: the 8-column K = 8 instance and the 4-column K = 16 instance at 32768^2.
set -o pipefail
D=${D:-gpurun_out/var}
mkdir -p $D
timeout -k 10 400 python3 -u tools/libsweep.py --size 32768 --steps 16 --rounds 2 --timeout 150 \
    --check-steps 19 --env '{"MM_WIDE": 1, "MM_WIDE_COLS": 8, "MM_STEPS_PER_PASS": 8}' \
    var/*/libmpimodel_hip.so > $D/sweep_w8k8.log 2>&1 || { tail -20 $D/sweep_w8k8.log; exit 1; }
grep -A20 summary $D/sweep_w8k8.log
timeout -k 10 400 python3 -u tools/libsweep.py --size 32768 --steps 32 --rounds 2 --timeout 150 \
    --check-steps 35 --env '{"MM_WIDE": 1, "MM_STEPS_PER_PASS": 16}' \
    var/*/libmpimodel_hip.so > $D/sweep_k16.log 2>&1 || { tail -20 $D/sweep_k16.log; exit 1; }
grep -A20 summary $D/sweep_k16.log
