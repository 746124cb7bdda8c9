# Slabs between 2^25 and 2^28 cells (8192^2; 4096 x 32768 = the per-GPU slab of an 8-GPU
# c3 run): mm_passk_kernel K = 7/8 against the wide kernel at K = 8..20.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/midslab}
mkdir -p $D
timeout -k 10 300 python3 -u tools/kernel_table.py --sizes 4096x32768,8192x8192,2048x32768 \
    --old 7,8 --wide 8,12,16,20 --reps 6 > $D/table.log 2>&1 || { tail -20 $D/table.log; exit 1; }
cat $D/table.log
