# C2 (4096^2): per-step pass time of mm_passk_kernel K = 6..8 and mm_wide_kernel K = 4 / 8
# across segment sizings (MM_SEG_WAVES) -- what bounds the short-segment plan.
set -o pipefail
export TMPDIR=/tmp
D=${D:-gpurun_out/c2sweep}
mkdir -p $D
for sw in 0 1 1.5 2 3 6; do
  if [ "$sw" = 0 ]; then unset MM_SEG_WAVES; else export MM_SEG_WAVES=$sw; fi
  echo "# MM_SEG_WAVES=$sw" >> $D/table.log
  timeout -k 10 120 python3 -u tools/kernel_table.py --sizes 4096x4096 --old 6,7,8 --wide 4,8,12 \
      --reps 20 >> $D/table.log 2>&1 || { tail -20 $D/table.log; exit 1; }
done
cat $D/table.log
