# The 4096 x 32768 slab of an 8-GPU c3 run (2^27 cells): mm_passk_kernel 7 + 7 + 6 (the
# default) against the level-split kernel's planner (MM_WIDE=1: one K = 20 pass), plain
# and with the split schedule + RCCL self-exchange, the driver's 20 steps, 3 rounds.
export D=${D:-gpurun_out/midslab}
for rep in 1 2 3; do
  for mode in "" "--self-halo"; do
    t=${mode:+self}; t=${t:-plain}
    TAG=passk_${t}_$rep bash tools/gpu.sh bench c3 20 5 --grid 4096 32768 --no-cpu-baseline $mode || exit 3
    MM_WIDE=1 TAG=wide_${t}_$rep bash tools/gpu.sh bench c3 20 5 --grid 4096 32768 --no-cpu-baseline $mode || exit 3
  done
done
