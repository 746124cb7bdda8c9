# c4 (16384^2, K = 20) segment-length sweep: MM_SEG_WAVES 4 (auto), 2, 1, two rounds
export D=${D:-gpurun_out/segw_c4}
for r in 1 2; do
    TAG=auto_r$r bash tools/gpu.sh bench c4 1000 50 --no-cpu-baseline || exit 3
    for sw in 2 1; do
        MM_SEG_WAVES=$sw TAG=sw${sw}_r$r bash tools/gpu.sh bench c4 1000 50 --no-cpu-baseline || exit 3
    done
done
