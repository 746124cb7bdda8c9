# C2 segment-length sweep: MM_SEG_WAVES (workgroups per resident slot; auto = 1 at 4096^2)
# and MM_SEG_EDGE (edge-strip segment length / interior, auto 0.5), 2 rounds
export D=${D:-gpurun_out/segw}
for r in 1 2; do
    TAG=auto_r$r bash tools/gpu.sh bench c2 1000 50 --no-cpu-baseline || exit 3
    for sw in 0.67 0.8 1.33; do
        MM_SEG_WAVES=$sw TAG=sw${sw}_r$r bash tools/gpu.sh bench c2 1000 50 --no-cpu-baseline || exit 3
    done
    for se in 0.35 0.7; do
        MM_SEG_EDGE=$se TAG=se${se}_r$r bash tools/gpu.sh bench c2 1000 50 --no-cpu-baseline || exit 3
    done
done
