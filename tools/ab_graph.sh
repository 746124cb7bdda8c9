# Graph length A/B on one box: 2-pass graphs (MM_GRAPH_MAX_LAUNCHES=2, the round-3 length)
# against the default (the longest graph dividing the run), c2 and c5, alternating, 3 rounds
export D=${D:-gpurun_out/abgraph}
for r in 1 2 3; do
    for wl in c2 c5; do
        MM_GRAPH_MAX_LAUNCHES=2 TAG=g2_r$r bash tools/gpu.sh bench $wl 1000 50 --no-cpu-baseline || exit 3
        TAG=gmax_r$r bash tools/gpu.sh bench $wl 1000 50 --no-cpu-baseline || exit 3
    done
done
