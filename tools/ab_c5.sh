# C5 chain-kernel lines: C5 (ring instance), C5 on the run-time-operand chain, the
# reordered ring, a program with a post-chain and two of four attributes diffusing
export D=${D:-gpurun_out/c5ab}
TAG=ring bash tools/gpu.sh bench c5 1000 50 --no-cpu-baseline || exit 3
MM_CHAIN_RING=0 TAG=runtime bash tools/gpu.sh bench c5 1000 50 --no-cpu-baseline || exit 3
TAG=reordered bash tools/gpu.sh bench c5 1000 50 --no-cpu-baseline --program reordered || exit 3
TAG=post bash tools/gpu.sh bench c5 1000 50 --no-cpu-baseline --program post || exit 3
