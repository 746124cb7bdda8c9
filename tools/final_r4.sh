# Round-4 evidence on the committed tree, part 1: GPU suite + smoke, every bench line with
# its CPU baseline (tools/gpu.sh lines), rocprofv3 trace + PMC traffic of each workload on
# the plan and length its line times (c3: the driver's 20 steps; c4 / c5 / c2: 1000).
export D=${D:-gpurun_out/final_r4}
bash tools/gpu.sh test || exit 3
bash tools/gpu.sh lines || exit 3
