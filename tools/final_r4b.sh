# Round-4 evidence, part 2: rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of each
# workload on the plan and length its bench line times, and the SQ split of the c3 pass.
export D=${D:-gpurun_out/final_r4}
bash tools/gpu.sh prof c3_k20 c3 20 5 || exit 3
bash tools/gpu.sh prof c4_k20 c4 1000 50 || exit 3
bash tools/gpu.sh prof c5_k8 c5 1000 50 || exit 3
bash tools/gpu.sh prof c2_k8 c2 1000 50 || exit 3
bash tools/gpu.sh sq c3_k20 c3 20 5 || exit 3
