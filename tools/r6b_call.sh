set -o pipefail
D=gpurun_out/r6b
export D
B=mpi-model_amd/libmpimodel_hip.so
bash tools/gpu.sh ab spin c3 20 4 "MM_SYNC_SPIN=0" "MM_SYNC_SPIN=1" > $D.spin.txt 2>&1; cat $D.spin.txt
bash tools/gpu.sh ab b6 c3 100 3 "MM_LIB_PATH=$B" "MM_LIB_PATH=abx/b6/libmpimodel_hip.so" > $D.b6.txt 2>&1; cat $D.b6.txt
bash tools/gpu.sh ab k8asc c2 1000 3 "MM_LIB_PATH=$B" "MM_LIB_PATH=abx/k8asc/libmpimodel_hip.so" > $D.k8asc.txt 2>&1; cat $D.k8asc.txt
bash tools/gpu.sh ab k8asc4 c2 1000 3 "MM_LIB_PATH=$B" "MM_LIB_PATH=abx/k8asc4/libmpimodel_hip.so" > $D.k8asc4.txt 2>&1; cat $D.k8asc4.txt
bash tools/gpu.sh trace spin c3 20 5
