#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bw_probe > gpurun_out/bw_probe.log 2>&1 || { echo "bw_probe rc=$?"; exit 3; }
cat gpurun_out/bw_probe.log
timeout -k 10 200 python -u tools/sweep.py --size 4096 > gpurun_out/sweep_4096.log 2>&1 || { echo "sweep4096 rc=$?"; tail gpurun_out/sweep_4096.log; exit 3; }
head -12 gpurun_out/sweep_4096.log
timeout -k 10 300 python -u tools/sweep.py --size 16384 --ths 16,32,64,128,256 --variants 0,2,3,4,6 --steps 30 --rounds 2 > gpurun_out/sweep_16384.log 2>&1 || { echo "sweep16384 rc=$?"; tail gpurun_out/sweep_16384.log; exit 3; }
head -10 gpurun_out/sweep_16384.log
timeout -k 10 200 python -u tests/../tools/sweep.py --size 32768 --ths 64,256,512 --variants 0,3,4 --steps 10 --rounds 2 > gpurun_out/sweep_32768.log 2>&1 || { echo "sweep32768 rc=$?"; tail gpurun_out/sweep_32768.log; exit 3; }
head -9 gpurun_out/sweep_32768.log
