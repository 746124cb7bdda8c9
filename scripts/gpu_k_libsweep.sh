cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/k10b
for K in 8 9 10; do
  timeout -k 10 300 python3 -u tools/libsweep.py --size 32768 --steps $((K*3)) --rounds 2 --env "{\"MM_STEPS_PER_PASS\": $K}" var/*/libmpimodel_hip.so > gpurun_out/k10b/libsweep_k$K.log 2>&1 || { echo "k$K failed"; tail gpurun_out/k10b/libsweep_k$K.log; exit 3; }
  grep variant gpurun_out/k10b/libsweep_k$K.log
done
timeout -k 10 300 python3 -u tools/libsweep.py --size 32768 --steps 24 --rounds 2 --env '{"MM_STEPS_PER_PASS": 8, "MM_SEG_WAVES": 3}' var/*/libmpimodel_hip.so > gpurun_out/k10b/libsweep_k8sw3.log 2>&1 || exit 3
grep variant gpurun_out/k10b/libsweep_k8sw3.log
