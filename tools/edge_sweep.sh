#!/bin/bash
# Edge-strip segment length (MM_SEG_EDGE: edge segment rows / interior segment rows) of the
# wide kernel's segment plan on every bench shape: GCUPS and kernel us per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
D=${D:-gpurun_out/edge}; mkdir -p $D
one() {  # tag edge args...
    local tag=$1 e=$2; shift 2
    MM_SEG_EDGE=$e timeout -k 10 300 python3 -u bench.py "$@" --no-cpu-baseline > $D/${tag}_e$e.log 2>&1 || exit 3
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['roofline']['kernel_avg_us'])" $D/${tag}_e$e.log "$tag edge=$e"
}
if [ "${ONLY:-}" = c5 ]; then  # the four-attribute line alone
    for rep in 0 1; do
        for e in ${EDGES:-0.25 0.35 0.5}; do one c5_$rep $e --workload c5 --steps 1000 --warmup 50; done
    done
    exit 0
fi
for rep in 0 1; do
    for e in ${EDGES:-0.5 1.0}; do
        one c4_$rep $e --workload c4 --steps 1000 --warmup 50
        one c5_$rep $e --workload c5 --steps 1000 --warmup 50
        one s4096_$rep $e --workload c3 --steps 200 --warmup 5 --grid 4096 32768 --self-halo
        one s8192_$rep $e --workload c3 --steps 200 --warmup 5 --grid 8192 32768 --self-halo
        one c3k_$rep $e --workload c3 --steps 1000 --warmup 50
    done
done
