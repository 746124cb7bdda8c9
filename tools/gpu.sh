#!/bin/bash
# The one GPU runner of this repository (replaces the per-round one-off scripts).
#
#   bash tools/gpu.sh test [pytest args]      GPU test suite (pytest -m gpu), then smoke()
#   bash tools/gpu.sh bench WL STEPS WARMUP [bench.py args]   one bench.py line
#   bash tools/gpu.sh lines                   every workload's bench line: the driver's
#                                             command (c3, 20 steps) and 1000-step c2..c5
#   bash tools/gpu.sh prof NAME WL STEPS WARMUP [bench.py args]
#                                             rocprofv3 --kernel-trace --stats of bench.py,
#                                             then two PMC passes (FETCH_SIZE, WRITE_SIZE),
#                                             summarised by tools/prof_summary.py
#   bash tools/gpu.sh trace NAME WL STEPS WARMUP [bench.py args]
#                                             rocprofv3 --kernel-trace only (per-dispatch timeline)
#   bash tools/gpu.sh sq NAME WL STEPS WARMUP [bench.py args]
#                                             SQ wave-cycle split + effective clock (PMC)
#   bash tools/gpu.sh pmc NAME WL STEPS WARMUP "COUNTERS" [bench.py args]
#                                             one --pmc pass, mean counters per dispatch
#   bash tools/gpu.sh selfhalo                bench.py --self-halo beside the plain run on the
#                                             slab shapes of the N > 1 runs (price of the
#                                             interior / border split + RCCL exchange)
#   bash tools/gpu.sh final                   a round's evidence on the committed tree: test, lines
#                                             (FINAL_PART=a), then prof / sq / L2 counters of each
#                                             line's own plan and length (FINAL_PART=b)
#   bash tools/gpu.sh self20                  every scaling slab plain and --self-halo at 20 steps
#   bash tools/gpu.sh trace20                 HIP-runtime trace of a 20-step split run
#   bash tools/gpu.sh ab TAG WL STEPS REPS "ENV_A" "ENV_B" [bench.py args]
#                                             A/B of two environments on one box, alternating
#                                             A B A B ... REPS times (GCUPS per run)
#   bash tools/gpu.sh thin                    segment-plan sweep of the thin split slabs of the
#                                             c3 N = 8 / N = 4 runs (4096 / 8192 x 32768,
#                                             self-halo, 200 steps) against the 32768^2 slab
#   bash tools/gpu.sh thintrace               rocprofv3 kernel traces of the same slabs, split and
#                                             plain, per pass decomposed (tools/thin_trace.py)
#   bash tools/gpu.sh scale WL [N...]         the driver's multi-GPU command, N = 1 2 4 8 by
#                                             default (needs N GPUs; never run on the 1-GPU box)
#
# Output under $D (default gpurun_out/run). Every GPU step runs under its own time limit and
# a failing step ends the script (no retries): read its log under $D.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
set -o pipefail
D=${D:-gpurun_out/run}
mkdir -p "$D"

fail() { echo "FAILED: $1 (rc=$2), log $3"; tail -30 "$3"; exit 3; }

gpu_test() {
    timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread "$@" > "$D/pytest_gpu.log" 2>&1 || fail pytest $? "$D/pytest_gpu.log"
    tail -3 "$D/pytest_gpu.log"
    timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$D/smoke.log" 2>&1 \
        || fail smoke $? "$D/smoke.log"
    cat "$D/smoke.log"
}

bench() {  # WL STEPS WARMUP [args]
    local wl=$1 steps=$2 warm=$3
    shift 3
    local log="$D/bench_${wl}_${steps}${TAG:+_$TAG}.log"
    timeout -k 10 600 python3 -u bench.py --workload "$wl" --steps "$steps" --warmup "$warm" "$@" \
        > "$log" 2>&1 || fail "bench $wl" $? "$log"
    grep '^{' "$log"
}

lines() {
    bench c3 20 5
    bench c3 1000 50
    bench c4 1000 50
    bench c2 1000 50
    bench c5 1000 50
}

prof() {  # NAME WL STEPS WARMUP [args]
    local name=$1 wl=$2 steps=$3 warm=$4
    shift 4
    local out="$D/prof_$name" args="--workload $wl --steps $steps --warmup $warm --no-cpu-baseline $*"
    mkdir -p "$out"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
        -- python3 bench.py $args > "$out/trace.log" 2>&1 || fail "prof trace $name" $? "$out/trace.log"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run \
        -- python3 bench.py $args > "$out/fetch.log" 2>&1 || fail "prof fetch $name" $? "$out/fetch.log"
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run \
        -- python3 bench.py $args > "$out/write.log" 2>&1 || fail "prof write $name" $? "$out/write.log"
    python3 tools/prof_summary.py "$out" "$wl" > "$out/summary.json" && cat "$out/summary.json"
}

trace() {  # NAME WL STEPS WARMUP [args]
    local name=$1 wl=$2 steps=$3 warm=$4
    shift 4
    local out="$D/trace_$name"
    mkdir -p "$out"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
        -- python3 bench.py --workload "$wl" --steps "$steps" --warmup "$warm" --no-cpu-baseline "$@" \
        > "$out/trace.log" 2>&1 || fail "trace $name" $? "$out/trace.log"
    grep '^{' "$out/trace.log" | cut -c1-200
}

sq() {  # NAME WL STEPS WARMUP [args]: SQ wave-cycle split + effective clock (one --pmc pass:
        # 6 SQ + 1 GRBM counters fit gfx950's slots), after a trace run for the kernel time
    local name=$1 wl=$2 steps=$3 warm=$4
    shift 4
    local out="$D/sq_$name" args="--workload $wl --steps $steps --warmup $warm --no-cpu-baseline $*"
    mkdir -p "$out"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
        -- python3 bench.py $args > "$out/trace.log" 2>&1 || fail "sq trace $name" $? "$out/trace.log"
    local avg
    avg=$(python3 tools/prof_summary.py "$out" "$wl" | python3 -c "import json,sys; print(json.load(sys.stdin)['steady_avg_us'])")
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
        SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc" -o run \
        -- python3 bench.py $args > "$out/pmc.log" 2>&1 || fail "sq pmc $name" $? "$out/pmc.log"
    python3 tools/pmc_sq_summary.py "$out/pmc" "$avg" > "$out/summary.json" && cat "$out/summary.json"
}

pmc() {  # NAME WL STEPS WARMUP "COUNTERS" [args]: one --pmc pass of up to 8 SQ counters
    local name=$1 wl=$2 steps=$3 warm=$4 counters=$5
    shift 5
    local out="$D/pmc_$name" args="--workload $wl --steps $steps --warmup $warm --no-cpu-baseline $*"
    mkdir -p "$out"
    timeout -s KILL 300 rocprofv3 --pmc $counters --output-format csv -d "$out/pmc" -o run \
        -- python3 bench.py $args > "$out/pmc.log" 2>&1 || fail "pmc $name" $? "$out/pmc.log"
    python3 tools/pmc_sq_summary.py "$out/pmc" > "$out/summary.json" && cat "$out/summary.json"
}

selfhalo() {
    # slab shapes of the scaling runs: c3 N = 1 / 2 / 4 / 8 (32768 columns, 32768 / 16384 /
    # 8192 / 4096 rows) and the c4 per-GPU slab (16384^2); each plain and with the split
    # schedule + RCCL self-exchange, 20 steps (the driver's) and 200
    local g
    for g in "32768 32768" "16384 32768" "8192 32768" "4096 32768" "16384 16384"; do
        set -- $g
        for steps in 20 200; do
            TAG="${1}x${2}_plain" bench c3 $steps 5 --grid $1 $2 --no-cpu-baseline
            TAG="${1}x${2}_self" bench c3 $steps 5 --grid $1 $2 --no-cpu-baseline --self-halo
        done
    done
}

final() {  # part a (FINAL_PART=a, default): suite + lines; part b: profiles (each fits a call)
    if [ "${FINAL_PART:-a}" = a ]; then
        gpu_test
        lines
        MM_CHAIN_RING=0 TAG=runtime_chain bench c5 1000 50
        TAG=4096x32768 bench c3 20 5 --grid 4096 32768 --no-cpu-baseline
    else
        prof c3_k20 c3 20 5
        prof c4_k20 c4 1000 50
        prof c2_k8 c2 1000 50
        prof c5_k8 c5 1000 50
        sq c3_k20 c3 20 5
        sq c2 c2 1000 50
        sq c5_k8 c5 1000 50
        pmc c3tcc c3 20 5 "TCC_HIT_sum TCC_MISS_sum"
    fi
}

self20() {  # the split's price at the driver's 20 steps: every scaling slab plain and split
    local g
    for g in "32768 32768" "16384 32768" "8192 32768" "4096 32768" "16384 16384"; do
        set -- $g
        TAG="${1}x${2}_plain" bench c3 20 5 --grid $1 $2 --no-cpu-baseline
        TAG="${1}x${2}_self" bench c3 20 5 --grid $1 $2 --no-cpu-baseline --self-halo
    done
}

trace20() {  # HIP-runtime + kernel trace of one 20-step split run (launch-to-start latencies)
    local out="$D/hiptrace20"
    mkdir -p "$out"
    timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$out" -o run \
        -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --grid 8192 32768 --self-halo \
        > "$out/trace.log" 2>&1 || fail trace20 $? "$out/trace.log"
    python3 tools/launch_latency.py "$out" > "$out/launch_latency.txt" && cat "$out/launch_latency.txt"
}

ab() {  # TAG WL STEPS REPS ENVA ENVB [args]
    local tag=$1 wl=$2 steps=$3 reps=$4 ea=$5 eb=$6 r
    shift 6
    for ((r = 0; r < reps; r++)); do
        env $ea TAG="${tag}_A$r" bash "$0" bench "$wl" "$steps" 5 --no-cpu-baseline "$@" | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A', '$ea', d['value'], d['roofline']['kernel_avg_us'])"
        env $eb TAG="${tag}_B$r" bash "$0" bench "$wl" "$steps" 5 --no-cpu-baseline "$@" | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B', '$eb', d['value'], d['roofline']['kernel_avg_us'])"
    done
}

thin() {
    local steps=${THIN_STEPS:-200} v
    TAG=32768x32768_plain bench c3 $steps 5 --no-cpu-baseline
    for g in "4096 32768" "8192 32768"; do
        set -- $g
        TAG="${1}x${2}_self" bench c3 $steps 5 --grid $1 $2 --no-cpu-baseline --self-halo
        for v in ${THIN_SW:-1 2 3 6}; do
            MM_SEG_WAVES=$v TAG="${1}x${2}_self_sw$v" bench c3 $steps 5 --grid $1 $2 \
                --no-cpu-baseline --self-halo
        done
        for v in ${THIN_K:-12 16}; do
            MM_STEPS_PER_PASS=$v TAG="${1}x${2}_self_k$v" bench c3 $steps 5 --grid $1 $2 \
                --no-cpu-baseline --self-halo
        done
    done
}

thintrace() {  # per-pass decomposition of the thin split slabs (tools/thin_trace.py)
    local steps=${THIN_STEPS:-200} g
    for g in "4096 32768" "8192 32768"; do
        set -- $g
        trace "${1}x${2}_self" c3 $steps 5 --grid $1 $2 --self-halo
        python3 tools/thin_trace.py "$D/trace_${1}x${2}_self" "${1}x${2} split" \
            > "$D/trace_${1}x${2}_self/summary.json" && cat "$D/trace_${1}x${2}_self/summary.json"
        trace "${1}x${2}_plain" c3 $steps 5 --grid $1 $2
        python3 tools/thin_trace.py "$D/trace_${1}x${2}_plain" "${1}x${2} plain" \
            > "$D/trace_${1}x${2}_plain/summary.json" && cat "$D/trace_${1}x${2}_plain/summary.json"
    done
    trace 32768x32768_plain c3 $steps 5
    python3 tools/thin_trace.py "$D/trace_32768x32768_plain" "32768x32768 plain" \
        > "$D/trace_32768x32768_plain/summary.json" && cat "$D/trace_32768x32768_plain/summary.json"
}

scale() {  # WL [N...]
    local wl=$1
    shift
    local ns=${*:-1 2 4 8} n
    for n in $ns; do
        local log="$D/scale_${wl}_n$n.log"
        timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
            --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus "$n" \
            --workload "$wl" --steps 20 --warmup 5 > "$log" 2>&1 || fail "scale $wl N=$n" $? "$log"
        grep '^{' "$log"
    done
}

cmd=${1:-test}
shift || true
case "$cmd" in
    test) gpu_test "$@" ;;
    bench) bench "$@" ;;
    lines) lines ;;
    prof) prof "$@" ;;
    sq) sq "$@" ;;
    trace) trace "$@" ;;
    pmc) pmc "$@" ;;
    selfhalo) selfhalo ;;
    self20) self20 ;;
    trace20) trace20 ;;
    thin) thin ;;
    thintrace) thintrace ;;
    ab) ab "$@" ;;
    final) final ;;
    scale) scale "$@" ;;
    *) echo "unknown command $cmd"; exit 2 ;;
esac
