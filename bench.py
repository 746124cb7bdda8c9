#!/usr/bin/env python3
"""Benchmark of the MI355X engine on the reference's headline metric.

metric  : cell-updates/s (GCUPS) of the generalised Exponencial flow step
          (BASELINE.json), whole job over all ranks, + % of the HBM roofline
workload: default "c3" = BASELINE.json configs[2], the north_star grid: 32768 x 32768 fp64
          cells, one Exponencial flow (rate 0.1, src/Main.cpp:33). With --gpus N the
          grid is cut into N row slabs, one per GPU, with the border rows exchanged over
          RCCL every K steps (strong scaling). Other workloads: c2 (4096^2 per GPU, weak:
          Infinity-Cache resident), c4 (16384^2 per GPU, weak), c5 (4 attributes, chained
          transfers + 4 diffusions, per-step sums).
step    : one pass of the flow over the whole grid (all passes of the program).
timing  : W untimed warmup steps, then exactly K steps on the production path (hipGraph
          replay of K-step kernel passes) bracketed by a barrier and a device-wide
          synchronize (hipDeviceSynchronize) on both sides; the max over ranks is reported. Inputs are resident in HBM
          (generated on the device) before timing. Then the same K steps again, launched
          eagerly with a HIP event pair around every step kernel on its own stream: the
          kernel's average duration for the roofline object.

Launch: python bench.py [--gpus 1] [--steps 1000] [--warmup 50]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
        (--halo host: the host transport over gloo, N ranks on however many GPUs exist)
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))

import mpimodel as mm  # noqa: E402

# Load the engine (and with it ROCm 7.2's libamdhip64 / librccl) BEFORE torch: torch
# bundles its own HIP 7.0 runtime and librccl.so.1 under the same sonames, and whichever
# is loaded first serves the whole process. With torch's RCCL the engine's halo path
# crashes; with ROCm's runtime torch.cuda sees no device. So the process runs on ROCm
# 7.2 only, torch is used for the launcher and the gloo control plane, and the device
# synchronize around the timed region is hipDeviceSynchronize via the engine
# (the same operation torch.cuda.synchronize performs).
mm.lib()

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
RATE = 0.1             # src/Main.cpp:33

WORKLOADS = {
    # name: (rows per GPU or global rows, cols, scaling, n_attr)
    "c2": dict(rows=4096, cols=4096, scaling="weak", n_attr=1,
               desc="4096x4096 fp64 per GPU, one Exponencial flow (BASELINE configs[1])"),
    "c3": dict(rows=32768, cols=32768, scaling="strong", n_attr=1,
               desc="32768x32768 fp64 global, row slabs (BASELINE configs[2])"),
    "c4": dict(rows=16384, cols=16384, scaling="weak", n_attr=1,
               desc="16384x16384 fp64 per GPU (BASELINE configs[3])"),
    "c5": dict(rows=4096, cols=4096, scaling="weak", n_attr=4,
               desc="4 attributes, 4 chained transfers + 4 diffusions, per-step sums "
                    "(BASELINE configs[4])"),
}

C5_FLOWS = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
            (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]
# other four-attribute programs for --program (measurements of the chain kernels; the C5
# line is C5_FLOWS): the same transfers in another order, and a pass with a post-chain
# (tests/test_gpu_parity.py WIDE_PROGRAMS[2] and [1])
PROGRAMS = {
    "c5": C5_FLOWS,
    "reordered": [C5_FLOWS[1], C5_FLOWS[0], C5_FLOWS[2], C5_FLOWS[3]] + C5_FLOWS[4:],
    "post": [(2, 0, 1, 0.1), (1, 0, 0, 0.1), (1, 2, 2, 0.2), (2, 3, 1, 0.05), (2, 2, -1, 0.01)],
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--self-halo", action="store_true",
                    help="N=1 only: run the RCCL halo path against itself (MM_SELF_HALO) to "
                         "price the exchange + interior/border split")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-baseline sample length (oracle port, rank 0, N=1)")
    ap.add_argument("--halo", default="rccl", choices=("rccl", "host"),
                    help="N>1: RCCL K-row exchange (one GPU per rank), or the host transport "
                         "over gloo between passes (any number of ranks on the GPUs present, "
                         "e.g. N ranks sharing one GPU)")
    ap.add_argument("--grid", type=int, nargs=2, metavar=("H", "W"),
                    help="tests: override the workload's grid")
    ap.add_argument("--dump", help="tests: save each rank's slab to DUMP.rank<r>.npy")
    ap.add_argument("--program", default="c5", choices=sorted(PROGRAMS),
                    help="c5 workload: the flow program (default C5's own)")
    return ap.parse_args()


def cpu_ranks():
    """Host cores for the CPU baseline: MM_CPU_RANKS, else min(16, cpu_count) -- the GPU
    box gives one GPU's job a 16-CPU share while os.cpu_count() shows the whole machine."""
    n = int(os.environ.get("MM_CPU_RANKS", "0"))
    return n if n > 0 else max(1, min(16, os.cpu_count() or 1))


def cpu_baseline(H, W, seconds):
    """The reference's CPU decomposition over the oracle's step (oracle/mm_cpu_mpi.c: row
    slabs, one MPI rank per core, blocking border-row exchange every step) on the same grid
    and inputs, as many whole steps as fit in about `seconds`. Without an MPI it falls back
    to the scalar single-core port (oracle/mm_oracle.c or_field_step)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    ranks = cpu_ranks()
    if os.path.exists(os.path.join(oracle.MPI_HOME, "bin", "mpirun")):
        r = oracle.cpu_mpi(H, W, RATE, seconds, ranks, timeout=max(120, 10 * seconds))
        return {"value": r["GCUPS"], "unit": "GCUPS", "cores": r["ranks"], "kind": "port",
                "sample": f"{r['steps']} timed steps (after {r['warmup_steps']} untimed) of the "
                          f"{H}x{W} fp64 grid, {r['ranks']} MPI ranks x 1 core, row slabs + "
                          f"blocking border-row MPI_Sendrecv per step (the reference's "
                          f"decomposition), oracle step (oracle/mm_cpu_mpi.c, -O3), "
                          f"{r['seconds']:.1f} s"}
    import numpy as np
    v = oracle.fill_random(H, W)
    o = np.empty_like(v)
    L = oracle.lib()
    ptr = oracle._ptr
    steps = 0
    t0 = time.perf_counter()
    while True:
        L.or_field_step(H, W, ptr(v), ptr(o), RATE)
        v, o = o, v
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 10000:
            break
    return {"value": H * W * steps / el / 1e9, "unit": "GCUPS", "cores": 1, "kind": "port",
            "sample": f"{steps} steps of the {H}x{W} fp64 grid, oracle/mm_oracle.c "
                      f"or_field_step (scalar C, -O2, no MPI found), {el:.1f} s"}


def cpu_baseline_program(H, W, na, flows, seconds):
    """C5's CPU baseline: the same reference decomposition as cpu_baseline (row slabs, one
    MPI rank per core, blocking border-row exchange before every diffusion) running the
    oracle's flow program (or_program_step's semantics) plus the per-step attribute sums
    combined in rank order (src/Model.hpp:88-92). Without an MPI: the scalar single-core
    or_program_step."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    ranks = cpu_ranks()
    if os.path.exists(os.path.join(oracle.MPI_HOME, "bin", "mpirun")):
        r = oracle.cpu_mpi(H, W, RATE, seconds, ranks, timeout=max(120, 10 * seconds),
                           program=flows)
        return {"value": r["GCUPS"], "unit": "GCUPS", "cores": r["ranks"], "kind": "port",
                "sample": f"{r['steps']} timed steps (after {r['warmup_steps']} untimed) of the "
                          f"{H}x{W} grid with {r['n_attr']} fp64 attributes and the C5 flow "
                          f"program ({r['n_flows']} flows) + per-step sums, {r['ranks']} MPI "
                          f"ranks x 1 core, row slabs + blocking border-row MPI_Sendrecv before "
                          f"every diffusion (the reference's decomposition), oracle step "
                          f"(oracle/mm_cpu_mpi.c, -O3), {r['seconds']:.1f} s"}
    import ctypes
    import numpy as np
    fields = [oracle.fill_random(H, W, seed=oracle.SEED + a) for a in range(na)]
    arr = (ctypes.c_void_p * na)(*[f.ctypes.data for f in fields])
    fl = (oracle.OrFlow * len(flows))(*[oracle.OrFlow(*f) for f in flows])
    scratch = np.empty((H, W), dtype=np.float64)
    L = oracle.lib()

    def step():
        L.or_program_step(H, W, na, arr, fl, len(flows), oracle._ptr(scratch))
        return [float(np.sum(f, dtype=np.float64)) for f in fields]

    step()  # untimed warm-up
    steps = 0
    t0 = time.perf_counter()
    while True:
        step()
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 1000:
            break
    return {"value": H * W * steps / el / 1e9, "unit": "GCUPS", "cores": 1, "kind": "port",
            "sample": f"{steps} steps of the {H}x{W} grid with {na} fp64 attributes and the "
                      f"C5 flow program + per-step sums, oracle/mm_oracle.c or_program_step "
                      f"(scalar C, one core, no MPI found), {el:.1f} s"}


def level_row_cycles(cols, n_diffuse=1, n_transfers=0, chain_kernel=0):
    """VALU cycles one wave issues per level-row of its strip: per diffusing
    attribute 5 fp64 instructions per column of a lane on average (4 cycles each on a SIMD:
    the box-sum step of oracle/mm_oracle.h -- the column triple 2 adds on an even row, 1 on
    the odd row after it, which reuses the pair's sum; the box sum 1.5 adds, the lane's
    columns paired alike; 2 fma) and the two fp64 DPP neighbour moves (4 v_mov_dpp, 2 cycles
    each); per transfer of a chain and
    column, 3 fp64 instructions (out = r*u_a, u_a - out, u_b + out) -- with compile-time
    operands (mm.MM_CHAIN_RING) and with chain_asm's run-time operands (mm.MM_CHAIN_RUNTIME)
    alike: chain_asm indexes the fp64 instructions' own operands, no moves."""
    del chain_kernel  # both chain kernels issue the same instructions per transfer
    diff = n_diffuse * (5 * cols * 4 + 4 * 2)
    return diff + n_transfers * cols * 3 * 4


def valu_roof(passes, h, W, kern_avg_ms, lr_cycles=None):
    """The K-step kernels' other roof: the steady-state loop's VALU cycles
    per SIMD. `passes`: (k, kernel, columns per lane, strips) of every launch the timed
    average covers (mm_pass_kernel); a launch runs k levels over every row of its strips
    (segment overlap, LDS hand-offs and the edge strips' slower body not counted), each
    level-row costing `lr_cycles(k, cols)` (level_row_cycles; default one diffusion). frac: the
    launches' mean cycles per SIMD / the mean launch's cycles at the 2.4 GHz peak clock.
    None unless every launch is a K-step kernel."""
    if not passes or kern_avg_ms <= 0 or any(kern not in (2, 3) for _, kern, _, _ in passes):
        return None
    lr = lr_cycles or (lambda k, cols: level_row_cycles(cols))
    cyc = sum(h * k * strips * lr(k, cols) / (256 * 4)
              for k, _, cols, strips in passes) / len(passes)
    return {"bound": "valu", "cycles_per_simd_per_launch": round(cyc), "peak_clock_mhz": 2400,
            "frac": round(cyc / (kern_avg_ms * 1e-3 * 2.4e9), 4)}


def make_line(*, workload, wl, N, ranks, H, W, h, na, steps, warmup, el, plan, info,
              kern_ms, n_launch, timing_steps, bytes_per_launch, passes, traffic, cons, halo,
              self_halo, lr_cycles=None, graph_captures_timed=None):
    """The driver's JSON line (no I/O): value = whole-job GCUPS = all ranks' cell-updates /
    the max-over-ranks wall time `el` of exactly `steps` steps."""
    gcups = H * W * steps / el / 1e9
    kern_avg_ms = kern_ms / max(n_launch, 1)
    spl = max(plan) if info["kernel"] in (2, 3) and plan else 1  # steps of the longest pass
    kname = {0: "mm_pass_kernel", 2: "mm_passk_kernel", 3: "mm_wide_kernel"}[info["kernel"]]
    achieved = bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9 if kern_ms > 0 else None
    if info["graph_state"] == 1:
        path = f"hipGraph replay ({info['graph_launches']} graph launches)"
    elif info["graph_state"] == -1:
        path = f"eager launches: graph capture refused ({info['graph_note']})"
    else:
        path = "eager launches (no graph)"
    if N == 1:
        par = "row-slab x1" + (" (self-halo: RCCL exchange with itself)" if self_halo else "")
    elif halo == "host":
        par = (f"row-slab x{N} ranks on {ranks['gpus']} GPU(s), host halo: K border rows "
               f"over gloo between passes")
    else:
        par = f"row-slab x{N} + RCCL halo"
    plan_s = '+'.join(map(str, plan)) if len(plan) <= 8 else f"{spl} (x{len(plan)})"
    line = {
        "metric": "cell-updates/s (GCUPS) per step + % of HBM roofline",
        "value": round(gcups, 3),
        "unit": "GCUPS",
        "n_gpus": ranks["gpus"],
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(el * 1e3 / steps, 5),
        "higher_is_better": True,
        "scaling": wl["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: v0 = 1 + U[0,1) from splitmix64 keyed by global cell index, "
                "seed 0x4D50494D, generated on the device",
        "config": {"workload": f"{workload}: {wl['desc']}", "grid": [H, W],
                   "path": f"{path}, {kname}, {len(plan)} pass(es) of {plan_s} fused steps",
                   "ranks": N, "rows_per_gpu": h, "n_attr": na, "rate": RATE,
                   "parallelism": par,
                   "passes_per_step": info["n_passes"],
                   "rows_per_wave": info["rows_per_wave"]},
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
            "traffic": traffic,
            "kernel": kname,
            "kernel_avg_us": round(kern_avg_ms * 1e3, 3),
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "steps_per_launch": spl,
            "launches_per_step": n_launch / max(timing_steps, 1),
            # BASELINE.md's formula: GCUPS x 16 B x A / 8 TB/s (per GPU); above 1.0
            # when K steps share one HBM round trip (temporal blocking)
            "equivalent_frac": round(gcups / ranks["gpus"] * 16.0 * na / HBM_PEAK_GBS, 4),
        },
        "check": {"total_rel_drift": cons},
    }
    v = valu_roof(passes, h, W, kern_avg_ms, lr_cycles)
    if v:
        line["roofline"]["valu"] = v
    if graph_captures_timed is not None:
        # graphs captured inside the timed region (0: every graph was prepared ahead)
        line["config"]["graph_captures_timed"] = graph_captures_timed
    return line


def gloo_exchange(rank, N):
    """Host transport of the K-row halo between passes (src/Model.hpp:202-204,224-235 made
    whole-row and K deep): this slab's first rows go to rank-1, its last rows to rank+1, the
    neighbours' rows come back for the ghost rows above / below."""
    import torch
    import torch.distributed as dist

    def ex(top, bottom, k):
        reqs, above, below = [], None, None
        if rank > 0:
            above = torch.empty(top.shape, dtype=torch.float64)
            reqs += [dist.isend(torch.from_numpy(top), rank - 1), dist.irecv(above, rank - 1)]
        if rank < N - 1:
            below = torch.empty(bottom.shape, dtype=torch.float64)
            reqs += [dist.isend(torch.from_numpy(bottom), rank + 1), dist.irecv(below, rank + 1)]
        for r in reqs:
            r.wait()
        return (None if above is None else above.numpy(),
                None if below is None else below.numpy())
    return ex


def main():
    args = parse()
    wl = WORKLOADS[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("--gpus N > 1 needs one process per GPU (torch.distributed.run)")
    N = world
    host = N > 1 and args.halo == "host"

    import torch
    import torch.distributed as dist
    if N > 1:
        dist.init_process_group("gloo")  # control plane (and the host halo); data on RCCL

    if wl["scaling"] == "weak":
        H = wl["rows"] * N
    else:
        H = wl["rows"]
    W = wl["cols"]
    if args.grid:  # tests: a small grid through the same machinery
        H, W = args.grid
    x0, h = mm.partition_rows(H, N, rank)

    ndev = max(1, mm.device_count())
    dev = local % ndev if host else local
    if host:
        eng = mm.Engine(H, W, x0, h, n_attr=wl["n_attr"], device=dev, rank=rank, nranks=N,
                        halo_mode=mm.MM_HALO_HOST)
    elif N > 1:
        ids = [mm.comm_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        eng = mm.Engine(H, W, x0, h, n_attr=wl["n_attr"], device=local, rank=rank, nranks=N,
                        halo_mode=mm.MM_HALO_RCCL, comm_id_bytes=ids[0])
    elif args.self_halo:
        os.environ["MM_SELF_HALO"] = "1"
        eng = mm.Engine(H, W, n_attr=wl["n_attr"], device=local, halo_mode=mm.MM_HALO_RCCL,
                        comm_id_bytes=mm.comm_id())
    else:
        eng = mm.Engine(H, W, n_attr=wl["n_attr"], device=local)
    sync = lambda: mm.device_synchronize(dev)  # noqa: E731
    exchange = gloo_exchange(rank, N) if host else None

    def run(n, reduce_every):
        if host:
            mm.run_host_halo(eng, n, exchange, reduce_every)
        else:
            eng.run(n, reduce_every)

    na = wl["n_attr"]
    for a in range(na):
        eng.fill_random(a, seed=mm.SEED + a)
    flows = PROGRAMS[args.program]
    if args.workload == "c5":
        for kind, a, b, r in flows:
            if kind == 1:
                eng.add_diffuse(a, r)
            else:
                eng.add_transfer(a, b, r)
        reduce_every = 1
    else:
        eng.add_diffuse(0, RATE)
        reduce_every = 0

    def global_total(e):
        # total over attributes and ranks: what the flows conserve (src/Model.hpp:95)
        t = torch.tensor([float(sum(e.sums()))], dtype=torch.float64)
        if N > 1:
            dist.all_reduce(t)
        return float(t.item())

    s_before = global_total(eng)

    # the timed run's one-time work -- its hipGraphs (both buffer parities) and the plan of
    # its eager passes -- done ahead (mm_prepare runs no step); then the warmup steps, which
    # end right before the timed region: an idle GPU drops its clock within milliseconds,
    # and the first ~1 ms of a run after an idle gap is slower (tools/timed_gap.py,
    # profiles/r03/timed_gap.log: 9.5-9.9 ms for the 20-step run after idle, 8.3-8.4 ms
    # back to back)
    if not host:
        eng.prepare(args.steps, reduce_every)
    run(args.warmup, reduce_every)
    eng.synchronize()
    graphs_before = eng.info()["graph_count"]

    # timed region: the production path
    if N > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run(args.steps, reduce_every)
    eng.synchronize()
    sync()
    el = time.perf_counter() - t0
    graphs_timed = eng.info()["graph_count"] - graphs_before
    if N > 1:
        dist.barrier()
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    s_after = global_total(eng)
    if args.dump:  # tests: this rank's slab after warmup + steps
        import numpy as np
        np.save(f"{args.dump}.rank{rank}.npy", np.stack([eng.download(a) for a in range(na)]))

    # kernel pass: the timed run's own passes (mm_pass_plan), repeated eagerly until at
    # least 3 launches, each step kernel bracketed by HIP events on its stream -- the
    # launches rocprofv3 averages
    plan = eng.pass_plan(args.steps)
    reps = max(1, -(-3 // max(len(plan), 1)))
    eng.set_timing(True)
    for _ in range(reps):
        run(args.steps, reduce_every)
    n_launch, kern_ms, bytes_per_launch = eng.timing()
    eng.set_timing(False)
    info = eng.info()
    passes = [(k, *eng.pass_kernel(k)) for k in plan] * reps
    gpus = [dev] if N == 1 else None
    if N > 1:
        got = [None] * N
        dist.all_gather_object(got, dev)
        gpus = got

    if rank == 0:
        spl = max(plan) if info["kernel"] in (2, 3) and plan else 1
        kname = {0: "mm_pass_kernel", 2: "mm_passk_kernel", 3: "mm_wide_kernel"}[info["kernel"]]
        traffic, traffic_src = None, None
        tf = os.path.join(REPO, "profiles", "pmc_traffic.json")
        # only when it was measured on this kernel and on the workload's own grid
        if os.path.exists(tf) and not args.grid:
            with open(tf) as f:
                pmc = json.load(f)
            key = f"{args.workload}_n{N}_k{spl}"
            if kname in pmc.get(f"{key}_kernel", ""):
                traffic = pmc.get(f"{key}_bytes_per_launch")
                # not measured in this run: the PMC passes of tools/gpu.sh prof on this
                # kernel and workload, recorded by tools/pmc_traffic.py
                traffic_src = (f"profiles/pmc_traffic.json {key} (rocprofv3 FETCH_SIZE / "
                               f"WRITE_SIZE passes, {pmc.get(f'{key}_source', 'unrecorded')})")
        lr = None
        if na > 1:  # C5: the program's diffusions and transfers (K = 8: its chain kernel)
            n_diff = sum(1 for f in flows if f[0] == 1)
            n_tr = sum(1 for f in flows if f[0] == 2)
            ck = info["chain_kernel"]
            lr = lambda k, cols: level_row_cycles(  # noqa: E731
                cols, n_diff, n_tr, ck if k == info["steps_per_launch"] else 3)
        line = make_line(workload=args.workload, wl=wl, N=N, ranks={"gpus": len(set(gpus))},
                         H=H, W=W, h=h, na=na, steps=args.steps, warmup=args.warmup, el=el,
                         plan=plan, info=info, kern_ms=kern_ms, n_launch=n_launch,
                         timing_steps=reps * args.steps, bytes_per_launch=bytes_per_launch, passes=passes, traffic=traffic,
                         cons=abs(s_after - s_before) / abs(s_before), halo=args.halo,
                         self_halo=args.self_halo, lr_cycles=lr,
                         graph_captures_timed=None if host else graphs_timed)
        line["roofline"]["traffic_source"] = traffic_src
        if args.workload == "c5" and args.program != "c5":
            line["config"]["program"] = f"{args.program}: {flows}"
        if N == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(wl["rows"], W, args.cpu_seconds) \
                if na == 1 else cpu_baseline_program(wl["rows"], W, na, flows,
                                                     args.cpu_seconds)
        print(json.dumps(line), flush=True)
    eng.close()
    if N > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
