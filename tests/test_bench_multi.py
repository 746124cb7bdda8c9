"""bench.py's N>1 machinery.

CPU (gloo, no GPU): the JSON line's multi-rank fields -- n_gpus, ranks, rows_per_gpu,
scaling, value from the max-over-ranks time -- for RCCL runs (one GPU per rank, c3 strong /
c4 weak) and host-halo runs (N ranks sharing one GPU); and the host transport's K-row
exchange between ranks (bench.gloo_exchange), world sizes 2 and 4.

GPU: `torchrun --nproc-per-node N bench.py --gpus N --halo host` on the one GPU, N = 2 and 4
ranks (each one engine slab, K border rows moved over gloo before every pass: the engine's
split schedule across processes, bench.py's barrier, max-reduce and global_total), on a
small grid: the gathered slabs bit-exact against the oracle's single-process steps.
Reference: src/Model.hpp:70-95 (slabs, border exchange, rank-order sums).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as tmp

from conftest import REPO
from test_distributed_cpu import free_port

INFO = {"kernel": 3, "graph_state": 1, "graph_launches": 1, "graph_note": "", "n_passes": 1,
        "rows_per_wave": 2535}


def line_for(bench, workload, N, gpus, halo="rccl", el=0.01, steps=20):
    wl = bench.WORKLOADS[workload]
    H = wl["rows"] * N if wl["scaling"] == "weak" else wl["rows"]
    W = wl["cols"]
    _, h = bench.mm.partition_rows(H, N, 0)
    return bench.make_line(workload=workload, wl=wl, N=N, ranks={"gpus": gpus}, H=H, W=W, h=h,
                           na=1, steps=steps, warmup=5, el=el, plan=[20], info=INFO,
                           kern_ms=8.0, n_launch=1, timing_steps=steps,
                           bytes_per_launch=16.0 * h * W,
                           passes=[(20, 3, 4, 152)], traffic=None, cons=0.0, halo=halo,
                           self_halo=False), H, W, h


@pytest.mark.parametrize("workload,N", [("c3", 1), ("c3", 2), ("c3", 8), ("c4", 4), ("c2", 8)])
def test_line_fields_rccl(workload, N):
    import bench
    d, H, W, h = line_for(bench, workload, N, gpus=N)
    assert d["n_gpus"] == N and d["config"]["ranks"] == N
    assert d["scaling"] == bench.WORKLOADS[workload]["scaling"]
    assert d["config"]["grid"] == [H, W]
    if workload == "c3":  # strong: the global grid is fixed, each GPU holds H/N rows
        assert H == 32768 and h == 32768 // N
    else:  # weak: rows per GPU fixed
        assert h == bench.WORKLOADS[workload]["rows"] and H == h * N
    # whole-job throughput over all ranks, from the max-over-ranks wall time
    assert abs(d["value"] - H * W * 20 / 0.01 / 1e9) <= 1e-3 * d["value"]
    assert d["ms_per_step"] == pytest.approx(0.5)
    assert ("RCCL halo" in d["config"]["parallelism"]) == (N > 1)
    assert d["roofline"]["equivalent_frac"] == pytest.approx(d["value"] / N * 16 / 8000, rel=1e-3)
    assert d["roofline"]["valu"]["bound"] == "valu"


@pytest.mark.parametrize("N", [2, 4])
def test_line_fields_host_halo(N):
    import bench
    d, H, W, h = line_for(bench, "c3", N, gpus=1, halo="host")
    assert d["n_gpus"] == 1 and d["config"]["ranks"] == N and d["config"]["rows_per_gpu"] == h
    assert "host halo" in d["config"]["parallelism"] and f"x{N} ranks on 1 GPU" in \
        d["config"]["parallelism"]
    assert d["roofline"]["equivalent_frac"] == pytest.approx(d["value"] * 16 / 8000, rel=1e-3)


def test_valu_roof_mixed_plan():
    """The VALU roof averages the launches of a mixed plan (7 + 7 + 6) instead of dropping it."""
    import bench
    h, W = 4096, 4096
    p = [(7, 2, 2, 35), (7, 2, 2, 35), (6, 2, 2, 34)]
    v = bench.valu_roof(p, h, W, 0.08)
    want = sum(h * k * s * (5 * c * 4 + 8) / 1024 for k, _, c, s in p) / 3
    assert v["cycles_per_simd_per_launch"] == round(want)
    assert v["frac"] == pytest.approx(want / (0.08e-3 * 2.4e9), rel=1e-3)
    assert bench.valu_roof([(1, 0, 1, 0)], h, W, 0.08) is None


def test_valu_roof_four_attributes():
    """C5's line carries a VALU roof too: per level-row of a lane 4 diffusions (5 fp64 per
    column on average + 2 fp64 DPP moves each) and 4 transfers (3 fp64 per column; with
    run-time operands no more with chain_asm) -- 288 cycles at 2 columns."""
    import bench
    assert bench.level_row_cycles(4) == 88
    assert bench.level_row_cycles(2, 4, 4, 2) == 4 * (40 + 8) + 4 * 2 * 12 == 288
    assert bench.level_row_cycles(2, 4, 4, 3) == 288
    h, W = 4096, 4096
    info = dict(INFO, chain_kernel=2, steps_per_launch=8)
    lr = lambda k, cols: bench.level_row_cycles(cols, 4, 4, 2 if k == 8 else 1)  # noqa: E731
    d = bench.make_line(workload="c5", wl=bench.WORKLOADS["c5"], N=1, ranks={"gpus": 1}, H=h,
                        W=W, h=h, na=4, steps=1000, warmup=5, el=0.06, plan=[8] * 125,
                        info=info, kern_ms=0.43 * 125, n_launch=125, timing_steps=1000,
                        bytes_per_launch=64.0 * h * W, passes=[(8, 3, 2, 37)] * 125,
                        traffic=None, cons=0.0, halo="rccl", self_halo=False, lr_cycles=lr,
                        graph_captures_timed=0)
    v = d["roofline"]["valu"]
    want = h * 8 * 37 * 288 / 1024
    assert v["cycles_per_simd_per_launch"] == round(want)
    assert v["frac"] == pytest.approx(want / (0.43e-3 * 2.4e9), rel=1e-3)
    assert d["config"]["graph_captures_timed"] == 0


def _exchange_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    ex = bench.gloo_exchange(rank, world)
    k, W = 3, 7
    top = np.full((1, k, W), 100.0 * rank + 1)
    bottom = np.full((1, k, W), 100.0 * rank + 2)
    above, below = ex(top, bottom, k)
    res = {"above": None if above is None else float(above.mean()),
           "below": None if below is None else float(below.mean()),
           "shape": None if above is None else list(above.shape)}
    with open(f"{out}.{rank}.json", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_exchange(tmp_path, world):
    out = str(tmp_path / "ex")
    tmp.start_processes(_exchange_worker, args=(world, free_port(), out), nprocs=world,
                        join=True, start_method="spawn")
    for r in range(world):
        with open(f"{out}.{r}.json") as f:
            res = json.load(f)
        # the ghost rows above come from rank-1's LAST rows, those below from rank+1's FIRST
        assert res["above"] == (None if r == 0 else 100.0 * (r - 1) + 2)
        assert res["below"] == (None if r == world - 1 else 100.0 * (r + 1) + 1)
        if r > 0:
            assert res["shape"] == [1, 3, 7]


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,steps,workload", [(2, 300, 1000, 23, "c3"),
                                                  (4, 301, 700, 17, "c3"),
                                                  (2, 130, 300, 5, "c5")])
def test_host_halo_bench_bit_exact(gpu, O, tmp_path, N, H, W, steps, workload):
    dump = str(tmp_path / "slab")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={N}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", str(N), "--halo", "host",
           "--workload", workload, "--grid", str(H), str(W), "--steps", str(steps),
           "--warmup", "0", "--dump", dump]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["ranks"] == N and d["steps"] == steps
    assert d["check"]["total_rel_drift"] <= 1e-12
    got = np.concatenate([np.load(f"{dump}.rank{r}.npy") for r in range(N)], axis=1)
    if workload == "c5":
        import bench
        fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
        want = np.stack(O.program_step(fields, bench.C5_FLOWS, steps=steps))
    else:
        want = O.field_step(O.fill_random(H, W), 0.1, steps=steps)[None]
    assert got.shape == want.shape
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))
