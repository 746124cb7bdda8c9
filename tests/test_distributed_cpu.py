"""Multi-process decomposition on CPU (gloo): the N>1 structure of the engine, checked
without GPUs.

Each rank owns the slab mm_partition_rows gives it, keeps `depth` ghost rows above and
below, and before every `depth` steps sends its first `depth` rows to rank-1 and its
last `depth` rows to rank+1 -- the exchange the engine does with ncclSend/ncclRecv
(mm_engine.hip halo_rccl; depth K for the K-step kernel, K <= 10). Steps are computed
with the oracle on the slab; the gathered grid must equal the single-process oracle
bit for bit (src/Model.hpp's row slabs, generalised to every cell and every step).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as tmp

from conftest import ORACLE, PKG


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def slab_steps(O, H, W, x0, h, rank, world, v_own, rate, steps, depth):
    """Advance this rank's slab `steps` steps, exchanging `depth` rows every `depth` steps."""
    import torch
    v = v_own.copy()
    done = 0
    while done < steps:
        k = min(depth, steps - done)
        # ghost rows from the neighbours (rows outside the grid stay zero / unused)
        up = np.zeros((k, W))
        down = np.zeros((k, W))
        reqs = []
        t_up, t_down = torch.zeros(k * W, dtype=torch.float64), torch.zeros(k * W, dtype=torch.float64)
        s_up = torch.tensor(v[:k].ravel(), dtype=torch.float64)       # kept alive until wait
        s_down = torch.tensor(v[h - k:].ravel(), dtype=torch.float64)
        if rank > 0:
            reqs.append(dist.isend(s_up, rank - 1, tag=1))
            reqs.append(dist.irecv(t_up, rank - 1, tag=2))
        if rank < world - 1:
            reqs.append(dist.isend(s_down, rank + 1, tag=2))
            reqs.append(dist.irecv(t_down, rank + 1, tag=1))
        for r in reqs:
            r.wait()
        if rank > 0:
            up = t_up.numpy().reshape(k, W)
        if rank < world - 1:
            down = t_down.numpy().reshape(k, W)
        # k steps on the extended slab [x0-k, x0+h+k): each step shrinks the valid band
        ext = np.vstack([up, v, down])
        lo = x0 - k
        for _ in range(k):
            n = ext.shape[0]
            vg = np.zeros((n + 2, W))
            vg[1:-1] = ext
            new = O.field_step_slab(H, W, lo, vg, rate)
            # rows outside the grid must stay inert: zero them like the engine's ghosts
            for i in range(n):
                if not (0 <= lo + i < H):
                    new[i] = 0.0
            ext = new
        v = ext[k:k + h]
        done += k
    return v


def worker(rank, world, port, H, W, rate, steps, depth, out_q):
    sys.path.insert(0, ORACLE)
    sys.path.insert(0, PKG)
    import oracle as O
    import mpimodel as mm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x0, h = mm.partition_rows(H, world, rank)
        v_own = O.fill_random(H, W, x0, h)  # keyed by global index: same input on every rank
        v = slab_steps(O, H, W, x0, h, rank, world, v_own, rate, steps, depth)
        gathered = [None] * world if rank == 0 else None
        dist.gather_object((x0, v), gathered, dst=0)
        if rank == 0:
            out_q.put(gathered)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H,W,steps,depth", [
    (2, 37, 53, 5, 1), (2, 40, 29, 6, 2), (3, 41, 33, 7, 2), (3, 30, 20, 4, 1),
    # the K-step kernel's depths (mm_engine.hip halo_depth): 3, 4 and 8 with ragged last
    # passes, and slabs exactly as thin as the depth (the engine caps K by min slab rows)
    (2, 40, 29, 9, 3), (3, 41, 33, 10, 4), (4, 16, 21, 9, 4), (2, 16, 19, 17, 8),
    (3, 13, 17, 7, 4),
    # the planner's deepest passes (K = 10): two passes of 10 on slabs of 12 and 13 rows
    (2, 25, 19, 20, 10),
])
def test_row_slabs_with_halo_exchange_bit_exact(O, world, H, W, steps, depth):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, H, W, 0.1, steps, depth, q))
             for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.vstack([v for _, v in sorted(gathered, key=lambda t: t[0])])
    want = O.field_step(O.fill_random(H, W), 0.1, steps=steps)
    assert np.array_equal(got, want)


def test_partition_covers_grid_without_overlap(mm):
    for H in (4096 * 8, 32768, 37):
        for G in (1, 2, 4, 8):
            parts = [mm.partition_rows(H, G, g) for g in range(G)]
            assert parts[0][0] == 0
            for (a, h), (b, _) in zip(parts, parts[1:]):
                assert a + h == b
            assert parts[-1][0] + parts[-1][1] == H
