#!/usr/bin/env python3
"""Probe: can two RCCL ranks share the one GPU of the test box? If they can, run the real-
neighbour K-row exchange (halo_rccl's r-1 / r+1 branches, which a single rank never takes)
on a small grid and compare the gathered slabs with the oracle.

  python tools/rccl_same_gpu.py [H W steps]

Two processes (spawned, not torchrun), one engine each, slab g of mm_partition_rows on
device 0, MM_HALO_RCCL with a comm id from rank 0 passed through a file. Prints one JSON
line per rank and a final verdict line.
"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(rank, nranks, H, W, steps, tmp):
    sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
    import numpy as np
    import mpimodel as mm
    mm.lib()
    idf = os.path.join(tmp, "id")
    if rank == 0:
        with open(idf + ".tmp", "wb") as f:
            f.write(mm.comm_id())
        os.rename(idf + ".tmp", idf)
    else:
        import time
        for _ in range(600):
            if os.path.exists(idf):
                break
            time.sleep(0.1)
    cid = open(idf, "rb").read()
    x0, h = mm.partition_rows(H, nranks, rank)
    out = {"rank": rank}
    try:
        with mm.Engine(H, W, x0, h, device=0, rank=rank, nranks=nranks,
                       halo_mode=mm.MM_HALO_RCCL, comm_id_bytes=cid) as e:
            e.fill_random(0)
            e.add_diffuse(0, 0.1)
            e.run(steps, 1)
            e.synchronize()
            np.save(os.path.join(tmp, f"slab{rank}.npy"), e.download())
            np.save(os.path.join(tmp, f"hist{rank}.npy"), e.sums_history())
            out["info"] = {k: v for k, v in e.info().items() if k in (
                "kernel", "steps_per_launch", "graph_state", "graph_launches", "graph_note")}
        out["ok"] = True
    except Exception as ex:  # RCCL refusing two ranks on one device lands here
        out["ok"] = False
        out["error"] = str(ex)[:400]
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        r, n, H, W, s = map(int, sys.argv[2:7])
        child(r, n, H, W, s, sys.argv[7])
        return
    H, W, steps = (int(a) for a in (sys.argv[1:4] if len(sys.argv) >= 4 else (301, 700, 25)))
    tmp = tempfile.mkdtemp()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    ps = [subprocess.Popen([sys.executable, __file__, "--child", str(r), "2", str(H), str(W),
                            str(steps), tmp], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True, env=env) for r in range(2)]
    outs = []
    for p in ps:
        try:
            o, _ = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
            o += "\n{\"timeout\": true}"
        outs.append(o)
        print(o.strip().splitlines()[-1] if o.strip() else "(no output)", flush=True)
    verdict = {"two_ranks_one_gpu": all('"ok": true' in o for o in outs)}
    if verdict["two_ranks_one_gpu"]:
        import numpy as np
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        got = np.vstack([np.load(os.path.join(tmp, f"slab{r}.npy")) for r in range(2)])
        want = O.field_step(O.fill_random(H, W), 0.1, steps=steps)
        verdict["bit_exact"] = bool(np.array_equal(got, want))
        verdict["cells_differing"] = int(np.count_nonzero(got != want))
    print(json.dumps(verdict), flush=True)


if __name__ == "__main__":
    main()
