#!/usr/bin/env python3
"""Price the RCCL halo path on one GPU (MM_SELF_HALO: the rank exchanges border rows
with itself). Prints wall time per step for eager / graph and fused / single-step
launches, with and without the exchange. Run under rocprofv3 --kernel-trace to see
whether the RCCL kernel overlaps the interior kernel."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402


def run(n, steps, halo, graph, fuse):
    os.environ["MM_SELF_HALO"] = "1" if halo else "0"
    os.environ["MM_GRAPH"] = str(graph)
    os.environ["MM_FUSE"] = str(fuse)
    kw = dict(halo_mode=mm.MM_HALO_RCCL, comm_id_bytes=mm.comm_id()) if halo else {}
    e = mm.Engine(n, n, **kw)
    e.fill_random(0)
    e.add_diffuse(0, 0.1)
    e.run(20)
    e.synchronize()
    t0 = time.perf_counter()
    e.run(steps)
    e.synchronize()
    dt = (time.perf_counter() - t0) / steps
    e.close()
    return dt


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    for halo in (0, 1):
        for graph in (0, 1):
            for fuse in (0, 1):
                dt = run(n, steps, halo, graph, fuse)
                print(json.dumps({"n": n, "halo": halo, "graph": graph, "fuse": fuse,
                                  "us_per_step": round(dt * 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
