#!/usr/bin/env python3
"""Is the K = 20 pass's clock set by the data? The same pass (32768^2, default plan: one
mm_wide_kernel K = 20 launch per 20 steps) on the reference's uniform 1.0 initial state,
on zeros and on the bench's random fill, each warmed for 40 steps and then HIP-event
timed over 3 launches; two rounds in alternating order.

  python tools/power_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402

mm.lib()
N = 32768


def one(e, kind):
    if kind == "random":
        e.fill_random(0)
    else:
        e.fill(0, mm.MM_FILL_UNIFORM, 1.0 if kind == "uniform 1.0" else 0.0)
    e.run(40)
    e.set_timing(True)
    e.run(60)
    n, ms, _ = e.timing()
    e.set_timing(False)
    e.synchronize()
    return {"fill": kind, "launches": n, "pass_us": round(1e3 * ms / n, 1)}


def main():
    e = mm.Engine(N, N)
    e.add_diffuse(0, 0.1)
    for order in (("random", "uniform 1.0", "zeros"), ("zeros", "uniform 1.0", "random")):
        for kind in order:
            print(json.dumps(one(e, kind)), flush=True)
    e.close()


if __name__ == "__main__":
    main()
