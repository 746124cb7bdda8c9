#!/usr/bin/env python3
"""Where the driver's timed region spends the time the kernels do not: the bench's
sequence (fill, warmup, prepare, timed run) at 32768^2, then the same timed run repeated
back to back, after an idle gap, and the kernels' own HIP-event time.

  python tools/timed_gap.py [--steps 20] [--warmup 5]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402

mm.lib()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    N = a.size
    e = mm.Engine(N, N)
    e.fill_random(0)
    e.add_diffuse(0, 0.1)

    def timed(label):
        mm.device_synchronize(0)
        t0 = time.perf_counter()
        e.run(a.steps)
        t1 = time.perf_counter()
        e.synchronize()
        mm.device_synchronize(0)
        t2 = time.perf_counter()
        print(json.dumps({"what": label, "enqueue_ms": round((t1 - t0) * 1e3, 3),
                          "total_ms": round((t2 - t0) * 1e3, 3)}), flush=True)

    e.run(a.warmup)
    e.prepare(a.steps)
    e.synchronize()
    timed("bench sequence: first timed run")
    timed("back to back")
    timed("back to back")
    time.sleep(1.0)
    timed("after 1 s idle")
    time.sleep(0.05)
    timed("after 50 ms idle")
    e.set_timing(True)
    e.run(a.steps)
    n, ms, _ = e.timing()
    e.set_timing(False)
    print(json.dumps({"what": "kernel events", "launches": n, "kernel_ms": round(ms, 3),
                      "plan": e.pass_plan(a.steps), "info_graph": e.info()["graph_state"]}))
    e.close()


if __name__ == "__main__":
    main()
