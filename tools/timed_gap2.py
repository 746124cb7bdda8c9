#!/usr/bin/env python3
"""The 20-step timed run after different warmups (what the ~1 ms between the driver's
timed region and its kernels is): each scenario idles 0.3 s, runs its warmup, then times
the 20-step run (host clock around run + device sync) and repeats it back to back.

  python tools/timed_gap2.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402

mm.lib()
N, STEPS = 32768, 20


def timed(e):
    mm.device_synchronize(0)
    t0 = time.perf_counter()
    e.run(STEPS)
    e.synchronize()
    mm.device_synchronize(0)
    return round((time.perf_counter() - t0) * 1e3, 3)


def main():
    e = mm.Engine(N, N)
    e.fill_random(0)
    e.add_diffuse(0, 0.1)
    s = mm.Engine(4096, 32768)  # scratch slab: the same kernel on other buffers
    s.fill_random(0)
    s.add_diffuse(0, 0.1)
    e.prepare(STEPS)
    scenarios = {
        "warmup 5 steps (bench)": lambda: e.run(5),
        "warmup 5 + one 20-step pass": lambda: (e.run(5), e.run(20)),
        "warmup 5 + 20-step pass on a scratch slab": lambda: (e.run(5), s.run(20), s.run(20)),
        "warmup 40 steps": lambda: e.run(40),
        "no warmup": lambda: None,
    }
    for rep in range(2):
        for name, warm in scenarios.items():
            time.sleep(0.3)
            warm()
            e.synchronize()
            s.synchronize()
            a = timed(e)
            b = timed(e)
            print(json.dumps({"rep": rep, "scenario": name, "timed_ms": a, "again_ms": b}),
                  flush=True)
    e.set_timing(True)
    e.run(STEPS)
    n, ms, _ = e.timing()
    print(json.dumps({"kernel_ms": round(ms / n, 3), "plan": e.pass_plan(STEPS),
                      "plan5": e.pass_plan(5)}))


if __name__ == "__main__":
    main()
