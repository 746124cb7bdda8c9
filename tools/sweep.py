#!/usr/bin/env python3
"""Tuning sweep of the step kernel (rows per wave x kernel variant) in ONE process,
interleaved rounds (cdna_hip_programming.md 5.4 rule 24). Prints one JSON line per
configuration with the median kernel time over rounds. Each variant's result is
also checked bit-exact against variant 0 on the same input."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import numpy as np  # noqa: E402

import mpimodel as mm  # noqa: E402


def make(H, W, th, variant, fuse):
    os.environ["MM_ROWS_PER_WAVE"] = str(th)
    os.environ["MM_KERNEL_VARIANT"] = str(variant)
    os.environ["MM_FUSE"] = str(fuse)
    e = mm.Engine(H, W)
    e.fill_random(0)
    e.add_diffuse(0, 0.1)
    return e


def time_engine(e, steps):
    e.set_timing(True)
    e.run(steps)
    n, ms, b = e.timing()
    e.set_timing(False)
    return ms / n, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--ths", default="8,16,32")
    ap.add_argument("--variants", default="0,1,3")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--fuse", default="0,1")
    a = ap.parse_args()
    H = W = a.size
    ths = [int(x) for x in a.ths.split(",")]
    vs = [int(x) for x in a.variants.split(",")]
    fs = [int(x) for x in a.fuse.split(",")]
    ref = None
    res = {}
    for rnd in range(a.rounds):
        for f in fs:
            for th in ths:
                if f and th == 32:
                    continue
                for v in vs:
                    if f and v == 3:
                        continue
                    e = make(H, W, th, v, f)
                    e.run(10)
                    t, b = time_engine(e, a.steps)
                    per = e.info()["steps_per_launch"]
                    res.setdefault((f, th, v, per), []).append(t)
                    if rnd == 0:
                        out = e.download()
                        if ref is None:
                            ref = out
                        elif not np.array_equal(out, ref):
                            print(json.dumps({"MISMATCH": [f, th, v]}), flush=True)
                    e.close()
    for (f, th, v, per), ts in sorted(res.items(), key=lambda kv: statistics.median(kv[1]) / kv[0][3]):
        med = statistics.median(ts)
        print(json.dumps({"size": H, "fuse": f, "th": th, "variant": v,
                          "us_per_step": round(med * 1e3 / per, 2),
                          "GCUPS": round(H * W * per / (med * 1e-3) / 1e9, 1),
                          "kernel_us_med": round(med * 1e3, 2),
                          "GBps_per_launch": round(16.0 * H * W / (med * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
