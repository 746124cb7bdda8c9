#!/usr/bin/env python3
"""HIP-event time of one K-step pass per grid size and kernel (mm_passk_kernel at K, or
mm_wide_kernel at K), the table the pass planner's cost model is fitted to.

  python tools/kernel_table.py --sizes 32768x32768,16384x16384 --old 7,8,10 --wide 8,12,16,20
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402

mm.lib()


def one(H, W, k, wide, reps):
    env = {"MM_STEPS_PER_PASS": str(k), "MM_WIDE": "1" if wide else "0"}
    old = {key: os.environ.get(key) for key in env}
    os.environ.update(env)
    try:
        e = mm.Engine(H, W)
    finally:
        for key, v in old.items():
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v
    e.fill_random(0)
    e.add_diffuse(0, 0.1)
    e.run(k)
    e.set_timing(True)
    e.run(k * reps)
    n, ms, _ = e.timing()
    e.set_timing(False)
    info = e.info()
    kern, c, strips = e.pass_kernel(k)
    e.close()
    us = ms / n * 1e3
    return {"H": H, "W": W, "k": k, "kernel": kern, "cols": c, "strips": strips, "pass_us": round(us, 1),
            "us_per_step": round(us / k, 2), "GCUPS": round(H * W * k / us / 1e3, 1),
            "rows_per_wave": info["rows_per_wave"], "waves": info["waves_per_pass"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="32768x32768,16384x16384,8192x32768,4096x32768,4096x4096")
    ap.add_argument("--old", default="7,8,10")
    ap.add_argument("--wide", default="4,8,12,16,20")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    for sz in a.sizes.split(","):
        H, W = (int(x) for x in sz.split("x"))
        for k in [int(x) for x in a.old.split(",") if x]:
            print(json.dumps(one(H, W, k, False, a.reps)), flush=True)
        for k in [int(x) for x in a.wide.split(",") if x]:
            print(json.dumps(one(H, W, k, True, a.reps)), flush=True)


if __name__ == "__main__":
    main()
