#!/usr/bin/env python3
"""Level-split kernel (mm_wide_kernel, MM_WIDE=1) against the oracle and against
mm_passk_kernel: bit-exactness at every K on awkward shapes, then the HIP-event kernel time
of one pass at --size^2.

  python tools/wide_probe.py --size 32768 --ks 8,12,16,20
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import mpimodel as mm  # noqa: E402

mm.lib()
import oracle as O  # noqa: E402


def engine(H, W, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return mm.Engine(H, W)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def check(ks, shapes):
    bad = 0
    for H, W in shapes:
        v0 = O.fill_random(H, W)
        want = {}
        ref = v0
        for s in range(1, 2 * max(ks) + 4):
            ref = O.field_step(ref, 0.3)
            want[s] = ref
        for k in ks:
            e = engine(H, W, {"MM_WIDE": 1, "MM_STEPS_PER_PASS": k})
            e.fill_random(0)
            e.add_diffuse(0, 0.3)
            info = e.info()
            done = 0
            for n in (k, k + 3):
                e.run(n)
                done += n
                ok = np.array_equal(e.download(), want[done])
                if not ok:
                    bad += 1
                    d = np.argwhere(e.download() != want[done])
                    print(json.dumps({"shape": [H, W], "k": k, "steps": done, "ok": False,
                                      "kernel": info["kernel"], "ndiff": int(len(d)),
                                      "first": d[:4].tolist()}), flush=True)
            e.close()
        print(json.dumps({"shape": [H, W], "checked": ks}), flush=True)
    return bad


def sums_check(k):
    import math
    H, W, steps = 300, 700, 2 * k
    v = O.fill_random(H, W)
    e = engine(H, W, {"MM_WIDE": 1, "MM_STEPS_PER_PASS": k})
    e.upload(v)
    e.add_diffuse(0, 0.1)
    e.run(steps, 1)
    hist = e.sums_history()
    got = e.download()
    e.close()
    ref = v
    worst = 0.0
    for s in range(steps):
        ref = O.field_step(ref, 0.1)
        want = math.fsum(ref.ravel())
        worst = max(worst, abs(hist[s, 0] - want) / want)
    ok = np.array_equal(got, ref) and worst <= 1e-12
    print(json.dumps({"sums_k": k, "ok": bool(ok), "worst_rel": worst}), flush=True)
    return 0 if ok else 1


def perf(size, k, wide, steps_mult=2):
    env = {"MM_STEPS_PER_PASS": k}
    if wide:
        env["MM_WIDE"] = 1
    e = engine(size, size, env)
    e.fill_random(0)
    e.add_diffuse(0, 0.1)
    e.run(k)
    e.set_timing(True)
    e.run(k * steps_mult)
    n, ms, b = e.timing()
    e.set_timing(False)
    info = e.info()
    e.close()
    us = ms / n * 1e3
    r = {"size": size, "k": k, "wide": wide, "kernel": info["kernel"], "kernel_us": round(us, 1),
         "us_per_step": round(us / k, 2), "GCUPS": round(size * size * k / us / 1e3, 1),
         "GBps_pass": round(b / us / 1e3, 1), "rows": info["rows_per_wave"],
         "waves": info["waves_per_pass"], "slots": info["seg_waves_per_cu"]}
    print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--ks", default="4,8,12,16,20")
    ap.add_argument("--old", default="8,10")
    ap.add_argument("--skip-check", action="store_true")
    a = ap.parse_args()
    ks = [int(x) for x in a.ks.split(",") if x]
    bad = 0
    if not a.skip_check:
        shapes = [(1, 1), (2, 3), (5, 2), (37, 53), (130, 257), (64, 1000), (300, 233),
                  (45, 700), (257, 512), (70, 1025)]
        bad += check(ks, shapes)
        for k in ks:
            bad += sums_check(k)
        print(json.dumps({"check_failures": bad}), flush=True)
    for k in [int(x) for x in a.old.split(",") if x]:
        perf(a.size, k, False)
    for k in ks:
        perf(a.size, k, True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
