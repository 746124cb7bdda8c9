#!/usr/bin/env python3
"""Tuning sweep of the single-attribute step kernels in ONE process, interleaved rounds
(cdna_hip_programming.md 5.4 rule 24). Each configuration is a set of engine environment
variables (MM_FUSE, MM_PASSK, MM_STEPS_PER_PASS, MM_ROWS_PER_WAVE[_K|2],
MM_KERNEL_VARIANT, MM_XCD_REMAP). Prints one JSON line per configuration with the
median kernel time per launch (HIP events) and the GCUPS it implies, fastest first.
Every configuration's result is checked bit-exact against the first one."""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import numpy as np  # noqa: E402

import mpimodel as mm  # noqa: E402

ENV_KEYS = ("MM_FUSE", "MM_PASSK", "MM_STEPS_PER_PASS", "MM_ROWS_PER_WAVE",
            "MM_ROWS_PER_WAVE2", "MM_KERNEL_VARIANT", "MM_XCD_REMAP", "MM_SEG_WAVES",
            "MM_SEG_EDGE", "MM_BORDER_SEG", "MM_SELF_HALO", "MM_PASS_PLAN")

PRESETS = {
    # segment-scheduled K-step kernel: K x waves per slot x edge-strip length x
    # non-temporal stores, plus the older kernels for comparison
    "seg": [{"MM_FUSE": 0}, {"MM_PASSK": 0}]
           + [{"MM_STEPS_PER_PASS": k, "MM_SEG_WAVES": f, "MM_KERNEL_VARIANT": nt}
              for k in (2, 3, 4) for f in (1, 2) for nt in (0, 1)]
           + [{"MM_STEPS_PER_PASS": 4, "MM_SEG_EDGE": 1.0}, {"MM_STEPS_PER_PASS": 4, "MM_SEG_WAVES": 4},
              {"MM_STEPS_PER_PASS": 4, "MM_SEG_WAVES": 0.75}, {"MM_STEPS_PER_PASS": 4, "MM_XCD_REMAP": 1}],
    "k-small": [{"MM_PASSK": 0}] + [{"MM_STEPS_PER_PASS": k} for k in (1, 2, 3, 4)],
}


def make(H, W, env):
    saved = {k: os.environ.pop(k) for k in ENV_KEYS if k in os.environ}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        e = mm.Engine(H, W)
    finally:
        for k in env:
            os.environ.pop(k, None)
        os.environ.update(saved)
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
    ap.add_argument("--rows", type=int, default=0, help="rows (default: --size)")
    ap.add_argument("--preset", default="seg", choices=sorted(PRESETS))
    ap.add_argument("--configs", default="", help="JSON list of env dicts (overrides --preset)")
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    H = a.rows or a.size
    W = a.size
    cfgs = json.loads(a.configs) if a.configs else PRESETS[a.preset]
    ref = None
    res = {}
    for rnd in range(a.rounds):
        for ci, env in enumerate(cfgs):
            e = make(H, W, env)
            e.run(8)
            t, _ = time_engine(e, a.steps)
            info = e.info()
            per = info["steps_per_launch"]
            res.setdefault(ci, []).append((t, per))
            if rnd == 0:
                cfgs[ci] = dict(cfgs[ci], _rows=info["rows_per_wave"], _waves=info["waves_per_pass"])
            if rnd == 0:
                out = e.download()
                if ref is None:
                    ref = out
                elif not np.array_equal(out, ref):
                    print(json.dumps({"MISMATCH": env}), flush=True)
            e.close()
    rows = []
    for ci, ts in res.items():
        med = statistics.median(t for t, _ in ts)
        per = ts[0][1]
        rows.append((med / per, {"H": H, "W": W, "env": cfgs[ci], "steps_per_launch": per,
                                 "kernel_us_med": round(med * 1e3, 2),
                                 "us_per_step": round(med * 1e3 / per, 2),
                                 "GCUPS": round(H * W * per / (med * 1e-3) / 1e9, 1),
                                 "GBps_per_launch": round(16.0 * H * W / (med * 1e-3) / 1e9, 1)}))
    for _, r in sorted(rows, key=lambda t: t[0]):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
