#!/usr/bin/env python3
"""Where a GPU result departs from the oracle: for each case, the cells that differ
(count, rows, columns) per slab. Cases: host-halo chains (tests/test_gpu_halo.py's
helpers, without pytest) and single engines, under MM_* environment overrides.

usage: python3 tools/diag_parity.py
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import mpimodel as gpu  # noqa: E402
import oracle as O  # noqa: E402


def chain(H, W, G, steps, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        es = []
        for g in range(G):
            x0, h = gpu.partition_rows(H, G, g)
            es.append(gpu.Engine(H, W, x0, h, rank=g, nranks=G,
                                 halo_mode=gpu.MM_HALO_HOST if G > 1 else 0))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for e in es:
        e.fill_random(0)
        e.add_diffuse(0, 0.3)
    plan = es[0].pass_plan(steps)
    for k in plan:
        if G > 1:
            halos = [e.halo_export(k) for e in es]
            for g, e in enumerate(es):
                e.halo_import(halos[g - 1][1] if g > 0 else None,
                              halos[g + 1][0] if g < G - 1 else None, nrows=k)
        for e in es:
            e.run(k)
    got = np.vstack([e.download() for e in es])
    info = es[0].info()
    for e in es:
        e.close()
    return got, plan, info


def report(name, H, W, G, steps, env):
    got, plan, info = chain(H, W, G, steps, env)
    want = O.field_step(O.fill_random(H, W), 0.3, steps=steps)
    bad = got != want
    n = int(np.count_nonzero(bad))
    print(f"{name}: H={H} W={W} G={G} steps={steps} env={env} plan={plan} "
          f"kernel={info['kernel']} depth={info['halo_depth']}: {n} cells differ", flush=True)
    if n:
        rows = np.nonzero(bad.any(axis=1))[0]
        cols = np.nonzero(bad.any(axis=0))[0]
        print(f"   rows {rows[:40].tolist()}{' ...' if len(rows) > 40 else ''}")
        print(f"   cols {cols[:40].tolist()}{' ...' if len(cols) > 40 else ''}")
        r, c = np.argwhere(bad)[0]
        print(f"   first ({r},{c}): got {got[r, c]!r} want {want[r, c]!r}")


CASES = [
    ("fail", 27, 257, 3, 19, {"MM_STEPS_PER_PASS": 10, "MM_WIDE": 0}),
    ("evenW", 27, 256, 3, 19, {"MM_STEPS_PER_PASS": 10, "MM_WIDE": 0}),
    ("evenX", 36, 257, 3, 19, {"MM_STEPS_PER_PASS": 10, "MM_WIDE": 0}),
    ("one-k9", 27, 257, 1, 9, {"MM_STEPS_PER_PASS": 9, "MM_WIDE": 0}),
    ("one-k1", 27, 257, 1, 1, {"MM_STEPS_PER_PASS": 1, "MM_WIDE": 0}),
    ("one-k2", 27, 257, 1, 2, {"MM_STEPS_PER_PASS": 2, "MM_WIDE": 0}),
    ("one-pass", 27, 257, 1, 2, {"MM_PASSK": 0}),
    ("chain-k1", 27, 257, 3, 3, {"MM_STEPS_PER_PASS": 1, "MM_WIDE": 0}),
    ("chain-k9", 27, 257, 3, 9, {"MM_STEPS_PER_PASS": 9, "MM_WIDE": 0}),
    ("chain-k9-256", 27, 256, 3, 9, {"MM_STEPS_PER_PASS": 9, "MM_WIDE": 0}),
    ("wide-k8", 27, 257, 3, 16, {"MM_STEPS_PER_PASS": 8, "MM_WIDE": 1}),
]

if __name__ == "__main__":
    for c in CASES:
        report(*c)
