#!/usr/bin/env python3
"""Compare builds of libmpimodel_hip.so (tools/build_variants.sh) on the GPU.

Each library runs in its own child process (one HIP module set per process), in
interleaved rounds: first a bit-exact check of K-step passes against the oracle on a
small grid, then the median HIP-event time of the step kernel at --size^2 (the
production path's plan: default engine settings, or --env). One JSON line per library,
fastest first.

  python tools/libsweep.py --size 32768 --steps 16 var/*/libmpimodel_hip.so
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import mpimodel as mm
    mm.LIB_PATH = a.lib
    mm.lib()
    import oracle as O
    os.environ.update({k: str(v) for k, v in json.loads(a.env).items()})
    out = {}
    # correctness: K-step passes + a shorter tail against the oracle
    H, W = 301, 1000
    cs = a.check_steps
    with mm.Engine(H, W) as e:
        e.fill_random(0)
        e.add_diffuse(0, 0.3)
        e.run(cs)
        ok = np.array_equal(e.download(), O.field_step(O.fill_random(H, W), 0.3, steps=cs))
    out["bit_exact"] = bool(ok)
    H = W = a.size
    if a.program == "c5":  # config C5: 4 attributes, chained transfers + 4 diffusions, sums
        flows = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
                 (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]
        h, w = 67, 300
        fields = [O.fill_random(h, w, seed=O.SEED + k) for k in range(4)]
        want = O.program_step(fields, flows, steps=5)
        with mm.Engine(h, w, n_attr=4) as e:
            for k in range(4):
                e.fill_random(k, seed=O.SEED + k)
            for kind, x, y, r in flows:
                (e.add_diffuse(x, r) if kind == 1 else e.add_transfer(x, y, r))
            e.run(5, 1)
            out["bit_exact"] = out["bit_exact"] and all(
                np.array_equal(e.download(k), want[k]) for k in range(4))
        with mm.Engine(H, W, n_attr=4) as e:
            for k in range(4):
                e.fill_random(k, seed=O.SEED + k)
            for kind, x, y, r in flows:
                (e.add_diffuse(x, r) if kind == 1 else e.add_transfer(x, y, r))
            e.run(8, 1)
            e.set_timing(True)
            e.run(a.steps, 1)
            n, ms, b = e.timing()
            e.set_timing(False)
            info = e.info()
        out.update(kernel_ms=ms / n, bytes=b, spl=info["steps_per_launch"],
                   rows=info["rows_per_wave"], waves=info["waves_per_pass"])
        print("RESULT " + json.dumps(out), flush=True)
        return
    with mm.Engine(H, W) as e:
        e.fill_random(0)
        e.add_diffuse(0, 0.1)
        e.run(8)
        e.set_timing(True)
        e.run(a.steps)
        n, ms, b = e.timing()
        e.set_timing(False)
        info = e.info()
    out.update(kernel_ms=ms / n, bytes=b, spl=info["steps_per_launch"], rows=info["rows_per_wave"],
               waves=info["waves_per_pass"])
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="*")
    ap.add_argument("--size", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--env", default="{}")
    ap.add_argument("--program", default="", help="c5: the 4-attribute flow program")
    ap.add_argument("--lib", default="")
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("--check-steps", type=int, default=9)
    a = ap.parse_args()
    if a.lib:
        return child(a)
    res = {}
    for rnd in range(a.rounds):
        for lib in a.libs:
            cmd = [sys.executable, "-u", __file__, "--lib", lib, "--size", str(a.size),
                   "--steps", str(a.steps), "--env", a.env, "--program", a.program,
                   "--check-steps", str(a.check_steps)]
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
            if p.returncode != 0 or not line:
                print(json.dumps({"lib": lib, "error": p.returncode, "tail": p.stderr[-400:]}),
                      flush=True)
                sys.exit(3)
            r = json.loads(line[0][7:])
            res.setdefault(lib, []).append(r)
            print(json.dumps({"round": rnd, "lib": lib, **r}), flush=True)
    rows = []
    for lib, rs in res.items():
        med = statistics.median(r["kernel_ms"] for r in rs)
        r0 = rs[0]
        name = os.path.basename(os.path.dirname(lib))
        flags = ""
        fp = os.path.join(os.path.dirname(lib), "flags.txt")
        if os.path.exists(fp):
            flags = open(fp).read().strip()
        rows.append((med, {"variant": name, "flags": flags, "bit_exact": all(r["bit_exact"] for r in rs),
                           "kernel_us_med": round(med * 1e3, 1),
                           "GBps_per_launch": round(r0["bytes"] / (med * 1e-3) / 1e9, 1),
                           "GCUPS": round(a.size * a.size * r0["spl"] / (med * 1e-3) / 1e9, 1),
                           "spl": r0["spl"], "rows": r0["rows"], "waves": r0["waves"]}))
    print("== summary (fastest first)")
    for _, r in sorted(rows, key=lambda t: t[0]):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
