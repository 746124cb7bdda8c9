#!/usr/bin/env python3
"""C5 (4096^2, 4 attributes, bench.py's flow program) on variant builds of the library
(tools/build_variants.sh): HIP-event time of the K = 8 pass, and a digest of the state after
the run -- every variant must match the first library's digest bit for bit.

  python tools/c5_variants.py LIB [LIB ...]
"""
import hashlib
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path):
    sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
    sys.path.insert(0, REPO)
    import mpimodel as mm
    mm.LIB_PATH = path
    mm.lib()
    from bench import C5_FLOWS
    e = mm.Engine(4096, 4096, n_attr=4)
    for a in range(4):
        e.fill_random(a, seed=mm.SEED + a)
    for kind, a, b, r in C5_FLOWS:
        if kind == 1:
            e.add_diffuse(a, r)
        else:
            e.add_transfer(a, b, r)
    e.run(16, 1)
    e.set_timing(True)
    e.run(160, 1)
    n, ms, _ = e.timing()
    e.set_timing(False)
    h = hashlib.sha256()
    for a in range(4):
        h.update(e.download(a).tobytes())
    print(json.dumps({"lib": path, "launches": n, "pass_us": round(1e3 * ms / n, 1),
                      "plan": e.pass_plan(8), "digest": h.hexdigest()[:16]}), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    ref = None
    for path in sys.argv[1:]:
        out = subprocess.run([sys.executable, __file__, "--child", path], capture_output=True,
                             text=True, timeout=150)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-500:]
        print(line, flush=True)
        d = json.loads(line)
        ref = ref or d["digest"]
        if d["digest"] != ref:
            print(json.dumps({"MISMATCH": path}), flush=True)


if __name__ == "__main__":
    main()
