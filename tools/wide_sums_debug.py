#!/usr/bin/env python3
"""Debug: per-step sums of the wide kernel vs the oracle (prints every entry)."""
import json, math, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np
import mpimodel as mm
mm.lib()
import oracle as O

for (H, W, k, steps, re) in [(300, 700, 4, 8, 1), (300, 700, 4, 8, 2), (300, 700, 4, 4, 1),
                             (64, 200, 4, 4, 1), (300, 700, 8, 8, 1), (300, 700, 4, 8, 4)]:
    os.environ["MM_WIDE"] = "1"
    os.environ["MM_STEPS_PER_PASS"] = str(k)
    v = O.fill_random(H, W)
    e = mm.Engine(H, W)
    e.upload(v)
    e.add_diffuse(0, 0.1)
    e.run(steps, re)
    hist = e.sums_history()
    got = e.download()
    info = e.info()
    e.close()
    ref = v
    want = []
    for s in range(1, steps + 1):
        ref = O.field_step(ref, 0.1)
        if s % re == 0:
            want.append(math.fsum(ref.ravel()))
    print(json.dumps({"H": H, "W": W, "k": k, "steps": steps, "re": re,
                      "field_ok": bool(np.array_equal(got, ref)), "graph": info["graph_state"],
                      "hist": hist[:, 0].tolist(), "want": want}), flush=True)
