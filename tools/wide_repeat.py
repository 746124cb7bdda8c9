#!/usr/bin/env python3
"""Debug: repeat small wide-kernel runs and report how often / how they differ."""
import json, math, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np
import mpimodel as mm
mm.lib()
import oracle as O

H, W = 300, 700
v = O.fill_random(H, W)
refs = {}
for k in (4, 8, 12):
    ref = v
    for s in range(k):
        ref = O.field_step(ref, 0.1)
    refs[k] = ref
for k, re, graph in [(8, 1, 0), (8, 0, 0), (4, 1, 0), (12, 1, 0), (8, 1, 1)]:
    os.environ["MM_WIDE"] = "1"
    os.environ["MM_STEPS_PER_PASS"] = str(k)
    os.environ["MM_GRAPH"] = str(graph)
    bad = []
    for rep in range(12):
        e = mm.Engine(H, W)
        e.upload(v)
        e.add_diffuse(0, 0.1)
        e.run(k, re)
        got = e.download()
        hist = e.sums_history() if re else None
        info = e.info()
        e.close()
        d = got != refs[k]
        if d.any():
            idx = np.argwhere(d)
            bad.append({"rep": rep, "ndiff": int(d.sum()), "rows": [int(idx[:, 0].min()), int(idx[:, 0].max())],
                        "cols": [int(idx[:, 1].min()), int(idx[:, 1].max())],
                        "zeros": int((got == 0).sum()), "hist0": (hist[0, 0] if re else None),
                        "waves": info["waves_per_pass"], "rows_per": info["rows_per_wave"]})
    print(json.dumps({"k": k, "re": re, "graph": graph, "nbad": len(bad), "bad": bad[:3]}), flush=True)
