#!/usr/bin/env python3
"""Probe of the linked-pass launch (mm_wide_link_kernel) on one small grid: run, sync,
compare with the oracle, print the engine info. Run it under `timeout`: a hang ends there.
usage: link_probe.py H W STEPS   (env: MM_LINK_PASSES, MM_LINK_DEBUG, MM_GRAPH)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mpi-model_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import mpimodel as mm  # noqa: E402
import oracle as O  # noqa: E402

H, W, steps = (int(a) for a in sys.argv[1:4])
t0 = time.time()
with mm.Engine(H, W) as e:
    e.fill_random(0)
    e.add_diffuse(0, 0.1)
    print("created", flush=True)
    e.run(steps)
    print("enqueued", flush=True)
    try:
        e.synchronize()
        print("synced %.2fs" % (time.time() - t0), flush=True)
    except mm.MMError as x:
        print("sync error:", x, flush=True)
    info = e.info()
    print({k: info[k] for k in ("kernel", "steps_per_launch", "linked_launches", "graph_launches",
                                "rows_per_wave", "waves_per_pass")}, flush=True)
    got = e.download()
want = O.field_rows(H, W, 0, H, steps, 0.1)
print("cells differing:", int(np.count_nonzero(got != want)), flush=True)
