#!/usr/bin/env python3
"""Segment plan (rows per wave) of the c3 engine when torch is imported before the first
engine exists (bench.py's order) vs not: the plan comes from the occupancy API."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402

mm.lib()
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401
    import torch.distributed  # noqa: F401
for _ in range(2):
    with mm.Engine(32768, 32768) as e:
        e.add_diffuse(0, 0.1)
        i = e.info()
        print(sys.argv[1:], "rows_per_wave", i["rows_per_wave"], "waves", i["waves_per_pass"],
              "waves_per_cu", i["seg_waves_per_cu"], flush=True)
