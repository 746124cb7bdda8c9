#!/usr/bin/env python3
"""Why does bench.py's step kernel run slower than tools/sweep.py's? Times whole K-step
passes of the 32768^2 c3 grid (HIP events) under bench.py's exact call sequence, one
ingredient at a time: `import torch.distributed`, mm_sums before the run, graph warmup."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mpi-model_amd"))
import mpimodel as mm  # noqa: E402

mm.lib()


def timed(tag, sums=False, warm=16, n=32768):
    with mm.Engine(n, n) as e:
        e.fill_random(0)
        if sums:
            e.sums()
        e.add_diffuse(0, 0.1)
        e.run(warm)
        e.synchronize()
        mm.device_synchronize(0)
        t0 = time.perf_counter()
        e.run(96)
        e.synchronize()
        el = time.perf_counter() - t0
        e.set_timing(True)
        e.run(96)
        k, ms, b = e.timing()
        e.set_timing(False)
        spl = e.info()["steps_per_launch"]
    print(f"{tag}: K={spl} kernel {ms / k * 1e3:.1f} us, graph run {el / 96 * 1e3:.4f} ms/step", flush=True)


what = sys.argv[1:] or ["plain"]
timed("plain")
timed("sums first", sums=True)
if "dist" in what:
    import torch  # noqa: F401
    import torch.distributed  # noqa: F401
    timed("after import torch.distributed")
    timed("after import torch.distributed, sums first", sums=True)
