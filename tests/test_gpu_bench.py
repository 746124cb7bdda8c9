"""bench.py's output line, end to end on the GPU: the driver's JSON contract (metric, value,
steps, roofline with HBM and VALU roofs, cpu_baseline), the pass plan it reports, and the
conservation check. Small workload (c2, 4096^2) and a short CPU leg, in a child process as
the driver runs it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args):
    p = subprocess.run([sys.executable, "-u", os.path.join(REPO, "bench.py"), *args],
                       cwd=REPO, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_line_contract():
    d = run_bench("--workload", "c2", "--steps", "20", "--warmup", "5", "--cpu-seconds", "1")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline", "check"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 5
    assert d["unit"] == "GCUPS" and d["dtype"] == "f64" and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0
    # value is whole-run throughput: cells x steps / (steps x ms_per_step)
    H, W = d["config"]["grid"]
    assert abs(d["value"] - H * W / (d["ms_per_step"] * 1e-3) / 1e9) <= 0.01 * d["value"]
    assert d["config"]["workload"].startswith("c2")
    # 4096^2: K = 8 passes of mm_wide_kernel and the K = 4 rest (no planner on a small slab)
    assert "mm_wide_kernel, 3 pass(es) of 8+8+4" in d["config"]["path"], d["config"]["path"]
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert r["steps_per_launch"] == 8 and r["algorithmic_bytes_per_launch"] == 16.0 * H * W
    assert r["valu"]["bound"] == "valu" and 0 < r["valu"]["frac"] < 1
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] == "port" and c["cores"] >= 1 and c["sample"]
    assert d["check"]["total_rel_drift"] <= 1e-12
