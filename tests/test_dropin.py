"""Drop-in tests: Main.cpp-style MPI programs built against mpi-model_amd/api/ run on
the GPU under mpirun, and their output files are compared with the reference's.

* oracle/_ref/dropin_ref_main is the reference's own src/Main.cpp, UNCHANGED, compiled
  against our headers (mpi-model_amd/api/Makefile; built in the build container).
* examples/drop_in_main.cpp is our Main.cpp-style program.
The reference writes ../output/comm_rank%d.txt per worker plus a merged file
(src/Model.hpp:97-131,245-260); golden sha256s come from the reference itself
(tests/golden/c1_default_text.json).
"""
import glob
import hashlib
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, golden

pytestmark = pytest.mark.gpu

MPIRUN = os.environ.get("MPIRUN", "/opt/conda/bin/mpirun")


def run_mpi(tmp_path, binary, np_, args=(), timeout=120, env=None):
    run = tmp_path / "run"
    out = tmp_path / "output"
    run.mkdir()
    out.mkdir()
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run([MPIRUN, "-np", str(np_), binary] + [str(a) for a in args], cwd=run,
                       capture_output=True, text=True, timeout=timeout, env=e)
    assert p.returncode == 0, p.stdout + p.stderr
    files = {os.path.basename(f): open(f, "rb").read() for f in glob.glob(str(out / "*"))}
    return p.stdout, files


def binaries():
    out = []
    ref = os.path.join(REPO, "oracle", "_ref", "dropin_ref_main")
    if os.path.exists(ref):
        out.append(ref)
    out.append(os.path.join(REPO, "examples", "drop_in_main"))
    return out


@pytest.mark.parametrize("binary", binaries(), ids=os.path.basename)
def test_default_run_matches_reference_output_files(tmp_path, binary):
    g = golden("c1_default_text.json")
    stdout, files = run_mpi(tmp_path, binary, 6)
    for name, want in g["rank_files"].items():
        assert hashlib.sha256(files[name]).hexdigest() == want["sha256"], name
    merged = [v for k, v in files.items() if k.startswith("output ")]
    assert len(merged) == 1
    assert hashlib.sha256(merged[0]).hexdigest() == g["concat_sha256"]
    for line in ["1|19:3|0.100000", "19 3 8", "1: 0.22"]:
        assert line in stdout.splitlines()


@pytest.mark.parametrize("np_", [1, 3])
def test_default_run_other_layouts(tmp_path, np_):
    # one process (master = only worker) and 2 workers: same cells, same bytes in order
    g = golden("c1_default_text.json")
    _, files = run_mpi(tmp_path, os.path.join(REPO, "examples", "drop_in_main"), np_)
    ranks = sorted(k for k in files if k.startswith("comm_rank"))
    assert len(ranks) == max(np_ - 1, 1)
    cat = b"".join(files[k] for k in sorted(ranks, key=lambda s: int(s[9:-4])))
    assert hashlib.sha256(cat).hexdigest() == g["concat_sha256"]


@pytest.mark.parametrize("np_", [1, 3, 4])
def test_whole_grid_flow_program(tmp_path, O, np_):
    # Exponencial(rate) on every cell, 51 steps (time 10, dt 0.2: src/Model.hpp:47-51);
    # workers sharing the one GPU exchange border rows through MPI (MM_HALO_HOST)
    import json
    H, W = 100, 100
    stdout, files = run_mpi(tmp_path, os.path.join(REPO, "examples", "grid_flow_main"), np_,
                            [H, W, 10.0, 0.2, 0.1])
    rep = json.loads([ln for ln in stdout.splitlines() if ln.startswith("{")][-1])
    assert rep["steps"] == 51
    v = np.ones((H, W))
    sums = []
    for _ in range(51):
        v = O.field_step(v, 0.1)
        sums.append(math.fsum(v.ravel()))
    got = [float.fromhex(s) for s in rep["sums"]]
    assert len(got) == 51
    for a, b in zip(got, sums):
        assert abs(a - b) <= 1e-12 * b
    lines = []
    for k in sorted((k for k in files if k.startswith("comm_rank")), key=lambda s: int(s[9:-4])):
        lines.extend(files[k].decode().splitlines())
    want = [f"{x}\t{y}\t{v[x, y]:g}" for x in range(H) for y in range(W)]
    assert lines == want
