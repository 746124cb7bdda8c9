import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mpi-model_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


# Load the engine (ROCm's HIP runtime and librccl) before any test module imports torch,
# which bundles its own librccl.so.1 / libamdhip64 under the same sonames (bench.py does
# the same). Loading needs no GPU.
try:
    import mpimodel as _mm
    _mm.lib()
except Exception:  # library not built yet: the tests that need it fail on their own
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def O():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def mm():
    import mpimodel
    return mpimodel


@pytest.fixture(scope="session")
def gpu(mm):
    """The HIP engine on cuda:0. No fallback: a GPU test without the library or a
    device fails instead of silently running something else."""
    n = mm.device_count()
    assert n >= 1, "no HIP device visible"
    return mm


def golden(name):
    import json
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def golden_points():
    import glob
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "point_*.json")))


def golden_strict():
    """Sources off the reference's valid domain that it still completes (no cell changed)."""
    import glob
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "strict_*.json")))
