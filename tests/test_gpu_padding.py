"""GPU: no result depends on the pitch padding.

Each attribute buffer is (h + 2 kGhost) x pitch doubles with pitch = roundup(W, 128)
(DESIGN.md section 3); columns W..pitch-1 are padding that the strips read (whole lanes
past the grid, and the grid's last lane when W % C != 0). Zeroed at creation, but the
kernels must not rely on it: a column outside the grid weighs 0 by select (mm_passk /
mm_pass kernels), enters the GEN body as 0 (mm_wide_kernel), and the step sums exclude
lanes that own no cell. Here the padding is poisoned with NaN (mm_debug_fill_padding)
before the run; cells must stay bit-exact with the oracle and every step sum finite and
within 1e-12.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C5_FLOWS = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
            (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]

# W % 4: 2 (a partial lane, GEN strip), 1, 3, 0 (the EDGE body's last-column lane);
# (37, 130): one strip holding both edges at K = 20
SHAPES = [(37, 130), (130, 257), (70, 125), (45, 700), (9, 300)]
ENVS = [{}, {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 20}, {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 4},
        {"MM_WIDE": 0}, {"MM_WIDE": 0, "MM_STEPS_PER_PASS": 3}, {"MM_PASSK": 0}]


def env_id(env):
    return ",".join(f"{k[3:]}={v}" for k, v in env.items()) or "default"


def engine(gpu, monkeypatch, H, W, n_attr=1, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    e = gpu.Engine(H, W, n_attr=n_attr)
    for k in env:
        monkeypatch.delenv(k)
    return e


@pytest.mark.parametrize("env", ENVS, ids=env_id)
@pytest.mark.parametrize("shape", SHAPES)
def test_nan_padding_changes_nothing(gpu, O, monkeypatch, env, shape):
    H, W = shape
    steps = 23
    e = engine(gpu, monkeypatch, H, W, **env)
    e.fill_random(0)
    e.fill_padding(float("nan"))
    e.add_diffuse(0, 0.1)
    e.run(steps, reduce_every=1)
    got, hist = e.download(), e.sums_history()
    e.close()
    ref, want = O.fill_random(H, W), []
    for _ in range(steps):
        ref = O.field_step(ref, 0.1)
        want.append(math.fsum(ref.ravel()))
    assert np.array_equal(got, ref)
    assert np.all(np.isfinite(hist))
    for a, b in zip(hist[:, 0], want):
        assert abs(a - b) <= 1e-12 * b


@pytest.mark.parametrize("env", [{}, {"MM_STEPS_PER_PASS": 4}, {"MM_CHAIN_RING": 0},
                                 {"MM_WIDE": 0}], ids=env_id)
@pytest.mark.parametrize("shape", [(37, 130), (67, 301)])
def test_nan_padding_four_attributes(gpu, O, monkeypatch, env, shape):
    H, W = shape
    steps = 9
    e = engine(gpu, monkeypatch, H, W, n_attr=4, **env)
    for a in range(4):
        e.fill_random(a, seed=O.SEED + a)
    e.fill_padding(float("nan"))
    for kind, a, b, r in C5_FLOWS:
        if kind == 1:
            e.add_diffuse(a, r)
        else:
            e.add_transfer(a, b, r)
    e.run(steps, reduce_every=1)
    got = [e.download(a) for a in range(4)]
    hist = e.sums_history()
    e.close()
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    want, sums = O.program_step(fields, C5_FLOWS, steps=steps, sums_per_step=True)
    for a in range(4):
        assert np.array_equal(got[a], want[a]), a
    assert np.all(np.isfinite(hist))
    for s in range(steps):
        for a in range(4):
            assert abs(hist[s, a] - sums[s][a]) <= 1e-12 * abs(sums[s][a]), (s, a)
