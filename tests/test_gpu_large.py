"""Full-size configs on the GPU (BASELINE.json configs[2..3]): C3 = 32768^2 and
C4 = 16384^2 fp64, 8 steps (two K=4 passes) of the production path.

The whole grid is far too big for the oracle, so parity is pinned by
  * three 64-row bands -- the top edge, the rows around an interior segment boundary of
    the K-step kernel's wave plan, the bottom edge -- compared BIT-EXACTLY with the
    oracle run on the band widened by the 8-row dependency cone of 8 steps (every column,
    so every strip boundary and both edge strips are covered). At pitch 32768 these rows
    sit at buffer offsets up to ~2^31 from a wave's descriptor base: exactly the
    large-offset indexing (passk_max_rows, num_records) a small grid never reaches;
  * conservation of the total (1e-12 relative);
  * exact mirror symmetry: the step commutes with flipping both axes.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STEPS = 8
RATE = 0.1


def band_oracle(O, H, W, lo, hi, steps, rate):
    """Rows [lo, hi) after `steps` steps, exact on [lo+steps, hi-steps) (inner rows of
    the dependency cone; rows next to a grid edge are exact up to that edge)."""
    v = O.fill_random(H, W, lo, hi - lo)
    for _ in range(steps):
        vg = np.zeros((v.shape[0] + 2, W))
        vg[1:-1] = v
        v = O.field_step_slab(H, W, lo, vg, rate)
    return v


def bands_for(H, info):
    r = info["rows_per_wave"]
    nseg = (H + r - 1) // r
    mid = (nseg // 2) * r  # an interior segment boundary of the wave plan
    return [0, mid - 32, H - 64]


@pytest.mark.parametrize("N", [16384, 32768])
def test_full_size_bands_conservation_symmetry(gpu, O, N):
    H = W = N
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        s0 = e.sums()[0]
        e.add_diffuse(0, RATE)
        info = e.info()
        assert info["steps_per_launch"] >= 4 and info["kernel"] == 2
        e.run(STEPS)
        e.synchronize()
        s1 = e.sums()[0]
        bands = {b: e.read_rows(b, 64) for b in bands_for(H, info)}
        mirror_src = {b: e.read_rows(H - 64 - b, 64) for b in bands}
    # conservation (src/Model.hpp:95, made two-sided and relative)
    assert abs(s1 - s0) <= 1e-12 * s0
    for b, got in bands.items():
        lo, hi = max(0, b - STEPS), min(H, b + 64 + STEPS)
        want = band_oracle(O, H, W, lo, hi, STEPS, RATE)[b - lo:b - lo + 64]
        assert np.array_equal(got, want), (N, b, int(np.count_nonzero(got != want)))
    # mirror: run the flipped input and compare the same bands flipped back
    v0 = O.fill_random(H, W)
    vf = np.ascontiguousarray(v0[::-1, ::-1])
    del v0
    with gpu.Engine(H, W) as e:
        e.upload(vf)
        del vf
        e.add_diffuse(0, RATE)
        e.run(STEPS)
        for b, got in mirror_src.items():
            flipped = e.read_rows(b, 64)
            assert np.array_equal(flipped, got[::-1, ::-1]), (N, b)




def test_pass_planner_plans(gpu, monkeypatch):
    """mm_pass_plan on an 8192 x 32768 slab: short runs take fewer, deeper passes (20
    steps: 10 + 10), long runs stay at K = 8; MM_PASS_PLAN=0 and slabs with fewer strips
    (16384^2) or cells (4096^2) give balanced passes of K."""
    with gpu.Engine(8192, 32768) as e:
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [10, 10]
        assert e.pass_plan(16) == [8, 8]
        assert e.pass_plan(9) == [9]
        assert e.pass_plan(1000) == [8] * 125
        assert e.pass_plan(0) == []
    monkeypatch.setenv("MM_PASS_PLAN", "0")
    with gpu.Engine(8192, 32768) as e:
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [7, 7, 6]
    monkeypatch.delenv("MM_PASS_PLAN")
    with gpu.Engine(16384, 16384) as e:  # 152 strips: no planner
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [7, 7, 6]
    with gpu.Engine(4096, 4096) as e:  # small slab: K = 7, no planner
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [7, 7, 6]


def test_driver_length_run_two_deep_passes(gpu, O):
    """A 20-step run on an 8192 x 32768 slab (the rows one GPU of a 4-GPU c3 run holds):
    two K = 10 passes (the planner), equal to 20 single steps bit for bit on three bands
    widened by the 20-row cone (top edge, middle, bottom edge: every column, so both edge
    strips), total conserved."""
    H, W = 8192, 32768
    steps = 20
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        s0 = e.sums()[0]
        e.add_diffuse(0, RATE)
        e.set_timing(True)
        e.run(steps)
        n_launch, _, _ = e.timing()
        e.set_timing(False)
        assert n_launch == 2
        s1 = e.sums()[0]
        bands = {b: e.read_rows(b, 64) for b in (0, H // 2 - 32, H - 64)}
    assert abs(s1 - s0) <= 1e-12 * s0
    for b, got in bands.items():
        lo, hi = max(0, b - steps), min(H, b + 64 + steps)
        want = band_oracle(O, H, W, lo, hi, steps, RATE)[b - lo:b - lo + 64]
        assert np.array_equal(got, want), (b, int(np.count_nonzero(got != want)))
