"""Full-size configs on the GPU (BASELINE.json configs[2..3]): C3 = 32768^2 and
C4 = 16384^2 fp64 on the production path: 8 steps, and the driver's exact 20-step run
(bench.py --steps 20: the default planner's passes, one K = 20 pass of the level-split
kernel; with MM_WIDE=0 round 2's 10 + 10 passes of mm_passk_kernel).

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
        assert info["steps_per_launch"] >= 4 and info["kernel"] in (2, 3)
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




WIDE_K = (4, 8, 12, 16, 20)


def test_pass_planner_plans(gpu, monkeypatch):
    """mm_pass_plan. Slabs of >= 2^28 cells run the level-split kernel: the planner's
    cheapest plan over both kernels' lengths -- one K = 20 pass for the driver's 20 steps,
    K = 20 passes for long runs. MM_PASS_PLAN=0: passes of K = 20 and a tail.
    MM_WIDE=0 (round 2): 10 + 10 on 8192 x 32768, K = 8 for long runs. Smaller slabs
    (4096^2) keep mm_passk_kernel's balanced passes of K = 7."""
    for H, W in ((8192, 32768), (16384, 16384)):
        with gpu.Engine(H, W) as e:
            e.add_diffuse(0, RATE)
            assert e.info()["kernel"] == 3
            assert e.pass_plan(20) == [20]
            assert e.pass_plan(16) == [16]
            assert e.pass_plan(12) == [12]
            assert e.pass_plan(9) == [9]
            assert e.pass_plan(0) == []
            p = e.pass_plan(1000)
            assert sum(p) == 1000 and len(p) <= 51
            assert all(k in WIDE_K or k <= 10 for k in p)
            assert p.count(20) >= 45
    monkeypatch.setenv("MM_PASS_PLAN", "0")
    with gpu.Engine(8192, 32768) as e:
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [20]
        assert e.pass_plan(45) == [20, 20, 5]
    monkeypatch.delenv("MM_PASS_PLAN")
    monkeypatch.setenv("MM_WIDE", "0")
    with gpu.Engine(8192, 32768) as e:
        e.add_diffuse(0, RATE)
        assert e.info()["kernel"] == 2
        assert e.pass_plan(20) == [10, 10]
        assert e.pass_plan(1000) == [8] * 125
    with gpu.Engine(16384, 16384) as e:  # 152 strips: no planner
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [7, 7, 6]
    monkeypatch.delenv("MM_WIDE")
    with gpu.Engine(4096, 4096) as e:  # small slab: mm_wide_kernel, K = 8, no planner
        e.add_diffuse(0, RATE)
        assert e.info()["kernel"] == 3 and e.info()["steps_per_launch"] == 8
        assert e.pass_plan(20) == [8, 8, 4]
        assert e.pass_plan(1000) == [8] * 125
    with gpu.Engine(8192, 8192) as e:  # between: mm_passk_kernel, K = 7
        e.add_diffuse(0, RATE)
        assert e.info()["kernel"] == 2
        assert e.pass_plan(20) == [7, 7, 6]


def driver_run_bands(gpu, O, monkeypatch, H, W, wide, plan):
    """`steps` = sum(plan) steps under the default planner (or MM_WIDE=0): the planned
    passes, each one launch; three bands -- top edge, an interior segment boundary of the
    pass's plan, bottom edge: every column, so both edge strips -- against 20 single steps
    of the oracle on the band widened by the dependency cone; total conserved."""
    steps = sum(plan)
    if not wide:
        monkeypatch.setenv("MM_WIDE", "0")
    # the segment plan of the run's first pass (info describes the configured K's plan)
    monkeypatch.setenv("MM_STEPS_PER_PASS", str(plan[0]))
    with gpu.Engine(H, W) as probe:
        probe.add_diffuse(0, RATE)
        seg_info = probe.info()
    monkeypatch.delenv("MM_STEPS_PER_PASS")
    with gpu.Engine(H, W) as e:
        if not wide:
            monkeypatch.delenv("MM_WIDE")
        e.fill_random(0)
        s0 = e.sums()[0]
        e.add_diffuse(0, RATE)
        assert e.pass_plan(steps) == plan
        info = e.info()
        assert info["kernel"] == (3 if wide else 2)
        e.set_timing(True)
        e.run(steps)
        n_launch, _, _ = e.timing()
        e.set_timing(False)
        assert n_launch == len(plan)
        s1 = e.sums()[0]
        bands = {b: e.read_rows(b, 64) for b in sorted(set(bands_for(H, seg_info)))}
    assert abs(s1 - s0) <= 1e-12 * s0
    for b, got in bands.items():
        lo, hi = max(0, b - steps), min(H, b + 64 + steps)
        want = band_oracle(O, H, W, lo, hi, steps, RATE)[b - lo:b - lo + 64]
        assert np.array_equal(got, want), (b, int(np.count_nonzero(got != want)))


@pytest.mark.parametrize("wide,plan", [(1, [20]), (0, [10, 10])], ids=["wide", "passk"])
def test_driver_length_run_slab(gpu, O, monkeypatch, wide, plan):
    """The 8192 x 32768 slab one GPU of a 4-GPU c3 run holds, 20 steps."""
    driver_run_bands(gpu, O, monkeypatch, 8192, 32768, wide, plan)


@pytest.mark.parametrize("wide,plan", [(1, [20]), (0, [10, 10])], ids=["wide", "passk"])
def test_driver_config_full_grid(gpu, O, monkeypatch, wide, plan):
    """The exact configuration the driver times (bench.py --steps 20, c3): the whole
    32768^2 grid, 20 steps under the default planner -- one K = 20 pass of the level-split
    kernel -- and under MM_WIDE=0 the 10 + 10 passes round 2's driver line timed."""
    driver_run_bands(gpu, O, monkeypatch, 32768, 32768, wide, plan)


def test_c4_production_pass_full_grid(gpu, O, monkeypatch):
    """C4's production pass (BASELINE configs[3], 16384^2 per GPU): the K = 20 pass of the
    level-split kernel the 1000-step line repeats (50 x 20), at full size."""
    driver_run_bands(gpu, O, monkeypatch, 16384, 16384, 1, [20])


def test_mid_slab_takes_the_k20_planner(gpu):
    """Slabs of 2^27 - 2^28 cells (rank 0 of an 8-rank c3 chain: 4096 x 32768) plan the
    level-split kernel's K = 20 pass, with a halo (the interior / border split) and, since
    the box-sum kernels, without one (profiles/r06/self20: 2532 GCUPS split against 1194
    for mm_passk_kernel's 7 + 7 + 6)."""
    with gpu.Engine(32768, 32768, 0, 4096, rank=0, nranks=8, halo_mode=gpu.MM_HALO_HOST) as e:
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [20]
        assert e.pass_kernel(20)[0] == 3 and e.info()["halo_depth"] == 20
    with gpu.Engine(4096, 32768) as e:
        e.add_diffuse(0, RATE)
        assert e.pass_plan(20) == [20] and e.info()["kernel"] == 3


def test_standalone_mid_slab_takes_k20(gpu, O, monkeypatch):
    """A standalone 4096 x 32768 grid (2^27 cells, NO halo -- the slab of an N = 8 c3 rank
    without its interior / border split, tests/test_gpu_fullsize.py c3_n8): the default
    planner's 20 steps are one K = 20 pass of the level-split kernel (round 4 kept
    mm_passk_kernel's 7 + 7 + 6 here; the box-sum kernels run it twice as fast)."""
    driver_run_bands(gpu, O, monkeypatch, 4096, 32768, 1, [20])


# ---- C5 at the size it is benchmarked at (bench.py --workload c5) ------------------------
C5_FLOWS = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
            (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]
# the ring's transfers in another order: the same four transfers, not the ring
C5_REORDERED = [C5_FLOWS[1], C5_FLOWS[0], C5_FLOWS[2], C5_FLOWS[3]] + C5_FLOWS[4:]


@pytest.mark.parametrize("flows,chain,env", [(C5_FLOWS, "MM_CHAIN_RING", {}),
                                             (C5_REORDERED, "MM_CHAIN_RUNTIME", {}),
                                             (C5_FLOWS, "MM_CHAIN_RUNTIME", {"MM_CHAIN_RING": "0"})],
                         ids=["ring", "reordered", "ring_runtime_operands"])
def test_c5_bench_size_bit_exact(gpu, O, monkeypatch, flows, chain, env):
    """bench.py's C5 configuration at its own size (4096^2, 4 attributes, per-step sums,
    the default engine: K = 8 passes of the level-split kernel, the bench's segment plan):
    21 steps (8 + 8 + 4 + 1, one graph) and then 48 more replayed as 16-step hipGraphs,
    every attribute bit-exact against the oracle's flow program, every step's sums within
    1e-12 (src/Attribute.hpp:8-9, src/Exponencial.hpp:18-20, src/Model.hpp:88-95)."""
    H = W = 4096
    from test_gpu_parity import add_flows
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    # graphs of 2 passes (the engine would take all 48 steps as one graph): replays
    # alternating between the two buffer parities
    env = dict(env, MM_GRAPH_MAX_LAUNCHES="2")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with gpu.Engine(H, W, n_attr=4) as e:
        for k in env:
            monkeypatch.delenv(k)
        for a in range(4):
            e.fill_random(a, seed=O.SEED + a)
        add_flows(e, flows)
        info = e.info()
        assert info["kernel"] == 3 and info["steps_per_launch"] == 8, info
        assert info["chain_kernel"] == getattr(gpu, chain), info
        assert e.pass_plan(21) == [8, 8, 4, 1]
        e.run(21, reduce_every=1)
        want, sums = O.program_step(fields, flows, steps=21, sums_per_step=True)
        for a in range(4):
            got = e.download(a)
            assert np.array_equal(got, want[a]), (a, int(np.count_nonzero(got != want[a])))
        e.run(48, reduce_every=1)
        i1 = e.info()
        assert i1["graph_state"] == 1 and i1["graph_launches"] >= 3, i1
        want, sums2 = O.program_step(want, flows, steps=48, sums_per_step=True)
        for a in range(4):
            got = e.download(a)
            assert np.array_equal(got, want[a]), (a, int(np.count_nonzero(got != want[a])))
        hist = e.sums_history()
    sums = sums + sums2
    assert hist.shape == (69, 4)
    for s, row in enumerate(sums):
        for a in range(4):
            assert abs(hist[s, a] - row[a]) <= 1e-12 * abs(row[a]), (s, a)
