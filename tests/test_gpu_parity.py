"""GPU parity: the HIP path (through the C ABI) against the oracle, bit for bit.

Bar (BASELINE.json north_star): bit-exact cell indexing and partition bookkeeping;
attribute values within 1e-12 relative (fp64). The step's arithmetic order is
shared with the oracle (oracle/mm_oracle.h), so values are compared BIT-EXACTLY
here; only sums (whose summation order differs by design) use the 1e-12 bound.
"""
import math

import numpy as np
import pytest

from conftest import golden, golden_points, golden_strict

pytestmark = pytest.mark.gpu

RATE = 0.1  # src/Main.cpp:33

SHAPES = [(1, 1), (1, 9), (2, 2), (3, 5), (5, 3), (37, 53), (100, 100), (64, 128), (63, 129),
          (130, 257), (257, 300), (33, 1000)]


def run_field(gpu, v, rate, steps, reduce_every=0):
    H, W = v.shape
    with gpu.Engine(H, W) as e:
        e.upload(v)
        e.add_diffuse(0, rate)
        e.run(steps, reduce_every)
        e.synchronize()
        return e.download(), (e.sums_history() if reduce_every else None)


@pytest.mark.parametrize("shape", SHAPES)
def test_one_step_bit_exact(gpu, O, shape):
    v = O.fill_random(*shape)
    got, _ = run_field(gpu, v, RATE, 1)
    assert np.array_equal(got, O.field_step(v, RATE))


@pytest.mark.parametrize("shape,steps", [((37, 53), 2), ((100, 100), 7), ((130, 257), 10),
                                          ((64, 128), 51)])
def test_multi_step_bit_exact(gpu, O, shape, steps):
    v = O.fill_random(*shape)
    got, _ = run_field(gpu, v, 0.25, steps)
    assert np.array_equal(got, O.field_step(v, 0.25, steps=steps))


def test_device_fill_matches_oracle_input(gpu, O):
    H, W = 77, 300
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        assert np.array_equal(e.download(), O.fill_random(H, W))
        e.fill(0, value=1.0)
        assert np.array_equal(e.download(), np.ones((H, W)))


@pytest.mark.parametrize("name", golden_points())
def test_point_flow_matches_reference_golden(gpu, name):
    # src/Model.hpp:176-235 on the device, against the grid the reference itself wrote
    g = golden(name)
    H, W = g["dimx"], g["dimy"]
    with gpu.Engine(H, W) as e:
        e.fill(0, value=1.0)
        e.point_apply(g["src_x"], g["src_y"], float.fromhex(g["value_hex"]),
                      float.fromhex(g["rate_hex"]))
        v = e.download()
        s = e.sums()[0]
    changed = sorted([x, y, val.hex()] for (x, y), val in np.ndenumerate(v) if val != 1.0)
    assert changed == g["changed"]
    want = float.fromhex(g["sum_fsum_hex"])
    assert abs(s - want) <= 1e-12 * abs(want)
    assert s - H * W < 0.001  # the reference's own check, src/Model.hpp:95


@pytest.mark.parametrize("name", golden_points())
def test_point_flow_on_reference_partition(gpu, name):
    # the same golden grid computed by P slabs laid out exactly as the reference's
    # workers (src/Model.hpp:70-76), each applying the flow to the cells it owns
    g = golden(name)
    H, W, P = g["dimx"], g["dimy"], g["nworkers"]
    parts = []
    for k in range(1, P + 1):
        x0, _, hh, _ = gpu.partition_reference(H, W, P, k)
        assert (x0, hh) == gpu.partition_rows(H, P, k - 1)
        with gpu.Engine(H, W, x0, hh, rank=k - 1, nranks=P, halo_mode=gpu.MM_HALO_HOST) as e:
            e.fill(0, value=1.0)
            e.point_apply(g["src_x"], g["src_y"], float.fromhex(g["value_hex"]),
                          float.fromhex(g["rate_hex"]))
            parts.append(e.download())
    v = np.vstack(parts)
    changed = sorted([x, y, val.hex()] for (x, y), val in np.ndenumerate(v) if val != 1.0)
    assert changed == g["changed"]


@pytest.mark.parametrize("name", golden_points() + golden_strict())
def test_strict_point_mode_matches_reference(gpu, name):
    # opt-in strict-reference mode: exactly the reference's grid, including sources off
    # its valid domain where it changes nothing (src/Model.hpp:189-216)
    g = golden(name)
    H, W = g["dimx"], g["dimy"]
    with gpu.Engine(H, W) as e:
        e.fill(0, value=1.0)
        applied = e.point_apply_strict(g["src_x"], g["src_y"], float.fromhex(g["value_hex"]),
                                       float.fromhex(g["rate_hex"]), g["nworkers"])
        v = e.download()
    changed = sorted([x, y, val.hex()] for (x, y), val in np.ndenumerate(v) if val != 1.0)
    assert changed == g["changed"]
    assert applied == bool(g["changed"])


@pytest.mark.parametrize("H,W,G,steps", [(37, 53, 2, 3), (100, 100, 5, 4), (41, 300, 8, 2),
                                         (9, 130, 3, 5)])
def test_slabs_with_host_halo_bit_exact(gpu, O, H, W, G, steps):
    v = O.fill_random(H, W)
    engines = []
    for g in range(G):
        x0, h = gpu.partition_rows(H, G, g)
        e = gpu.Engine(H, W, x0, h, rank=g, nranks=G, halo_mode=gpu.MM_HALO_HOST)
        e.fill_random(0)
        e.add_diffuse(0, RATE)
        engines.append(e)
    for _ in range(steps):
        halos = [e.halo_export() for e in engines]
        for g, e in enumerate(engines):
            top = halos[g - 1][1] if g > 0 else None
            bot = halos[g + 1][0] if g < G - 1 else None
            e.halo_import(top, bot)
        for e in engines:
            e.run(1)
    got = np.vstack([e.download() for e in engines])
    for e in engines:
        e.close()
    assert np.array_equal(got, O.field_step(v, RATE, steps=steps))


def test_step_sums_history(gpu, O):
    H, W, steps = 130, 257, 6
    v = O.fill_random(H, W)
    got, hist = run_field(gpu, v, RATE, steps, reduce_every=1)
    assert hist.shape == (steps, 1)
    ref = v
    for k in range(steps):
        ref = O.field_step(ref, RATE)
        want = math.fsum(ref.ravel())
        assert abs(hist[k, 0] - want) <= 1e-12 * want
    assert np.array_equal(got, ref)


def test_sums_every_third_step(gpu, O):
    v = O.fill_random(64, 128)
    _, hist = run_field(gpu, v, RATE, 9, reduce_every=3)
    assert hist.shape == (3, 1)
    ref = v
    for k in range(9):
        ref = O.field_step(ref, RATE)
        if (k + 1) % 3 == 0:
            want = math.fsum(ref.ravel())
            assert abs(hist[(k + 1) // 3 - 1, 0] - want) <= 1e-12 * want


def test_timed_eager_path_equals_graph_path(gpu, O):
    H, W = 257, 300
    with gpu.Engine(H, W) as a, gpu.Engine(H, W) as b:
        for e in (a, b):
            e.fill_random(0)
            e.add_diffuse(0, RATE)
        a.set_timing(True)
        a.run(20)
        b.run(20)
        n, ms, bytes_per = a.timing()
        per = a.info()["steps_per_launch"]
        assert per >= 4  # one attribute, one diffusion: K >= 4 fused steps per pass
        assert n == -(-20 // per) and ms > 0 and bytes_per == 16.0 * H * W
        assert np.array_equal(a.download(), b.download())
        assert np.array_equal(a.download(), O.field_step(O.fill_random(H, W), RATE, steps=20))


def make_env_engine(gpu, monkeypatch, H, W, n_attr=1, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    e = gpu.Engine(H, W, n_attr=n_attr)
    for k in env:
        monkeypatch.delenv(k)
    return e


# every way the engine can run a single-diffusion program: one step per pass, and the
# K-step overlapped-strip kernel at each K / row block / block order
# (the default {} on these small slabs: mm_wide_kernel K = 8 passes; MM_WIDE=0 pins
# mm_passk_kernel)
FUSE_ENVS = [{"MM_PASSK": 0}, {}, {"MM_WIDE": 0}] + [
    {"MM_WIDE": 0, "MM_STEPS_PER_PASS": k} for k in (1, 2, 3, 5, 6, 7, 8, 9, 10)
] + [{"MM_WIDE": 0, **e} for e in (
    {"MM_SEG_WAVES": 64}, {"MM_SEG_WAVES": 0.01}, {"MM_SEG_EDGE": 1.0}, {"MM_XCD_REMAP": 1},
    {"MM_KERNEL_VARIANT": 1}, {"MM_STEPS_PER_PASS": 3, "MM_SEG_WAVES": 16})]
# the level-split kernel (mm_wide_kernel) at each of its K, and its plan / order knobs
WIDE_ENVS = [{"MM_WIDE": 1}] + [{"MM_WIDE": 1, "MM_STEPS_PER_PASS": k} for k in (4, 8, 12, 16, 20)] + [
    {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 8, "MM_SEG_WAVES": 64},
    {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 12, "MM_SEG_WAVES": 0.01},
    {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 16, "MM_SEG_EDGE": 1.0},
    {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 20, "MM_SEG_WAVES": 3},
    {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 12, "MM_KERNEL_VARIANT": 1},
    {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 4, "MM_KERNEL_VARIANT": 1}]


def env_id(env):
    return ",".join(f"{k[3:]}={v}" for k, v in env.items()) or "default"


FUSE_SHAPES = [(1, 1), (2, 3), (3, 5), (5, 2), (37, 53), (130, 257), (257, 300), (64, 1000),
               (9, 124), (70, 125), (33, 241), (100, 488)]


@pytest.mark.parametrize("env", FUSE_ENVS + WIDE_ENVS, ids=env_id)
@pytest.mark.parametrize("shape", FUSE_SHAPES + [(45, 700), (257, 512), (70, 1025), (300, 233)])
def test_fused_steps_equal_single_steps(gpu, O, monkeypatch, env, shape):
    # K steps per pass (temporal blocking) against the oracle's single steps; step counts
    # that are not multiples of K end with a shorter pass. Run lengths: 1, 3, 5 (the
    # passes of mm_passk_kernel), then K and K + 3 (a whole pass of the configured K, then
    # one with a tail)
    H, W = shape
    k = int(env.get("MM_STEPS_PER_PASS", 20 if env.get("MM_WIDE") else 10))
    runs = (1, 3, 5, k, k + 3)
    v0 = O.fill_random(H, W)
    want = {}
    ref = v0
    for s in range(1, sum(runs) + 1):
        ref = O.field_step(ref, 0.3)
        want[s] = ref
    e = make_env_engine(gpu, monkeypatch, H, W, **env)
    e.fill_random(0)
    e.add_diffuse(0, 0.3)
    done = 0
    for steps in runs:
        e.run(steps)
        done += steps
        assert np.array_equal(e.download(), want[done]), (env, shape, done)
    e.close()


@pytest.mark.parametrize("env", [{}, {"MM_WIDE": 0}]
                         + [{"MM_WIDE": 0, "MM_STEPS_PER_PASS": k} for k in (3, 2, 8, 6, 7, 10)]
                         + [{"MM_PASSK": 0}]
                         + [{"MM_WIDE": 1, "MM_STEPS_PER_PASS": k} for k in (4, 8, 12, 16, 20)],
                         ids=env_id)
@pytest.mark.parametrize("reduce_every", [1, 2, 3, 4, 5])
def test_fused_steps_step_sums(gpu, O, monkeypatch, env, reduce_every):
    H, W = 130, 257
    steps = max(12, 2 * int(env.get("MM_STEPS_PER_PASS", 0)) + 3)
    v = O.fill_random(H, W)
    e = make_env_engine(gpu, monkeypatch, H, W, **env)
    e.upload(v)
    e.add_diffuse(0, RATE)
    e.run(steps, reduce_every)
    hist = e.sums_history()
    got = e.download()
    e.close()
    want = []
    ref = v
    for k in range(1, steps + 1):
        ref = O.field_step(ref, RATE)
        if k % reduce_every == 0:
            want.append(math.fsum(ref.ravel()))
    assert np.array_equal(got, ref)
    assert hist.shape == (len(want), 1)
    for a, b in zip(hist[:, 0], want):
        assert abs(a - b) <= 1e-12 * b


@pytest.mark.parametrize("k,wide", [(k, 0) for k in (2, 3, 4, 6, 7, 8, 9, 10)]
                         + [(k, 1) for k in (4, 8, 12, 16, 20)])
def test_fused_steps_graph_replay_many_steps(gpu, O, monkeypatch, k, wide):
    # hipGraph replay of K-step passes with sums every 3rd step; 50 steps is not a
    # multiple of the graph length, so the tail runs eagerly (K >= 10: a graph holds
    # 6K steps -- an even number of flips and whole reduction periods -- so run 13K)
    H, W, steps = 300, 700, (50 if k < 10 else 13 * k)
    e = make_env_engine(gpu, monkeypatch, H, W, MM_STEPS_PER_PASS=k, MM_WIDE=wide)
    e.fill_random(0)
    e.add_diffuse(0, 0.2)
    e.run(steps, 3)
    got = e.download()
    hist = e.sums_history()
    info = e.info()
    e.close()
    # the steps really were replayed as hipGraphs (a refused capture would run eagerly)
    assert info["graph_state"] == 1 and info["graph_launches"] >= 1, info
    assert info["hist_entries"] == steps // 3
    ref = O.fill_random(H, W)
    sums = []
    for s in range(1, steps + 1):
        ref = O.field_step(ref, 0.2)
        if s % 3 == 0:
            sums.append(math.fsum(ref.ravel()))
    assert np.array_equal(got, ref)
    assert hist.shape == (len(sums), 1)
    for a, b in zip(hist[:, 0], sums):
        assert abs(a - b) <= 1e-12 * b


@pytest.mark.parametrize("max_launches,launches", [(None, 1), (3, 4), (1, 6)])
def test_graph_length_divides_run(gpu, O, monkeypatch, max_launches, launches):
    # a run that is a whole number of passes replays as the longest graph dividing it (up
    # to MM_GRAPH_MAX_LAUNCHES step kernels): 96 steps of K = 8 with per-step sums are one
    # graph of 12 passes by default; 3 passes per graph (an odd number of buffer flips, so
    # launches alternate between the two parities' graphs) replay more; a cap under the
    # 16 steps of MM_GRAPH_MIN_STEPS leaves 2-pass graphs
    H, W, steps = 300, 700, 96
    env = {"MM_STEPS_PER_PASS": 8, "MM_WIDE": 1}
    if max_launches is not None:
        env["MM_GRAPH_MAX_LAUNCHES"] = max_launches
    e = make_env_engine(gpu, monkeypatch, H, W, **env)
    e.fill_random(0)
    e.add_diffuse(0, 0.2)
    e.prepare(steps, 1)
    e.run(steps, 1)
    got = e.download()
    hist = e.sums_history()
    info = e.info()
    e.close()
    assert info["graph_state"] == 1 and info["graph_launches"] == launches, info
    want, sums = O.program_step([O.fill_random(H, W)], [(1, 0, 0, 0.2)], steps=steps,
                                sums_per_step=True)
    assert np.array_equal(got, want[0])
    assert hist.shape == (steps, 1)
    for s, row in enumerate(sums):
        assert abs(hist[s, 0] - row[0]) <= 1e-12 * abs(row[0]), s


C5_FLOWS = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
            (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]


def add_flows(e, flows):
    for kind, a, b, r in flows:
        if kind == 1:
            e.add_diffuse(a, r)
        else:
            e.add_transfer(a, b, r)


@pytest.mark.parametrize("env", [{}, {"MM_STEPS_PER_PASS": 1}, {"MM_PASSK": 0},
                                 {"MM_SEG_WAVES": 64}, {"MM_WIDE": 0}], ids=env_id)
@pytest.mark.parametrize("flows,n_attr", [
    (C5_FLOWS, 4),
    ([(1, 0, 0, 0.1), (2, 0, 1, 0.2), (1, 1, 1, 0.3)], 2),       # post-chain, then a 2nd pass
    ([(2, 0, -1, 0.01), (1, 0, 0, 0.1), (1, 0, 0, 0.2)], 1),      # sink, two diffusions of a
    ([(2, 2, 0, 0.5), (1, 1, 1, 0.1), (2, 1, 2, 0.1)], 3),        # pre + post chain, one pass
    ([(1, 0, 0, 0.2), (1, 1, 1, 0.3)], 2),                        # two diffusions, one pass
    ([(2, 0, 1, 0.1), (2, 2, 3, 0.2), (2, 3, -1, 0.05)], 4),     # four attributes, transfers only
    ([(2, 3, 1, 0.1), (1, 3, 3, 0.2), (1, 1, 1, 0.1)], 4),       # diffusing attributes last
])
@pytest.mark.parametrize("shape", [(67, 300), (5, 130), (130, 9)])
def test_flow_program_bit_exact(gpu, O, monkeypatch, env, flows, n_attr, shape):
    H, W = shape
    steps = 5
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(n_attr)]
    want, sums = O.program_step(fields, flows, steps=steps, sums_per_step=True)
    e = make_env_engine(gpu, monkeypatch, H, W, n_attr=n_attr, **env)
    for a in range(n_attr):
        e.fill_random(a, seed=O.SEED + a)
    add_flows(e, flows)
    e.run(steps, reduce_every=1)
    got = [e.download(a) for a in range(n_attr)]
    hist = e.sums_history()
    e.close()
    for a in range(n_attr):
        assert np.array_equal(got[a], want[a]), a
    assert hist.shape == (steps, n_attr)
    for k in range(steps):
        for a in range(n_attr):
            w = sums[k][a]
            assert abs(hist[k, a] - w) <= 1e-12 * abs(w), (k, a)


# four-attribute one-pass programs on the level-split kernel (mm_wide_kernel, 2 columns per
# lane, K = 8 / 4 passes): C5, and a pre-chain + two of four attributes diffusing + a post-
# chain with a sink -- the non-diffusing attributes pass through every level
WIDE_PROGRAMS = [
    C5_FLOWS,  # its pre-chain is the ring t -> t+1 mod 4: the compile-time-chain instance
    [(2, 0, 1, 0.1), (1, 0, 0, 0.1), (1, 2, 2, 0.2), (2, 3, 1, 0.05), (2, 2, -1, 0.01)],
    # the ring's transfers in another order: not the ring, the generic chain
    [C5_FLOWS[1], C5_FLOWS[0], C5_FLOWS[2], C5_FLOWS[3]] + C5_FLOWS[4:],
    # a self-transfer (a -> a: u_a - out, then + out), a sink, repeated operands, a post-
    # chain of four
    [(2, 2, 2, 0.3), (2, 0, -1, 0.02), (2, 0, 3, 0.1), (2, 3, 0, 0.2), (1, 0, 0, 0.1),
     (1, 1, 1, 0.2), (1, 3, 3, 0.05), (2, 1, 2, 0.1), (2, 2, 1, 0.15), (2, 1, -1, 0.01),
     (2, 3, 3, 0.5)],
    # four diffusions, no transfer at all (every chain slot on the pad)
    C5_FLOWS[4:],
]


@pytest.mark.parametrize("env", [{"MM_WIDE": 1}, {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 4},
                                 {"MM_WIDE": 1, "MM_SEG_WAVES": 0.01},
                                 {"MM_WIDE": 1, "MM_KERNEL_VARIANT": 1},
                                 # variant bits beyond 0 must not select the ring instance
                                 # for a program that is not the ring
                                 {"MM_WIDE": 1, "MM_KERNEL_VARIANT": 3},
                                 # C5's ring on the run-time-operand chain too
                                 {"MM_WIDE": 1, "MM_CHAIN_RING": 0}],
                         ids=env_id)
@pytest.mark.parametrize("prog", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("shape", [(67, 300), (5, 130), (130, 9), (45, 700), (257, 512)])
def test_flow_program_wide_kernel(gpu, O, monkeypatch, env, prog, shape):
    H, W = shape
    flows = WIDE_PROGRAMS[prog]
    steps = 21  # 8 + 8 + 4 + 1 at K = 8
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    want, sums = O.program_step(fields, flows, steps=steps, sums_per_step=True)
    e = make_env_engine(gpu, monkeypatch, H, W, n_attr=4, **env)
    for a in range(4):
        e.fill_random(a, seed=O.SEED + a)
    add_flows(e, flows)
    assert e.info()["kernel"] == 3
    k = int(env.get("MM_STEPS_PER_PASS", 8))
    # K = 8: the ring instance for C5's chain, the run-time-operand chain otherwise
    ring = prog == 0 and k == 8 and env.get("MM_CHAIN_RING", 1) != 0
    assert e.info()["chain_kernel"] == (gpu.MM_CHAIN_RING if ring else gpu.MM_CHAIN_RUNTIME)
    plan = e.pass_plan(steps)
    assert sum(plan) == steps and plan[0] == k
    assert all(e.pass_kernel(p)[0] == (3 if p in (4, 8) else 2) for p in plan)
    e.run(steps, reduce_every=1)
    got = [e.download(a) for a in range(4)]
    hist = e.sums_history()
    e.close()
    for a in range(4):
        assert np.array_equal(got[a], want[a]), (a, int(np.count_nonzero(got[a] != want[a])))
    assert hist.shape == (steps, 4)
    for s_ in range(steps):
        for a in range(4):
            w = sums[s_][a]
            assert abs(hist[s_, a] - w) <= 1e-12 * abs(w), (s_, a)


def test_fill_after_freed_engine(gpu, O):
    """A new engine's zeroing (hipMemset on the null stream) must be complete before its
    fill runs on the engine's non-blocking stream: with memory another engine just freed
    the fill used to be partly zeroed (found by a host-halo chain after C5 runs)."""
    for rep in range(4):
        with gpu.Engine(257, 512, n_attr=4) as big:
            for a in range(4):
                big.fill_random(a, seed=O.SEED + a)
            big.add_diffuse(0, 0.1)
            big.run(2, 1)
        H, W = 64 + rep, 300
        with gpu.Engine(H, W, 0, H // 2, rank=0, nranks=2, halo_mode=gpu.MM_HALO_HOST) as e:
            e.fill_random(0)
            assert np.array_equal(e.download(), O.fill_random(H, W)[:H // 2]), rep


def test_large_grid_properties(gpu, O):
    # full-size checks via size-independent properties: conservation and exact
    # mirror symmetry of the 4096^2 (config C2 shape) step, plus the top and bottom
    # 64-row blocks (every column: both edge strips) compared with the oracle run on
    # the block widened by the 20-row dependency cone
    H = W = 4096
    steps = 20
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        s0 = e.sums()[0]
        e.add_diffuse(0, RATE)
        e.run(steps)
        v = e.download()
        s1 = e.sums()[0]
    assert abs(s1 - s0) <= 1e-12 * s0
    for lo, hi, blk in ((0, 64 + steps, slice(0, 64)), (H - 64 - steps, H, slice(steps, None))):
        band = O.fill_random(H, W, lo, hi - lo)
        for _ in range(steps):
            vg = np.zeros((band.shape[0] + 2, W))
            vg[1:-1] = band
            band = O.field_step_slab(H, W, lo, vg, RATE)
        assert np.array_equal(v[lo:hi][blk], band[blk]), lo
    v0 = O.fill_random(H, W)
    assert abs(math.fsum(v0.ravel()) - s0) <= 1e-12 * s0
    with gpu.Engine(H, W) as e:
        e.upload(v0[::-1, ::-1].copy())
        e.add_diffuse(0, RATE)
        e.run(steps)
        vf = e.download()
    assert np.array_equal(vf, v[::-1, ::-1])


def test_uniform_field_interior_fixed_point(gpu):
    with gpu.Engine(512, 640) as e:
        e.fill(0, value=1.0)
        e.add_diffuse(0, 0.25)
        e.run(10)
        v = e.download()
    assert np.all(v[11:-11, 11:-11] == 1.0)


def test_engine_rejects_bad_shapes(gpu):
    with pytest.raises(gpu.MMError):
        gpu.Engine(10, 10, x_init=5, h=6, nranks=2, rank=1, halo_mode=gpu.MM_HALO_HOST)
    with pytest.raises(gpu.MMError):
        gpu.Engine(10, 10, n_attr=5)
    with gpu.Engine(8, 8) as e:
        with pytest.raises(gpu.MMError):
            e.run(1)  # no flow
        with pytest.raises(gpu.MMError):
            e.point_apply(8, 0, 1.0, 0.1)


@pytest.mark.parametrize("k,wide", [(k, 0) for k in (1, 2, 3, 4, 6, 7, 8, 9, 10)]
                         + [(k, 1) for k in (4, 8, 12, 16, 20)])
@pytest.mark.parametrize("graph", [0, 1])
def test_rccl_halo_path_single_rank(gpu, O, monkeypatch, k, graph, wide):
    # The RCCL halo path on one GPU: one rank whose two neighbours are itself
    # (MM_SELF_HALO). Border rows go through ncclSend/ncclRecv on the comm stream, the
    # interior rows run meanwhile, the border rows after the event join -- eagerly and
    # captured in a hipGraph. The received rows land in ghost rows outside the grid, so
    # the cells must still match the oracle bit for bit. k = 1 runs the one-step
    # kernel; k >= 2 the K-step kernel with a k-row halo every k steps.
    H, W = 64, 300
    depth = k
    steps = 2 * depth  # two passes: afterwards the current buffer's ghost rows hold the
                       # rows exchanged in the first pass (the initial state's)
    env = {"MM_SELF_HALO": 1, "MM_GRAPH": graph, "MM_WIDE": wide}
    env.update({"MM_PASSK": 0} if k == 1 else {"MM_STEPS_PER_PASS": k})
    for key, v in env.items():
        monkeypatch.setenv(key, str(v))
    e = gpu.Engine(H, W, halo_mode=gpu.MM_HALO_RCCL, comm_id_bytes=gpu.comm_id())
    for key in env:
        monkeypatch.delenv(key)
    v0 = O.fill_random(H, W)
    e.fill_random(0)
    e.add_diffuse(0, RATE)
    assert e.info()["steps_per_launch"] == k
    e.run(steps, reduce_every=1)
    got = e.download()
    top = e.read_rows(-depth, depth)
    bot = e.read_rows(H, depth)
    hist = e.sums_history()
    info = e.info()
    e.close()
    # graph=1: the RCCL calls were captured and replayed, not silently run eagerly
    if graph:
        assert info["graph_state"] == 1 and info["graph_launches"] == 1, info
    else:
        assert info["graph_state"] == 0 and info["graph_launches"] == 0, info
    ref = v0
    sums = []
    for _ in range(steps):
        ref = O.field_step(ref, RATE)
        sums.append(math.fsum(ref.ravel()))
    assert np.array_equal(got, ref)
    assert np.array_equal(bot, v0[:depth])        # first rows -> bottom ghost rows
    assert np.array_equal(top, v0[H - depth:])    # last rows -> top ghost rows
    for a, b in zip(hist[:, 0], sums):
        assert abs(a - b) <= 1e-12 * b


def test_rccl_halo_path_many_steps(gpu, O, monkeypatch):
    # graph replay of RCCL calls over many steps, odd step count (fused pairs + one single)
    monkeypatch.setenv("MM_SELF_HALO", "1")
    H, W, steps = 200, 520, 25
    e = gpu.Engine(H, W, halo_mode=gpu.MM_HALO_RCCL, comm_id_bytes=gpu.comm_id())
    monkeypatch.delenv("MM_SELF_HALO")
    e.fill_random(0)
    e.add_diffuse(0, RATE)
    e.run(steps)
    got = e.download()
    e.close()
    assert np.array_equal(got, O.field_step(O.fill_random(H, W), RATE, steps=steps))


@pytest.mark.parametrize("wide", [0, 1])
@pytest.mark.parametrize("G", [1, 2])
def test_prepare_primes_eager_passes_without_running(gpu, O, monkeypatch, wide, G):
    """mm_prepare's priming: with graphs off, every planned pass is eager, and prepare
    dispatches each planned kernel once with no work -- on the compute stream, and on the
    comm stream for a split slab (G = 2: host-halo chain) -- without touching a buffer."""
    H, W, steps = 240, 700, 17
    monkeypatch.setenv("MM_GRAPH", "0")
    monkeypatch.setenv("MM_WIDE", str(wide))
    monkeypatch.setenv("MM_STEPS_PER_PASS", "8" if wide else "6")
    es = []
    try:
        for g in range(G):
            x0, h = gpu.partition_rows(H, G, g)
            es.append(gpu.Engine(H, W, x0, h, rank=g, nranks=G,
                                 halo_mode=gpu.MM_HALO_HOST if G > 1 else 0))
        for e in es:
            e.fill_random(0)
            e.add_diffuse(0, 0.2)
        plan = es[0].pass_plan(steps)
        for e in es:
            if G == 1:
                e.prepare(steps)
            else:  # the host transport runs one pass per call: prepare each pass length
                for k in sorted(set(plan)):
                    e.prepare(k)
            assert e.info()["steps_done"] == 0
        assert np.array_equal(np.vstack([e.download() for e in es]), O.fill_random(H, W))
        for k in plan:
            if G > 1:
                halos = [e.halo_export(k) for e in es]
                for g, e in enumerate(es):
                    e.halo_import(halos[g - 1][1] if g > 0 else None,
                                  halos[g + 1][0] if g < G - 1 else None, nrows=k)
            for e in es:
                e.run(k)
        got = np.vstack([e.download() for e in es])
    finally:
        for e in es:
            e.close()
    assert np.array_equal(got, O.field_step(O.fill_random(H, W), 0.2, steps=steps))


@pytest.mark.parametrize("warmup", [0, 3])
def test_prepare_captures_graph_without_running(gpu, O, warmup):
    # mm_prepare does a run's one-time work (graph capture for both buffer parities, tail
    # plan) and runs no step; warmup steps after it (bench.py's order) leave the state at
    # either parity, and the timed run still replays a prepared graph without capturing
    H, W, steps = 300, 700, 20
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        e.add_diffuse(0, 0.2)
        e.prepare(steps)
        i0 = e.info()
        assert i0["graph_count"] == 2 and i0["steps_done"] == 0 and i0["graph_launches"] == 0
        assert np.array_equal(e.download(), O.fill_random(H, W))
        e.run(warmup)
        n_graphs = e.info()["graph_count"]
        e.run(steps)
        i1 = e.info()
        got = e.download()
    assert i1["graph_count"] == n_graphs and i1["graph_launches"] >= 1
    assert np.array_equal(got, O.field_step(O.fill_random(H, W), 0.2, steps=warmup + steps))
