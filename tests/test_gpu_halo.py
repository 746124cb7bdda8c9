"""The N>1 engine path on one GPU: G engines, one row slab each, exchanging `halo_depth`
border rows between K-step passes through the host transport (MM_HALO_HOST).

Each engine runs exactly the schedule it runs with RCCL -- interior segments on the
compute stream beside the border blocks on the comm stream, joined by events, per-wave
partials at partial_base offsets -- with the neighbours' K rows already in its ghost rows
instead of arriving by ncclRecv. So everything but the transport of the multi-GPU path
(src/Model.hpp:202-204,224-235 made whole-row and K deep) is checked here, bit for bit
against the oracle's single-process steps, with the per-step sums of all slabs against
math.fsum of the whole grid.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def make_chain(gpu, monkeypatch, H, W, G, n_attr=1, env=None):
    env = env or {}
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    engines = []
    try:
        for g in range(G):
            x0, h = gpu.partition_rows(H, G, g)
            engines.append(gpu.Engine(H, W, x0, h, n_attr=n_attr, rank=g, nranks=G,
                                      halo_mode=gpu.MM_HALO_HOST))
    finally:
        for k in env:
            monkeypatch.delenv(k)
    return engines


def run_chain(engines, steps, reduce_every=0):
    """Advance every slab `steps` steps: before each pass of the engines' (common) plan,
    that pass's depth of border rows is exchanged (mpimodel.run_host_halo's schedule)."""
    G = len(engines)
    depth = engines[0].info()["halo_depth"]
    assert all(e.info()["halo_depth"] == depth for e in engines)
    plan = engines[0].pass_plan(steps)
    assert all(e.pass_plan(steps) == plan for e in engines)
    for k in plan:
        halos = [e.halo_export(k) for e in engines]
        for g, e in enumerate(engines):
            e.halo_import(halos[g - 1][1] if g > 0 else None,
                          halos[g + 1][0] if g < G - 1 else None, nrows=k)
        for e in engines:
            e.run(k, reduce_every)
    return depth


def gather(engines, attr=0):
    return np.vstack([e.download(attr) for e in engines])


def close(engines):
    for e in engines:
        e.close()


# (H, W, G): slabs well above 2*depth+1 rows (interior / border split), barely above it,
# below it (one launch after the exchange), and thinner than K (K capped to min h)
CHAINS = [(64, 300, 2), (37, 130, 3), (27, 257, 3), (100, 488, 3), (41, 200, 8),
          (24, 257, 8), (16, 130, 8), (9, 124, 8), (300, 700, 2)]


WIDE_K = (4, 8, 12, 16, 20)  # mm_wide_kernel instances


@pytest.mark.parametrize("k,wide", [(k, 0) for k in (10, 9, 8, 7, 6, 5, 4, 3, 2, 1)]
                         + [(k, 1) for k in WIDE_K])
@pytest.mark.parametrize("H,W,G", CHAINS)
def test_deep_halo_chain_bit_exact(gpu, O, monkeypatch, H, W, G, k, wide):
    check_deep_chain(gpu, O, monkeypatch, H, W, G, k, wide)


def check_deep_chain(gpu, O, monkeypatch, H, W, G, k, wide, extra=None):
    # wide = 1: the level-split kernel wherever the depth is one of its K (a thinner
    # slab caps the depth to min h, which may leave mm_passk_kernel to run it)
    env = {"MM_STEPS_PER_PASS": k, "MM_WIDE": wide, **(extra or {})}
    engines = make_chain(gpu, monkeypatch, H, W, G, env=env)
    try:
        for e in engines:
            e.fill_random(0)
            e.add_diffuse(0, 0.3)
        info = engines[0].info()
        min_h = H // G
        assert info["halo_depth"] == min(k, min_h) == info["steps_per_launch"]
        assert info["kernel"] == (3 if wide and info["halo_depth"] in WIDE_K else 2)
        steps = 2 * info["halo_depth"] + 1  # two full passes and a shorter one
        run_chain(engines, steps)
        got = gather(engines)
    finally:
        close(engines)
    assert np.array_equal(got, O.field_step(O.fill_random(H, W), 0.3, steps=steps))


@pytest.mark.parametrize("env", [{}, {"MM_WIDE": 0}, {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 8},
                                 {"MM_WIDE": 1, "MM_STEPS_PER_PASS": 12}],
                         ids=lambda e: ",".join(f"{k[3:]}={v}" for k, v in e.items()) or "default")
@pytest.mark.parametrize("reduce_every", [1, 3])
@pytest.mark.parametrize("H,W,G", [(100, 488, 3), (41, 200, 8), (300, 700, 2), (130, 257, 4)])
def test_deep_halo_chain_step_sums(gpu, O, monkeypatch, H, W, G, reduce_every, env):
    # per-step sums of every slab (partials at partial_base offsets: interior segments
    # first, then the border blocks) summed over the slabs in rank order
    steps = 2 * env["MM_STEPS_PER_PASS"] + 1 if "MM_STEPS_PER_PASS" in env else 9
    engines = make_chain(gpu, monkeypatch, H, W, G, env=env)
    try:
        for e in engines:
            e.fill_random(0)
            e.add_diffuse(0, 0.1)
        run_chain(engines, steps, reduce_every)
        got = gather(engines)
        hists = [e.sums_history() for e in engines]
    finally:
        close(engines)
    ref = O.fill_random(H, W)
    want = []
    for s in range(1, steps + 1):
        ref = O.field_step(ref, 0.1)
        if s % reduce_every == 0:
            want.append(math.fsum(ref.ravel()))
    assert np.array_equal(got, ref)
    for hst in hists:
        assert hst.shape == (len(want), 1)
    tot = np.zeros(len(want))
    for hst in hists:  # rank order, as src/Model.hpp:89-92
        tot = tot + hst[:, 0]
    for a, b in zip(tot, want):
        assert abs(a - b) <= 1e-12 * b


C5_FLOWS = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
            (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]


@pytest.mark.parametrize("H,W,G", [(67, 300, 3), (40, 130, 8)])
def test_deep_halo_chain_flow_program(gpu, O, monkeypatch, H, W, G):
    # four attributes, chained transfers + four diffusions (config C5) on slabs: passes of
    # the level-split kernel (K = 8, 8, 4 on 22-row slabs; 4 on 5-row slabs), then a 1-step
    # mm_passk_kernel pass
    steps = 21
    na = 4
    engines = make_chain(gpu, monkeypatch, H, W, G, n_attr=na)
    try:
        for e in engines:
            for a in range(na):
                e.fill_random(a, seed=O.SEED + a)
            for kind, a, b, r in C5_FLOWS:
                if kind == 1:
                    e.add_diffuse(a, r)
                else:
                    e.add_transfer(a, b, r)
        # the level-split kernel's K = 8 for four attributes, capped by the thinnest slab
        assert engines[0].info()["halo_depth"] == min(8, H // G)
        run_chain(engines, steps, 1)
        got = [gather(engines, a) for a in range(na)]
        hists = [e.sums_history() for e in engines]
    finally:
        close(engines)
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(na)]
    want, sums = O.program_step(fields, C5_FLOWS, steps=steps, sums_per_step=True)
    for a in range(na):
        assert np.array_equal(got[a], want[a]), a
    tot = sum(h for h in hists)
    for s in range(steps):
        for a in range(na):
            assert abs(tot[s, a] - sums[s][a]) <= 1e-12 * abs(sums[s][a])


def test_one_step_kernel_chain(gpu, O, monkeypatch):
    # MM_PASSK=0: the one-step kernel with a 1-row halo on the same split schedule
    H, W, G, steps = 77, 300, 4, 5
    engines = make_chain(gpu, monkeypatch, H, W, G, env={"MM_PASSK": 0})
    try:
        for e in engines:
            e.fill_random(0)
            e.add_diffuse(0, 0.2)
        assert run_chain(engines, steps) == 1
        got = gather(engines)
    finally:
        close(engines)
    assert np.array_equal(got, O.field_step(O.fill_random(H, W), 0.2, steps=steps))


def test_host_halo_rejects_more_steps_than_depth(gpu, monkeypatch):
    engines = make_chain(gpu, monkeypatch, 64, 130, 2)
    try:
        e = engines[0]
        e.fill_random(0)
        e.add_diffuse(0, 0.1)
        d = e.info()["halo_depth"]
        with pytest.raises(gpu.MMError):
            e.run(d + 1)
        with pytest.raises(gpu.MMError):
            e.halo_export(21)  # more rows than the ghost zone (kGhost = 20) holds
    finally:
        close(engines)


def test_history_grows_past_initial_capacity(gpu, O):
    # more reduced steps than the history's first allocation: nothing is dropped
    H, W, steps = 8, 130, 5000
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        e.add_diffuse(0, 0.1)
        e.run(steps, 1)
        hist = e.sums_history(max_entries=steps)
        got = e.download()
        assert e.info()["hist_entries"] == steps
    assert hist.shape == (steps, 1)
    ref = O.fill_random(H, W)
    for s in range(steps):
        ref = O.field_step(ref, 0.1)
        if s in (0, 4095, 4096, steps - 1):
            assert abs(hist[s, 0] - math.fsum(ref.ravel())) <= 1e-12 * abs(hist[s, 0]), s
    assert np.array_equal(got, ref)
