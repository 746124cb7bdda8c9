"""The production schedules of every N > 1 rank at full size, whole grids bit-exact.

Each multi-GPU configuration the driver runs (BASELINE.json configs[2..3]) is run here on
one GPU as a chain of engines, one per rank, exchanging the K-row halo through the host
transport (MM_HALO_HOST). A host-halo engine runs exactly the schedule it runs with RCCL
-- the interior workgroups on the compute stream beside the border segments on the comm
stream, joined by events -- with the neighbours' K rows already in its ghost rows instead
of arriving by ncclRecv (src/Model.hpp:202-204,224-235 made whole-row and K deep). So
each slab below is exactly the slab one GPU of that run holds, with its plan:

  * c3 at N = 8: 32768^2 as eight 4096 x 32768 slabs (one K = 20 pass of the level-split
    kernel per 20 steps, interior / border split; ranks 1..6 have both neighbours);
  * c3 at N = 4 and N = 2: four 8192-row and two 16384-row slabs;
  * c4 at N = 2 (weak: 16384^2 per GPU): 32768 x 16384 as two 16384^2 slabs;
  * one engine, 16384^2, 120 steps = 6 K = 20 passes replayed as one hipGraph.

Every slab is compared cell for cell with the oracle: oracle.field_rows computes the
slab's rows on their dependency cone in row chunks over the host's cores (bit-identical
to or_field_step, tests/test_oracle.py). The per-pass sums of all slabs, added in rank
order (src/Model.hpp:89-92), must match the oracle's to 1e-12.
"""
import numpy as np
import pytest

from test_gpu_halo import make_chain, run_chain, close

pytestmark = pytest.mark.gpu

RATE = 0.1  # src/Main.cpp:33


def check_chain(gpu, O, monkeypatch, H, W, G, steps, env=None):
    engines = make_chain(gpu, monkeypatch, H, W, G, env=env)
    try:
        for e in engines:
            e.fill_random(0)
            e.add_diffuse(0, RATE)
        info = engines[0].info()
        assert info["halo_depth"] == 20 and info["kernel"] == 3, info
        plan = engines[0].pass_plan(steps)
        assert plan == [20] * (steps // 20), plan
        assert all(e.pass_kernel(20)[0] == 3 for e in engines)
        run_chain(engines, steps, reduce_every=20)
        hists = [e.sums_history() for e in engines]
        tot = np.zeros(len(plan))
        want_tot = 0.0
        for g, e in enumerate(engines):
            x0, h = gpu.partition_rows(H, G, g)
            got = e.download()
            want = O.field_rows(H, W, x0, x0 + h, steps, RATE)
            bad = int(np.count_nonzero(got != want))
            assert bad == 0, (H, W, G, g, bad)
            want_tot += O.csum(want)
            del got, want
            assert hists[g].shape == (len(plan), 1)
            tot = tot + hists[g][:, 0]
    finally:
        close(engines)
    # the last pass's sums of all slabs against the oracle's grid (conserved: every pass
    # sums to the same total up to rounding)
    assert abs(tot[-1] - want_tot) <= 1e-12 * want_tot, (tot[-1], want_tot)
    assert np.all(np.abs(tot - want_tot) <= 1e-12 * want_tot)


@pytest.mark.parametrize("H,W,G", [(32768, 32768, 8), (32768, 32768, 4), (32768, 32768, 2),
                                   (32768, 16384, 2)],
                         ids=["c3_n8", "c3_n4", "c3_n2", "c4_n2"])
def test_rank_schedules_full_size(gpu, O, monkeypatch, H, W, G):
    """Two K = 20 passes (40 steps: the exchange before each) on every rank's slab."""
    check_chain(gpu, O, monkeypatch, H, W, G, 40)


def test_graph_replayed_k20_passes_full_size(gpu, O):
    """16384^2 (C4's per-GPU grid), 120 steps: six K = 20 passes of the level-split kernel
    captured into ONE hipGraph and replayed, against the oracle on the whole grid."""
    H = W = 16384
    steps = 120
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        e.add_diffuse(0, RATE)
        assert e.pass_plan(steps) == [20] * 6
        e.run(steps)
        e.synchronize()
        info = e.info()
        assert info["graph_state"] == 1 and info["graph_launches"] == 1, info
        got = e.download()
    want = O.field_rows(H, W, 0, H, steps, RATE)
    assert int(np.count_nonzero(got != want)) == 0
