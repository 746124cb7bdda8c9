"""Linked passes (mm_wide_link_kernel): the K = 8 passes of a one-rank run without step
sums in ONE launch, workgroups taking (pass, segment) tickets and waiting on the previous
pass's neighbouring segments through per-segment flags. Every case is compared bit for
bit with the oracle AND with the same run launched one pass per kernel
(MM_LINK_PASSES=0), so a stale read anywhere in a hand-off shows as a changed cell.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RATE = 0.1  # src/Main.cpp:33


def run(gpu, O, monkeypatch, H, W, steps, link, reduce_every=0, runs=1):
    monkeypatch.setenv("MM_LINK_PASSES", "1" if link else "0")
    with gpu.Engine(H, W) as e:
        e.fill_random(0)
        e.add_diffuse(0, RATE)
        for _ in range(runs):
            e.run(steps, reduce_every)
        e.synchronize()  # fails if a segment's wait timed out
        info = e.info()
        return e.download(), (e.sums_history() if reduce_every else None), info


# ragged and tiny grids (one or two strips: seg_map's ns < 3 branch; a few rows per
# segment), the C2 grid (18 strips, 760 segments per pass: every workgroup slot busy)
@pytest.mark.parametrize("H,W,steps", [(130, 257, 40), (37, 53, 24), (300, 1000, 64),
                                       (1000, 130, 32), (9, 700, 16), (2048, 2048, 48),
                                       (4096, 4096, 40)])
def test_linked_passes_bit_exact(gpu, O, monkeypatch, H, W, steps):
    got, _, info = run(gpu, O, monkeypatch, H, W, steps, True)
    assert info["kernel"] == 3 and info["steps_per_launch"] == 8, info
    assert info["linked_launches"] >= 1, info
    want = O.field_rows(H, W, 0, H, steps, RATE)
    assert int(np.count_nonzero(got != want)) == 0
    ref, _, info0 = run(gpu, O, monkeypatch, H, W, steps, False)
    assert info0["linked_launches"] == 0
    assert np.array_equal(got, ref)


def test_linked_graph_replays_keep_epochs(gpu, O, monkeypatch):
    """Five runs of 64 steps: the first captures a graph (one linked launch of 8 passes),
    the others replay it -- each launch must start from the ticket / epoch the previous one
    left (the last workgroup out resets them)."""
    H, W = 1024, 1536
    got, _, info = run(gpu, O, monkeypatch, H, W, 64, True, runs=5)
    assert info["graph_launches"] >= 4 and info["linked_launches"] >= 1, info
    want = O.field_rows(H, W, 0, H, 320, RATE)
    assert int(np.count_nonzero(got != want)) == 0


def test_linked_run_with_final_sums(gpu, O, monkeypatch):
    """Sums only after the last step: the passes before it link, the last one reduces."""
    H, W, steps = 512, 700, 64
    got, hist, info = run(gpu, O, monkeypatch, H, W, steps, True, reduce_every=steps)
    assert info["linked_launches"] >= 1
    want = O.field_rows(H, W, 0, H, steps, RATE)
    assert int(np.count_nonzero(got != want)) == 0
    assert hist.shape == (1, 1)
    tot = O.csum(want)
    assert abs(hist[0, 0] - tot) <= 1e-12 * tot


def test_sums_every_pass_do_not_link(gpu, O, monkeypatch):
    H, W, steps = 256, 300, 32
    got, hist, info = run(gpu, O, monkeypatch, H, W, steps, True, reduce_every=8)
    assert info["linked_launches"] == 0
    assert hist.shape == (4, 1)
    assert int(np.count_nonzero(got != O.field_rows(H, W, 0, H, steps, RATE))) == 0
