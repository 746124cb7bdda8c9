"""CPU tests: the oracle against the reference's golden grids, and its invariants.

The reference (daviidsilvaa/MPI-Model) has no tests of its own;
its only built-in check is the conservation assert src/Model.hpp:95. These tests
pin the C restatement (oracle/mm_oracle.c) to fixtures produced by the reference
itself (tests/golden/make_golden.py), then check the generalised step's invariants.
"""
import math
import os

import numpy as np
import pytest

from conftest import golden, golden_points


@pytest.mark.parametrize("name", golden_points())
def test_point_apply_matches_reference_golden(O, name):
    g = golden(name)
    H, W = g["dimx"], g["dimy"]
    v = np.ones((H, W))
    v = O.point_apply(v, g["src_x"], g["src_y"], float.fromhex(g["value_hex"]),
                      float.fromhex(g["rate_hex"]))
    changed = sorted([x, y, val.hex()] for (x, y), val in np.ndenumerate(v) if val != 1.0)
    assert changed == g["changed"]
    assert math.fsum(v.ravel()).hex() == g["sum_fsum_hex"]


def test_default_golden_values_section0(O):
    # source 0.78, its 8 neighbours 1.0275 (3 of them via halo)
    g = golden("point_100_100_5_0.json")
    vals = {(x, y): float.fromhex(h) for x, y, h in g["changed"]}
    assert vals[(19, 3)].hex() == "0x1.8f5c28f5c28f6p-1"
    for c in [(18, 2), (18, 3), (18, 4), (19, 2), (19, 4), (20, 2), (20, 3), (20, 4)]:
        assert vals[c].hex() == "0x1.070a3d70a3d71p+0"


@pytest.mark.parametrize("name", golden_points())
def test_general_step_with_point_outflow_is_reference_update(O, name):
    # the generalised step with outflow zero everywhere but the source IS the
    # reference's single-source update (src/Model.hpp:176-235), bit for bit
    g = golden(name)
    H, W = g["dimx"], g["dimy"]
    v = np.ones((H, W))
    outf = np.zeros((H, W))
    outf[g["src_x"], g["src_y"]] = float.fromhex(g["rate_hex"]) * float.fromhex(g["value_hex"])
    o = O.field_step_general(v, outf)
    assert np.array_equal(o, O.point_apply(v, g["src_x"], g["src_y"],
                                           float.fromhex(g["value_hex"]),
                                           float.fromhex(g["rate_hex"])))


@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (2, 2), (3, 5), (37, 53), (64, 130)])
def test_uniform_rate_step_equals_general_form(O, shape):
    H, W = shape
    v = O.fill_random(H, W)
    # a cell without neighbours (1x1 grid) cannot emit: its outflow is 0
    emits = np.array([[O.neighbor_count(H, W, x, y) > 0 for y in range(W)] for x in range(H)])
    outf = np.where(emits, 0.1 * v, 0.0)
    # the reference's update written per emitter (shares) against the whole-grid step's
    # per-receiver form (r/8 factored out of the neighbours' weights): the same sum,
    # rounded differently -- a few ulp (mm_oracle.h)
    got, want = O.field_step(v, 0.1), O.field_step_general(v, outf)
    assert np.max(np.abs(got - want) / np.abs(want)) <= 1e-14


def _contract_step(O, v, rate):
    """oracle/mm_oracle.h's arithmetic contract restated in plain Python, the two fma exact
    (Fraction, then one rounding): w = v * 8/cnt; row-paired column triples; column-paired
    box sums S; v' = fma(fma(v, -(8 + 8/cnt), S), r/8, v)."""
    from fractions import Fraction

    def fma(a, b, c):
        return float(Fraction(a) * Fraction(b) + Fraction(c))

    H, W = v.shape

    def c8(c):
        return 1.0 if c == 8 else (8.0 / c if c > 0 else 0.0)

    w = np.zeros((H + 2, W + 2))
    for x in range(H):
        for y in range(W):
            w[x + 1, y + 1] = v[x, y] * c8(O.neighbor_count(H, W, x, y))
    cw = np.zeros((H, W + 2))
    for x in range(H):
        for y in range(W + 2):
            a, b, c = w[x, y], w[x + 1, y], w[x + 2, y]
            cw[x, y] = a + (b + c) if x % 2 == 0 else (a + b) + c
    out = v.copy()
    for x in range(H):
        for y in range(W):
            n = O.neighbor_count(H, W, x, y)
            if n == 0:
                continue
            a, b, c = cw[x, y], cw[x, y + 1], cw[x, y + 2]
            s = a + (b + c) if y % 2 == 0 else (a + b) + c
            out[x, y] = fma(fma(v[x, y], -(8.0 + c8(n)), s), rate * 0.125, v[x, y])
    return out


@pytest.mark.parametrize("shape", [(1, 1), (1, 6), (5, 1), (2, 2), (3, 3), (7, 9), (8, 10),
                                   (13, 6)])
@pytest.mark.parametrize("rate", [0.1, 0.37])
def test_oracle_step_is_the_written_contract(O, shape, rate):
    v = O.fill_random(*shape)
    assert np.array_equal(O.field_step(v, rate), _contract_step(O, v, rate))


def _emitter_steps(O, v, rate, steps):
    """The reference's own update iterated: every cell with neighbours emits out = r*v and
    each neighbour receives out/cnt (or_field_step_general, src/Model.hpp:199,206-211,234;
    src/Exponencial.hpp:14-16)."""
    H, W = v.shape
    emits = np.array([[O.neighbor_count(H, W, x, y) > 0 for y in range(W)] for x in range(H)])
    for _ in range(steps):
        v = O.field_step_general(v, np.where(emits, rate * v, 0.0))
    return v


# 2-row, 2-column, 2x2 and 3x3 grids are all edge / corner cells (the rounded 8/5 and 8/3
# weights of the per-receiver form dominate); 64x96 and 130x97 mix every count class
@pytest.mark.parametrize("shape,steps", [((2, 50), 1000), ((50, 2), 1000), ((2, 2), 1000),
                                         ((3, 3), 1000), ((64, 96), 1000), ((130, 97), 1000),
                                         ((200, 300), 20), ((1, 9), 20)])
@pytest.mark.parametrize("rate", [0.1, 0.3])
def test_whole_grid_step_tracks_reference_update_over_bench_steps(O, shape, steps, rate):
    """The kernels' (and the oracle's) per-receiver step against the reference's
    per-emitter update, iterated over the bench runs' step counts (20: the driver's line;
    1000: the long lines). Bound: north_star's 1e-12 relative per cell; measured <= 3.6e-14
    (DESIGN.md section 2). Both forms conserve the total to the same bound."""
    v = O.fill_random(*shape)
    got, want = O.field_step(v, rate, steps=steps), _emitter_steps(O, v, rate, steps)
    assert np.max(np.abs(got - want) / np.abs(want)) <= 1e-12
    s0 = math.fsum(v.ravel())
    for f in (got, want):
        assert abs(math.fsum(f.ravel()) - s0) <= 1e-12 * s0


@pytest.mark.parametrize("shape", [(2, 50), (3, 3), (64, 96)])
def test_program_diffusions_track_reference_update_over_1000_steps(O, shape):
    """C5's flow program (transfer ring, then four diffusions) with each diffusion as the
    reference's per-emitter update, against or_program_step (the kernels' per-receiver
    form), 1000 steps: every attribute within 1e-12 relative (measured <= 8.2e-15)."""
    H, W = shape
    emits = np.array([[O.neighbor_count(H, W, x, y) > 0 for y in range(W)] for x in range(H)])
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    want = [f.copy() for f in fields]
    for _ in range(1000):
        for kind, a, b, r in C5_FLOWS:
            if kind == O.DIFFUSE:
                want[a] = O.field_step_general(want[a], np.where(emits, r * want[a], 0.0))
            else:  # or_program_step's transfer: out = r*u_a; u_a -= out; u_b += out
                out = r * want[a]
                want[a] = want[a] - out
                want[b] = want[b] + out
    got = O.program_step(fields, C5_FLOWS, steps=1000)
    for g, w in zip(got, want):
        assert np.max(np.abs(g - w) / np.abs(w)) <= 1e-12


def test_step_count_matches_reference_loop(O):
    # fp64 accumulation of src/Model.hpp:48
    assert O.step_count(10.0, 0.2) == 51
    assert O.step_count(1.0, 0.1) == 11
    assert O.step_count(100.0, 0.1) == 1001
    assert O.step_count(1000.0, 1.0) == 1000


def test_neighbor_counts_match_cell_hpp(O):
    # src/Cell.hpp:71-157: corners 3, edges 5, interior 8 (grids >= 2x2)
    for H, W in [(2, 2), (3, 3), (100, 100), (5, 9)]:
        for x in range(H):
            for y in range(W):
                corner = x in (0, H - 1) and y in (0, W - 1)
                edge = (x in (0, H - 1) or y in (0, W - 1)) and not corner
                want = 3 if corner else (5 if edge else 8)
                if H == 2 or W == 2:  # 2-wide grids: no interior, edges as in Cell.hpp
                    want = 3 if corner else 5
                assert O.neighbor_count(H, W, x, y) == want


def test_conservation_and_uniform_fixed_point(O):
    v = O.fill_random(61, 47)
    o = O.field_step(v, 0.1, steps=20)
    s0, s1 = math.fsum(v.ravel()), math.fsum(o.ravel())
    assert abs(s1 - s0) <= 1e-12 * abs(s0)
    u = O.field_step(np.ones((20, 30)), 0.25, steps=5)
    # cells farther than steps+1 from the edge receive exactly what they emit
    # (rate 0.25: every share 1/32 is exact)
    assert np.all(u[6:-6, 6:-6] == 1.0)
    assert not np.all(u == 1.0)


def test_flip_symmetry_is_exact(O):
    # the rows and the columns are paired from an even index (oracle/mm_oracle.h), so a flip
    # of an axis of even length maps pairs onto pairs
    v = O.fill_random(34, 46)
    a = O.field_step(v, 0.25, steps=3)
    assert np.array_equal(O.field_step(v[::-1].copy(), 0.25, steps=3), a[::-1])
    assert np.array_equal(O.field_step(v[:, ::-1].copy(), 0.25, steps=3), a[:, ::-1])


@pytest.mark.parametrize("H,G", [(37, 1), (37, 2), (37, 3), (40, 4), (41, 8), (9, 9)])
def test_slab_decomposition_is_bit_exact(O, H, G):
    W = 29
    v = O.fill_random(H, W)
    want = O.field_step(v, 0.1)
    parts = []
    for g in range(G):
        x0, h = O.partition_rows(H, G, g)
        vg = np.zeros((h + 2, W))
        lo, hi = max(x0 - 1, 0), min(x0 + h + 1, H)
        vg[lo - (x0 - 1):hi - (x0 - 1)] = v[lo:hi]
        parts.append(O.field_step_slab(H, W, x0, vg, 0.1))
    assert np.array_equal(np.vstack(parts), want)


@pytest.mark.parametrize("H,W,steps", [(1, 1, 3), (2, 5, 2), (3, 3, 4), (5, 1, 3), (1, 7, 2),
                                       (37, 130, 7), (64, 300, 20), (130, 257, 9), (300, 700, 25)])
def test_field_rows_cone_is_the_full_step(O, H, W, steps):
    # or_field_rows (the full-size GPU tests' checker: rows on their dependency cone, the
    # counts hoisted, the fma on the FMA unit, row chunks in threads) against or_field_step
    # on the whole grid, bit for bit, for row ranges at both edges, inside, and one row
    want = O.field_step(O.fill_random(H, W), 0.3, steps=steps)
    for lo, hi in ((0, H), (H // 3, H - H // 4), (H - 1, H), (0, 1), (H // 2, H // 2 + 1)):
        for chunk in (None, 1, 5):
            got = O.field_rows(H, W, lo, hi, steps, 0.3, chunk=chunk)
            assert np.array_equal(got, want[lo:hi]), (H, W, steps, lo, hi, chunk)


@pytest.mark.parametrize("H,W,P,steps", [(37, 29, 3, 5), (16, 130, 4, 3), (9, 7, 2, 4)])
def test_cpu_mpi_baseline_is_the_oracle(O, tmp_path, H, W, P, steps):
    """The MPI CPU baseline (oracle/mm_cpu_mpi.c, bench.py's cpu_baseline leg) reproduces the
    oracle's whole-grid steps bit for bit across its row slabs and border-row exchange."""
    if not os.path.exists(os.path.join(O.MPI_HOME, "bin", "mpirun")):
        pytest.skip("no MPI")
    out = tmp_path / "grid.bin"
    r = O.cpu_mpi(H, W, 0.1, 0, P, maxsteps=-steps, dump=str(out), timeout=120)
    assert r["ranks"] == P and r["steps"] == steps
    got = np.fromfile(out, dtype=np.float64).reshape(H, W)
    want = O.field_step(O.fill_random(H, W), 0.1, steps=steps)
    assert np.array_equal(got, want)


C5_FLOWS = [(2, 0, 1, 0.05), (2, 1, 2, 0.03), (2, 2, 3, 0.02), (2, 3, 0, 0.01),
            (1, 0, 0, 0.1), (1, 1, 1, 0.1), (1, 2, 2, 0.05), (1, 3, 3, 0.2)]


@pytest.mark.parametrize("H,W,P,steps", [(37, 29, 3, 4), (16, 130, 4, 3)])
def test_cpu_mpi_program_baseline_is_the_oracle(O, tmp_path, H, W, P, steps):
    """The MPI CPU baseline's flow-program mode (config C5: 4 attributes, chained
    transfers + diffusions, per-step sums) reproduces or_program_step bit for bit."""
    if not os.path.exists(os.path.join(O.MPI_HOME, "bin", "mpirun")):
        pytest.skip("no MPI")
    out = tmp_path / "grid.bin"
    r = O.cpu_mpi(H, W, 0.1, 0, P, maxsteps=-steps, dump=str(out), timeout=120,
                  program=C5_FLOWS)
    assert r["ranks"] == P and r["steps"] == steps and r["n_attr"] == 4 and r["n_flows"] == 8
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    want = O.program_step(fields, C5_FLOWS, steps=steps)
    got = np.fromfile(out, dtype=np.float64).reshape(H, W)
    assert np.array_equal(got, want[0])
    total = math.fsum(np.concatenate([f.ravel() for f in want]))
    assert abs(r["total"] - total) <= 1e-12 * total


def test_program_step_conserves_total(O):
    H, W = 24, 40
    fields = [O.fill_random(H, W, seed=O.SEED + a) for a in range(4)]
    flows = [(O.TRANSFER, 0, 1, 0.05), (O.TRANSFER, 1, 2, 0.03), (O.TRANSFER, 2, 3, 0.02),
             (O.TRANSFER, 3, 0, 0.01), (O.DIFFUSE, 0, 0, 0.1), (O.DIFFUSE, 1, 1, 0.1),
             (O.DIFFUSE, 2, 2, 0.05), (O.DIFFUSE, 3, 3, 0.2)]
    out = O.program_step(fields, flows, steps=10)
    t0 = math.fsum(np.concatenate([f.ravel() for f in fields]))
    t1 = math.fsum(np.concatenate([f.ravel() for f in out]))
    assert abs(t1 - t0) <= 1e-12 * t0


def test_oracle_under_address_and_ub_sanitizers(O):
    """the restatement under ASan + UBSan (oracle/oracle_selftest.c:
    every function on degenerate and ragged grids, slab = whole-grid step, conservation)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", O.HERE, "asan"], check=True)
    r = subprocess.run([os.path.join(O.HERE, "_build", "oracle_selftest_asan")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle selftest ok" in r.stdout
