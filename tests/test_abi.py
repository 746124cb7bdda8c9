"""CPU tests of the drop-in boundary: libmpimodel_hip.so loads, exports every symbol
include/mpimodel.h declares, and its host-only bookkeeping is bit-exact with the
reference (src/Model.hpp:47-80, src/Cell.hpp:71-157). No compute call is made
here: without a GPU the engine must refuse to start (it never falls back).
"""
import os
import re

import pytest

from conftest import REPO


def declared_functions():
    text = open(os.path.join(REPO, "include", "mpimodel.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mm_[a-z_]+)\s*\(", text)))


def test_header_and_binding_agree(mm):
    assert declared_functions() == sorted(mm.EXPORTS)


def test_library_exports_every_declared_symbol(mm):
    L = mm.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.mm_abi_version() == 2


def test_step_count(mm, O):
    for t, dt in [(10.0, 0.2), (1.0, 0.1), (100.0, 0.1), (1000.0, 1.0), (0.0, 1.0), (3.3, 0.7)]:
        assert mm.step_count(t, dt) == O.step_count(t, dt)
    assert mm.step_count(1.0, 0.0) == -1


def test_reference_partition_bit_exact(mm, O):
    for H, W, P in [(100, 100, 5), (40, 64, 4), (10, 10, 3), (10, 3, 4), (37, 11, 6), (7, 7, 7)]:
        for k in range(1, P + 1):
            assert mm.partition_reference(H, W, P, k) == O.partition_reference(H, W, P, k)
        for x in range(H):
            assert mm.owner_reference(H, P, x) == O.owner_reference(H, P, x)


def test_engine_partition_equals_reference_when_divisible(mm):
    for H, W, G in [(100, 100, 5), (32768, 32768, 8), (4096, 4096, 4), (16384 * 8, 16384, 8)]:
        if H * W >= 2 ** 31:  # the reference's int arithmetic overflows; compare rows only
            for g in range(G):
                assert mm.partition_rows(H, G, g) == (g * (H // G), H // G)
            continue
        for g in range(G):
            x0, y0, hh, ww = mm.partition_reference(H, W, G, g + 1)
            assert mm.partition_rows(H, G, g) == (x0, hh)


def test_engine_partition_covers_every_row(mm):
    for H in [1, 7, 37, 100, 4097]:
        for G in range(1, 9):
            if G > H:
                continue
            rows = []
            for g in range(G):
                x0, h = mm.partition_rows(H, G, g)
                assert h >= 1
                rows.extend(range(x0, x0 + h))
            assert rows == list(range(H))


def test_neighbor_count(mm, O):
    for H, W in [(1, 1), (1, 5), (2, 2), (3, 7), (100, 100)]:
        for x in range(-1, H + 1):
            for y in range(-1, W + 1):
                assert mm.neighbor_count(H, W, x, y) == O.neighbor_count(H, W, x, y)


def test_bad_arguments_are_errors(mm):
    with pytest.raises(mm.MMError):
        mm.partition_rows(10, 0, 0)
    with pytest.raises(mm.MMError):
        mm.partition_reference(10, 10, 3, 4)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_engine_refuses_to_start_without_gpu(mm):
    with pytest.raises(mm.MMError):
        mm.Engine(16, 16)
