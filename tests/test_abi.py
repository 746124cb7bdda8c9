"""CPU tests of the drop-in boundary: libmpimodel_hip.so loads, exports every symbol
include/mpimodel.h declares, and its host-only bookkeeping is bit-exact with the
reference (src/Model.hpp:47-80, src/Cell.hpp:71-157). No compute call is made
here: without a GPU the engine must refuse to start (it never falls back).
"""
import os
import re
import subprocess

import pytest

from conftest import REPO


def declared_functions():
    text = open(os.path.join(REPO, "include", "mpimodel.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mm_[a-z_]+)\s*\(", text)))


def test_header_and_binding_agree(mm):
    assert declared_functions() == sorted(mm.EXPORTS)


def test_header_constants_match_binding_and_engine(mm):
    # every #define value of the boundary (flow kinds, fill modes, halo modes, the
    # mm_info.chain_kernel codes) is the binding's, and the engine reports chain kernels
    # by those names only (the GPU tests compare mm_engine_info with the binding's values)
    text = open(os.path.join(REPO, "include", "mpimodel.h")).read()
    defines = dict(re.findall(r"#define\s+(MM_[A-Z_]+)\s+(-?\d+)\b", text))
    defines.update(re.findall(r"\b(MM_[A-Z_]+)\s*=\s*(-?\d+)", text))  # enumerators
    for name in ("MM_CHAIN_NONE", "MM_CHAIN_RING", "MM_CHAIN_RUNTIME", "MM_FLOW_DIFFUSE",
                 "MM_FLOW_TRANSFER", "MM_FILL_UNIFORM", "MM_FILL_RANDOM", "MM_HALO_NONE",
                 "MM_HALO_RCCL", "MM_HALO_HOST", "MM_OK"):
        assert name in defines, name
        assert int(defines[name]) == getattr(mm, name), name
    engine = open(os.path.join(REPO, "mpi-model_amd", "csrc", "mm_engine.hip")).read()
    sets = re.findall(r"chain_kernel\s*=\s*([^;]+);", engine)
    assert sets, "mm_engine_info no longer sets chain_kernel"
    for v in sets:  # `cond ? A : B` or `A`: every value a name from the header
        values = v.split("?", 1)[-1].split(":")
        assert all(x.strip() in ("MM_CHAIN_NONE", "MM_CHAIN_RING", "MM_CHAIN_RUNTIME")
                   for x in values), v


def test_library_exports_every_declared_symbol(mm):
    L = mm.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.mm_abi_version() == 3


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


# ---- the reference's control plane, pinned by its own MPI traffic -------------------
# tests/golden/wire_*.json: every MPI_Send of the reference, recorded by
# oracle/ref_wire_harness.cpp (MPI_Send interposed over the unmodified reference headers).

def wire_fixtures():
    import glob
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(REPO, "tests", "golden", "wire_*.json")))


def master_messages(g, tag):
    return [(d, data) for d, t, typ, n, data in g["sends_by_rank"]["0"] if t == tag and typ == "char"]


@pytest.mark.parametrize("name", wire_fixtures())
def test_wire_partition_descriptors_match_reference(mm, name):
    from conftest import golden
    g = golden(name)
    msgs = master_messages(g, mm.TAG_PARTITION)
    P = g["np"] - 1
    assert [d for d, _ in msgs] == list(range(1, P + 1))
    for k, data in msgs:
        if g["model"] == "row":
            desc = mm.partition_reference(g["dimx"], g["dimy"], P, k)
        else:
            desc = mm.partition_rect_reference(g["dimx_rec"], g["dimy_rec"], g["lines_rec"],
                                               g["columns_rec"], k)
        raw = mm.wire_partition(*desc)
        assert len(raw) == mm.WIRE_LEN and raw.rstrip(b"\0").decode() == data, (k, desc, data)
        assert mm.parse_wire_partition(data.encode()) == desc  # src/Model.hpp:139-146


@pytest.mark.parametrize("name", wire_fixtures())
def test_wire_flow_descriptors_match_reference(mm, name):
    from conftest import golden
    g = golden(name)
    msgs = master_messages(g, mm.TAG_FLOW)
    P = g["np"] - 1
    sx, sy, rate = g["src_x"], g["src_y"], float(g["rate"])
    if g["model"] == "row":
        owner = mm.owner_reference(g["dimx"], P, sx)  # src/Model.hpp:80
    else:
        owner = mm.owner_rect_reference(g["space"][0], sx, sy)  # src/ModelRectangular.hpp:85
    want = mm.wire_flow(owner, sx, sy, rate).rstrip(b"\0").decode()
    assert [d for d, _ in msgs] == list(range(1, P + 1))
    assert all(data == want for _, data in msgs)
    # the worker's parse: owner, x, y by atoi, and the rate read back as an int (atoi)
    assert mm.parse_wire_flow(want.encode())[:4] == (owner, sx, sy, int(rate) if rate >= 1 else 0)
    assert mm.parse_wire_flow(want.encode())[4] == float(f"{rate:f}")
    # the master prints the descriptor (src/Model.hpp:82; ModelRectangular adds the owner)
    line = want if g["model"] == "row" else f"{want} {owner}"
    assert line in g["reference_stdout_lines"]


def test_wire_format_refuses_overflow(mm):
    with pytest.raises(mm.MMError):  # the reference's sprintf would overrun its 23 chars
        mm.wire_partition(2 ** 30, 2 ** 30, 2 ** 30, 2 ** 30)
    with pytest.raises(mm.MMError):
        mm.parse_wire_flow(b"12")


def test_rect_partition_without_wrap(mm):
    # DIMY_REC % COLUMNS_REC != 0: the column offset never lands on DIMY_REC, so the
    # reference never moves to the second band of rows (src/ModelRectangular.hpp:76-79)
    assert [mm.partition_rect_reference(20, 61, 2, 3, k)[:2] for k in range(1, 7)] == \
        [(0, 0), (0, 20), (0, 40), (0, 60), (0, 80), (0, 100)]


def point_fixtures(prefix):
    import glob
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(REPO, "tests", "golden", prefix + "_*.json")))


@pytest.mark.parametrize("name", point_fixtures("point") + point_fixtures("strict"))
def test_strict_point_decision_matches_reference(mm, name):
    # src/Model.hpp:176-235: the reference changes cells only for an interior source on
    # its owner's last row; off that domain (strict_*: sources the reference still
    # completes) it changes nothing
    from conftest import golden
    g = golden(name)
    applies = mm.point_strict_applies(g["dimx"], g["dimy"], g["nworkers"], g["src_x"], g["src_y"])
    assert applies == (1 if g["changed"] else 0)
REF_MAIN = "/root/reference/src/Main.cpp"


@pytest.mark.skipif(not os.path.exists(REF_MAIN), reason="the reference exists only in the "
                    "build container (its sources and binaries do not travel to the GPU box)")
def test_reference_main_compiles_and_links_unchanged(tmp_path):
    """CPU side of the drop-in claim: the reference's own src/Main.cpp,
    byte for byte (fed on stdin, so none of its directory's headers is seen), compiles
    against mpi-model_amd/api/ and links against libmpimodel_hip.so -- the recipe of
    mpi-model_amd/api/Makefile, into a scratch path. Running it needs the GPU; the GPU runs
    of the drop-in use examples/drop_in_main (the binary built from the reference stays in
    this container: .gpurunignore)."""
    api = os.path.join(REPO, "mpi-model_amd", "api")
    exe = str(tmp_path / "ref_main")
    mpi = os.environ.get("MM_MPI_HOME", "/opt/conda")
    with open(REF_MAIN, "rb") as src:
        p = subprocess.run(
            ["g++", "-O2", "-std=c++14", "-Wall", f"-I{api}", f"-I{REPO}/include", f"-I{mpi}/include",
             "-x", "c++", "-", "-x", "none", os.path.join(api, "MPIImpl.cpp"), "-o", exe,
             f"-L{REPO}/mpi-model_amd", "-lmpimodel_hip", f"{mpi}/lib/libmpicxx.so",
             f"{mpi}/lib/libmpi.so", "-Wl,--disable-new-dtags",
             f"-Wl,-rpath,{REPO}/mpi-model_amd:/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:{mpi}/lib"],
            stdin=src, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    assert os.path.getsize(exe) > 0
    # every engine entry point the drop-in calls is bound from the product library
    syms = subprocess.run(["nm", "-D", "--undefined-only", exe], capture_output=True,
                          text=True).stdout
    assert "mm_engine_create" in syms and "mm_run" in syms


