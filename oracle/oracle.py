"""ctypes front-end of the C oracle (oracle/mm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker. The product path never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libmm_oracle.so")

SEED = 0x4D50494D

_lib = None


class OrFlow(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("a", ctypes.c_int), ("b", ctypes.c_int),
                ("rate", ctypes.c_double)]


DIFFUSE = 1
TRANSFER = 2


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


MPI_HOME = os.environ.get("MM_MPI_HOME", "/opt/conda")
CPU_MPI_PATH = os.path.join(HERE, "_build", "mm_cpu_mpi")


def cpu_mpi(H, W, rate, seconds, ranks, maxsteps=100000, dump=None, timeout=600, program=None):
    """Run the MPI CPU baseline (mm_cpu_mpi.c: row slabs, one rank per core, blocking
    border-row exchange, the oracle's step) as a child process; returns its JSON dict.
    program: [(kind, a, b, rate)] runs that flow program (config C5) instead of one
    diffusion, with per-step sums; dump then holds attribute 0."""
    import json
    if not os.path.exists(CPU_MPI_PATH):
        subprocess.run(["make", "-s", "-C", HERE, "cpu_mpi"], check=True)
    cmd = [os.path.join(MPI_HOME, "bin", "mpirun"), "-np", str(ranks), CPU_MPI_PATH,
           str(H), str(W), repr(float(rate)), repr(float(seconds)), str(maxsteps)]
    if dump:
        cmd.append(dump)
    env = dict(os.environ)
    env.pop("MM_PROGRAM", None)
    if program:
        env["MM_PROGRAM"] = ",".join(f"{k}:{a}:{b}:{float(r)!r}" for k, a, b, r in program)
    r = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=timeout, env=env)
    return json.loads(r.stdout.strip().splitlines()[-1])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        LL, D, I, P = ctypes.c_longlong, ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        L.or_step_count.restype = LL
        L.or_step_count.argtypes = [D, D]
        L.or_partition_reference.argtypes = [I, I, I, I] + [ctypes.POINTER(I)] * 4
        L.or_owner_reference.restype = I
        L.or_owner_reference.argtypes = [I, I, I]
        L.or_partition_rows.argtypes = [LL, I, I, ctypes.POINTER(LL), ctypes.POINTER(LL)]
        L.or_neighbor_count.restype = I
        L.or_neighbor_count.argtypes = [LL, LL, LL, LL]
        L.or_fill_random.argtypes = [LL, LL, LL, LL, ctypes.c_uint64, P]
        L.or_point_apply.argtypes = [LL, LL, P, LL, LL, D, D]
        L.or_field_step.restype = I
        L.or_field_step.argtypes = [LL, LL, P, P, D]
        L.or_field_step_slab.restype = I
        L.or_field_step_slab.argtypes = [LL, LL, LL, LL, P, P, D]
        L.or_field_step_general.restype = I
        L.or_field_step_general.argtypes = [LL, LL, P, P, P]
        L.or_program_step.restype = I
        L.or_program_step.argtypes = [LL, LL, I, P, ctypes.POINTER(OrFlow), I, P]
        L.or_field_rows.restype = I
        L.or_field_rows.argtypes = [LL, LL, LL, LL, I, D, ctypes.c_uint64, P]
        L.or_sum.restype = D
        L.or_sum.argtypes = [P, ctypes.c_size_t]
        _lib = L
    return _lib


def _ok(rc, what):
    if rc != 0:
        raise MemoryError(f"{what}: out of memory")


def _ptr(a):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def step_count(time, dt):
    return lib().or_step_count(time, dt)


def partition_reference(H, W, P, k):
    o = [ctypes.c_int() for _ in range(4)]
    lib().or_partition_reference(H, W, P, k, *[ctypes.byref(x) for x in o])
    return tuple(x.value for x in o)  # x_init, y_init, height, width


def owner_reference(H, P, x):
    return lib().or_owner_reference(H, P, x)


def partition_rows(H, G, g):
    a, h = ctypes.c_longlong(), ctypes.c_longlong()
    lib().or_partition_rows(H, G, g, ctypes.byref(a), ctypes.byref(h))
    return a.value, h.value


def neighbor_count(H, W, x, y):
    return lib().or_neighbor_count(H, W, x, y)


def fill_random(H, W, x_init=0, h=None, seed=SEED):
    h = H if h is None else h
    out = np.empty((h, W), dtype=np.float64)
    lib().or_fill_random(H, W, x_init, h, seed, _ptr(out))
    return out


def point_apply(v, sx, sy, captured, rate):
    v = np.ascontiguousarray(v, dtype=np.float64).copy()
    H, W = v.shape
    lib().or_point_apply(H, W, _ptr(v), sx, sy, captured, rate)
    return v


def field_step(v, rate, steps=1):
    v = np.ascontiguousarray(v, dtype=np.float64).copy()
    H, W = v.shape
    o = np.empty_like(v)
    for _ in range(steps):
        _ok(lib().or_field_step(H, W, _ptr(v), _ptr(o), rate), "or_field_step")
        v, o = o, v
    return v


def field_step_general(v, outf):
    v = np.ascontiguousarray(v, dtype=np.float64)
    outf = np.ascontiguousarray(outf, dtype=np.float64)
    H, W = v.shape
    o = np.empty_like(v)
    _ok(lib().or_field_step_general(H, W, _ptr(v), _ptr(outf), _ptr(o)), "or_field_step_general")
    return o


def field_step_slab(H, W, x_init, vg, rate):
    """vg: (h+2, W) slab with ghost rows; returns (h, W)."""
    vg = np.ascontiguousarray(vg, dtype=np.float64)
    h = vg.shape[0] - 2
    o = np.empty((h, W), dtype=np.float64)
    _ok(lib().or_field_step_slab(H, W, x_init, h, _ptr(vg), _ptr(o), rate), "or_field_step_slab")
    return o


def field_rows(H, W, lo, hi, steps, rate, seed=SEED, threads=None, chunk=None):
    """Rows [lo, hi) of fill_random(H, W) after `steps` field steps: or_field_rows on the
    dependency cone of row chunks, the chunks in parallel threads (ctypes releases the GIL).
    Bit-identical to field_step(fill_random(H, W), rate, steps)[lo:hi], at a cost that
    fits full-size GPU checks (32768^2, 40 steps: ~1 min on 16 cores)."""
    from concurrent.futures import ThreadPoolExecutor
    lo, hi = max(0, lo), min(H, hi)
    out = np.empty((max(hi - lo, 0), W), dtype=np.float64)
    if hi <= lo:
        return out
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    # chunks several times the cone's depth (the cone costs ~steps extra rows per chunk)
    chunk = chunk or max(64, 8 * steps, -(-(hi - lo) // (4 * threads)))
    starts = list(range(lo, hi, chunk))
    L = lib()

    def one(a):
        b = min(hi, a + chunk)
        view = out[a - lo:b - lo]
        rc = L.or_field_rows(H, W, a, b, steps, rate, seed, view.ctypes.data_as(ctypes.c_void_p))
        if rc != 0:
            raise MemoryError(f"or_field_rows rows [{a}, {b}): out of memory")

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, starts))
    return out


def program_step(fields, flows, steps=1, sums_per_step=False):
    """fields: list of (H, W) arrays (one per attribute); flows: [(kind, a, b, rate)]."""
    fields = [np.ascontiguousarray(f, dtype=np.float64).copy() for f in fields]
    H, W = fields[0].shape
    arr = (ctypes.c_void_p * len(fields))(*[f.ctypes.data for f in fields])
    fl = (OrFlow * len(flows))(*[OrFlow(k, a, b, r) for k, a, b, r in flows])
    scratch = np.empty((H, W), dtype=np.float64)
    sums = []
    for _ in range(steps):
        _ok(lib().or_program_step(H, W, len(fields), arr, fl, len(flows), _ptr(scratch)),
            "or_program_step")
        if sums_per_step:
            sums.append([float(np.sum(f, dtype=np.float64)) for f in fields])
    return (fields, sums) if sums_per_step else fields


def csum(v):
    v = np.ascontiguousarray(v, dtype=np.float64).ravel()
    return lib().or_sum(_ptr(v), v.size)
