"""ctypes binding of the C ABI in include/mpimodel.h (libmpimodel_hip.so).

Host-side mirror of the reference's Model/CellularSpace/Exponencial interface for
Python callers (bench.py, tests). The C++ mirror for Main.cpp-style programs is
mpi-model_amd/api/. There is no fallback: if the HIP library is missing or no
GPU is visible, these calls raise -- nothing here computes on the CPU.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MM_LIB_PATH: a tuning variant of the library (tools/build_variants.sh) for A/B runs
LIB_PATH = os.environ.get("MM_LIB_PATH") or os.path.join(HERE, "libmpimodel_hip.so")

MM_OK = 0
MM_FLOW_DIFFUSE = 1
MM_FLOW_TRANSFER = 2
MM_FILL_UNIFORM = 0
MM_FILL_RANDOM = 1
MM_HALO_NONE = 0
MM_HALO_RCCL = 1
MM_HALO_HOST = 2
MM_CHAIN_NONE = 0  # mm_info.chain_kernel (include/mpimodel.h)
MM_CHAIN_RING = 2
MM_CHAIN_RUNTIME = 3
SEED = 0x4D50494D

# every symbol include/mpimodel.h declares
EXPORTS = [
    "mm_abi_version", "mm_last_error", "mm_step_count", "mm_partition_reference",
    "mm_owner_reference", "mm_partition_rows", "mm_neighbor_count", "mm_comm_id_size",
    "mm_comm_id_create", "mm_device_count", "mm_device_synchronize", "mm_engine_create", "mm_engine_destroy",
    "mm_engine_info", "mm_fill", "mm_upload", "mm_download", "mm_clear_flows", "mm_add_flow",
    "mm_point_apply", "mm_run", "mm_prepare", "mm_pass_plan", "mm_pass_kernel", "mm_synchronize", "mm_sums", "mm_sums_history",
    "mm_clear_history", "mm_halo_export_rows", "mm_halo_import_rows", "mm_halo_export",
    "mm_halo_import", "mm_debug_read_rows", "mm_debug_fill_padding",
    "mm_set_timing", "mm_timing", "mm_partition_rect_reference", "mm_owner_rect_reference",
    "mm_wire_format_partition", "mm_wire_format_flow", "mm_wire_parse_partition",
    "mm_wire_parse_flow", "mm_point_strict_applies", "mm_point_apply_strict",
]

WIRE_LEN = 23
TAG_PARTITION = 0
TAG_FLOW = 999


class MMError(RuntimeError):
    """Non-zero mm_status; the C++ API raises std::runtime_error the same way
    (reference convention: src/MPIImpl.cpp:7-8,13-14)."""


class Desc(ctypes.Structure):
    _fields_ = [("H", ctypes.c_longlong), ("W", ctypes.c_longlong),
                ("x_init", ctypes.c_longlong), ("h", ctypes.c_longlong),
                ("n_attr", ctypes.c_int), ("device", ctypes.c_int),
                ("rank", ctypes.c_int), ("nranks", ctypes.c_int),
                ("halo_mode", ctypes.c_int), ("comm_id", ctypes.c_void_p)]


class Info(ctypes.Structure):
    _fields_ = [("pitch", ctypes.c_longlong), ("bytes_device", ctypes.c_longlong),
                ("n_passes", ctypes.c_int), ("rows_per_wave", ctypes.c_int),
                ("waves_per_pass", ctypes.c_longlong), ("steps_done", ctypes.c_longlong),
                ("fused_attrs", ctypes.c_int), ("steps_per_launch", ctypes.c_int),
                ("kernel", ctypes.c_int), ("halo_depth", ctypes.c_int),
                ("graph_state", ctypes.c_int), ("graph_count", ctypes.c_int),
                ("graph_launches", ctypes.c_longlong), ("hist_entries", ctypes.c_longlong),
                ("graph_note", ctypes.c_char * 160), ("seg_waves_per_cu", ctypes.c_int),
                ("chain_kernel", ctypes.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MMError(f"{LIB_PATH} not built: run `make -C mpi-model_amd` "
                          "(or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        LL, D, I, P = ctypes.c_longlong, ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        pLL, pI = ctypes.POINTER(LL), ctypes.POINTER(I)
        sig = {
            "mm_abi_version": (I, []),
            "mm_last_error": (ctypes.c_char_p, []),
            "mm_step_count": (LL, [D, D]),
            "mm_partition_reference": (I, [I, I, I, I, pI, pI, pI, pI]),
            "mm_owner_reference": (I, [I, I, I]),
            "mm_partition_rows": (I, [LL, I, I, pLL, pLL]),
            "mm_neighbor_count": (I, [LL, LL, LL, LL]),
            "mm_comm_id_size": (I, []),
            "mm_comm_id_create": (I, [P, I]),
            "mm_device_count": (I, [pI]),
            "mm_device_synchronize": (I, [I]),
            "mm_engine_create": (I, [ctypes.POINTER(Desc), ctypes.POINTER(P)]),
            "mm_engine_destroy": (I, [P]),
            "mm_engine_info": (I, [P, ctypes.POINTER(Info)]),
            "mm_fill": (I, [P, I, I, D, ctypes.c_ulonglong]),
            "mm_upload": (I, [P, I, P]),
            "mm_download": (I, [P, I, P]),
            "mm_clear_flows": (I, [P]),
            "mm_add_flow": (I, [P, I, I, I, D]),
            "mm_point_apply": (I, [P, I, LL, LL, D, D]),
            "mm_run": (I, [P, LL, LL]),
            "mm_prepare": (I, [P, LL, LL]),
            "mm_pass_plan": (I, [P, LL, pI, I, pI]),
            "mm_pass_kernel": (I, [P, I, pI, pI, pLL]),
            "mm_synchronize": (I, [P]),
            "mm_sums": (I, [P, P]),
            "mm_sums_history": (I, [P, P, LL, pLL]),
            "mm_clear_history": (I, [P]),
            "mm_halo_export_rows": (I, [P, I, P, P]),
            "mm_halo_import_rows": (I, [P, I, P, P]),
            "mm_halo_export": (I, [P, P, P]),
            "mm_halo_import": (I, [P, P, P]),
            "mm_debug_read_rows": (I, [P, I, LL, LL, P]),
            "mm_debug_fill_padding": (I, [P, D]),
            "mm_set_timing": (I, [P, I]),
            "mm_partition_rect_reference": (I, [I, I, I, I, I, pI, pI, pI, pI]),
            "mm_point_strict_applies": (I, [I, I, I, I, I]),
            "mm_point_apply_strict": (I, [P, I, LL, LL, D, D, I, pI]),
            "mm_owner_rect_reference": (I, [I, I, I]),
            "mm_wire_format_partition": (I, [ctypes.c_char_p, I, I, I, I, I]),
            "mm_wire_format_flow": (I, [ctypes.c_char_p, I, I, I, I, D]),
            "mm_wire_parse_partition": (I, [ctypes.c_char_p, I, pI, pI, pI, pI]),
            "mm_wire_parse_flow": (I, [ctypes.c_char_p, I, pI, pI, pI, pI,
                                       ctypes.POINTER(D)]),
            "mm_timing": (I, [P, pLL, ctypes.POINTER(D), ctypes.POINTER(D)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc != MM_OK:
        raise MMError(f"mm error {rc}: {lib().mm_last_error().decode(errors='replace')}")


def _dptr(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


# ---- host-only bookkeeping (src/Model.hpp:47-80, src/Cell.hpp:71-157) ----------
def step_count(time, time_step):
    return lib().mm_step_count(time, time_step)


def partition_reference(H, W, P, k):
    o = [ctypes.c_int() for _ in range(4)]
    check(lib().mm_partition_reference(H, W, P, k, *[ctypes.byref(x) for x in o]))
    return tuple(x.value for x in o)


def owner_reference(H, P, x):
    return lib().mm_owner_reference(H, P, x)


def partition_rows(H, G, g):
    a, h = ctypes.c_longlong(), ctypes.c_longlong()
    check(lib().mm_partition_rows(H, G, g, ctypes.byref(a), ctypes.byref(h)))
    return a.value, h.value


def neighbor_count(H, W, x, y):
    return lib().mm_neighbor_count(H, W, x, y)


def partition_rect_reference(H, W, lines, columns, k):
    o = [ctypes.c_int() for _ in range(4)]
    check(lib().mm_partition_rect_reference(H, W, lines, columns, k, *[ctypes.byref(x) for x in o]))
    return tuple(x.value for x in o)  # x_init, y_init, height, width


def point_strict_applies(H, W, P, x, y):
    return lib().mm_point_strict_applies(H, W, P, x, y)


def owner_rect_reference(space_height, x, y):
    return lib().mm_owner_rect_reference(space_height, x, y)


def wire_partition(x_init, y_init, height, width, length=WIRE_LEN):
    buf = ctypes.create_string_buffer(length)
    check(lib().mm_wire_format_partition(buf, length, x_init, y_init, height, width))
    return buf.raw


def wire_flow(owner, x, y, rate, length=WIRE_LEN):
    buf = ctypes.create_string_buffer(length)
    check(lib().mm_wire_format_flow(buf, length, owner, x, y, rate))
    return buf.raw


def parse_wire_partition(msg):
    o = [ctypes.c_int() for _ in range(4)]
    check(lib().mm_wire_parse_partition(msg, len(msg), *[ctypes.byref(x) for x in o]))
    return tuple(x.value for x in o)


def parse_wire_flow(msg):
    o = [ctypes.c_int() for _ in range(4)]
    r = ctypes.c_double()
    check(lib().mm_wire_parse_flow(msg, len(msg), *[ctypes.byref(x) for x in o], ctypes.byref(r)))
    return tuple(x.value for x in o) + (r.value,)  # owner, x, y, rate as atoi, rate


def comm_id():
    n = lib().mm_comm_id_size()
    buf = ctypes.create_string_buffer(n)
    check(lib().mm_comm_id_create(buf, n))
    return buf.raw


def device_synchronize(device=0):
    check(lib().mm_device_synchronize(device))


def device_count():
    n = ctypes.c_int()
    check(lib().mm_device_count(ctypes.byref(n)))
    return n.value


def run_host_halo(eng, nsteps, exchange, reduce_every=0):
    """nsteps steps of a MM_HALO_HOST slab in a chain of ranks: before every K-step pass of
    the engine's plan (mm_pass_plan) the slab's first / last K rows go out and the
    neighbours' K rows come in (`exchange(top, bottom, k) -> (above, below)`, None where the
    slab has no neighbour), then the pass runs. Every rank's plan is the same (it is sized
    by the chain's thinnest slab), so the exchanges pair up."""
    single = {}
    for k in eng.pass_plan(nsteps):
        if k not in single:  # a k-step run is exactly one k-step pass
            single[k] = eng.pass_plan(k) == [k]
            if not single[k]:
                raise RuntimeError(f"run_host_halo: a {k}-step run is not one pass")
        top, bottom = eng.halo_export(k)
        above, below = exchange(top, bottom, k)
        eng.halo_import(above, below, nrows=k)
        eng.run(k, reduce_every)


class Engine:
    """One row slab [x_init, x_init+h) of an H x W grid on one GPU."""

    def __init__(self, H, W, x_init=0, h=None, n_attr=1, device=0, rank=0, nranks=1,
                 halo_mode=MM_HALO_NONE, comm_id_bytes=None):
        h = H if h is None else h
        self._id = None
        if comm_id_bytes is not None:
            self._id = ctypes.create_string_buffer(comm_id_bytes, len(comm_id_bytes))
        d = Desc(H, W, x_init, h, n_attr, device, rank, nranks, halo_mode,
                 ctypes.cast(self._id, ctypes.c_void_p) if self._id is not None else None)
        p = ctypes.c_void_p()
        check(lib().mm_engine_create(ctypes.byref(d), ctypes.byref(p)))
        self.ptr = p
        self.H, self.W, self.x_init, self.h, self.n_attr = H, W, x_init, h, n_attr

    def close(self):
        if getattr(self, "ptr", None):
            check(lib().mm_engine_destroy(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def info(self):
        i = Info()
        check(lib().mm_engine_info(self.ptr, ctypes.byref(i)))
        out = {k: getattr(i, k) for k, _ in Info._fields_}
        out["graph_note"] = i.graph_note.decode(errors="replace")
        return out

    def fill(self, attr=0, mode=MM_FILL_UNIFORM, value=1.0, seed=SEED):
        check(lib().mm_fill(self.ptr, attr, mode, value, seed))

    def fill_random(self, attr=0, seed=SEED):
        self.fill(attr, MM_FILL_RANDOM, 0.0, seed)

    def upload(self, host, attr=0):
        a = np.ascontiguousarray(host, dtype=np.float64)
        assert a.shape == (self.h, self.W)
        check(lib().mm_upload(self.ptr, attr, _dptr(a)))

    def download(self, attr=0):
        out = np.empty((self.h, self.W), dtype=np.float64)
        check(lib().mm_download(self.ptr, attr, _dptr(out)))
        return out

    def clear_flows(self):
        check(lib().mm_clear_flows(self.ptr))

    def add_diffuse(self, attr, rate):
        check(lib().mm_add_flow(self.ptr, MM_FLOW_DIFFUSE, attr, attr, rate))

    def add_transfer(self, a, b, rate):
        check(lib().mm_add_flow(self.ptr, MM_FLOW_TRANSFER, a, b, rate))

    def point_apply(self, sx, sy, captured, rate, attr=0):
        check(lib().mm_point_apply(self.ptr, attr, sx, sy, captured, rate))

    def point_apply_strict(self, sx, sy, captured, rate, workers, attr=0):
        """Strict-reference mode: applied only where the reference's run on `workers`
        workers applies it (src/Model.hpp:189-216); returns whether it was applied."""
        applied = ctypes.c_int()
        check(lib().mm_point_apply_strict(self.ptr, attr, sx, sy, captured, rate, workers,
                                          ctypes.byref(applied)))
        return bool(applied.value)

    def run(self, nsteps, reduce_every=0):
        check(lib().mm_run(self.ptr, nsteps, reduce_every))

    def prepare(self, nsteps, reduce_every=0):
        """Capture / plan what run(nsteps, reduce_every) will launch, running no step."""
        check(lib().mm_prepare(self.ptr, nsteps, reduce_every))

    def pass_plan(self, nsteps):
        """Steps of each kernel pass run(nsteps) launches (mm_pass_plan)."""
        cnt = ctypes.c_int()
        check(lib().mm_pass_plan(self.ptr, nsteps, None, 0, ctypes.byref(cnt)))
        buf = (ctypes.c_int * max(cnt.value, 1))()
        check(lib().mm_pass_plan(self.ptr, nsteps, buf, cnt.value, ctypes.byref(cnt)))
        return list(buf[:cnt.value])

    def pass_kernel(self, k):
        """(kernel, columns per lane, strips) of a k-step pass (mm_pass_kernel): kernel 0 =
        mm_pass_kernel, 2 = mm_passk_kernel, 3 = mm_wide_kernel."""
        kern, cols, strips = ctypes.c_int(), ctypes.c_int(), ctypes.c_longlong()
        check(lib().mm_pass_kernel(self.ptr, k, ctypes.byref(kern), ctypes.byref(cols),
                                   ctypes.byref(strips)))
        return kern.value, cols.value, strips.value

    def synchronize(self):
        check(lib().mm_synchronize(self.ptr))

    def sums(self):
        out = np.empty(self.n_attr, dtype=np.float64)
        check(lib().mm_sums(self.ptr, _dptr(out)))
        return out

    def sums_history(self, max_entries=1 << 16):
        out = np.empty((max_entries, self.n_attr), dtype=np.float64)
        n = ctypes.c_longlong()
        check(lib().mm_sums_history(self.ptr, _dptr(out), max_entries, ctypes.byref(n)))
        return out[:min(n.value, max_entries)].copy()

    def clear_history(self):
        check(lib().mm_clear_history(self.ptr))

    def halo_export(self, nrows=1):
        """First / last nrows owned rows of every attribute: two (n_attr, nrows, W) arrays."""
        top = np.empty((self.n_attr, nrows, self.W), dtype=np.float64)
        bot = np.empty((self.n_attr, nrows, self.W), dtype=np.float64)
        check(lib().mm_halo_export_rows(self.ptr, nrows, _dptr(top), _dptr(bot)))
        return top, bot

    def halo_import(self, top=None, bottom=None, nrows=1):
        """Neighbour rows (n_attr, nrows, W) into the ghost rows above / below."""
        t = None if top is None else np.ascontiguousarray(top, dtype=np.float64)
        b = None if bottom is None else np.ascontiguousarray(bottom, dtype=np.float64)
        for x in (t, b):
            assert x is None or x.size == self.n_attr * nrows * self.W
        check(lib().mm_halo_import_rows(self.ptr, nrows, _dptr(t), _dptr(b)))

    def read_rows(self, row0, nrows, attr=0):
        out = np.empty((nrows, self.W), dtype=np.float64)
        check(lib().mm_debug_read_rows(self.ptr, attr, row0, nrows, _dptr(out)))
        return out

    def fill_padding(self, value):
        """Test hook: write value into every row's pitch padding (columns W..pitch-1)."""
        check(lib().mm_debug_fill_padding(self.ptr, float(value)))

    def set_timing(self, on):
        check(lib().mm_set_timing(self.ptr, 1 if on else 0))

    def timing(self):
        n, ms, b = ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
        check(lib().mm_timing(self.ptr, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(b)))
        return n.value, ms.value, b.value
