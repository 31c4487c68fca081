"""ctypes binding of libhdbmi (include/hdbmi.h).

The product path: every call goes to the HIP library.  There is no CPU fallback -- if the
library is missing or no HIP device is visible, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HDBMI_LIB") or os.path.join(HERE, "lib", "libhdbmi.so")  # override: A/B builds

HDB_OK = 0
ERRORS = {
    -1: "HDB_EINVAL", -2: "HDB_EDEVICE", -3: "HDB_ENOMEM", -10: "HDB_EREF_NPE", -11: "HDB_EREF_OOB",
    -12: "HDB_EREF_NEGATIVE_CLUSTER", -13: "HDB_EREF_DIVZERO", -14: "HDB_EREF_NUMBER_FORMAT",
    -20: "HDB_EUNSUPPORTED",
}

METRIC = {"euclidean": 0, "cosine": 1, "pearson": 2, "manhattan": 3, "supremum": 4}
CORE_INCL_SELF_CUMULATIVE, CORE_INCL_SELF, CORE_EXCL_SELF = 0, 1, 2
EDGES_SELF, EDGES_MERGED = 1, 2  # hdb_exact_mst edge flags (include/hdbmi.h)
BUBBLE_COMBINESTEP, BUBBLE_CF = 0, 1
JMAX = float(np.finfo(np.float64).max)

# Java exceptions the reference raises on the same inputs.
class HdbError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class NullPointerException(HdbError):
    pass


class ArrayIndexOutOfBoundsException(HdbError):
    pass


class IllegalStateException(HdbError):
    """Clusters.java:45-46 "Cluster cannot have less than 0 points."."""


class ArithmeticException(HdbError):
    pass


class NumberFormatException(HdbError):
    """Double.parseDouble / Integer.parseInt on a malformed field."""


_EXC = {-10: NullPointerException, -11: ArrayIndexOutOfBoundsException, -12: IllegalStateException,
        -13: ArithmeticException, -14: NumberFormatException}

_lib = None
_lock = threading.Lock()


def lib():
    """Load libhdbmi.so; raise loudly when it is absent (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 (SONAME
        # libamdhip64.so.7).  Loading torch first lets this library's NEEDED entry bind to
        # that runtime, so device pointers of torch tensors are valid here.  Loading us
        # first would map /opt/rocm's runtime and torch would then map a second one.
        try:
            import torch  # noqa: F401
        except ImportError:  # pragma: no cover - standalone use: /opt/rocm runtime
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libhdbmi.so not built ({LIB_PATH}); run build_lib.py / __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        vp, dp, ip, lp = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p
        i64, i32 = C.c_int64, C.c_int32
        sig = {
            "hdb_ctx_create": [C.c_int, C.POINTER(vp)],
            "hdb_ctx_set_stream": [vp, vp],
            "hdb_ctx_set_timing": [vp, C.c_int],
            "hdb_ctx_kernel_time": [vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.c_int],
            "hdb_ctx_synchronize": [vp],
            "hdb_ctx_set_option": [vp, C.c_char_p, C.c_int64],
            "hdb_ctx_get_stat": [vp, C.c_char_p, C.POINTER(C.c_int64)],
            "hdb_distance_rows": [vp, dp, dp, i64, i32, i32, dp],
            "hdb_core_distances": [vp, dp, i64, i32, i32, i32, i32, dp],
            "hdb_knn": [vp, dp, i64, i32, i32, i32, i32, dp, ip],
            "hdb_prim_mst": [vp, dp, i64, i32, dp, ip, i32, i32, ip, ip, dp],
            "hdb_prim_mst_batched": [vp, dp, lp, i32, i32, dp, ip, i32, i32, ip, ip, dp],
            "hdb_leaf_msts": [vp, dp, lp, i32, i32, ip, i32, i32, dp, ip, ip, dp],
            "hdb_mst_boruvka": [vp, dp, i64, i32, dp, i32, i32, ip, ip, dp],
            "hdb_exact_mst": [vp, dp, i64, i32, i32, i32, i32, i32, dp, ip, ip, dp],
            "hdb_nearest_sample": [vp, dp, i64, dp, i64, i32, i32, ip, ip, ip, dp],
            "hdb_bubble_stats": [vp, dp, i64, i32, ip, i64, i32, dp, dp, dp, dp],
            "hdb_bubble_partials": [vp, dp, i64, i32, ip, i64, lp, i32, dp, dp, dp],
            "hdb_bubble_combine": [vp, dp, dp, dp, i32, i64, i32, dp, dp, dp, dp],
            "hdb_bubble_core_distances": [vp, dp, ip, dp, dp, i64, i32, i32, i32, dp],
            "hdb_bubble_prim_mst": [vp, dp, dp, dp, ip, dp, i64, i32, i32, i32, ip, ip, dp],
            "hdb_local_model": [vp, dp, dp, i64, i32, i32, i32, i32, ip, ip, ip, dp, ip, ip, dp, lp],
            "hdb_local_model_cores": [vp, dp, dp, i64, i32, i32, i32, i32, dp, ip, ip, ip, dp, ip, ip, dp, lp],
            "hdb_quicksort_edges": [ip, ip, dp, i64],
            "hdb_sort_edges_desc": [vp, ip, ip, dp, i64],
            "hdb_merge_sorted_runs": [vp, ip, ip, dp, lp, i32, ip, ip, dp],
            "hdb_flat_labels": [vp, ip, ip, dp, i64, i64, i32, ip, lp],
            "hdb_local_mst_ids": [vp, ip, i64, ip, ip, dp, i64, i32, ip, ip, ip],
            "hdb_comm_unique_id": [vp, i32],
            "hdb_comm_init": [vp, i32, i32, vp, C.POINTER(vp)],
            "hdb_free": [vp],
            "hdb_copy": [vp, vp, vp, i64],
            "hdb_merge_edges": [vp, ip, ip, dp, lp, i64, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp),
                                C.POINTER(C.c_int64)],
            "hdb_format_double": [C.c_double, C.c_char_p, i32],
            "hdb_parse_points": [C.c_char_p, i64, i32, i32, dp, i64, lp, ip],
            "hdb_format_mst_records": [ip, ip, dp, ip, ip, ip, i64, vp, i64, lp],
            "hdb_parse_mst_records": [C.c_char_p, i64, ip, ip, dp, ip, ip, ip, i64, lp],
        }
        for name, args in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = C.c_int
        L.hdb_ctx_destroy.argtypes = [vp]
        L.hdb_ctx_destroy.restype = None
        L.hdb_comm_destroy.argtypes = [vp]
        L.hdb_comm_destroy.restype = None
        L.hdb_last_error.restype = C.c_char_p
        L.hdb_version.restype = C.c_int
        _lib = L
    return _lib


EXPORTED = ["hdb_ctx_create", "hdb_ctx_destroy", "hdb_ctx_set_stream", "hdb_ctx_set_timing", "hdb_ctx_set_option",
            "hdb_ctx_get_stat", "hdb_ctx_kernel_time", "hdb_ctx_synchronize", "hdb_last_error", "hdb_version",
            "hdb_distance_rows", "hdb_core_distances", "hdb_knn", "hdb_prim_mst", "hdb_prim_mst_batched",
            "hdb_leaf_msts", "hdb_mst_boruvka", "hdb_exact_mst", "hdb_nearest_sample", "hdb_bubble_stats",
            "hdb_bubble_partials", "hdb_bubble_combine", "hdb_bubble_core_distances", "hdb_bubble_prim_mst", "hdb_local_model", "hdb_local_model_cores", "hdb_quicksort_edges",
            "hdb_merge_sorted_runs", "hdb_sort_edges_desc", "hdb_flat_labels", "hdb_format_double", "hdb_parse_points",
            "hdb_format_mst_records", "hdb_parse_mst_records", "hdb_comm_unique_id", "hdb_comm_init",
            "hdb_comm_destroy", "hdb_free", "hdb_copy", "hdb_merge_edges", "hdb_local_mst_ids"]


def check(rc: int, what: str):
    if rc != HDB_OK:
        msg = lib().hdb_last_error().decode(errors="replace")
        raise _EXC.get(rc, HdbError)(rc, f"{what}: {msg}")


class Context:
    """One hdb_ctx per (thread, device); owns a stream (or borrows torch's)."""

    _tls = threading.local()
    _all: list = []  # every context created (diagnostic stat totals across threads)

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().hdb_ctx_create(device, C.byref(h)), "hdb_ctx_create")
        self.h = h
        self.device = device
        self._stream = None
        Context._all.append(self)

    @classmethod
    def stat_total(cls, name: str) -> int:
        return sum(c.get_stat(name) for c in cls._all)

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        d = getattr(cls._tls, "ctxs", None)
        if d is None:
            d = cls._tls.ctxs = {}
        if device not in d:
            d[device] = Context(device)
        return d[device]

    def set_stream(self, stream_ptr: int | None):
        if stream_ptr != self._stream:
            check(lib().hdb_ctx_set_stream(self.h, C.c_void_p(stream_ptr) if stream_ptr else None),
                  "hdb_ctx_set_stream")
            self._stream = stream_ptr

    def use_torch_stream(self):
        import torch
        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def set_timing(self, on: bool):
        check(lib().hdb_ctx_set_timing(self.h, int(on)), "hdb_ctx_set_timing")

    def kernel_time(self, name: str, reset: bool = True):
        ms = C.c_double()
        n = C.c_int64()
        check(lib().hdb_ctx_kernel_time(self.h, name.encode(), C.byref(ms), C.byref(n), int(reset)),
              "hdb_ctx_kernel_time")
        return ms.value, n.value

    def set_option(self, name: str, value: int):
        check(lib().hdb_ctx_set_option(self.h, name.encode(), int(value)), "hdb_ctx_set_option")

    def get_stat(self, name: str) -> int:
        v = C.c_int64()
        check(lib().hdb_ctx_get_stat(self.h, name.encode(), C.byref(v)), "hdb_ctx_get_stat")
        return v.value

    def synchronize(self):
        check(lib().hdb_ctx_synchronize(self.h), "hdb_ctx_synchronize")

    def __del__(self):
        try:
            if self.h and _lib is not None:
                _lib.hdb_ctx_destroy(self.h)
        except Exception:
            pass


# ------------------------------------------------------------- array plumbing
def is_torch(x) -> bool:
    try:
        import torch
        return isinstance(x, torch.Tensor)
    except ImportError:  # pragma: no cover
        return False


class Arr:
    """A caller array as (pointer, keep-alive), numpy (host) or torch (host/HIP)."""

    def __init__(self, x, dtype):
        if is_torch(x):
            import torch
            tdt = {np.float64: torch.float64, np.int32: torch.int32, np.int64: torch.int64}[dtype]
            t = x.contiguous()
            if t.dtype != tdt:
                t = t.to(tdt)
            self.obj = t
            self.ptr = t.data_ptr()
            self.device = t.device
        else:
            a = np.ascontiguousarray(x, dtype=dtype)
            self.obj = a
            self.ptr = a.ctypes.data
            self.device = None

    @property
    def p(self):
        return C.c_void_p(self.ptr)


def new_like(ref: Arr, shape, dtype):
    if ref.device is not None and ref.device.type == "cuda":
        import torch
        tdt = {np.float64: torch.float64, np.int32: torch.int32, np.int64: torch.int64}[dtype]
        return torch.empty(shape, dtype=tdt, device=ref.device)
    return np.empty(shape, dtype=dtype)


def ptr(x):
    if x is None:
        return None
    if is_torch(x):
        return C.c_void_p(x.data_ptr())
    return C.c_void_p(x.ctypes.data)
