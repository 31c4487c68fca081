"""CPU oracle (TEST INFRASTRUCTURE ONLY).

ctypes binding of ``oracle/hdb_oracle.c`` -- the line-faithful restatement of the
reference's Java hot path (see that file's header for the file:line map and the parity
status).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module; the product path (the HIP library) never touches it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libhdb_oracle.so")

EUCLIDEAN, COSINE, PEARSON, MANHATTAN, SUPREMUM = range(5)
METRICS = {"euclidean": EUCLIDEAN, "cosine": COSINE, "pearson": PEARSON,
           "manhattan": MANHATTAN, "supremum": SUPREMUM}
INCL_SELF_CUMULATIVE, INCL_SELF, EXCL_SELF = range(3)
JMAX = np.finfo(np.float64).max

ERRORS = {-1: "EINVAL", -3: "ENOMEM", -10: "EREF_NPE", -11: "EREF_OOB",
          -12: "EREF_NEGATIVE_CLUSTER", -13: "EREF_DIVZERO", -20: "EUNSUPPORTED"}


class OracleError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what}: {ERRORS.get(code, code)}")
        self.code = code


def build() -> str:
    """Compile the oracle with its Makefile (-O2 -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        dp, ip, lp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int64)
        i64, i32 = C.c_int64, C.c_int
        L.orc_distance.restype = C.c_double
        L.orc_distance.argtypes = [dp, dp, i32, i32]
        L.orc_core_distances.argtypes = [dp, i64, i32, i32, i32, i32, dp]
        L.orc_knn_lists.argtypes = [dp, i64, i32, i32, i32, i32, dp]
        L.orc_prim_mst.argtypes = [dp, i64, i32, dp, ip, i32, i32, ip, ip, dp]
        L.orc_nearest_sample.argtypes = [dp, i64, dp, i64, i32, i32, ip, ip, ip, dp]
        L.orc_bubble_stats_combine.argtypes = [dp, i64, i32, ip, i64, dp, dp, dp, dp]
        L.orc_bubble_stats_cf.argtypes = [dp, i64, i32, ip, i64, dp, dp, dp, dp]
        L.orc_bubble_stats_combine_sliced.argtypes = [dp, i64, i32, ip, i64, lp, i32, dp, dp, dp, dp]
        L.orc_distance_bubbles.restype = C.c_double
        L.orc_distance_bubbles.argtypes = [C.c_double, dp, dp, i64, i64]
        L.orc_bubble_core_distances.argtypes = [dp, ip, dp, dp, i64, i32, i32, i32, dp]
        L.orc_bubble_prim_mst.argtypes = [dp, dp, dp, ip, dp, i64, i32, i32, i32, ip, ip, dp]
        L.orc_quicksort_edges.argtypes = [ip, ip, dp, i64]
        L.orc_merge_edges.argtypes = [ip, ip, dp, i64]
        L.orc_core_rows.argtypes = [dp, i64, i32, lp, i64, i32, i32, i32, dp]
        L.orc_create_local_mst.argtypes = [dp, i64, i32, dp, ip, i32, i32, i32, ip, ip, dp, ip, ip, ip]
        L.orc_core_rows_par.argtypes = [dp, i64, i32, lp, i64, i32, i32, i32, i32, dp]
        L.orc_prim_mst_par.argtypes = [dp, i64, i32, dp, i32, i32, ip, ip, dp]
        L.orc_local_model.argtypes = [dp, dp, i64, i32, i32, i32, i32, ip, ip, ip, dp, ip, ip, dp, lp]
        _lib = L
    return _lib


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(C.POINTER(C.c_int32))


def _chk(rc, what):
    if rc != 0:
        raise OracleError(rc, what)


def _metric(m):
    return METRICS[m] if isinstance(m, str) else int(m)


def distance(a, b, metric="euclidean"):
    a, pa = _d(a)
    b, pb = _d(b)
    return lib().orc_distance(pa, pb, a.shape[0], _metric(metric))


def core_distances(X, min_pts, metric="euclidean", semantics=INCL_SELF_CUMULATIVE):
    """HDBSCANStar.calculateCoreDistances (HDBSCANStar.java:71-106) and its variants."""
    X, px = _d(X)
    n, d = X.shape
    core = np.empty(n, np.float64)
    _chk(lib().orc_core_distances(px, n, d, min_pts, _metric(metric), semantics, _d(core)[1]),
         "core_distances")
    return core


def core_rows(X, rows, min_pts, metric="euclidean", excl_self=True):
    """Core distance of selected rows against all rows (bench.py cpu_baseline sample)."""
    X, px = _d(X)
    n, d = X.shape
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    out = np.empty(rows.shape[0], np.float64)
    _chk(lib().orc_core_rows(px, n, d, rows.ctypes.data_as(C.POINTER(C.c_int64)), rows.shape[0], min_pts,
                             _metric(metric), int(excl_self), _d(out)[1]), "core_rows")
    return out


def core_rows_par(X, rows, min_pts, nthreads, metric="euclidean", excl_self=True):
    """core_rows with OpenMP over the query rows (bench.py CPU-all baseline); same values."""
    X, px = _d(X)
    n, d = X.shape
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    out = np.empty(rows.shape[0], np.float64)
    _chk(lib().orc_core_rows_par(px, n, d, rows.ctypes.data_as(C.POINTER(C.c_int64)), rows.shape[0], min_pts,
                                 _metric(metric), int(excl_self), int(nthreads), _d(out)[1]), "core_rows_par")
    return out


def prim_mst_par(X, core, nthreads, metric="euclidean"):
    """orc_prim_mst (identity ids, no self edges) with an OpenMP-parallel scan per Prim step
    (bench.py CPU-all baseline); the same edges as prim_mst."""
    X, px = _d(X)
    n, d = X.shape
    core, pc = _d(core)
    va = np.zeros(n - 1, np.int32)
    vb = np.zeros(n - 1, np.int32)
    w = np.zeros(n - 1, np.float64)
    _chk(lib().orc_prim_mst_par(px, n, d, pc, _metric(metric), int(nthreads), _i(va)[1], _i(vb)[1], _d(w)[1]),
         "prim_mst_par")
    return va, vb, w


def knn_lists(X, min_pts, metric="euclidean", excl_self=False):
    X, px = _d(X)
    n, d = X.shape
    out = np.empty((n, min_pts - 1), np.float64)
    _chk(lib().orc_knn_lists(px, n, d, min_pts, _metric(metric), int(excl_self), _d(out)[1]),
         "knn_lists")
    return out


def prim_mst(X, core, ids=None, metric="euclidean", self_edges=True):
    """HDBSCANStar.constructMST (HDBSCANStar.java:124-205). Returns (va, vb, w)."""
    X, px = _d(X)
    n, d = X.shape
    core, pc = _d(core)
    if ids is None:
        ids = np.arange(n, dtype=np.int32)
    ids, pi = _i(ids)
    ne = (n - 1) + (n if self_edges else 0)
    va = np.zeros(ne, np.int32)
    vb = np.zeros(ne, np.int32)
    w = np.zeros(ne, np.float64)
    _chk(lib().orc_prim_mst(px, n, d, pc, pi, _metric(metric), int(self_edges),
                            _i(va)[1], _i(vb)[1], _d(w)[1]), "prim_mst")
    return va, vb, w


def create_local_mst(X, core, ids, node, metric="euclidean", self_edges=True):
    """CreateLocalMST.constructMST (CreateLocalMST.java:187-292) with its record fields:
    returns (va, vb, w, fake1, fake2, node) in the reference's edge order."""
    X, px = _d(X)
    n, d = X.shape
    core, pc = _d(core)
    ids, pi = _i(ids)
    ne = (n - 1) + (n if self_edges else 0)
    out = [np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne, np.float64), np.zeros(ne, np.int32),
           np.zeros(ne, np.int32), np.zeros(ne, np.int32)]
    _chk(lib().orc_create_local_mst(px, n, d, pc, pi, _metric(metric), int(self_edges), int(node), _i(out[0])[1],
                                    _i(out[1])[1], _d(out[2])[1], _i(out[3])[1], _i(out[4])[1], _i(out[5])[1]),
         "create_local_mst")
    return tuple(out)


def nearest_sample(X, S, metric="euclidean", x_key=None, s_key=None):
    """FirstStep.java:74-85 first-minimum nearest sample. Returns (idx, dist)."""
    X, px = _d(X)
    S, ps = _d(S)
    n, d = X.shape
    m = S.shape[0]
    nn = np.zeros(n, np.int32)
    dist = np.zeros(n, np.float64)
    xk = sk = None
    pxk = psk = None
    if x_key is not None:
        xk, pxk = _i(x_key)
        sk, psk = _i(s_key)
    _chk(lib().orc_nearest_sample(px, n, ps, m, d, _metric(metric), pxk, psk, _i(nn)[1], _d(dist)[1]),
         "nearest_sample")
    return nn, dist


def bubble_stats(X, bubble_of, nb, variant="combine", cuts=None):
    """CombineStep (CombineStep.java:18-64) or CF (ClusterFeatureDataBubbles.java:192-215).
    cuts (CombineStep only): S + 1 slice boundaries over the rows -- per-slice folds combined
    in slice order (D11, orc_bubble_stats_combine_sliced); None: one sequential fold.
    Returns dict(ls, ss, rep, info) with info[:, (extent, nnDist, n)]."""
    X, px = _d(X)
    n, d = X.shape
    bo, pb = _i(bubble_of)
    ls = np.zeros((nb, d))
    ss = np.zeros((nb, d))
    rep = np.zeros((nb, d))
    info = np.zeros((nb, 3))
    if cuts is not None:
        if variant != "combine":
            raise ValueError("slices apply to CombineStep only")
        cu = np.ascontiguousarray(cuts, np.int64)
        _chk(lib().orc_bubble_stats_combine_sliced(px, n, d, pb, nb, cu.ctypes.data_as(C.POINTER(C.c_int64)),
                                                   cu.shape[0] - 1, _d(ls)[1], _d(ss)[1], _d(rep)[1], _d(info)[1]),
             "bubble_stats_sliced")
        return dict(ls=ls, ss=ss, rep=rep, info=info)
    fn = lib().orc_bubble_stats_combine if variant == "combine" else lib().orc_bubble_stats_cf
    _chk(fn(px, n, d, pb, nb, _d(ls)[1], _d(ss)[1], _d(rep)[1], _d(info)[1]), "bubble_stats")
    return dict(ls=ls, ss=ss, rep=rep, info=info)


def distance_bubbles(dist, eB, nnB, p, q):
    eB, pe = _d(eB)
    nnB, pn = _d(nnB)
    return lib().orc_distance_bubbles(float(dist), pe, pn, p, q)


def bubble_core_distances(rep, nB, eB, nnB, min_pts, metric="euclidean"):
    """HdbscanDataBubbles.calculateCoreDistancesBubbles (HdbscanDataBubbles.java:75-146)."""
    rep, pr = _d(rep)
    b, d = rep.shape
    nB, pnb = _i(nB)
    eB, pe = _d(eB)
    nnB, pn = _d(nnB)
    core = np.zeros(b)
    _chk(lib().orc_bubble_core_distances(pr, pnb, pe, pn, b, d, min_pts, _metric(metric), _d(core)[1]),
         "bubble_core_distances")
    return core


def bubble_prim_mst(rep, eB, nnB, core, ids=None, metric="euclidean", self_edges=True):
    """HdbscanDataBubbles.constructMSTBubbles (HdbscanDataBubbles.java:165-254)."""
    rep, pr = _d(rep)
    b, d = rep.shape
    eB, pe = _d(eB)
    nnB, pn = _d(nnB)
    core, pc = _d(core)
    if ids is None:
        ids = np.arange(b, dtype=np.int32)
    ids, pi = _i(ids)
    ne = (b - 1) + (b if self_edges else 0)
    va = np.zeros(ne, np.int32)
    vb = np.zeros(ne, np.int32)
    w = np.zeros(ne)
    _chk(lib().orc_bubble_prim_mst(pr, pe, pn, pi, pc, b, d, _metric(metric), int(self_edges),
                                   _i(va)[1], _i(vb)[1], _d(w)[1]), "bubble_prim_mst")
    return va, vb, w


def quicksort_edges(va, vb, w):
    """UndirectedGraph.quicksortByEdgeWeight (UndirectedGraph.java:93-124), in a copy."""
    va, pa = _i(np.array(va, np.int32))
    vb, pb = _i(np.array(vb, np.int32))
    w, pw = _d(np.array(w, np.float64))
    _chk(lib().orc_quicksort_edges(pa, pb, pw, w.shape[0]), "quicksort_edges")
    return va, vb, w


def merge_edges(lists):
    """UnionFindReducer.call + SortMST (UnionFindReducer.java:19-69): concatenation in
    list order, stable sort by DESCENDING weight."""
    va = np.concatenate([np.asarray(l[0], np.int32) for l in lists]) if lists else np.zeros(0, np.int32)
    vb = np.concatenate([np.asarray(l[1], np.int32) for l in lists]) if lists else np.zeros(0, np.int32)
    w = np.concatenate([np.asarray(l[2], np.float64) for l in lists]) if lists else np.zeros(0)
    va, pa = _i(va)
    vb, pb = _i(vb)
    w, pw = _d(w)
    _chk(lib().orc_merge_edges(pa, pb, pw, w.shape[0]), "merge_edges")
    return va, vb, w


def local_model(rep, info, min_pts, min_cl_size, metric="euclidean"):
    """LocalModelReduceByKey.call body (LocalModelReduceByKey.java:88-104) with D4 ids.
    Returns dict(labels, mst=(va,vb,w) quicksorted, inter=(va,vb,w))."""
    rep, pr = _d(rep)
    b, d = rep.shape
    info, pinf = _d(info)
    ne = 2 * b - 1
    labels = np.zeros(b, np.int32)
    mva, mvb, mw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
    iva, ivb, iw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
    nic = np.zeros(1, np.int64)
    _chk(lib().orc_local_model(pr, pinf, b, d, min_pts, min_cl_size, _metric(metric), _i(labels)[1],
                               _i(mva)[1], _i(mvb)[1], _d(mw)[1], _i(iva)[1], _i(ivb)[1], _d(iw)[1],
                               nic.ctypes.data_as(C.POINTER(C.c_int64))), "local_model")
    k = int(nic[0])
    return dict(labels=labels, mst=(mva, mvb, mw), inter=(iva[:k], ivb[:k], iw[:k]))


def last_negative_cluster():
    """(label, level, numPoints) of the cluster whose detachPoints threw last on this thread
    (Clusters.java:45-46) -- test diagnostics."""
    lab, lev, pts = C.c_int32(), C.c_double(), C.c_int32()
    lib().orc_last_negative_cluster(C.byref(lab), C.byref(lev), C.byref(pts))
    return dict(label=lab.value, level=lev.value, num_points=pts.value)


def first_step_leaf(X, ids, min_pts, metric="euclidean"):
    """FirstStep.call leaf branch (FirstStep.java:104-120): cumulative cores (the live
    HDBSCANStar.calculateCoreDistances) + Prim with self edges, ids = global point ids."""
    core = core_distances(X, min_pts, metric, INCL_SELF_CUMULATIVE)
    return core, prim_mst(X, core, ids, metric, True)
