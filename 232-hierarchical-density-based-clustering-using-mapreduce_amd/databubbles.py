"""Mirror of databubbles/HdbscanDataBubbles.java and the live Spark operators of the hot
path (mappers/FirstStep.java, mappers/CombineStep.java, main/LocalModelReduceByKey.java)
over libhdbmi.  Method names follow the Java; bodies call the C-ABI.
"""
from __future__ import annotations

import numpy as np

from . import _capi as A
from .hdbscanstar import UndirectedGraph, _ctx, metric_of


class HdbscanDataBubbles:
    """databubbles/HdbscanDataBubbles.java."""

    def __init__(self, ctx: A.Context | None = None):
        self.ctx = ctx
        self.vertice1 = None
        self.vertice2 = None
        self.dmreach = None

    def calculateCoreDistancesBubbles(self, repB, nB, eB, nnDistB, k: int, distanceFunction=None):
        """HdbscanDataBubbles.java:75-146 (stale indexBubbles and int-division pow quirks)."""
        R = A.Arr(repB, np.float64)
        b, d = R.obj.shape
        nb_, e, nn = A.Arr(nB, np.int32), A.Arr(eB, np.float64), A.Arr(nnDistB, np.float64)
        core = A.new_like(R, (b,), np.float64)
        c = _ctx(R, self.ctx)
        A.check(A.lib().hdb_bubble_core_distances(c.h, R.p, nb_.p, e.p, nn.p, b, d, k, metric_of(distanceFunction),
                                                  A.ptr(core)), "calculateCoreDistancesBubbles")
        return core

    def constructMSTBubbles(self, dataRepB, nB, eB, nnDistB, idBubbles, coreDistances, selfEdges: bool,
                            distanceFunction=None) -> UndirectedGraph:
        """HdbscanDataBubbles.java:165-254."""
        R = A.Arr(dataRepB, np.float64)
        b, d = R.obj.shape
        e, nn = A.Arr(eB, np.float64), A.Arr(nnDistB, np.float64)
        ids = A.Arr(idBubbles, np.int32)
        core = A.Arr(coreDistances, np.float64)
        ne = (b - 1) + (b if selfEdges else 0)
        va = A.new_like(R, (ne,), np.int32)
        vb = A.new_like(R, (ne,), np.int32)
        w = A.new_like(R, (ne,), np.float64)
        c = _ctx(R, self.ctx)
        A.check(A.lib().hdb_bubble_prim_mst(c.h, R.p, e.p, nn.p, ids.p, core.p, b, d, metric_of(distanceFunction),
                                            int(bool(selfEdges)), A.ptr(va), A.ptr(vb), A.ptr(w)),
                "constructMSTBubbles")
        return UndirectedGraph(va, vb, w, b)

    def localModel(self, rep, info, minPts: int, minClSize: int, distanceFunction=None):
        """LocalModelReduceByKey.java:88-104 body: returns (labels, sorted mst, inter-cluster edges)."""
        R = np.ascontiguousarray(_host(rep), np.float64)
        I = np.ascontiguousarray(_host(info), np.float64)
        b, d = R.shape
        ne = 2 * b - 1
        labels = np.zeros(b, np.int32)
        mva, mvb, mw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
        iva, ivb, iw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
        nic = np.zeros(1, np.int64)
        c = self.ctx or A.Context.get(0)
        A.check(A.lib().hdb_local_model(c.h, A.ptr(R), A.ptr(I), b, d, minPts, minClSize,
                                        metric_of(distanceFunction), A.ptr(labels), A.ptr(mva), A.ptr(mvb),
                                        A.ptr(mw), A.ptr(iva), A.ptr(ivb), A.ptr(iw), A.ptr(nic)), "localModel")
        k = int(nic[0])
        self.vertice1, self.vertice2, self.dmreach = (iva[:k], ivb[:k], iw[:k]) if k else (None, None, None)
        return labels, UndirectedGraph(mva, mvb, mw, b), (iva[:k], ivb[:k], iw[:k])

    def getVertice1(self):
        return self.vertice1

    def getVertice2(self):
        return self.vertice2

    def getDmreach(self):
        return self.dmreach


def _host(x):
    if A.is_torch(x):
        return x.detach().cpu().numpy()
    return np.asarray(x)


# ------------------------------------------------------------ operators
def nearest_sample(X, S, distanceFunction=None, x_key=None, s_key=None, ctx=None, with_dist=False):
    """FirstStep.java:74-85 (first minimum over the sample list, strict '<').  Returns
    the winning LIST POSITION per point (FirstStep then reports that sample's per-key index)."""
    XX, SS = A.Arr(X, np.float64), A.Arr(S, np.float64)
    n, d = XX.obj.shape
    m = SS.obj.shape[0]
    out = A.new_like(XX, (n,), np.int32)
    dist = A.new_like(XX, (n,), np.float64) if with_dist else None
    xk = A.Arr(x_key, np.int32) if x_key is not None else None
    sk = A.Arr(s_key, np.int32) if s_key is not None else None
    c = _ctx(XX, ctx)
    A.check(A.lib().hdb_nearest_sample(c.h, XX.p, n, SS.p, m, d, metric_of(distanceFunction),
                                       xk.p if xk else None, sk.p if sk else None, A.ptr(out), A.ptr(dist)),
            "nearest_sample")
    return (out, dist) if with_dist else out


def bubble_stats(X, bubble_of, nb: int, variant: int = A.BUBBLE_COMBINESTEP, ctx=None):
    """Bulk CombineStep (CombineStep.java:18-64) over a partition, D5 member order.
    Returns (ls, ss, rep, info[extent, nnDist, n])."""
    XX = A.Arr(X, np.float64)
    n, d = XX.obj.shape
    bo = A.Arr(bubble_of, np.int32)
    ls = A.new_like(XX, (nb, d), np.float64)
    ss = A.new_like(XX, (nb, d), np.float64)
    rep = A.new_like(XX, (nb, d), np.float64)
    info = A.new_like(XX, (nb, 3), np.float64)
    c = _ctx(XX, ctx)
    A.check(A.lib().hdb_bubble_stats(c.h, XX.p, n, d, bo.p, nb, variant, A.ptr(ls), A.ptr(ss), A.ptr(rep),
                                     A.ptr(info)), "bubble_stats")
    return ls, ss, rep, info


class CombineStep:
    """mappers/CombineStep.java as a bulk operator over (points, bubble ids)."""

    def __init__(self, variant: int = A.BUBBLE_COMBINESTEP):
        self.variant = variant

    def call(self, X, bubble_of, nb, ctx=None):
        return bubble_stats(X, bubble_of, nb, self.variant, ctx)


class FirstStep:
    """mappers/FirstStep.java:18-122 -- per-subset first step of MR-HDBSCAN*.

    A subset with n <= processingUnits is a leaf: cumulative core distances +
    constructMST(selfEdges=true) over its rows (:104-120).  Otherwise every row goes to its
    nearest sample (:74-85) and becomes a singleton bubble seed (:87-101)."""

    def __init__(self, k: float, processingUnits: int, mpts: int, distanceFunction=None, samples=None,
                 sample_keys=None, ctx=None):
        self.k = k
        self.processingUnits = processingUnits
        self.mpts = mpts
        self.distanceFunction = distanceFunction
        self.samples = samples
        self.sample_keys = sample_keys
        self.ctx = ctx

    def leaf(self, X, ids, offsets):
        """Leaf branch for P subsets at once (offsets = CSR row ranges)."""
        XX = A.Arr(X, np.float64)
        n, d = XX.obj.shape
        off = np.ascontiguousarray(_host(offsets), np.int64)
        P = off.shape[0] - 1
        sizes = np.diff(off)
        ne = int(np.sum(np.where(sizes > 0, 2 * sizes - 1, 0)))
        idsA = A.Arr(ids, np.int32)
        core = A.new_like(XX, (n,), np.float64)
        va = A.new_like(XX, (ne,), np.int32)
        vb = A.new_like(XX, (ne,), np.int32)
        w = A.new_like(XX, (ne,), np.float64)
        c = _ctx(XX, self.ctx)
        A.check(A.lib().hdb_leaf_msts(c.h, XX.p, A.ptr(off), P, d, idsA.p, self.mpts, metric_of(self.distanceFunction),
                                      A.ptr(core), A.ptr(va), A.ptr(vb), A.ptr(w)), "FirstStep.leaf")
        return core, UndirectedGraph(va, vb, w)

    def nearest(self, X, x_key=None):
        return nearest_sample(X, self.samples, self.distanceFunction, x_key,
                              self.sample_keys if x_key is not None else None, self.ctx)


class LocalModelReduceByKey:
    """main/LocalModelReduceByKey.java:13-115 (once all bubbles of the subset are present)."""

    def __init__(self, mpts: int, mclSize: int, distanceFunction=None, ctx=None):
        self.mpts = mpts
        self.mclSize = mclSize
        self.distanceFunction = distanceFunction
        self.ctx = ctx

    def call(self, rep, info):
        model = HdbscanDataBubbles(self.ctx)
        labels, mst, inter = model.localModel(rep, info, self.mpts, self.mclSize, self.distanceFunction)
        return labels, mst, inter


def sort_edges_desc(va, vb, w, ctx=None):
    """UnionFindReducer + SortMST merge (stable, descending weight), in place."""
    a, b, ww = A.Arr(va, np.int32), A.Arr(vb, np.int32), A.Arr(w, np.float64)
    c = _ctx(a, ctx)
    A.check(A.lib().hdb_sort_edges_desc(c.h, a.p, b.p, ww.p, ww.obj.shape[0]), "sort_edges_desc")
    return a.obj, b.obj, ww.obj


def merge_sorted_runs(va, vb, w, run_off, ctx=None):
    """The same order as sort_edges_desc over a concatenation of runs that are each sorted
    descending already (per-rank sort_edges_desc outputs): stable merge, run order on ties.
    run_off: nruns + 1 offsets.  Returns new (va, vb, w) arrays of the input's kind."""
    a, b, ww = A.Arr(va, np.int32), A.Arr(vb, np.int32), A.Arr(w, np.float64)
    off = np.ascontiguousarray(np.asarray(run_off, np.int64))
    ne = ww.obj.shape[0]
    oa, ob, ow = A.new_like(a, (ne,), np.int32), A.new_like(a, (ne,), np.int32), A.new_like(a, (ne,), np.float64)
    c = _ctx(a, ctx)
    A.check(A.lib().hdb_merge_sorted_runs(c.h, a.p, b.p, ww.p, off.ctypes.data, len(off) - 1, A.ptr(oa), A.ptr(ob),
                                          A.ptr(ow)), "merge_sorted_runs")
    return oa, ob, ow
