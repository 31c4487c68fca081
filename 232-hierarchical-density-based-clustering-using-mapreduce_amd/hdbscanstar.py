"""Mirror of the reference's ``distance`` and ``hdbscanstar`` packages over libhdbmi.

Same class/method names and argument meaning as the Java (源代码/distance/*.java,
源代码/hdbscanstar/HDBSCANStar.java, UndirectedGraph.java); the bodies call the C-ABI.
Arrays may be numpy (host) or torch tensors (host or HIP device); results come back on the
side the input lives on.
"""
from __future__ import annotations

import numpy as np

from . import _capi as A


# --------------------------------------------------------------- distance
class DistanceCalculator:
    """distance/DistanceCalculator.java:9-21."""

    name = ""

    def getName(self) -> str:  # DistanceCalculator.java:20
        return self.name

    def computeDistance(self, attributesOne, attributesTwo) -> float:  # :17
        a = np.asarray(attributesOne, np.float64).reshape(1, -1)
        b = np.asarray(attributesTwo, np.float64).reshape(1, -1)
        return float(distance_rows(a, b, self)[0])

    @property
    def metric(self) -> int:
        return A.METRIC[self.getName()]


class EuclideanDistance(DistanceCalculator):
    name = "euclidean"  # EuclideanDistance.java:28-41


class CosineSimilarity(DistanceCalculator):
    name = "cosine"  # CosineSimilarity.java:28-45


class PearsonCorrelation(DistanceCalculator):
    name = "pearson"  # PearsonCorrelation.java:28-56


class ManhattanDistance(DistanceCalculator):
    name = "manhattan"  # ManhattanDistance.java:28-41


class SupremumDistance(DistanceCalculator):
    name = "supremum"  # SupremumDistance.java:28-43


def metric_of(distanceFunction) -> int:
    if distanceFunction is None:
        return 0
    if isinstance(distanceFunction, str):
        return A.METRIC[distanceFunction]
    if isinstance(distanceFunction, int):
        return distanceFunction
    return A.METRIC[distanceFunction.getName()]


def _ctx(ref: A.Arr, ctx=None) -> A.Context:
    if ctx is not None:
        return ctx
    dev = ref.device.index if (ref.device is not None and ref.device.type == "cuda") else 0
    c = A.Context.get(dev or 0)
    if ref.device is not None and ref.device.type == "cuda":
        c.use_torch_stream()
    return c


def distance_rows(a, b, distanceFunction=None, ctx=None):
    aa, bb = A.Arr(a, np.float64), A.Arr(b, np.float64)
    n, d = aa.obj.shape
    out = A.new_like(aa, (n,), np.float64)
    c = _ctx(aa, ctx)
    A.check(A.lib().hdb_distance_rows(c.h, aa.p, bb.p, n, d, metric_of(distanceFunction), A.ptr(out)),
            "hdb_distance_rows")
    return out


# ---------------------------------------------------------- UndirectedGraph
class UndirectedGraph:
    """hdbscanstar/UndirectedGraph.java: parallel edge arrays (+ adjacency on demand)."""

    def __init__(self, verticesA, verticesB, edgeWeights, numVertices: int | None = None):
        self.verticesA = verticesA
        self.verticesB = verticesB
        self.edgeWeights = edgeWeights
        self.numVertices = numVertices

    def _host(self):
        def h(x, dt):
            if A.is_torch(x):
                return np.ascontiguousarray(x.detach().cpu().numpy(), dtype=dt)
            return np.ascontiguousarray(x, dtype=dt)
        return h(self.verticesA, np.int32), h(self.verticesB, np.int32), h(self.edgeWeights, np.float64)

    def quicksortByEdgeWeight(self):
        """UndirectedGraph.java:93-124 (pivot = startIndex quirk), in place on host copies."""
        a, b, w = self._host()
        A.check(A.lib().hdb_quicksort_edges(A.ptr(a), A.ptr(b), A.ptr(w), w.shape[0]), "quicksortByEdgeWeight")
        self.verticesA, self.verticesB, self.edgeWeights = a, b, w

    def getNumVertices(self):
        return self.numVertices

    def getNumEdges(self):
        return int(self.edgeWeights.shape[0])

    def getFirstVertexAtIndex(self, i):
        return int(self.verticesA[i])

    def getSecondVertexAtIndex(self, i):
        return int(self.verticesB[i])

    def getEdgeWeightAtIndex(self, i):
        return float(self.edgeWeights[i])

    def getVerticeA(self):
        return self.verticesA

    def getVericeB(self):  # sic, UndirectedGraph.java:259
        return self.verticesB

    def getEges(self):  # sic, UndirectedGraph.java:263
        return self.edgeWeights


# --------------------------------------------------------------- HDBSCANStar
class HDBSCANStar:
    """hdbscanstar/HDBSCANStar.java -- the hot-path entry points."""

    def __init__(self, ctx: A.Context | None = None):
        self.ctx = ctx

    def calculateCoreDistances(self, dataSet, k: int, distanceFunction=None,
                               semantics: int = A.CORE_INCL_SELF_CUMULATIVE):
        """HDBSCANStar.java:71-106 (live: the k-NN buffer is never reset between points).
        semantics selects the reference's other variants (CORE_INCL_SELF:
        CoreDistanceMapper.java:71-109, CORE_EXCL_SELF: CreateLocalMST.java:138-185)."""
        X = A.Arr(dataSet, np.float64)
        n, d = X.obj.shape
        core = A.new_like(X, (n,), np.float64)
        c = _ctx(X, self.ctx)
        A.check(A.lib().hdb_core_distances(c.h, X.p, n, d, k, metric_of(distanceFunction), semantics,
                                           A.ptr(core)), "calculateCoreDistances")
        return core

    def constructMST(self, dataSet, coreDistances, selfEdges: bool, distanceFunction=None, indices=None,
                     totalLength=None) -> UndirectedGraph:
        """HDBSCANStar.java:124-205 -- exact reference Prim (totalLength unused, as in Java)."""
        X = A.Arr(dataSet, np.float64)
        n, d = X.obj.shape
        core = A.Arr(coreDistances, np.float64)
        ids = A.Arr(indices, np.int32) if indices is not None else None
        ne = (n - 1) + (n if selfEdges else 0)
        va = A.new_like(X, (ne,), np.int32)
        vb = A.new_like(X, (ne,), np.int32)
        w = A.new_like(X, (ne,), np.float64)
        c = _ctx(X, self.ctx)
        A.check(A.lib().hdb_prim_mst(c.h, X.p, n, d, core.p, ids.p if ids else None, metric_of(distanceFunction),
                                     int(bool(selfEdges)), A.ptr(va), A.ptr(vb), A.ptr(w)), "constructMST")
        return UndirectedGraph(va, vb, w)

    def constructLocalMST(self, dataSet, indices, coreDistances, selfEdges: bool, distanceFunction=None,
                          node: int = 0):
        """CreateLocalMST.constructMST (partition/mappers/CreateLocalMST.java:187-292): the
        reference Prim plus its MinimumSpanningTree record fields -- returns (va, vb, w, fake1,
        fake2, node) with fake1 = nearestneighborsID (:242), fake2 = otherVertexIndicesID
        (:266), node (:285); format with formats.format_local_mst (CreateLocalMST.java:110-123)."""
        g = self.constructMST(dataSet, coreDistances, selfEdges, distanceFunction, indices)
        va, vb, w = g.getVerticeA(), g.getVericeB(), g.getEges()
        n = A.Arr(dataSet, np.float64).obj.shape[0]
        ids = A.Arr(indices, np.int32) if indices is not None else None
        a, b, ww = A.Arr(va, np.int32), A.Arr(vb, np.int32), A.Arr(w, np.float64)
        ne = a.obj.shape[0]
        f1, f2, nd = (A.new_like(a, (ne,), np.int32) for _ in range(3))
        c = _ctx(a, self.ctx)
        A.check(A.lib().hdb_local_mst_ids(c.h, ids.p if ids else None, n, a.p, b.p, ww.p, ne, int(node), A.ptr(f1),
                                          A.ptr(f2), A.ptr(nd)), "hdb_local_mst_ids")
        return va, vb, w, f1, f2, nd

    def constructMSTBoruvka(self, dataSet, coreDistances, selfEdges: bool, distanceFunction=None) -> UndirectedGraph:
        """Large-graph MST (K2b): same sorted weights as constructMST, ties broken by
        (w, min id, max id); edges sorted by that key, then the self edges."""
        X = A.Arr(dataSet, np.float64)
        n, d = X.obj.shape
        core = A.Arr(coreDistances, np.float64)
        ne = (n - 1) + (n if selfEdges else 0)
        va = A.new_like(X, (ne,), np.int32)
        vb = A.new_like(X, (ne,), np.int32)
        w = A.new_like(X, (ne,), np.float64)
        c = _ctx(X, self.ctx)
        A.check(A.lib().hdb_mst_boruvka(c.h, X.p, n, d, core.p, metric_of(distanceFunction), int(bool(selfEdges)),
                                        A.ptr(va), A.ptr(vb), A.ptr(w)), "constructMSTBoruvka")
        return UndirectedGraph(va, vb, w)

    def exactMST(self, dataSet, k: int, distanceFunction=None, semantics: int = A.CORE_EXCL_SELF,
                 selfEdges: bool = True, merged: bool = False):
        """FirstStep's leaf branch on one large partition (FirstStep.java:104-108):
        calculateCoreDistances + the exact MRD MST (constructMSTBoruvka's weights and edge
        order) in one call sharing one spatial index.  Returns (core, UndirectedGraph).
        merged: the edges in the reducers' merge order (UnionFindReducer.java:19-69 +
        SortMST.java:9-17) -- what sort_edges_desc returns for the plain list -- without the
        re-sort (HDB_EDGES_MERGED)."""
        X = A.Arr(dataSet, np.float64)
        n, d = X.obj.shape
        ne = (n - 1) + (n if selfEdges else 0)
        core = A.new_like(X, (n,), np.float64)
        va = A.new_like(X, (ne,), np.int32)
        vb = A.new_like(X, (ne,), np.int32)
        w = A.new_like(X, (ne,), np.float64)
        c = _ctx(X, self.ctx)
        flags = (A.EDGES_SELF if selfEdges else 0) | (A.EDGES_MERGED if merged else 0)
        A.check(A.lib().hdb_exact_mst(c.h, X.p, n, d, k, metric_of(distanceFunction), semantics, flags,
                                      A.ptr(core), A.ptr(va), A.ptr(vb), A.ptr(w)), "exactMST")
        return core, UndirectedGraph(va, vb, w)

    def knn(self, dataSet, k: int, distanceFunction=None, exclSelf: bool = False, withIndices: bool = False):
        """Per-row k smallest distances (ascending, Double.MAX_VALUE padded) [+ indices]."""
        X = A.Arr(dataSet, np.float64)
        n, d = X.obj.shape
        dist = A.new_like(X, (n, k), np.float64)
        idx = A.new_like(X, (n, k), np.int32) if withIndices else None
        c = _ctx(X, self.ctx)
        A.check(A.lib().hdb_knn(c.h, X.p, n, d, k, metric_of(distanceFunction), int(exclSelf), A.ptr(dist),
                                A.ptr(idx)), "knn")
        return (dist, idx) if withIndices else dist


def flat_labels(va, vb, w, n: int, minClSize: int, ctx=None):
    """Global HDBSCAN* flat partition over a merged MST (the reference's
    Main.java:351-408 never completes it): HDBSCANStar.java:208-625 semantics, canonical tie
    rules.  Returns (labels[n] with 1..K by smallest member id and 0 = noise, K).
    Device tensors, or any arrays with a ctx, run the device algorithm (K6, csrc/flat.hip);
    host arrays without a ctx run the host algorithm (csrc/flat.cpp) with no device."""
    a, b, ww = A.Arr(va, np.int32), A.Arr(vb, np.int32), A.Arr(w, np.float64)
    labels = A.new_like(a, (n,), np.int32)
    k = np.zeros(1, np.int64)
    on_dev = a.device is not None and a.device.type == "cuda"
    h = ctx.h if ctx is not None else (A.Context.get(a.device.index or 0).h if on_dev else None)
    A.check(A.lib().hdb_flat_labels(h, a.p, b.p, ww.p, ww.obj.shape[0], n, minClSize, A.ptr(labels), A.ptr(k)),
            "flat_labels")
    return labels, int(k[0])
