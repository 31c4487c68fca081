"""TEST INFRASTRUCTURE ONLY -- a second, independent transcription of the reference's bubble
local model, written directly from the Java in pure Python (numpy only to evaluate
vectors of the same scalar expressions), with its own emulation of the JDK 8 collections
whose iteration order decides the labels.  Nothing here is derived from hdb_oracle.c or
from the product's local_model.cpp; tests/test_java_transcription.py cross-checks it against
the C oracle (the pin VERDICT r02 asked for).  Only tests/ may import it.

Transcribed (file:line under /root/reference/源代码/):
  distance/EuclideanDistance.java:28-36            euclidean_row
  databubbles/HdbscanDataBubbles.java:592-600      distance_bubbles
  databubbles/HdbscanDataBubbles.java:75-146       calculate_core_distances_bubbles
  databubbles/HdbscanDataBubbles.java:165-254      construct_mst_bubbles
  hdbscanstar/UndirectedGraph.java:44-124,157-234  UndirectedGraph (+ quicksort_by_edge_weight)
  hdbscanstar/Clusters.java:27-47                  Clusters.detach_points
  databubbles/HdbscanDataBubbles.java:256-375      construct_cluster_tree
  databubbles/HdbscanDataBubbles.java:377-504      find_prominent_clusters_and_classification_noise_bubbles
  databubbles/HdbscanDataBubbles.java:506-527      find_inter_cluster_edges
  main/LocalModelReduceByKey.java:76-108           local_model
JDK 8 semantics emulated from the published java.util sources (not vendored, OpenJDK 8):
  HashMap<Integer, V>: hash = h ^ (h >>> 16), table created at the first put with capacity
  16, threshold 0.75 * capacity, resize doubles and splits every bucket into (lo, hi) lists
  keeping their order, keySet() iterates buckets ascending and each bucket in list order; a
  bucket reaching 9 nodes is treeified when the table has >= 64 buckets (then the iteration
  order changes: JavaTreeifyError is raised -- unsupported) and triggers a resize otherwise.
  TreeSet<Integer>: add / pollFirst / isEmpty (a set plus a heap).
  ArrayList.remove(Object): first occurrence, no-op if absent.
  Collections.sort: stable merge sort (TimSort) -- identical to any stable sort for a
  consistent comparator; a NaN birth level makes comparatorA inconsistent and is refused.
Java exceptions are raised as JavaException with the hdbmi code (HDB_EREF_*) and a detail.
"""
from __future__ import annotations

import heapq
import math

import numpy as np

JMAX = float(np.finfo(np.float64).max)  # Double.MAX_VALUE

EREF_NPE, EREF_OOB, EREF_NEGATIVE_CLUSTER, EREF_DIVZERO = -10, -11, -12, -13


class JavaException(RuntimeError):
    def __init__(self, code: int, detail):
        super().__init__(f"java exception {code}: {detail}")
        self.code = code
        self.detail = detail


class JavaTreeifyError(RuntimeError):
    """A HashMap bin would become a tree bin: its iteration order is not emulated."""


class JavaHang(RuntimeError):
    """The Java loop would not terminate (e.g. a NaN edge weight in constructClusterTree)."""


# ----------------------------------------------------------------- java.lang helpers
def jidiv(a: int, b: int) -> int:
    """int / int (truncation toward zero); ArithmeticException on / by zero."""
    if b == 0:
        raise JavaException(EREF_DIVZERO, "/ by zero")
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def jrecip(x: float) -> float:
    """1 / x in IEEE double (Python raises on a zero divisor)."""
    if x == 0.0:
        return math.copysign(math.inf, x)
    return 1.0 / x


def jpow(a: float, b: float) -> float:
    """Math.pow for the exponents that occur here (the int quotients 0 and 1)."""
    if b == 0.0:
        return 1.0
    if b == 1.0:
        return a
    return math.pow(a, b)


def jarr(arr, i: int):
    """Java array read: ArrayIndexOutOfBoundsException outside [0, length)."""
    if i < 0 or i >= len(arr):
        raise JavaException(EREF_OOB, f"index {i} length {len(arr)}")
    return arr[i]


# ----------------------------------------------------------------- java.util emulation
class JavaHashMap:
    """java.util.HashMap<Integer, V> (JDK 8) -- enough for put/get/isEmpty/keySet order."""

    def __init__(self):
        self.table = None
        self.thr = 0
        self.size = 0

    @staticmethod
    def _hash(k: int) -> int:
        h = k & 0xFFFFFFFF
        return h ^ (h >> 16)

    def _resize(self):
        if self.table is None:
            self.table = [[] for _ in range(16)]
            self.thr = 12
            return
        old = self.table
        cap = len(old)
        new = [[] for _ in range(2 * cap)]
        for j, bucket in enumerate(old):
            for node in bucket:  # split keeps the order of each half
                (new[j] if (node[2] & cap) == 0 else new[j + cap]).append(node)
        self.table = new
        self.thr = self.thr * 2

    def get(self, k):
        if self.table is None:
            return None
        h = self._hash(k)
        for node in self.table[h & (len(self.table) - 1)]:
            if node[0] == k:
                return node[1]
        return None

    def put(self, k, v):
        if self.table is None:
            self._resize()
        h = self._hash(k)
        bucket = self.table[h & (len(self.table) - 1)]
        for node in bucket:
            if node[0] == k:
                node[1] = v
                return
        before = len(bucket)
        bucket.append([k, v, h])
        if before >= 8:  # binCount >= TREEIFY_THRESHOLD - 1
            if len(self.table) < 64:  # MIN_TREEIFY_CAPACITY: resize instead
                self._resize()
            else:
                raise JavaTreeifyError(f"HashMap bin with {before + 1} keys at capacity {len(self.table)}")
        self.size += 1
        if self.size > self.thr:
            self._resize()

    def is_empty(self):
        return self.size == 0

    def key_set(self):
        out = []
        if self.table is not None:
            for bucket in self.table:
                out.extend(node[0] for node in bucket)
        return out


class JavaTreeSet:
    """java.util.TreeSet<Integer>: add, remove, pollFirst, isEmpty, ascending iteration
    (a set plus a heap with lazy deletion)."""

    def __init__(self, items=()):
        self.s = set()
        self.h = []
        for x in items:
            self.add(x)

    def add(self, x):
        if x not in self.s:
            self.s.add(x)
            heapq.heappush(self.h, x)

    def remove(self, x):
        self.s.discard(x)

    def poll_first(self):
        while True:
            x = heapq.heappop(self.h)
            if x in self.s:
                self.s.discard(x)
                return x

    def is_empty(self):
        return not self.s

    def __contains__(self, x):
        return x in self.s

    def __iter__(self):
        return iter(sorted(self.s))

    def __len__(self):
        return len(self.s)


def array_list_remove(lst, value):
    """ArrayList.remove(Object): the first occurrence, false (no-op) if absent."""
    try:
        lst.remove(value)
    except ValueError:
        pass


# ----------------------------------------------------------------- distance
def euclidean_row(rep, p: int):
    """EuclideanDistance.computeDistance(rep[p], rep[q]) for every q at once: the same
    scalar sequence (0 + t0, then + t1, ...; separate multiply and add; sqrt)."""
    diff = rep[p][None, :] - rep
    s = diff[:, 0] * diff[:, 0]
    for c in range(1, rep.shape[1]):
        s = s + diff[:, c] * diff[:, c]
    return np.sqrt(s)


def euclidean(a, b) -> float:
    s = 0.0
    for x, y in zip(a, b):
        s += (float(x) - float(y)) * (float(x) - float(y))
    return math.sqrt(s)


def jmax(a: float, b: float) -> float:
    """Math.max(double, double): NaN if either is NaN, +0.0 over -0.0."""
    if a != a or b != b:
        return math.nan
    if a == b:
        return b if math.copysign(1.0, a) < 0 else a
    return a if a > b else b


def jmax_row(a: float, b):
    """Math.max(a, b[q]) for every q: NaN-propagating, +0.0 over -0.0."""
    b = np.asarray(b, np.float64)
    m = np.maximum(a, b)
    z = (m == 0.0) & (a == 0.0)
    if z.any():
        m = np.where(z & ~(np.signbit(a) & np.signbit(b)), 0.0, m)
    return m


def distance_bubbles(distance, eB, nnDistB, point, neighbor):
    """HdbscanDataBubbles.distanceBubbles (:592-600), scalar."""
    verify = distance - (eB[point] + eB[neighbor])
    if verify >= 0:
        return (distance - (eB[point] + eB[neighbor])) + (nnDistB[point] + nnDistB[neighbor])
    return jmax(float(nnDistB[point]), float(nnDistB[neighbor]))


def distance_bubbles_row(dist, eB, nnDistB, point):
    """distanceBubbles(dist[q], eB, nnDistB, point, q) for every q (numpy, same expressions)."""
    with np.errstate(invalid="ignore"):
        verify = dist - (eB[point] + eB)
        a = (dist - (eB[point] + eB)) + (nnDistB[point] + nnDistB)
        return np.where(verify >= 0, a, jmax_row(float(nnDistB[point]), nnDistB))


# ----------------------------------------------------------------- bubble cores (:75-146)
def calculate_core_distances_bubbles(repB, nB, eB, nnDistB, k):
    b = repB.shape[0]
    d = repB.shape[1]
    num_neighbors = k - 1
    index_bubbles = [0] * num_neighbors  # never reset across points (:79-83)
    core = [0.0] * b
    if k == 1:
        return np.asarray(core)
    for point in range(b):
        knn = [JMAX] * num_neighbors
        dist = distance_bubbles_row(euclidean_row(repB, point), eB, nnDistB, point)
        # the insertion loop (:97-120) in neighbour order; a neighbour whose distance is not
        # below the current (k-1)-th value writes nothing, and that value only falls, so
        # blocks are pre-filtered against the value at the block start
        lo, step = 0, 32
        while lo < b:
            blk = dist[lo:lo + step]
            with np.errstate(invalid="ignore"):
                cand = np.nonzero(blk < knn[num_neighbors - 1])[0]
            for off in cand:
                neighbor = lo + int(off)
                if neighbor == point:
                    continue
                distance = float(blk[off])
                ni = num_neighbors
                while ni >= 1 and distance < knn[ni - 1]:
                    ni -= 1
                if ni < num_neighbors:
                    for s in range(num_neighbors - 1, ni, -1):
                        knn[s] = knn[s - 1]
                    knn[ni] = distance
                    index_bubbles[ni] = neighbor
            lo += blk.shape[0]
            step = min(2 * step, 8192)
        if nB[point] >= num_neighbors:
            core[point] = jpow(float(jidiv(num_neighbors, int(nB[point]))), float(jidiv(1, d))) * float(eB[point])
        else:
            nX = int(nB[point])
            i = 0
            while nX < num_neighbors:
                nX += int(jarr(nB, jarr(index_bubbles, i)))
                i += 1
            s = int(nB[point])
            aux = 0
            for j in range(i):
                ij = index_bubbles[j]
                dc = euclidean(jarr(repB, ij), jarr(repB, i))
                dc = distance_bubbles(dc, eB, nnDistB, ij, i)
                if s < num_neighbors and knn[j] < dc:
                    aux = num_neighbors - s
                s += int(nB[ij])
            kv = jarr(knn, i)
            q = jidiv(aux, int(jarr(nB, i)))
            core[point] = kv + jpow(float(q), float(jidiv(1, jarr(repB, i).shape[0]))) * float(jarr(eB, i))
    return np.asarray(core, dtype=np.float64)


# ----------------------------------------------------------------- bubble Prim (:165-254)
def construct_mst_bubbles(repB, eB, nnDistB, idBubbles, core, self_edges=True):
    b = repB.shape[0]
    sec = b if self_edges else 0
    nbr = np.zeros(b - 1 + sec, np.int64)  # new int[]: zeros
    best = np.zeros(b - 1 + sec)
    best[: b - 1] = JMAX
    attached = np.zeros(b, bool)
    cur = b - 1
    attached[b - 1] = True
    n_att = 1
    while n_att < b:
        dist = distance_bubbles_row(euclidean_row(repB, cur), eB, nnDistB, cur)
        mrd = dist.copy()
        with np.errstate(invalid="ignore"):
            mrd = np.where(core[cur] > mrd, core[cur], mrd)
            mrd = np.where(core > mrd, core, mrd)
        free = ~attached
        free[cur] = False
        cand = np.nonzero(free)[0]
        m = mrd[cand]
        with np.errstate(invalid="ignore"):
            upd = m < best[cand]
        best[cand[upd]] = m[upd]
        nbr[cand[upd]] = idBubbles[cur]
        # argmin with <= in index order: the last index among the smallest values
        bv = best[cand]
        mn = bv.min() if cand.size else math.nan
        if not cand.size or not (mn <= JMAX):
            raise JavaException(EREF_OOB, "BitSet.set(-1)")
        nxt = int(cand[np.nonzero(bv == mn)[0][-1]])
        attached[nxt] = True
        n_att += 1
        cur = nxt
    other = np.zeros(b - 1 + sec, np.int64)
    other[: b - 1] = idBubbles[: b - 1]
    if self_edges:
        nbr[b - 1:] = idBubbles
        other[b - 1:] = idBubbles
        best[b - 1:] = core
    return UndirectedGraph(b, nbr.astype(np.int64).tolist(), other.astype(np.int64).tolist(), best.tolist())


# ----------------------------------------------------------------- UndirectedGraph
class UndirectedGraph:
    """UndirectedGraph(numVertices, A, B, W) (:51-84) and quicksortByEdgeWeight (:93-124)."""

    def __init__(self, num_vertices, va, vb, w):
        self.num_vertices = num_vertices
        self.va, self.vb, self.w = list(va), list(vb), list(w)
        self.edges = {}
        for a, b in zip(self.va, self.vb):
            self.edges.setdefault(a, []).append(b)
            if a != b:
                self.edges.setdefault(b, []).append(a)

    def _swap(self, i, j):
        if i == j:
            return
        self.va[i], self.va[j] = self.va[j], self.va[i]
        self.vb[i], self.vb[j] = self.vb[j], self.vb[i]
        self.w[i], self.w[j] = self.w[j], self.w[i]

    def _select_pivot_index(self, start, end):
        if start - end <= 1:  # (:158) always true for start <= end
            return start
        first, middle, last = self.w[start], self.w[start + (end - start) // 2], self.w[end]
        if first <= middle:
            if middle <= last:
                return start + (end - start) // 2
            return end if last >= first else start
        if first <= last:
            return start
        return end if last >= middle else start + (end - start) // 2

    def _partition(self, start, end, pivot):
        pv = self.w[pivot]
        self._swap(pivot, end)
        low = start
        if end - start > 64:  # exact shortcut: nothing in [start, end) below the pivot -> no swaps
            with np.errstate(invalid="ignore"):
                if not np.any(np.asarray(self.w[start:end]) < pv):
                    self._swap(low, end)
                    return low
        for i in range(start, end):
            if self.w[i] < pv:
                self._swap(i, low)
                low += 1
        self._swap(low, end)
        return low

    def quicksort_by_edge_weight(self):
        n = len(self.w)
        if n <= 1:
            return
        size = n // 2
        start_stack = [0] * size
        end_stack = [0] * size
        start_stack[0] = 0
        end_stack[0] = n - 1
        top = 0
        while top >= 0:
            s, e = start_stack[top], end_stack[top]
            top -= 1
            p = self._select_pivot_index(s, e)
            p = self._partition(s, e, p)
            if p > s + 1:
                if top + 1 >= size:
                    raise JavaException(EREF_OOB, "quicksort stack")
                start_stack[top + 1] = s
                end_stack[top + 1] = p - 1
                top += 1
            if p < e - 1:
                if top + 1 >= size:
                    raise JavaException(EREF_OOB, "quicksort stack")
                start_stack[top + 1] = p + 1
                end_stack[top + 1] = e
                top += 1


# ----------------------------------------------------------------- Clusters (:27-47)
class Clusters:
    __slots__ = ("label", "birth", "death", "num_points", "members", "stability", "parent_id", "has_children")

    def __init__(self, label, parent, birth, num_points, members):
        self.label = label
        self.birth = birth
        self.death = JMAX
        self.num_points = num_points
        self.members = members  # sorted list (TreeSet) or None
        self.stability = 0.0
        self.parent_id = parent
        self.has_children = False

    def detach_points(self, num_points, count_members, level):
        self.num_points -= num_points
        self.stability += float(num_points + count_members) * (jrecip(level) - jrecip(self.birth))
        if self.num_points == 0:
            self.death = level
        elif self.num_points < 0:
            raise JavaException(EREF_NEGATIVE_CLUSTER,
                                dict(label=self.label, level=level, num_points=self.num_points))


def _first_alive(clusters, label):
    for c in clusters:
        if c.label == label and c.death == JMAX:
            return c
    return None


# ----------------------------------------------------------------- cluster tree (:256-375)
def construct_cluster_tree(mst: UndirectedGraph, mcl_size, nB):
    cur = len(mst.w) - 1
    next_label = 2
    labels = [1] * mst.num_vertices
    clusters = [Clusters(1, -1, math.nan, int(sum(int(x) for x in nB)), None)]
    nv = mst.num_vertices
    while cur >= 0:
        affected = JavaHashMap()
        w = mst.w[cur]
        if w != w:
            raise JavaHang("NaN edge weight: the removal loop never advances")
        while cur >= 0 and mst.w[cur] == w:
            a, b = mst.va[cur], mst.vb[cur]
            la, lb = mst.edges.get(a), mst.edges.get(b)
            if la is None or lb is None:
                raise JavaException(EREF_NPE, "edge list of a vertex")
            array_list_remove(la, b)
            array_list_remove(lb, a)
            if jarr(labels, a) == 0:
                cur -= 1
                continue
            ts = affected.get(labels[a])
            if ts is None:
                ts = JavaTreeSet()
                affected.put(labels[a], ts)
            ts.add(a)
            ts.add(b)
            cur -= 1
        if affected.is_empty():
            continue
        for parent_label in affected.key_set():
            new_clusters = []
            ts = affected.get(parent_label)
            while not ts.is_empty():
                root = ts.poll_first()
                visited = bytearray(nv)
                visited[root] = 1
                comp = [root]
                stack = [root]
                while stack:  # TreeSet queue: the visit order does not change the set reached
                    v = stack.pop()
                    adj = mst.edges.get(v)
                    if adj is None:
                        raise JavaException(EREF_NPE, "getEdges().get(vertex)")
                    for u in adj:
                        if not visited[u]:
                            visited[u] = 1
                            stack.append(u)
                            comp.append(u)
                count = 0
                for v in comp:
                    count += int(nB[v])
                if count >= mcl_size:
                    new_clusters.append(Clusters(parent_label, parent_label, w, count, sorted(comp)))
                else:
                    for v in comp:
                        labels[v] = 0
                    c = _first_alive(clusters, parent_label)
                    if c is not None:
                        c.detach_points(count, 0, w)
            if len(new_clusters) >= 2:
                for cl in new_clusters:
                    cl.label = next_label
                    for m in cl.members:
                        labels[m] = next_label
                    next_label += 1
                    c = _first_alive(clusters, cl.parent_id)
                    if c is not None:
                        c.has_children = True
                        c.detach_points(cl.num_points, 0, cl.birth)
                    clusters.append(cl)
    return clusters


# ----------------------------------------------------------------- FOSC + noise (:377-504)
def find_prominent_clusters_and_classification_noise_bubbles(clusters, rep, nB, extent, nnDist, idBubbles):
    tree = clusters[1:]  # clusterTree.remove(0): the root
    adj = {}
    for parent in tree:
        if not parent.has_children and parent.label not in adj:
            adj[parent.label] = []
        for child in tree:
            if parent.label == child.parent_id:
                adj.setdefault(parent.label, []).append(
                    [parent.stability, float(child.label), child.stability, 1.0, float(parent.parent_id)])
    if any(c.birth != c.birth for c in tree):
        raise JavaTreeifyError("NaN birth level: comparatorA is inconsistent, TimSort order not emulated")
    tree = sorted(tree, key=lambda c: c.birth)  # Collections.sort (stable), -0.0 == 0.0
    b = len(nB)
    flat = [[int(idBubbles[o]), 0] for o in range(b)]
    solution = JavaTreeSet(c.label for c in tree)
    set_keys = [c.label for c in tree]
    for key in set_keys:
        lst = adj.get(key)
        if lst is None:
            raise JavaException(EREF_NPE, "adjListNodes.get(key)")
        children_stab = 0.0
        if lst:
            for info in lst:
                children_stab += info[2]
            if children_stab <= lst[0][0]:
                for i in range(len(lst)):
                    root = int(lst[i][1])
                    queue = JavaTreeSet([root])
                    visited = {root}
                    lst[i][3] = 0.0
                    solution.remove(root)
                    while not queue.is_empty():
                        v = queue.poll_first()
                        vl = adj.get(v)
                        if vl is not None:
                            for e in vl:
                                solution.remove(v)
                                c = int(e[1])
                                if c not in visited:
                                    queue.add(c)
                                    visited.add(c)
            else:
                lst[0][0] = children_stab
                gp = adj.get(int(lst[0][4]))
                if gp is not None:
                    for e in gp:
                        if int(e[1]) == key:
                            e[2] = children_stab
        else:
            solution.remove(key)
    sol = list(solution)
    for cl in tree:
        for prominent in sol:
            if cl.label == prominent:
                for m in cl.members:
                    jarr(flat, m)[1] = prominent
    # noise -> the first neighbour (index order) that is labelled at that moment and whose
    # bubble distance is below Double.MAX_VALUE (:485-502)
    lab = np.array([f[1] for f in flat], np.int64)
    for point in range(b):
        if lab[point] != 0:
            continue
        dist = distance_bubbles_row(euclidean_row(rep, point), extent, nnDist, point)
        with np.errstate(invalid="ignore"):
            ok = (lab != 0) & (dist < JMAX)
        ok[point] = False
        hit = np.nonzero(ok)[0]
        if hit.size:
            lab[point] = lab[hit[0]]
            flat[point][1] = int(lab[point])
    return flat


def find_inter_cluster_edges(mst: UndirectedGraph, flat):
    va, vb, w = [], [], []
    for i in range(len(mst.w)):
        if jarr(flat, mst.va[i])[1] != jarr(flat, mst.vb[i])[1]:
            va.append(mst.va[i])
            vb.append(mst.vb[i])
            w.append(mst.w[i])
    return va, vb, w


# ----------------------------------------------------------------- LocalModelReduceByKey
def local_model(rep, info, min_pts, min_cl_size):
    """LocalModelReduceByKey.call (:76-108) on one subset's bubbles (D4 ids 0..b-1):
    dict(labels, mst=(va, vb, w) after the quicksort, inter=(va, vb, w)); raises
    JavaException where the reference throws."""
    rep = np.ascontiguousarray(rep, np.float64)
    info = np.ascontiguousarray(info, np.float64)
    b = rep.shape[0]
    eB = info[:, 0].copy()
    nnB = info[:, 1].copy()
    nB = [int(x) for x in info[:, 2]]  # (int) infoBubbles[i][2]
    ids = np.arange(b, dtype=np.int64)
    core = calculate_core_distances_bubbles(rep, nB, eB, nnB, min_pts)
    mst = construct_mst_bubbles(rep, eB, nnB, ids, core, True)
    mst.quicksort_by_edge_weight()
    clusters = construct_cluster_tree(mst, min_cl_size, nB)
    flat = find_prominent_clusters_and_classification_noise_bubbles(clusters, rep, nB, eB, nnB, ids)
    iva, ivb, iw = find_inter_cluster_edges(mst, flat)
    return dict(core=core, labels=np.array([f[1] for f in flat], np.int32),
                mst=(np.array(mst.va, np.int32), np.array(mst.vb, np.int32), np.array(mst.w, np.float64)),
                inter=(np.array(iva, np.int32), np.array(ivb, np.int32), np.array(iw, np.float64)))
