"""Pins the CPU oracle (oracle/hdb_oracle.c) before it is trusted as the parity checker.

The reference has no tests or golden vectors and cannot run here (no JVM).
Pinning therefore uses: (1) known-answer tests hand-derived from the Java source
(SURVEY.md §8(c)); (2) an independent pure-Python transcription of the Java loops on small
inputs; (3) scipy / sklearn on the standard (EXCL_SELF) semantics; (4) the committed golden
fixtures (regression).
"""
import math

import numpy as np
import pytest

from conftest import blobs, golden, load_iris, load_skin

JMAX = np.finfo(np.float64).max


# ---------------------------------------------------- pure-Python transcription
def py_dist(a, b):  # EuclideanDistance.java:28-36
    s = 0.0
    for x, y in zip(a, b):
        s += (x - y) * (x - y)
    return math.sqrt(s)


def py_core(X, k, cumulative, excl):  # HDBSCANStar.java:71-106 / CreateLocalMST.java:138-185
    K = k - 1
    if k == 1:
        return [0.0] * len(X)
    buf = [JMAX] * K
    core = []
    for p in range(len(X)):
        if not cumulative:
            buf = [JMAX] * K
        for q in range(len(X)):
            if excl and p == q:
                continue
            dd = py_dist(X[p], X[q])
            idx = K
            while idx >= 1 and dd < buf[idx - 1]:
                idx -= 1
            if idx < K:
                buf[idx + 1:] = buf[idx:K - 1]
                buf[idx] = dd
        core.append(buf[K - 1])
    return core


def py_prim(X, core, ids):  # HDBSCANStar.java:124-205
    n = len(X)
    att = [False] * n
    best = [JMAX] * n
    par = [0] * n
    cur = n - 1
    att[cur] = True
    na = 1
    while na < n:
        nd, npnt = JMAX, -1
        for nb in range(n):
            if nb == cur or att[nb]:
                continue
            dd = py_dist(X[cur], X[nb])
            m = dd
            if core[cur] > m:
                m = core[cur]
            if core[nb] > m:
                m = core[nb]
            if m < best[nb]:
                best[nb] = m
                par[nb] = ids[cur]
            if best[nb] <= nd:
                nd, npnt = best[nb], nb
        att[npnt] = True
        na += 1
        cur = npnt
    va = par[:n - 1] + list(ids)
    vb = list(ids[:n - 1]) + list(ids)
    w = best[:n - 1] + list(core)
    return va, vb, w


def py_nearest(X, S):  # FirstStep.java:74-85
    out = []
    for x in X:
        mn, nn = JMAX, 0
        for j, s in enumerate(S):
            dd = py_dist(x, s)
            if dd < mn:
                mn, nn = dd, j
        out.append(nn)
    return out


# ---------------------------------------------------------------------- KATs
def test_iris_kats(oracle):
    """SURVEY.md §8(c) KATs on 数据集/dataset.txt at minPts = 4."""
    X = load_iris()
    core = oracle.core_distances(X, 4, semantics=oracle.INCL_SELF_CUMULATIVE)
    assert core[0] == 0.1414213562373093 and core[1] == 0.09999999999999998
    assert np.count_nonzero(core) == 2 and np.all(core[2:] == 0)  # core[i]=0 for i >= minPts-2
    va, vb, w = oracle.prim_mst(X, core)
    s = 0.0
    for x in w[:149]:
        s += x
    assert s == 43.56520099453603
    assert (va[0], vb[0], w[0]) == (39, 0, 0.14142135623730964)
    assert (va[1], vb[1], w[1]) == (34, 1, 0.14142135623730964)
    assert (va[2], vb[2], w[2]) == (47, 2, 0.14142135623730978)
    core2 = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    _, _, w2 = oracle.prim_mst(X, core2)
    s2 = 0.0
    for x in w2[:149]:
        s2 += x
    assert s2 == 58.0188251332504


def test_cumulative_zero_property(oracle):
    X = blobs(300, 3, 4, 1)
    for k in (2, 3, 4, 7):
        core = oracle.core_distances(X, k, semantics=oracle.INCL_SELF_CUMULATIVE)
        assert np.all(core[max(k - 2, 0):] == 0)


def test_min_pts_one_all_zero(oracle):
    X = blobs(50, 3, 2, 2)
    for sem in range(3):
        assert np.all(oracle.core_distances(X, 1, semantics=sem) == 0)


# ------------------------------------------------- independent transcription
@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_matches_python_transcription(oracle, seed):
    rng = np.random.default_rng(seed)
    X = np.round(rng.uniform(0, 5, size=(40, 3)), 1)  # rounding creates exact ties
    ids = np.arange(40, dtype=np.int32) + 7
    for cum, excl, sem in [(True, False, 0), (False, False, 1), (False, True, 2)]:
        c_py = py_core(X.tolist(), 4, cum, excl)
        c_or = oracle.core_distances(X, 4, semantics=sem)
        assert np.array_equal(np.asarray(c_py), c_or)
        va, vb, w = py_prim(X.tolist(), c_py, ids.tolist())
        ova, ovb, ow = oracle.prim_mst(X, c_or, ids)
        assert np.array_equal(va, ova) and np.array_equal(vb, ovb) and np.array_equal(w, ow)
    S = X[::5]
    assert np.array_equal(py_nearest(X.tolist(), S.tolist()), oracle.nearest_sample(X, S)[0])


# ------------------------------------------------------ independent libraries
def test_excl_self_core_vs_sklearn(oracle):
    from sklearn.neighbors import NearestNeighbors
    X = blobs(800, 3, 5, 3)
    core = oracle.core_distances(X, 5, semantics=oracle.EXCL_SELF)
    d, _ = NearestNeighbors(n_neighbors=5).fit(X).kneighbors(X)  # includes self at 0
    np.testing.assert_allclose(core, d[:, 4], rtol=1e-12)


def test_mst_weight_vs_scipy(oracle):
    from scipy.sparse.csgraph import minimum_spanning_tree
    from scipy.spatial.distance import cdist
    X = blobs(500, 3, 4, 4)
    core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    _, _, w = oracle.prim_mst(X, core, self_edges=False)
    D = cdist(X, X)
    M = np.maximum(D, np.maximum(core[:, None], core[None, :]))
    np.fill_diagonal(M, 0)
    t = minimum_spanning_tree(M).toarray()
    # sorted weights of any MST are identical
    np.testing.assert_allclose(np.sort(w), np.sort(t[t > 0]), rtol=1e-12)


def test_nearest_first_minimum_on_ties(oracle):
    X = np.array([[0.0, 0.0], [1.0, 0.0]])
    S = np.array([[2.0, 0.0], [-1.0, 0.0], [0.0, 1.0], [1.0, 1.0]])
    idx, dist = oracle.nearest_sample(X, S)
    assert idx.tolist() == [1, 0] and dist.tolist() == [1.0, 1.0]  # first of equal minima (1 vs 2; 0 vs 3)


def test_prim_select_last_index_on_ties(oracle):
    # four corners of a unit square: all MRDs tie -> '<=' select picks the LAST index
    X = np.array([[0.0, 0.0], [0.0, 1.0], [1.0, 0.0], [1.0, 1.0]])
    core = np.zeros(4)
    va, vb, w = oracle.prim_mst(X, core, self_edges=False)
    # start at 3: updates 1 and 2 (dist 1), 0 (sqrt2); select last min = 2, then 0 via 2, then 1
    assert va.tolist() == [2, 3, 3] and w.tolist() == [1.0, 1.0, 1.0]


# ------------------------------------------------------------ bubble formulas
def test_combine_step_singleton_and_pair(oracle):
    X = np.array([[1.0, 2.0], [3.0, 6.0], [5.0, 5.0]])
    st = oracle.bubble_stats(X, np.array([0, 0, 1], np.int32), 2)
    # bubble 1: never combined -> (rep=x, [0,0,1]) (FirstStep.java:87-101)
    assert st["rep"][1].tolist() == [5.0, 5.0] and st["info"][1].tolist() == [0, 0, 1]
    # bubble 0: n=2, ls=(4,8), ss=(10,40): extent = mean_i sqrt((2n ss - 2 ls^2)/(n(n-1)))
    e = (math.sqrt((4 * 10 - 2 * 16) / 2) + math.sqrt((4 * 40 - 2 * 64) / 2)) / 2
    assert st["rep"][0].tolist() == [2.0, 4.0]
    assert st["info"][0][0] == e and st["info"][0][1] == e and st["info"][0][2] == 2  # nnDist=extent, d>=2


def test_combine_step_d1_nndist(oracle):
    X = np.array([[1.0], [4.0], [9.0]])
    st = oracle.bubble_stats(X, np.zeros(3, np.int32), 1)
    ext = st["info"][0][0]
    assert st["info"][0][1] == (1 / 3) * ext  # pow(1/n, 1) * extent for d = 1


def test_cf_int_overflow(oracle):
    # n*(n-1) is a Java int: 46342*46341 wraps negative
    n = 46342
    X = np.ones((n, 1))
    st = oracle.bubble_stats(X, np.zeros(n, np.int32), 1, "cf")
    prod = np.int32(np.int64(n) * (n - 1) & 0xFFFFFFFF)
    assert prod < 0
    num = (2 * n * float(n)) - 2 * (float(n) * float(n))  # 0
    assert st["info"][0][0] == math.sqrt(num / float(prod))


def test_distance_bubbles_branches(oracle):
    e = np.array([1.0, 2.0])
    nn = np.array([0.5, 0.25])
    assert oracle.distance_bubbles(10.0, e, nn, 0, 1) == (10.0 - 3.0) + 0.75
    assert oracle.distance_bubbles(2.0, e, nn, 0, 1) == 0.5  # overlap -> max(nn)


# --------------------------------------------------------------- regression
@pytest.mark.parametrize("name", ["iris", "skin3k", "blobs2k"])
def test_oracle_against_golden(oracle, name):
    g = golden(name)
    X = g["X"]
    for sem, tag in [(0, "cum"), (1, "incl"), (2, "excl")]:
        core = oracle.core_distances(X, 4, semantics=sem)
        assert np.array_equal(core, g[f"core_{tag}"])
        va, vb, w = oracle.prim_mst(X, core, g["ids"])
        assert np.array_equal(va, g[f"prim_{tag}_va"]) and np.array_equal(w, g[f"prim_{tag}_w"])


def test_oracle_bubble_slice_against_golden(oracle):
    g = golden("iris")
    lm = oracle.local_model(g["b_rep"], g["b_info"], 4, 4)
    assert np.array_equal(lm["labels"], g["b_labels"])
    assert np.array_equal(lm["mst"][2], g["b_mst_w"])


def test_skin_parse_d1():
    X = load_skin(5)
    assert X.shape == (5, 3) and X[0].tolist() == [74.0, 85.0, 123.0]


def test_cpu_all_variants_equal_serial(oracle):
    """bench.py's CPU-all baseline (OpenMP over rows / over each Prim step's scan) computes
    exactly what the serial oracle does, ties included (Skin duplicates)."""
    from conftest import load_skin
    for X in (blobs(3000, 3, 6, 2), load_skin(2500)):
        n = X.shape[0]
        rows = np.arange(0, n, 7)
        ref = oracle.core_rows(X, rows, 4)
        core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
        va, vb, w = oracle.prim_mst(X, core, self_edges=False)
        for t in (1, 3, 8):
            assert np.array_equal(oracle.core_rows_par(X, rows, 4, t), ref)
            pa, pb, pw = oracle.prim_mst_par(X, core, t)
            assert np.array_equal(pa, va) and np.array_equal(pb, vb) and np.array_equal(pw, w)


def test_create_local_mst_record_fields(oracle):
    """CreateLocalMST.java:187-292: the tracked nearestneighborsID / otherVertexIndicesID are
    the local indices of each record's vertices; the edges are HDBSCANStar's Prim edges."""
    X = load_iris()
    core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    ids = (np.arange(X.shape[0], dtype=np.int32) * 7 + 3)
    va, vb, w, f1, f2, nd = oracle.create_local_mst(X, core, ids, 11)
    ra, rb, rw = oracle.prim_mst(X, core, ids)
    assert np.array_equal(va, ra) and np.array_equal(vb, rb) and np.array_equal(w, rw)
    assert np.array_equal(ids[f1], va) and np.array_equal(ids[f2], vb) and np.all(nd == 11)
    n = X.shape[0]
    assert np.array_equal(f2[:n - 1], np.arange(n - 1)) and np.array_equal(f1[n - 1:], np.arange(n))


def test_bubble_stats_slices_d11(oracle):
    """D11: one slice is the sequential CombineStep fold bit for bit; any slicing keeps the
    member counts and differs from the fold only by summation order (rounding)"""
    rng = np.random.default_rng(3)
    X = np.round(rng.normal(size=(6000, 5)) * 10, 3)
    bo = rng.integers(0, 900, 6000).astype(np.int32)
    a = oracle.bubble_stats(X, bo, 900)
    b = oracle.bubble_stats(X, bo, 900, cuts=[0, 6000])
    assert all(np.array_equal(a[k], b[k]) for k in a)
    c = oracle.bubble_stats(X, bo, 900, cuts=[0, 0, 1500, 3000, 6000])
    assert np.array_equal(a["info"][:, 2], c["info"][:, 2])
    np.testing.assert_allclose(c["ls"], a["ls"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(c["rep"], a["rep"], rtol=1e-12, atol=1e-12)
    with pytest.raises(oracle.OracleError):
        oracle.bubble_stats(X, bo, 900, cuts=[0, 7000])
