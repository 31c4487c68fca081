"""Global HDBSCAN* flat labels over a merged MST.

The oracle (oracle/flat_labels.py, the top-down restatement of HDBSCANStar.java:208-625) is
pinned against scikit-learn's independent HDBSCAN implementation (condensed tree + excess of
mass), fed the same MST: identical partitions wherever the two definitions coincide -- every
input without weight ties at split levels (single linkage on continuous data, minPts = 1) --
and near-identical with the MRD ties minPts > 1 creates (sklearn splits ties in binary
dendrogram order, the canonical rule removes a tie group at once).  The library's bottom-up
union-find (csrc/flat.cpp, host algorithm, ctx = NULL) must equal the oracle exactly,
including heavy ties, zero weights (duplicates), noise-only and single-cluster trees.
"""
import numpy as np
import pytest

from conftest import blobs, load_iris, load_skin


def sk_labels_on_mst(va, vb, w, n, mcs):
    from sklearn.cluster._hdbscan import _linkage as Lk, _tree as T
    m = va != vb
    mst = np.zeros(int(m.sum()), dtype=Lk.MST_edge_dtype)
    mst["current_node"], mst["next_node"], mst["distance"] = va[m], vb[m], w[m]
    mst = mst[np.argsort(mst["distance"], kind="mergesort")]
    return T.tree_to_labels(Lk.make_single_linkage(mst), min_cluster_size=mcs)[0]


def same_partition(a, b_sk):
    """a: 0 = noise, 1..K; b_sk: -1 = noise, 0..K-1 (any numbering)."""
    if not np.array_equal(a == 0, b_sk == -1):
        return False
    pairs = set(zip(a[a > 0].tolist(), b_sk[a > 0].tolist()))
    return len(pairs) == len(set(a[a > 0].tolist())) == len(set(b_sk[b_sk >= 0].tolist()))


def mst_of(oracle, X, min_pts):
    core = oracle.core_distances(X, min_pts, semantics=oracle.EXCL_SELF)
    return oracle.prim_mst(X, core)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_equals_sklearn_single_linkage(oracle, seed):
    from oracle.flat_labels import flat_labels
    X = blobs(1200, 2, 6, seed, spread=10.0)
    va, vb, w = mst_of(oracle, X, 1)  # minPts = 1: core 0, MRD = distance, no ties
    for mcs in (5, 15, 40):
        lab, k = flat_labels(X.shape[0], va, vb, w, mcs)
        assert same_partition(lab, sk_labels_on_mst(va, vb, w, X.shape[0], mcs)), mcs


@pytest.mark.parametrize("seed", range(4))
def test_oracle_close_to_sklearn_mrd(oracle, seed):
    from sklearn.metrics import adjusted_rand_score
    from oracle.flat_labels import flat_labels
    X = blobs(1500, 2, 6, seed, spread=10.0)
    va, vb, w = mst_of(oracle, X, 5)
    lab, _ = flat_labels(X.shape[0], va, vb, w, 10)
    sk = sk_labels_on_mst(va, vb, w, X.shape[0], 10)
    assert adjusted_rand_score(lab, sk) > 0.99


def lib_flat(pkg, va, vb, w, n, mcs):
    return pkg.flat_labels(np.asarray(va, np.int32), np.asarray(vb, np.int32), np.asarray(w, np.float64), n, mcs)


def cases(oracle):
    rng = np.random.default_rng(0)
    out = []
    for min_pts in (1, 4, 8):
        X = blobs(900, 3, 5, min_pts, spread=15.0)
        out.append(("blobs", X.shape[0], *mst_of(oracle, X, min_pts)))
    X = load_iris()
    out.append(("iris", X.shape[0], *mst_of(oracle, X, 4)))
    X = load_skin(1500)  # duplicates: zero-weight ties everywhere
    out.append(("skin", X.shape[0], *mst_of(oracle, X, 4)))
    # random trees with integer weights: huge tie groups, multi-way splits
    for t in range(6):
        n = int(rng.integers(2, 600))
        va = np.array([int(rng.integers(0, i)) for i in range(1, n)], np.int32)
        vb = np.arange(1, n, dtype=np.int32)
        w = rng.integers(0, 1 + t * 3, size=n - 1).astype(np.float64)
        perm = rng.permutation(n).astype(np.int32)
        out.append((f"rand{t}", n, perm[va], perm[vb], w))
    # star tree: one vertex, all other points tied
    n = 50
    out.append(("star", n, np.zeros(n - 1, np.int32), np.arange(1, n, dtype=np.int32), np.ones(n - 1)))
    return out


def test_library_equals_oracle_with_ties(pkg, oracle):
    from oracle.flat_labels import flat_labels
    for name, n, va, vb, w in cases(oracle):
        for mcs in (2, 4, 10, 30):
            ref, kr = flat_labels(n, va, vb, w, mcs)
            got, kg = lib_flat(pkg, va, vb, w, n, mcs)
            assert kg == kr and np.array_equal(got, ref), (name, mcs)


def test_library_self_edges_ignored_and_errors(pkg, oracle):
    X = load_iris()
    core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    va, vb, w = oracle.prim_mst(X, core, self_edges=True)  # with the n self edges
    va2, vb2, w2 = oracle.prim_mst(X, core, self_edges=False)
    a, _ = lib_flat(pkg, va, vb, w, X.shape[0], 4)
    b, _ = lib_flat(pkg, va2, vb2, w2, X.shape[0], 4)
    assert np.array_equal(a, b)
    with pytest.raises(pkg.HdbError):
        lib_flat(pkg, va2[:-1], vb2[:-1], w2[:-1], X.shape[0], 4)  # not spanning
    with pytest.raises(pkg.HdbError):
        lib_flat(pkg, va2, vb2, w2, X.shape[0], 1)  # minClSize < 2
    lab, k = lib_flat(pkg, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0), 1, 4)
    assert k == 0 and lab.tolist() == [0]


def test_library_large_tree_fast(pkg):
    """1M-point random tree: the bottom-up algorithm is O(E log E)."""
    import time
    rng = np.random.default_rng(1)
    n = 1_000_000
    va = (rng.random(n - 1) * np.arange(1, n)).astype(np.int32)
    vb = np.arange(1, n, dtype=np.int32)
    w = rng.random(n - 1)
    t = time.perf_counter()
    lab, k = lib_flat(pkg, va, vb, w, n, 20)
    assert time.perf_counter() - t < 10 and lab.shape == (n,)
