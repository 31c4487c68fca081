"""K1t (box-pruned k-NN over the Morton/BVH index, csrc/spatial.hip) parity: the lists and
all three core semantics must equal the oracle and the all-pairs K1 bit for bit, for every
d the index supports, every minPts bucket, duplicates, ties, non-finite values and ragged
tile counts.  The tree only skips pairs that provably fail the strict '<' insertion test
(HDBSCANStar.java:89), so any difference is a bug.
"""
import contextlib

import numpy as np
import pytest

from conftest import blobs, load_skin

pytestmark = pytest.mark.gpu


def eq(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(np.where(na, 0.0, a).view(np.uint64), np.where(nb, 0.0, b).view(np.uint64))


@contextlib.contextmanager
def options(ctx, **kw):
    defaults = {"knn_tree": 1, "knn_tree_min_n": 8192, "knn_fp32_screen": 1, "count_evals": 0,
                "leaf_seed_k": -1, "leaf_list_rounds": 2, "boruvka_seed": 1, "boruvka_wave_pts": 64,
                "boruvka_early_pts": 0, "boruvka_adj_seed": 1, "k1t_xcd_chunks": 8, "bor_xcd_chunks": 8}
    try:
        for k, v in kw.items():
            ctx.set_option(k, v)
        yield
    finally:
        for k in kw:
            ctx.set_option(k, defaults[k])


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(0)
    c.use_torch_stream()  # device tensors below are produced/consumed on torch's stream
    return c


@pytest.fixture(scope="module")
def star(pkg, ctx):
    return pkg.HDBSCANStar(ctx)


def tree_cores(ctx, star, X, mp, sem):
    with options(ctx, knn_tree=1, knn_tree_min_n=0):
        return star.calculateCoreDistances(X, mp, None, sem)


@pytest.mark.parametrize("d", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("min_pts", [2, 4, 8, 16, 32])
def test_tree_cores_vs_oracle(ctx, star, oracle, d, min_pts):
    X = blobs(2500, d, 6, 7 * d + min_pts)
    for sem in range(3):
        assert eq(tree_cores(ctx, star, X, min_pts, sem), oracle.core_distances(X, min_pts, semantics=sem)), sem


@pytest.mark.parametrize("n", [1, 2, 3, 5, 63, 64, 65, 511, 513, 4097])
def test_tree_ragged_sizes(ctx, star, oracle, n):
    X = blobs(n, 3, 3, n)
    for sem in range(3):
        assert eq(tree_cores(ctx, star, X, 4, sem), oracle.core_distances(X, 4, semantics=sem)), (n, sem)


def test_tree_duplicates_skin(ctx, star, oracle):
    X = load_skin(20000)  # integer RGB, max multiplicity in the hundreds: zero-distance ties
    for sem in range(3):
        assert eq(tree_cores(ctx, star, X, 4, sem), oracle.core_distances(X, 4, semantics=sem)), sem


def test_tree_lists_equal_dense(ctx, star):
    X = blobs(60000, 3, 12, 21)
    for k in (1, 3, 7, 15, 31):
        with options(ctx, knn_tree=1, knn_tree_min_n=0):
            a = star.knn(X, k, None, exclSelf=True)
        with options(ctx, knn_tree=0):
            b = star.knn(X, k, None, exclSelf=True)
        assert eq(a, b), k


@pytest.mark.parametrize("n", [1, 65, 4097, 70000])
def test_tree_xcd_chunks_lists_equal(ctx, star, n):
    """K1t's XCD-interleaved chunk map (k1t_xcd_chunks) only places workgroups: the lists are
    the same with it off, at the default 8 chunks per XCD and at 3 (uneven chunk counts)."""
    X = blobs(n, 3, 5, 31 + n)
    out = []
    for m in (0, 8, 3):
        with options(ctx, knn_tree=1, knn_tree_min_n=0, k1t_xcd_chunks=m):
            out.append(star.knn(X, 7, None, exclSelf=True))
    assert eq(out[0], out[1]) and eq(out[0], out[2])


@pytest.mark.parametrize("d", [2, 8, 16])
def test_tree_equals_dense_mid_size(ctx, star, d):
    X = blobs(30000, d, 30, 100 + d, spread=20.0)
    for sem in range(3):
        a = tree_cores(ctx, star, X, 8, sem)
        with options(ctx, knn_tree=0):
            b = star.calculateCoreDistances(X, 8, None, sem)
        assert eq(a, b), sem


def test_tree_uniform_and_scales(ctx, star, oracle):
    rng = np.random.default_rng(3)
    for scale in (1e-9, 1.0, 1e8, 1e150):
        X = rng.uniform(-1, 1, size=(3000, 3)) * scale
        X[10:20] = X[9]
        for sem in range(3):
            assert eq(tree_cores(ctx, star, X, 5, sem), oracle.core_distances(X, 5, semantics=sem)), (scale, sem)


def test_tree_nonfinite(ctx, star, oracle):
    X = blobs(2000, 3, 3, 5)
    X[7, 1] = np.nan
    X[100, 0] = np.inf
    X[101, 2] = -np.inf
    for sem in range(3):
        assert eq(tree_cores(ctx, star, X, 4, sem), oracle.core_distances(X, 4, semantics=sem)), sem


def test_tree_prunes(ctx, star):
    """Diagnostic counter: at 200k clustered points the tree evaluates a tiny fraction of n^2."""
    X = blobs(200_000, 3, 20, 1)
    with options(ctx, knn_tree=1, knn_tree_min_n=0, count_evals=1):
        star.calculateCoreDistances(X, 4, None, 2)
        ev = ctx.get_stat("last_evals")
    assert 0 < ev < 0.01 * 200_000 ** 2


def test_tree_full_size_rows(star):
    """1M x 3 (config 2) through the default path (tree): exact per-row check on a sample."""
    import torch
    X = blobs(1_000_000, 3, 20, 1)
    got = star.calculateCoreDistances(torch.from_numpy(X).cuda(), 4, None, 2).cpu().numpy()
    rng = np.random.default_rng(6)
    for r in rng.choice(X.shape[0], 24, replace=False):
        s = (X[r, 0] - X[:, 0]) * (X[r, 0] - X[:, 0])
        s = s + (X[r, 1] - X[:, 1]) * (X[r, 1] - X[:, 1])
        s = s + (X[r, 2] - X[:, 2]) * (X[r, 2] - X[:, 2])
        s[r] = np.inf
        assert got[r] == np.sqrt(np.partition(s, 2)[:3].max()), r


# ------------------------------------------- fused exact leaf (hdb_exact_mst)
def _sorted_edges(g):
    return g.getVerticeA(), g.getVericeB(), g.getEges()


@pytest.mark.parametrize("d", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("min_pts", [2, 4, 9])
def test_exact_mst_equals_two_calls(star, oracle, d, min_pts):
    """hdb_exact_mst (one index, kNN-seeded Boruvka round 0) == calculateCoreDistances +
    constructMSTBoruvka, bit for bit: cores for all three semantics, and the same edges in
    the same order (the (w, s, lo, hi) key makes the MST unique)."""
    X = np.round(blobs(6000, d, 8, 11 * d + min_pts), 1)  # rounded: heavy weight ties
    for sem in range(3):
        core, g = star.exactMST(X, min_pts, None, sem, selfEdges=True)
        ref_core = oracle.core_distances(X, min_pts, semantics=sem)
        assert eq(core, ref_core), sem
        b = star.constructMSTBoruvka(X, ref_core, True)
        for u, v in zip(_sorted_edges(g), _sorted_edges(b)):
            assert eq(np.asarray(u, dtype=np.float64), np.asarray(v, dtype=np.float64)), (d, sem)


def test_exact_mst_weights_equal_prim_skin(star, oracle):
    """Skin prefix (integer RGB, massive duplication): the sorted MST weights equal the
    reference Prim's (HDBSCANStar.java:124-205) exactly."""
    X = load_skin(12000)
    core, g = star.exactMST(X, 4, None, 2, selfEdges=False)
    ref_core = oracle.core_distances(X, 4, semantics=2)
    assert eq(core, ref_core)
    _, _, w = oracle.prim_mst(X, ref_core, self_edges=False)
    assert eq(np.sort(g.getEges()), np.sort(w))


@pytest.mark.parametrize("n", [1, 2, 3, 64, 65, 4097])
def test_exact_mst_ragged(star, oracle, n):
    X = blobs(n, 3, 3, n + 1)
    core, g = star.exactMST(X, 4, None, 2, selfEdges=True)
    assert eq(core, oracle.core_distances(X, 4, semantics=2))
    assert len(g.getEges()) == 2 * n - 1
    _, _, w = oracle.prim_mst(X, core, self_edges=False)
    assert eq(np.sort(g.getEges()[: n - 1]), np.sort(w))


def test_exact_mst_device_full_size(star):
    """1M x 3 (config 2) on device tensors: cores equal the split path, MST equals
    constructMSTBoruvka edge for edge."""
    import torch
    t = torch.from_numpy(blobs(1_000_000, 3, 20, 1)).cuda()
    core, g = star.exactMST(t, 4, None, 2, selfEdges=False)
    ref_core = star.calculateCoreDistances(t, 4, None, 2)
    assert torch.equal(core, ref_core)
    b = star.constructMSTBoruvka(t, ref_core, False)
    assert torch.equal(g.getEges(), b.getEges())
    assert torch.equal(g.getVerticeA(), b.getVerticeA()) and torch.equal(g.getVericeB(), b.getVericeB())


@pytest.mark.parametrize("d", [2, 3, 8])
def test_exact_mst_seeding_options_equal(ctx, star, d):
    """Every seeding knob (list length, rounds seeded from the lists, previous-round seeds and
    their carried bounds, the Morton-adjacency seeds) changes only which lanes search, never the MST: edge for edge
    equal to the plain constructMSTBoruvka on the same cores (tie-heavy rounded blobs)."""
    X = np.round(blobs(20000, d, 12, 7 * d), 1)
    core, _ = star.exactMST(X, 4, None, 2, selfEdges=False)
    ref = _sorted_edges(star.constructMSTBoruvka(X, core, False))
    for kw in ({}, dict(leaf_seed_k=0), dict(leaf_seed_k=7, leaf_list_rounds=64),
               dict(leaf_seed_k=15, leaf_list_rounds=1), dict(leaf_list_rounds=0),
               dict(boruvka_seed=0), dict(boruvka_seed=0, leaf_list_rounds=1),
               dict(boruvka_adj_seed=0), dict(boruvka_adj_seed=0, boruvka_seed=0, leaf_list_rounds=0),
               # workgroup placement only (XCD-interleaved chunks off, or one chunk per XCD)
               dict(k1t_xcd_chunks=0, bor_xcd_chunks=0), dict(k1t_xcd_chunks=1, bor_xcd_chunks=1),
               # the diagnostic pass at its largest per-wave record count (the
               # record buffer must fit its carve at 16 points per wave)
               dict(count_evals=1, boruvka_wave_pts=16, boruvka_early_pts=16),
               dict(count_evals=1, boruvka_wave_pts=32)):
        with options(ctx, **kw):
            c2, g = star.exactMST(X, 4, None, 2, selfEdges=False)
        assert eq(c2, core), kw
        for u, v in zip(_sorted_edges(g), ref):
            assert eq(np.asarray(u, dtype=np.float64), np.asarray(v, dtype=np.float64)), (d, kw)


def _spanning_tree(va, vb, n):
    """Host union-find: the n-1 edges connect all n points without a cycle."""
    p = np.arange(n)

    def find(x):
        while p[x] != x:
            p[x] = p[p[x]]
            x = p[x]
        return x
    assert va.shape[0] == n - 1
    for a, b in zip(va.tolist(), vb.tolist()):
        ra, rb = find(a), find(b)
        assert ra != rb, "cycle"
        p[rb] = ra
    return True


def test_exact_mst_1m_is_spanning_tree_with_prim_weights(star):
    """C2 at full size (1M x 3) checked independently of K2b: the edges form a spanning tree
    of the 1M points, the sorted weights equal those of the GPU stepwise reference Prim
    (prim_step_kernel, HDBSCANStar.java:124-205, bit-exact against the oracle up to 60k),
    which shares no code with the Boruvka path but the distance functor, and the flat labels
    of both trees are identical."""
    import time
    import torch
    t = torch.from_numpy(blobs(1_000_000, 3, 20, 1)).cuda()
    core, g = star.exactMST(t, 4, None, 2, selfEdges=False)
    va, vb = g.getVerticeA().cpu().numpy(), g.getVericeB().cpu().numpy()
    assert _spanning_tree(va, vb, 1_000_000)
    t0 = time.perf_counter()
    p = star.constructMST(t, core, False)
    torch.cuda.synchronize()
    print(f"stepwise Prim 1M: {time.perf_counter() - t0:.1f} s")
    assert torch.equal(torch.sort(g.getEges())[0], torch.sort(p.getEges())[0])
    # the C2 output itself: the flat labels of the K2b tree (device K6) equal those of the
    # reference Prim's tree (device K6 and the host algorithm, csrc/flat.cpp) -- the hierarchy
    # removes a tie group at once, so equal-weight topology differences cannot change them
    import importlib
    pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
    n = 1_000_000
    lab_k, k_k = pkg.flat_labels(g.getVerticeA(), g.getVericeB(), g.getEges(), n, 4)
    lab_p, k_p = pkg.flat_labels(p.getVerticeA(), p.getVericeB(), p.getEges(), n, 4)
    host, k_h = pkg.flat_labels(p.getVerticeA().cpu().numpy(), p.getVericeB().cpu().numpy(),
                                p.getEges().cpu().numpy(), n, 4)
    assert k_k == k_p == k_h and k_k >= 1
    assert torch.equal(lab_k, lab_p) and np.array_equal(lab_p.cpu().numpy(), host)


def test_exact_mst_full_skin_weights_equal_prim(star):
    """All 245,057 Skin rows (max multiplicity 1,598: zero-weight ties everywhere), live
    cumulative cores: K2b's sorted weights equal the GPU reference Prim's and its edges form
    a spanning tree."""
    import torch
    X = torch.from_numpy(load_skin()).cuda()
    n = X.shape[0]
    core, g = star.exactMST(X, 4, None, 0, selfEdges=False)
    assert _spanning_tree(g.getVerticeA().cpu().numpy(), g.getVericeB().cpu().numpy(), n)
    p = star.constructMST(X, core, False)
    assert torch.equal(torch.sort(g.getEges())[0], torch.sort(p.getEges())[0])
    import importlib
    pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
    lab_k, k_k = pkg.flat_labels(g.getVerticeA(), g.getVericeB(), g.getEges(), n, 4)
    lab_p, k_p = pkg.flat_labels(p.getVerticeA(), p.getVericeB(), p.getEges(), n, 4)
    assert k_k == k_p and torch.equal(lab_k, lab_p)  # zero-weight tie groups everywhere


def _merged_vs_sorted(pkg, star, ctx, X, min_pts, self_edges=True, sem=2):
    """hdb_exact_mst's HDB_EDGES_MERGED output must equal hdb_sort_edges_desc of its plain
    output bit for bit (the reducers' merge order, SortMST.java:9-17, ties included)"""
    import torch
    Xd = torch.from_numpy(np.ascontiguousarray(X)).cuda()
    c1, g1 = star.exactMST(Xd, min_pts, None, sem, self_edges)
    c2, g2 = star.exactMST(Xd, min_pts, None, sem, self_edges, merged=True)
    ref = pkg.sort_edges_desc(g1.getVerticeA(), g1.getVericeB(), g1.getEges(), ctx)
    got = (g2.getVerticeA(), g2.getVericeB(), g2.getEges())
    assert torch.equal(c1.view(torch.int64), c2.view(torch.int64))
    assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    assert torch.equal(got[2].view(torch.int64), ref[2].view(torch.int64))


@pytest.mark.parametrize("d", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("min_pts", [1, 2, 4, 9])
def test_exact_mst_merged_order_equals_sort(pkg, ctx, star, d, min_pts):
    """minPts 1: the two-call fallback path (re-sorted); the rest the fused leaf's merge-path order"""
    _merged_vs_sorted(pkg, star, ctx, blobs(20000, d, 8, 3 + d), min_pts)


@pytest.mark.parametrize("n", [1, 2, 3, 64, 65, 4097])
def test_exact_mst_merged_order_ragged_and_no_self(pkg, ctx, star, n):
    X = blobs(n, 3, 3, n)
    _merged_vs_sorted(pkg, star, ctx, X, 4)
    if n > 1:  # n = 1 without self edges: no edges at all (empty outputs are rejected as before)
        _merged_vs_sorted(pkg, star, ctx, X, 4, self_edges=False)


def test_exact_mst_merged_order_ties_full_size(pkg, ctx, star):
    """Skin (heavy duplication: huge zero-weight tie groups between tree and self edges) and
    1M blobs (the bench's partition)"""
    _merged_vs_sorted(pkg, star, ctx, load_skin(), 4)
    _merged_vs_sorted(pkg, star, ctx, blobs(1_000_000, 3, 20, 1), 4)
