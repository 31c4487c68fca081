"""Parity of the HIP path (through the C-ABI) against the CPU oracle and the committed
golden fixtures.  Bar: bit-exact for every value the reference computes in double
arithmetic with +,-,*,/,sqrt (core distances, MST weights, distances, bubble LS/SS/rep/
extent) and for every integer/index output (edges, nearest sample, labels); 1e-9 relative
for the CF variant's real-exponent Math.pow (ClusterFeatureDataBubbles.java:213).
"""
import numpy as np
import pytest
import torch

from conftest import blobs, golden, load_iris, load_skin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def star(pkg):
    return pkg.HDBSCANStar()


def eq(a, b):
    """Bit-exact equality (NaN == NaN regardless of payload, as Java's NaN is one value)."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype == np.float64:
        na, nb = np.isnan(a), np.isnan(b)
        if not np.array_equal(na, nb):
            return False
        a, b = np.where(na, 0.0, a), np.where(nb, 0.0, b)
        return np.array_equal(a.view(np.uint64), b.view(np.uint64))
    return np.array_equal(a, b)


# ------------------------------------------------------------------ distance
def test_distance_rows_bitexact_incl_sqrt_rounding(pkg, oracle):
    rng = np.random.default_rng(0)
    for d in (1, 2, 3, 8, 16):
        a = rng.normal(size=(20000, d)) * rng.choice([1e-3, 1, 1e3, 1e150], size=(20000, 1))
        b = a + rng.normal(size=(20000, d)) * 1e-2
        for name in ["euclidean", "cosine", "pearson", "manhattan", "supremum"]:
            got = pkg.distance_rows(a, b, name)
            ref = np.array([oracle.distance(a[i], b[i], name) for i in range(0, 20000, 97)])
            assert eq(got[::97], ref), (d, name)


# ------------------------------------------------------------ core distances
@pytest.mark.parametrize("name", ["iris", "skin3k", "blobs2k"])
def test_core_distances_golden(star, name):
    g = golden(name)
    for sem, tag in [(0, "cum"), (1, "incl"), (2, "excl")]:
        assert eq(star.calculateCoreDistances(g["X"], 4, None, sem), g[f"core_{tag}"]), tag


@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 6, 7, 8, 16])
@pytest.mark.parametrize("min_pts", [1, 2, 4, 8, 16, 32])
def test_core_distances_vs_oracle(star, oracle, d, min_pts):
    X = blobs(1500, d, 5, d * 100 + min_pts)
    for sem in range(3):
        assert eq(star.calculateCoreDistances(X, min_pts, None, sem), oracle.core_distances(X, min_pts, semantics=sem))


def test_core_distances_ragged_and_tiny(star, oracle):
    for n in (1, 2, 3, 5, 255, 257, 1023, 1025):
        X = blobs(n, 3, 2, n)
        for sem in range(3):
            assert eq(star.calculateCoreDistances(X, 4, None, sem), oracle.core_distances(X, 4, semantics=sem)), n


def test_core_distances_duplicates_skin(star, oracle):
    X = load_skin(6000)  # integer RGB with heavy duplication: exact zero distances
    for sem in range(3):
        assert eq(star.calculateCoreDistances(X, 4, None, sem), oracle.core_distances(X, 4, semantics=sem))


def test_core_distances_other_metrics(star):
    g = golden("metrics300")
    for name in ["euclidean", "cosine", "pearson", "manhattan", "supremum"]:
        for tag, sem in [("incl", 1), ("excl", 2), ("cum", 0)]:
            assert eq(star.calculateCoreDistances(g["X"], 5, name, sem), g[f"{name}_core_{tag}"]), (name, tag)


def test_knn_lists_and_indices(star, oracle):
    X = blobs(3000, 3, 4, 9)
    for k in (1, 3, 7, 15):
        ref = oracle.knn_lists(X, k + 1, excl_self=True)
        dist, idx = star.knn(X, k, None, exclSelf=True, withIndices=True)
        assert eq(dist, ref)
        # indices point at a row with exactly that distance
        for r in range(0, 3000, 137):
            for c in range(k):
                j = idx[r, c]
                assert j != r and oracle.distance(X[r], X[j]) == dist[r, c]


def test_core_distances_device_tensors(star, oracle):
    import torch
    X = blobs(5000, 3, 6, 1)
    t = torch.from_numpy(X).cuda()
    got = star.calculateCoreDistances(t, 4, None, 2)
    assert got.is_cuda
    assert eq(got.cpu().numpy(), oracle.core_distances(X, 4, semantics=2))


def test_core_distances_full_size_rows(star):
    """BASELINE config 2 size (1M x 3): exact per-row check on a row sample -- numpy
    elementwise ops follow the Java order (no FMA), sqrt is correctly rounded."""
    import torch
    X = blobs(1_000_000, 3, 20, 1)
    got = star.calculateCoreDistances(torch.from_numpy(X).cuda(), 4, None, 2).cpu().numpy()
    rng = np.random.default_rng(5)
    for r in rng.choice(X.shape[0], 24, replace=False):
        s = (X[r, 0] - X[:, 0]) * (X[r, 0] - X[:, 0])
        s = s + (X[r, 1] - X[:, 1]) * (X[r, 1] - X[:, 1])
        s = s + (X[r, 2] - X[:, 2]) * (X[r, 2] - X[:, 2])
        s[r] = np.inf
        ref = np.sqrt(np.partition(s, 2)[:3].max())
        assert got[r] == ref, r


# ----------------------------------------------------------------------- MST
@pytest.mark.parametrize("name", ["iris", "skin3k", "blobs2k"])
def test_prim_golden(star, name):
    g = golden(name)
    for tag in ["cum", "incl", "excl"]:
        mst = star.constructMST(g["X"], g[f"core_{tag}"], True, None, g["ids"])
        assert eq(mst.getVerticeA(), g[f"prim_{tag}_va"]), tag
        assert eq(mst.getVericeB(), g[f"prim_{tag}_vb"]), tag
        assert eq(mst.getEges(), g[f"prim_{tag}_w"]), tag


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 256, 257, 1024, 1025, 4096, 4097, 7000])
def test_prim_sizes_vs_oracle(star, oracle, n):
    X = np.round(blobs(n, 3, 4, n), 2)  # rounding -> many exact MRD ties
    core = oracle.core_distances(X, 4, semantics=2)
    ids = np.arange(n, dtype=np.int32) * 3 + 1
    mst = star.constructMST(X, core, True, None, ids)
    va, vb, w = oracle.prim_mst(X, core, ids)
    assert eq(mst.getVerticeA(), va) and eq(mst.getVericeB(), vb) and eq(mst.getEges(), w)


def test_prim_other_metrics_golden(star):
    g = golden("metrics300")
    for name in ["euclidean", "cosine", "pearson", "manhattan", "supremum"]:
        mst = star.constructMST(g["X"], g[f"{name}_core_incl"], True, name)
        assert eq(mst.getVerticeA(), g[f"{name}_va"]) and eq(mst.getEges(), g[f"{name}_w"]), name


def test_prim_batched_partitions(pkg, oracle):
    import ctypes as C
    sizes = [1, 5, 50, 64, 300, 1000, 4100, 2]
    X = np.round(blobs(sum(sizes), 3, 4, 77), 2)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    core = oracle.core_distances(X, 4, semantics=2)  # any cores
    ids = np.arange(X.shape[0], dtype=np.int32) + 100
    ne = sum(2 * s - 1 for s in sizes)
    va, vb, w = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
    ctx = pkg.Context.get(0)
    A = pkg._capi
    A.check(A.lib().hdb_prim_mst_batched(ctx.h, A.ptr(X), A.ptr(off), len(sizes), 3, A.ptr(core), A.ptr(ids), 0, 1,
                                         A.ptr(va), A.ptr(vb), A.ptr(w)), "batched")
    e = 0
    for p, s in enumerate(sizes):
        ra, rb, rw = oracle.prim_mst(X[off[p]:off[p + 1]], core[off[p]:off[p + 1]], ids[off[p]:off[p + 1]])
        assert eq(va[e:e + 2 * s - 1], ra) and eq(vb[e:e + 2 * s - 1], rb) and eq(w[e:e + 2 * s - 1], rw), p
        e += 2 * s - 1


def test_first_step_leaf_batched(pkg, oracle):
    """FirstStep leaf branch (FirstStep.java:104-120) for many partitions at once."""
    sizes = [50, 49, 1, 2, 37, 50, 3, 4100]
    X = load_skin(sum(sizes))
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    ids = np.arange(X.shape[0], dtype=np.int32) + 5
    fs = pkg.FirstStep(0.2, 50, 4)
    core, mst = fs.leaf(X, ids, off)
    e = 0
    for p, s in enumerate(sizes):
        rc, (ra, rb, rw) = oracle.first_step_leaf(X[off[p]:off[p + 1]], ids[off[p]:off[p + 1]], 4)
        assert eq(core[off[p]:off[p + 1]], rc), p
        sl = slice(e, e + 2 * s - 1)
        assert eq(mst.getVerticeA()[sl], ra) and eq(mst.getVericeB()[sl], rb) and eq(mst.getEges()[sl], rw), p
        e += 2 * s - 1


def _check_spanning_tree(n, va, vb):
    parent = list(range(n))

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x
    for a, b in zip(va, vb):
        ra, rb = find(int(a)), find(int(b))
        assert ra != rb, "cycle"
        parent[ra] = rb
    assert len({find(i) for i in range(n)}) == 1


@pytest.mark.parametrize("n,d", [(2, 3), (100, 3), (5000, 3), (6000, 2), (3000, 8), (20000, 3)])
def test_boruvka_weights_equal_prim(star, oracle, n, d):
    X = np.round(blobs(n, d, 6, n + d), 1)  # heavy ties
    core = oracle.core_distances(X, 4, semantics=2)
    mst = star.constructMSTBoruvka(X, core, False)
    _, _, w = oracle.prim_mst(X, core, self_edges=False)
    assert eq(np.sort(mst.getEges()), np.sort(w))  # MST weight multiset is unique
    _check_spanning_tree(n, mst.getVerticeA(), mst.getVericeB())
    # edges are reported sorted by (w, lo, hi)
    k = np.lexsort((mst.getVericeB(), mst.getVerticeA(), mst.getEges()))
    assert np.array_equal(k, np.arange(n - 1))


def test_boruvka_large_vs_gpu_prim(star):
    """Borůvka vs the (exact) stepwise GPU Prim on a 60k graph: identical sorted weights."""
    import torch
    X = blobs(60000, 3, 20, 1)
    t = torch.from_numpy(X).cuda()
    core = star.calculateCoreDistances(t, 4, None, 2)
    wb = star.constructMSTBoruvka(t, core, False).getEges().cpu().numpy()
    wp = star.constructMST(t, core, False).getEges().cpu().numpy()
    assert eq(np.sort(wb), np.sort(wp))


# ------------------------------------------------------------ nearest sample
@pytest.mark.parametrize("name", ["iris", "skin3k"])
def test_nearest_golden(pkg, name):
    g = golden(name)
    idx, dist = pkg.nearest_sample(g["X"], g["ns_S"], with_dist=True)
    assert eq(idx, g["ns_idx"]) and eq(dist, g["ns_dist"])


def test_nearest_other_metrics(pkg):
    g = golden("metrics300")
    for name in ["euclidean", "cosine", "pearson", "manhattan", "supremum"]:
        idx, dist = pkg.nearest_sample(g["X"], g["S"], name, with_dist=True)
        assert eq(idx, g[f"{name}_ns_idx"]) and eq(dist, g[f"{name}_ns_dist"]), name


@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 6, 7, 8, 16])
def test_nearest_vs_oracle(pkg, oracle, d):
    X = np.round(blobs(4000, d, 5, d), 1)
    S = X[::7].copy()
    idx, dist = pkg.nearest_sample(X, S, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S)
    assert eq(idx, r_idx) and eq(dist, r_dist)


def test_nearest_keyed(pkg, oracle):
    rng = np.random.default_rng(4)
    X = np.round(blobs(5000, 3, 5, 4), 1)
    xk = rng.integers(0, 7, 5000).astype(np.int32)
    S = X[::9].copy()
    sk = xk[::9].copy()
    sk[sk == 6] = 5  # key 6 has no samples -> index 0 / MAX as the Java init
    idx, dist = pkg.nearest_sample(X, S, None, xk, sk, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S, x_key=xk, s_key=sk)
    assert eq(idx, r_idx) and eq(dist, r_dist)


def test_nearest_sqrt_ties(pkg, oracle):
    """Two samples whose squared distances differ but whose sqrt values are equal: Java's
    strict '<' on sqrt values keeps the FIRST; an argmin on squares would pick the second."""
    rng = np.random.default_rng(11)
    c = rng.normal(size=(400000, 2))
    c /= np.sqrt((c * c).sum(1))[:, None]
    s = c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]
    r = np.sqrt(s)
    order = np.lexsort((s, r))
    found = None
    for a, b in zip(order[:-1], order[1:]):
        if r[a] == r[b] and s[a] < s[b]:
            found = (b, a)  # larger square first
            break
    assert found is not None
    S = np.stack([c[found[0]], c[found[1]], [5.0, 5.0]])
    X = np.zeros((3, 2))
    idx, dist = pkg.nearest_sample(X, S, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S)
    assert eq(idx, r_idx) and idx[0] == 0 and eq(dist, r_dist)


# ------------------------------------------------------------- bubble stats
@pytest.mark.parametrize("name", ["iris", "skin_bubbles2k", "blobs2k"])
def test_bubble_stats_golden(pkg, name):
    g = golden(name)
    ls, ss, rep, info = pkg.bubble_stats(g["X"], g["b_bubble_of"], g["b_used"].shape[0])
    assert eq(ls, g["b_ls"]) and eq(ss, g["b_ss"]) and eq(rep, g["b_rep"]) and eq(info, g["b_info"])


def test_bubble_stats_cf(pkg):
    g = golden("blobs2k")
    ls, ss, rep, info = pkg.bubble_stats(g["X"], g["b_bubble_of"], g["b_used"].shape[0], pkg.BUBBLE_CF)
    assert eq(rep, g["cf_rep"]) and eq(ls, g["cf_ls"]) and eq(info[:, 0], g["cf_info"][:, 0])
    np.testing.assert_allclose(info[:, 1], g["cf_info"][:, 1], rtol=1e-9)  # real-exponent pow


@pytest.mark.parametrize("d", [1, 3, 8])
def test_bubble_partials_combine_vs_oracle_slices(pkg, oracle, d):
    """D11 CombineStep over slices: hdb_bubble_partials (per-slice folds, here in two calls as
    two ranks would make them) + hdb_bubble_combine (slice order, empty partials skipped) equal
    the oracle's sliced fold bit for bit -- empty slices, a one-slice bubble, empty bubbles --
    and one slice equals hdb_bubble_stats"""
    import ctypes
    import torch
    A = pkg._capi
    rng = np.random.default_rng(40 + d)
    n, nb = 20000, 3000
    X = np.round(rng.normal(size=(n, d)) * 30, 3)
    bo = rng.integers(0, nb, n).astype(np.int32)
    bo[bo == 11] = 12                           # bubble 11 empty
    bo[bo == 2999] = 7
    bo[5000:5003] = 2999                        # bubble 2999: three members, all in one slice
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    c = A.Context.get(0)
    c.use_torch_stream()
    for cuts in ([0, n], [0, 2500, 2500, 9000, 13000, n], [0, 4000, 8000, 12000, 16000, n], [0, 0, n, n]):
        S = len(cuts) - 1
        pl = torch.empty(S * nb * d, dtype=torch.float64, device="cuda")
        pq, pn = torch.empty_like(pl), torch.empty(S * nb, dtype=torch.float64, device="cuda")
        h = S // 2  # slices [0, h) and [h, S) folded by two calls ("ranks")
        for s0, s1 in ((0, h), (h, S)):
            if s1 == s0:
                continue
            r0, r1 = cuts[s0], cuts[s1]
            lc = np.array([cuts[s] - r0 for s in range(s0, s1 + 1)], np.int64)
            Xd, bd = dev(X[r0:r1]), dev(bo[r0:r1])
            A.check(A.lib().hdb_bubble_partials(c.h, Xd.data_ptr(), r1 - r0, d, bd.data_ptr(), nb, lc.ctypes.data,
                                                s1 - s0, pl[s0 * nb * d:].data_ptr(), pq[s0 * nb * d:].data_ptr(),
                                                pn[s0 * nb:].data_ptr()), "partials")
        out = [torch.empty((nb, d), dtype=torch.float64, device="cuda") for _ in range(3)]
        info = torch.empty((nb, 3), dtype=torch.float64, device="cuda")
        A.check(A.lib().hdb_bubble_combine(c.h, pl.data_ptr(), pq.data_ptr(), pn.data_ptr(), S, nb, d,
                                           *(o.data_ptr() for o in out), info.data_ptr()), "combine")
        r = oracle.bubble_stats(X, bo, nb, cuts=cuts)
        got = dict(ls=out[0], ss=out[1], rep=out[2], info=info)
        for k in ("ls", "ss", "rep", "info"):
            assert eq(got[k].cpu().numpy(), r[k]), (cuts, k)
        if S == 1:
            ls, ss, rep, inf = pkg.bubble_stats(X, bo, nb)
            assert eq(rep, r["rep"]) and eq(inf, r["info"]) and eq(ls, r["ls"])
    assert r["info"][11, 2] == 0 and r["info"][2999, 2] == 3


def test_bubble_stats_empty_and_d1(pkg, oracle):
    X = np.random.default_rng(1).normal(size=(1000, 1))
    bo = np.random.default_rng(2).integers(0, 300, 1000).astype(np.int32)
    bo[bo == 7] = 8  # bubble 7 empty
    ls, ss, rep, info = pkg.bubble_stats(X, bo, 300)
    r = oracle.bubble_stats(X, bo, 300)
    assert eq(ls, r["ls"]) and eq(ss, r["ss"]) and eq(rep, r["rep"]) and eq(info, r["info"])


# -------------------------------------------------------------- bubble model
@pytest.mark.parametrize("name", ["iris", "skin_bubbles2k", "blobs2k"])
def test_bubble_core_and_prim_vs_oracle(pkg, oracle, name):
    g = golden(name)
    rep, info = g["b_rep"], g["b_info"]
    nB, eB, nnB = info[:, 2].astype(np.int32), info[:, 0].copy(), info[:, 1].copy()
    model = pkg.HdbscanDataBubbles()
    core = model.calculateCoreDistancesBubbles(rep, nB, eB, nnB, 4)
    assert eq(core, oracle.bubble_core_distances(rep, nB, eB, nnB, 4))
    ids = np.arange(rep.shape[0], dtype=np.int32)
    mst = model.constructMSTBubbles(rep, nB, eB, nnB, ids, core, True)
    va, vb, w = oracle.bubble_prim_mst(rep, eB, nnB, core, ids)
    assert eq(mst.getVerticeA(), va) and eq(mst.getEges(), w)


@pytest.mark.parametrize("name", ["iris", "skin_bubbles2k", "blobs2k"])
def test_local_model_golden(pkg, name):
    g = golden(name)
    op = pkg.LocalModelReduceByKey(4, 4)
    labels, mst, (iva, ivb, iw) = op.call(g["b_rep"], g["b_info"])
    assert eq(labels, g["b_labels"])
    assert eq(mst.getVerticeA(), g["b_mst_va"]) and eq(mst.getEges(), g["b_mst_w"])
    assert eq(iva, g["b_ic_va"]) and eq(ivb, g["b_ic_vb"]) and eq(iw, g["b_ic_w"])


@pytest.mark.parametrize("seed,min_pts,mcl", [(12, 4, 4), (13, 4, 16), (16, 4, 4), (17, 8, 8)])
def test_local_model_larger_vs_oracle(pkg, oracle, seed, min_pts, mcl):
    """~5k-bubble models (stepwise bubble Prim path, b > 4096).  When the reference itself
    throws (duplicate components -> "Cluster cannot have less than 0 points",
    Clusters.java:45-46) the product must raise the same exception."""
    X = blobs(30000, 3, 8, seed)
    rng = np.random.default_rng(seed)
    sids = np.sort(rng.choice(30000, 5000, replace=False))
    near, _ = oracle.nearest_sample(X, X[sids])
    used = np.unique(near)
    remap = -np.ones(5000, np.int32)
    remap[used] = np.arange(used.shape[0], dtype=np.int32)
    st = oracle.bubble_stats(X, remap[near], used.shape[0])
    try:
        lm = oracle.local_model(st["rep"], st["info"], min_pts, mcl)
    except oracle.OracleError as e:
        assert e.code == -12
        with pytest.raises(pkg.IllegalStateException):
            pkg.LocalModelReduceByKey(min_pts, mcl).call(st["rep"], st["info"])
        return
    labels, mst, inter = pkg.LocalModelReduceByKey(min_pts, mcl).call(st["rep"], st["info"])
    assert eq(labels, lm["labels"]) and eq(mst.getEges(), lm["mst"][2]) and eq(inter[2], lm["inter"][2])


# --------------------------------------------------------------------- merge
def test_sort_edges_desc_golden(pkg):
    g = golden("merge")
    va, vb, w = pkg.sort_edges_desc(g["in_va"].copy(), g["in_vb"].copy(), g["in_w"].copy())
    assert eq(va, g["va"]) and eq(vb, g["vb"]) and eq(w, g["w"])


def test_sort_edges_desc_large_stable(pkg, oracle):
    rng = np.random.default_rng(8)
    n = 300000
    w = np.round(rng.uniform(0, 50, n), 2)
    a = rng.integers(0, 1 << 30, n).astype(np.int32)
    b = rng.integers(0, 1 << 30, n).astype(np.int32)
    ga, gb, gw = pkg.sort_edges_desc(a.copy(), b.copy(), w.copy())
    ra, rb, rw = oracle.merge_edges([(a, b, w)])
    assert eq(ga, ra) and eq(gb, rb) and eq(gw, rw)


@pytest.mark.parametrize("p,r,levels", [(200_000, 200_001, 40), (300_000, 0, 7), (100_000, 290_000, 0),
                                         (60_000, 180_000, 3), (5_000, 20_000, 2)])
def test_sort_edges_desc_runs(pkg, oracle, p, r, levels):
    """the run-aware merge (non-decreasing prefix + radix-sorted rest, merged): a prefix with
    heavy tie groups (levels > 0: weights on a grid, incl. -0.0 next to +0.0), a rest that ties
    with it, no rest at all, and a prefix below the run threshold -- equal to the oracle's
    stable sort"""
    rng = np.random.default_rng(p + r)
    if levels:
        pw = np.sort(rng.integers(0, levels + 1, p)).astype(np.float64) * 0.5
    else:
        pw = np.sort(rng.uniform(0, 50, p))
    pw[pw == 0] = np.where(rng.random((pw == 0).sum()) < 0.5, -0.0, 0.0)
    rw = rng.integers(0, max(levels, 1) + 1, r) * 0.5 if levels else rng.uniform(0, 50, r)
    w = np.r_[pw, rw]
    a = rng.integers(0, 1 << 30, p + r).astype(np.int32)
    b = rng.integers(0, 1 << 30, p + r).astype(np.int32)
    for dev in (False, True):
        args = (a.copy(), b.copy(), w.copy())
        if dev:
            args = tuple(torch.from_numpy(x).cuda() for x in args)
        ga, gb, gw = pkg.sort_edges_desc(*args)
        if dev:
            ga, gb, gw = (x.cpu().numpy() for x in (ga, gb, gw))
        ra, rb, rw2 = oracle.merge_edges([(a, b, w)])
        assert eq(ga, ra) and eq(gb, rb) and eq(gw, rw2) and np.array_equal(np.signbit(gw), np.signbit(rw2))


@pytest.mark.parametrize("sizes,levels", [([300_000, 250_000, 1, 0, 180_000, 300_000, 7, 64_000], 25),
                                          ([1_000_000, 1_000_000], 0), ([5_000, 3_000, 9_000], 2), ([12_345], 4)])
def test_merge_sorted_runs_equals_stable_sort(pkg, oracle, sizes, levels):
    """hdb_merge_sorted_runs: the ranks' individually sorted lists merged (merge-path tiles,
    run order on ties) equal the stable descending sort of the raw rank-major concatenation --
    heavy ties across runs, empty and one-edge runs, an odd run count, one run; and the
    precondition errors"""
    rng = np.random.default_rng(sum(sizes) + levels)
    raw, srt = [], []
    for k, m in enumerate(sizes):
        w = (rng.integers(0, levels + 1, m) * 0.25) if levels else rng.uniform(0, 50, m)
        a = rng.integers(0, 1 << 30, m).astype(np.int32)
        b = rng.integers(0, 1 << 30, m).astype(np.int32)
        raw.append((a, b, w))
        t = tuple(torch.from_numpy(x.copy()).cuda() for x in (a, b, w))
        srt.append(pkg.sort_edges_desc(*t))
    off = np.r_[0, np.cumsum(sizes)]
    cat = [torch.cat([s_[i] for s_ in srt]) for i in range(3)]
    ga, gb, gw = (x.cpu().numpy() for x in pkg.merge_sorted_runs(*cat, off))
    ra, rb, rw = oracle.merge_edges(raw)
    assert eq(ga, ra) and eq(gb, rb) and eq(gw, rw)
    ha, hb, hw = pkg.merge_sorted_runs(*(x.cpu().numpy() for x in cat), off)  # host arrays, staged
    assert eq(ha, ra) and eq(hb, rb) and eq(hw, rw)
    if sum(sizes) > 10:
        bad = cat[2].clone()
        bad[1] = bad[0] + 1.0  # run 0 no longer descending
        with pytest.raises(pkg.HdbError):
            pkg.merge_sorted_runs(cat[0], cat[1], bad, off)
        bad = cat[2].clone()
        bad[3] = float("nan")
        with pytest.raises(pkg.HdbError):
            pkg.merge_sorted_runs(cat[0], cat[1], bad, off)


def test_sort_edges_desc_exact_mst_list_and_nan(pkg, oracle):
    """the exact leaf's own output (tree edges ascending, then self edges) and a NaN weight
    (the run path is skipped: the radix order of NaN keys is kept)"""
    X = np.random.default_rng(4).normal(size=(50_000, 3))
    star = pkg.HDBSCANStar(pkg.Context.get(0))
    _, g = star.exactMST(torch.from_numpy(X).cuda(), 4, None, 2, selfEdges=True)
    a, b, w = (x.cpu().numpy() for x in (g.getVerticeA(), g.getVericeB(), g.getEges()))
    ga, gb, gw = pkg.sort_edges_desc(a.copy(), b.copy(), w.copy())
    ra, rb, rw = oracle.merge_edges([(a, b, w)])
    assert eq(ga, ra) and eq(gb, rb) and eq(gw, rw)
    w2 = w.copy()
    w2[len(w2) // 2] = np.nan
    ga, gb, gw = pkg.sort_edges_desc(a.copy(), b.copy(), w2.copy())
    ha, hb, hw = pkg.sort_edges_desc(a.copy(), b.copy(), w2.copy())  # deterministic
    assert eq(ga, ha) and eq(gb, hb) and np.isnan(gw).sum() == 1


# -------------------------------------------------------------------- errors
def test_errors_map_to_reference_exceptions(pkg, star):
    with pytest.raises(pkg.HdbError):
        star.calculateCoreDistances(np.zeros((10, 3)), 0)  # minPts < 1
    with pytest.raises(pkg.HdbError):
        star.calculateCoreDistances(np.zeros((10, 3)), 40)  # > 32 unsupported


# ------------------------------------------------- K1 FP32 screen (exactness)
@pytest.mark.parametrize("scale", [1e-8, 1.0, 1e6, 1e17])
def test_knn_fp32_screen_equals_fp64_path(pkg, oracle, scale):
    """The FP32 screen only skips provably rejected pairs: both K1 paths equal the oracle
    (including huge magnitudes, where the screen disables itself, and near-duplicates)."""
    rng = np.random.default_rng(int(np.log10(scale) + 20))
    X = blobs(4000, 3, 5, 3) * scale + 12345.0 * scale
    X[100:140] = X[99]  # exact duplicates
    X[200:240] = X[199] + rng.normal(size=(40, 3)) * scale * 1e-9  # near-duplicates
    ctx = pkg.Context.get(0)
    star = pkg.HDBSCANStar(ctx)
    for sem in range(3):
        ref = oracle.core_distances(X, 4, semantics=sem)
        ctx.set_option("knn_fp32_screen", 1)
        a = star.calculateCoreDistances(X, 4, None, sem)
        ctx.set_option("knn_fp32_screen", 0)
        b = star.calculateCoreDistances(X, 4, None, sem)
        ctx.set_option("knn_fp32_screen", 1)
        assert eq(a, ref) and eq(b, ref), sem


@pytest.mark.parametrize("case", range(24))
def test_local_model_stress_vs_oracle(pkg, oracle, case):
    """Random bubble sets over tie-heavy inputs (integer grids, Skin duplicates, blobs):
    the dendrogram-replay cluster tree must reproduce the reference's BFS walk exactly --
    labels, sorted MST, inter-cluster edges, or the same exception."""
    rng = np.random.default_rng(1000 + case)
    kind = case % 3
    n = int(rng.integers(300, 6000))
    if kind == 0:
        X = rng.integers(0, 6, size=(n, 2)).astype(np.float64)  # heavy exact ties
    elif kind == 1:
        X = load_skin(n)
    else:
        X = blobs(n, 3, int(rng.integers(2, 9)), case)
    m = int(rng.integers(20, max(21, n // 3)))
    sids = np.sort(rng.choice(n, m, replace=False))
    near, _ = oracle.nearest_sample(X, X[sids])
    used = np.unique(near)
    remap = -np.ones(m, np.int32)
    remap[used] = np.arange(used.shape[0], dtype=np.int32)
    st = oracle.bubble_stats(X, remap[near], used.shape[0])
    min_pts = int(rng.choice([2, 4, 8]))
    mcl = int(rng.choice([2, 4, 16, 64]))
    try:
        lm = oracle.local_model(st["rep"], st["info"], min_pts, mcl)
    except oracle.OracleError as e:
        with pytest.raises(pkg.HdbError) as ei:
            pkg.LocalModelReduceByKey(min_pts, mcl).call(st["rep"], st["info"])
        assert ei.value.code == e.code
        return
    labels, mst, inter = pkg.LocalModelReduceByKey(min_pts, mcl).call(st["rep"], st["info"])
    assert eq(labels, lm["labels"]) and eq(mst.getEges(), lm["mst"][2]) and eq(inter[2], lm["inter"][2])
    assert eq(inter[0], lm["inter"][0]) and eq(inter[1], lm["inter"][1])


@pytest.mark.parametrize("n,kind", [(4097, "blobs"), (12000, "blobs"), (30000, "blobs"), (20000, "skin")])
def test_prim_cooperative_vs_oracle(pkg, oracle, n, kind):
    """4096 < n <= 65536: the single-launch cooperative Prim (grid barrier per step) must be
    the reference Prim exactly, ties included (Skin: pervasive zero-weight ties); the
    stepwise multi-launch path must agree with it."""
    X = load_skin(n) if kind == "skin" else blobs(n, 3, 7, n)
    core = oracle.core_distances(X, 4, semantics=0)
    va, vb, w = oracle.prim_mst(X, core)
    ctx = pkg.Context.get(0)
    star = pkg.HDBSCANStar(ctx)
    for coop, slots in ((1, 6), (1, 5), (1, 4), (1, 3), (1, 2), (1, 1), (1, 0), (0, 0)):
        if not _slots_built(pkg, slots):
            continue
        ctx.set_option("prim_coop", coop)
        ctx.set_option("prim_coop_slots", slots)
        try:
            g = star.constructMST(X, core, True)
        finally:
            ctx.set_option("prim_coop", 1)
            ctx.set_option("prim_coop_slots", 4)
        assert eq(g.getVerticeA(), va) and eq(g.getVericeB(), vb) and eq(g.getEges(), w), (coop, slots)


def test_prim_coop_plain_timeout_retries_cooperatively(pkg, oracle):
    """A plain-launched cooperative Prim whose inter-workgroup waits time out (forced here with a
    2-poll limit) must report it -- key sweep and winner-row wait alike -- and the cooperative
    relaunch must give the reference Prim exactly (prim.hip row-wait timeout)."""
    X = blobs(12000, 3, 7, 77)
    core = oracle.core_distances(X, 4, semantics=0)
    va, vb, w = oracle.prim_mst(X, core)
    ctx = pkg.Context.get(0)
    star = pkg.HDBSCANStar(ctx)
    before = ctx.get_stat("prim_coop_plain_retries")
    for slots in (4, 5, 6):
        if not _slots_built(pkg, slots):
            continue
        ctx.set_option("prim_coop_slots", slots)
        ctx.set_option("prim_coop_plain_spin_log2", 0)
        try:
            g = star.constructMST(X, core, True)
        finally:
            ctx.set_option("prim_coop_plain_spin_log2", 20)
            ctx.set_option("prim_coop_slots", 4)
        assert eq(g.getVerticeA(), va) and eq(g.getVericeB(), vb) and eq(g.getEges(), w), slots
    assert ctx.get_stat("prim_coop_plain_retries") >= before + 1


@pytest.mark.parametrize("slots", [4, 6])
@pytest.mark.parametrize("d,metric,n", [(8, "euclidean", 9000), (16, "euclidean", 5000), (5, "cosine", 6000),
                                        (2, "manhattan", 4500), (8, "euclidean", 16384), (3, "euclidean", 65536)])
def test_prim_coop_slots_metrics_and_bubbles(pkg, oracle, d, metric, n, slots):
    """The step-tagged cooperative Prim (rows in registers, d <= 16; slots 4) and the
    speculative one (slots 6: many steps per exchange, undone past the first wrong pick) equal
    the reference Prim for every metric, and the bubble Prim (HdbscanDataBubbles.java:165-254,
    the C3/C5 bubble models they were written for) on > 4096 bubbles, up to 64 workgroups."""
    _need_slots(pkg, slots)
    pkg.Context.get(0).set_option("prim_coop_slots", slots)
    try:
        _coop_slots_case(pkg, oracle, d, metric, n)
    finally:
        pkg.Context.get(0).set_option("prim_coop_slots", 4)


def _slots_built(pkg, slots):
    """slots 6 (the speculative Prim) exists only in a -DHDB_PRIM_SPEC=1 build"""
    c = pkg.Context.get(0)
    try:
        c.set_option("prim_coop_slots", slots)
    except pkg.HdbError:
        return False
    finally:
        c.set_option("prim_coop_slots", 4)
    return True


def _need_slots(pkg, slots):
    if not _slots_built(pkg, slots):
        pytest.skip("speculative Prim not built (HDBMI_EXTRA_FLAGS=-DHDB_PRIM_SPEC=1)")


def _coop_slots_case(pkg, oracle, d, metric, n):
    X = blobs(n, d, 9, n + d, spread=20.0)
    core = oracle.core_distances(X, 4, metric=metric, semantics=0)
    ids = (np.arange(n, dtype=np.int32) * 3 + 1)
    va, vb, w = oracle.prim_mst(X, core, ids, metric=metric)
    star = pkg.HDBSCANStar(pkg.Context.get(0))
    dist = {"euclidean": pkg.EuclideanDistance(), "cosine": pkg.CosineSimilarity(),
            "manhattan": pkg.ManhattanDistance()}[metric]
    g = star.constructMST(X, core, True, dist, ids)
    assert eq(g.getVerticeA(), va) and eq(g.getVericeB(), vb) and eq(g.getEges(), w)
    if metric != "euclidean":
        return
    rng = np.random.default_rng(n)
    eB = np.abs(rng.normal(0.3, 0.1, n))
    nnB = np.abs(rng.normal(0.2, 0.05, n))
    nB = rng.integers(1, 9, n).astype(np.int32)
    bcore = oracle.bubble_core_distances(X, nB, eB, nnB, 4)
    ra, rb, rw = oracle.bubble_prim_mst(X, eB, nnB, bcore, ids)
    model = pkg.HdbscanDataBubbles()
    mst = model.constructMSTBubbles(X, nB, eB, nnB, ids, bcore, True)
    assert eq(mst.getVerticeA(), ra) and eq(mst.getVericeB(), rb) and eq(mst.getEges(), rw)


@pytest.mark.parametrize("case", ["ties", "descending"])
def test_bubble_core_split_scan_vs_oracle(pkg, oracle, case):
    """K5 in candidate chunks with the exact event replay (bubbles.hip): the bubble core
    distances -- which read the sequential scan's per-position insertion log through the stale
    indexBubbles epilogue (HdbscanDataBubbles.java:121-143) -- equal the oracle's on 9,000
    bubbles with massive distance ties (rounded coordinates, repeated extents), and on a 1-D
    descending layout where every candidate is a new nearest for the far points (the chunks'
    event buffers overflow and the sequential scan takes over)."""
    rng = np.random.default_rng(31)
    n = 9000
    if case == "ties":
        X = np.round(blobs(n, 4, 12, 77, spread=10.0), 0)
        eB = np.round(np.abs(rng.normal(0.3, 0.1, n)), 1)
        nnB = np.round(np.abs(rng.normal(0.2, 0.05, n)), 1)
    else:
        X = -np.arange(n, dtype=np.float64)[:, None] * np.ones((1, 2))
        eB = np.full(n, 0.1)
        nnB = np.full(n, 0.05)
    nB = rng.integers(1, 9, n).astype(np.int32)
    model = pkg.HdbscanDataBubbles()
    for k in (4, 8):
        core = model.calculateCoreDistancesBubbles(X, nB, eB, nnB, k)
        assert eq(core, oracle.bubble_core_distances(X, nB, eB, nnB, k)), (case, k)


# ------------------------------------------- K3g (grouped samples, box pruning) vs the scan
@pytest.mark.parametrize("d", [2, 3, 4, 8, 16])
def test_nearest_grouped_vs_oracle(pkg, oracle, d):
    """The recursive-sampling shape (n >= 8192 points, m >= 1024 samples) takes K3g: median-split
    sample groups scanned in home order with FP64 box pruning.  Rounded coordinates make exact
    distance ties between samples common; the first minimum in sample order must survive."""
    X = np.round(blobs(20000, d, 7, 40 + d), 1)
    S = X[::13].copy()
    assert S.shape[0] >= 1024
    idx, dist = pkg.nearest_sample(X, S, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S)
    assert eq(idx, r_idx) and eq(dist, r_dist)


def test_nearest_grouped_sqrt_ties(pkg, oracle):
    """Equal sqrt values from different squares, the larger square first in sample order, inside
    a 2k-sample set: the grouped scan must keep the first (index 0), like Java."""
    rng = np.random.default_rng(11)
    c = rng.normal(size=(400000, 2))
    c /= np.sqrt((c * c).sum(1))[:, None]
    s = c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]
    r = np.sqrt(s)
    order = np.lexsort((s, r))
    found = next((b, a) for a, b in zip(order[:-1], order[1:]) if r[a] == r[b] and s[a] < s[b])
    far = 5.0 + rng.random((2046, 2))
    S = np.concatenate([c[list(found)], far])
    X = np.concatenate([np.zeros((5000, 2)), 5.0 + rng.random((5000, 2))])
    idx, dist = pkg.nearest_sample(X, S, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S)
    assert eq(idx, r_idx) and np.all(idx[:5000] == 0) and eq(dist, r_dist)


def test_nearest_grouped_equals_scan_large(pkg):
    """C5's level shape at 1/8 size: 2M x 8 points against 16,384 samples, K3g vs the plain scan."""
    import torch
    X = torch.from_numpy(blobs(2_000_000, 8, 100, 5)).cuda()
    S = X[:: 2_000_000 // 16384][:16384].contiguous()
    ctx = pkg.Context.get(0)
    ctx.use_torch_stream()
    try:
        ctx.set_option("nearest_grouped", 1)
        a_i, a_d = pkg.nearest_sample(X, S, ctx=ctx, with_dist=True)
        ctx.set_option("nearest_grouped", 0)
        b_i, b_d = pkg.nearest_sample(X, S, ctx=ctx, with_dist=True)
    finally:
        ctx.set_option("nearest_grouped", 1)
    assert torch.equal(a_i, b_i) and torch.equal(a_d.view(torch.int64), b_d.view(torch.int64))


def test_nearest_grouped_keyed(pkg, oracle):
    """Keyed K3g (D3: the driver's one call over all big subsets): each key's samples get their
    own split tree; a key without samples gives index 0 / MAX, as the Java init."""
    rng = np.random.default_rng(9)
    X = np.round(blobs(30000, 3, 9, 12), 1)
    xk = rng.integers(0, 5, 30000).astype(np.int32)
    S = X[::11].copy()
    sk = xk[::11].copy()
    sk[sk == 4] = 3  # key 4 has no samples
    idx, dist = pkg.nearest_sample(X, S, None, xk, sk, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S, x_key=xk, s_key=sk)
    assert eq(idx, r_idx) and eq(dist, r_dist)


@pytest.mark.parametrize("d", [3, 8])
def test_nearest_grouped_keyed_vs_oracle(pkg, oracle, d):
    """Keyed K3g (the per-subset levels of C3/C5): uneven key sizes, so the runs of consecutive
    sample groups tested behind one union box (HDB_NNG_SB) straddle key boundaries, and a key
    without samples (index 0 / MAX, the Java init)."""
    rng = np.random.default_rng(50 + d)
    n = 24000
    X = np.round(blobs(n, d, 9, 60 + d), 1)
    xk = rng.choice(9, n, p=[0.3, 0.2, 0.15, 0.1, 0.08, 0.07, 0.05, 0.04, 0.01]).astype(np.int32)
    S = X[::11].copy()
    sk = xk[::11].copy()
    sk[sk == 8] = 7  # key 8 has no samples
    assert S.shape[0] >= 1024
    idx, dist = pkg.nearest_sample(X, S, None, xk, sk, with_dist=True)
    r_idx, r_dist = oracle.nearest_sample(X, S, x_key=xk, s_key=sk)
    assert eq(idx, r_idx) and eq(dist, r_dist)
