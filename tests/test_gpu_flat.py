"""K6 (csrc/flat.hip): the device hierarchy + flat labels over a merged MST must equal the host
algorithm (csrc/flat.cpp, ctx = NULL) and the oracle (oracle/flat_labels.py, the top-down
restatement of HDBSCANStar.java:208-625 pinned against scikit-learn in test_flat_labels.py)
exactly: same labels, same cluster count, on heavy ties, zero weights, stars, single-cluster
and noise-only trees, any input order, and the same errors on malformed input."""
import time

import numpy as np
import pytest
import torch

from conftest import blobs, load_iris, load_skin
from test_flat_labels import cases, lib_flat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pkg):
    return pkg.Context.get(0)


def dev_flat(pkg, ctx, va, vb, w, n, mcs, on_device=True):
    va, vb, w = np.asarray(va, np.int32), np.asarray(vb, np.int32), np.asarray(w, np.float64)
    if on_device:
        lab, k = pkg.flat_labels(torch.from_numpy(va).cuda(), torch.from_numpy(vb).cuda(),
                                 torch.from_numpy(w).cuda(), n, mcs, ctx=ctx)
        return lab.cpu().numpy(), k
    return pkg.flat_labels(va, vb, w, n, mcs, ctx=ctx)  # host arrays staged by the C-ABI


def orders(va, vb, w, rng):
    """the same tree in merged order (descending, stable), ascending, and shuffled"""
    va, vb, w = np.asarray(va, np.int32), np.asarray(vb, np.int32), np.asarray(w, np.float64)
    d = np.argsort(-w, kind="stable")
    a = np.argsort(w, kind="stable")
    p = rng.permutation(len(w))
    return [(va[d], vb[d], w[d]), (va[a], vb[a], w[a]), (va[p], vb[p], w[p])]


def test_device_equals_oracle_and_host_with_ties(pkg, oracle, ctx):
    from oracle.flat_labels import flat_labels
    rng = np.random.default_rng(3)
    for name, n, va, vb, w in cases(oracle):
        for mcs in (2, 4, 10, 30):
            ref, kr = flat_labels(n, va, vb, w, mcs)
            for i, (a, b, ww) in enumerate(orders(va, vb, w, rng)):
                got, kg = dev_flat(pkg, ctx, a, b, ww, n, mcs, on_device=i != 1)
                assert kg == kr and np.array_equal(got, ref), (name, mcs, i)


def test_device_self_edges_and_errors(pkg, oracle, ctx):
    X = load_iris()
    core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    va, vb, w = oracle.prim_mst(X, core, self_edges=True)
    va2, vb2, w2 = oracle.prim_mst(X, core, self_edges=False)
    n = X.shape[0]
    a, ka = dev_flat(pkg, ctx, va, vb, w, n, 4)
    b, kb = dev_flat(pkg, ctx, va2, vb2, w2, n, 4)
    h, kh = lib_flat(pkg, va2, vb2, w2, n, 4)
    assert np.array_equal(a, b) and np.array_equal(a, h) and ka == kb == kh
    bad = [
        (va2[:-1], vb2[:-1], w2[:-1], n, 4),                       # not spanning
        (np.r_[va2[:-1], va2[0]], np.r_[vb2[:-1], vb2[0]], np.r_[w2[:-1], 1.0], n, 4),  # cycle
        (va2, vb2, np.where(np.arange(n - 1) == 7, np.nan, w2), n, 4),                   # NaN
        (np.where(np.arange(n - 1) == 3, n + 5, va2), vb2, w2, n, 4),                    # range
        (va2, vb2, w2, n, 1),                                       # minClSize < 2
    ]
    for args in bad:
        with pytest.raises(pkg.HdbError):
            dev_flat(pkg, ctx, *args)
    lab, k = dev_flat(pkg, ctx, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0), 1, 4)
    assert k == 0 and lab.tolist() == [0]
    lab, k = dev_flat(pkg, ctx, [0], [1], [0.5], 2, 2)
    h2, k2 = lib_flat(pkg, [0], [1], [0.5], 2, 2)
    assert k == k2 and np.array_equal(lab, h2)


@pytest.mark.parametrize("n,wmax", [(1000, 0), (5000, 3), (20000, 50), (200_000, None)])
def test_device_random_trees_equal_host(pkg, ctx, n, wmax):
    """random trees (ragged depth, star-like hubs), integer weights (huge tie groups; wmax 0:
    every edge tied) or continuous weights"""
    rng = np.random.default_rng(n)
    hub = rng.random(n - 1) < 0.3
    par = np.where(hub, 0, (rng.random(n - 1) * np.arange(1, n)).astype(np.int64))
    va, vb = par.astype(np.int32), np.arange(1, n, dtype=np.int32)
    w = rng.random(n - 1) if wmax is None else rng.integers(0, wmax + 1, n - 1).astype(np.float64)
    perm = rng.permutation(n).astype(np.int32)
    va, vb = perm[va], perm[vb]
    d = np.argsort(-w, kind="stable")
    for mcs in (2, 5, 50):
        ref, kr = lib_flat(pkg, va[d], vb[d], w[d], n, mcs)
        got, kg = dev_flat(pkg, ctx, va[d], vb[d], w[d], n, mcs)
        assert kg == kr and np.array_equal(got, ref), (n, wmax, mcs)


def test_device_exact_mst_blobs_and_skin_equal_host(pkg, ctx):
    """real MSTs: 1M blobs (C2 shape, the bench's merged list) and full Skin (zero-weight ties)"""
    star = pkg.HDBSCANStar(ctx)
    for X, mcs in ((blobs(1_000_000, 3, 20, 1), 4), (load_skin(), 4)):
        t = torch.from_numpy(X).cuda()
        _, g = star.exactMST(t, 4, None, 2, selfEdges=True)
        va, vb, w = pkg.sort_edges_desc(g.getVerticeA(), g.getVericeB(), g.getEges(), ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got, kg = pkg.flat_labels(va, vb, w, X.shape[0], mcs, ctx=ctx)
        torch.cuda.synchronize()
        t_dev = time.perf_counter() - t0
        ha, hb, hw = va.cpu().numpy(), vb.cpu().numpy(), w.cpu().numpy()
        t0 = time.perf_counter()
        ref, kr = lib_flat(pkg, ha, hb, hw, X.shape[0], mcs)
        t_host = time.perf_counter() - t0
        print(f"flat labels n={X.shape[0]}: device {t_dev * 1e3:.2f} ms, host {t_host * 1e3:.1f} ms, K={kg}")
        assert kg == kr and np.array_equal(got.cpu().numpy(), ref)


@pytest.mark.parametrize("teeth,tie", [(3000, 1), (3000, 3), (700, 7)])
def test_device_comb_cluster_tree_equal_host(pkg, ctx, teeth, tie):
    """a comb: spine edges of increasing weight (`tie` consecutive ones equal: multi-way splits),
    a tooth of 5 points at every spine vertex (tight or loose) -- the condensed tree is a
    caterpillar thousands of clusters high (FOSC heavy paths much longer than a wave's chunk)"""
    rng = np.random.default_rng(teeth + tie)
    va, vb, w = [], [], []
    tooth = 5
    for i in range(teeth):
        base = i * tooth
        loose = float(1 + i // tie) * rng.uniform(0.001, 1.5)  # some teeth dissolve first
        for j in range(1, tooth):
            va.append(base)
            vb.append(base + j)
            w.append(loose * rng.random())
        if i:
            va.append(base - tooth)
            vb.append(base)
            w.append(float(1 + (i - 1) // tie) + (0.5 * rng.random() if tie == 1 else 0.0))
    n = teeth * tooth
    va, vb, w = np.array(va, np.int32), np.array(vb, np.int32), np.array(w)
    perm = rng.permutation(n).astype(np.int32)
    va, vb = perm[va], perm[vb]
    d = np.argsort(-w, kind="stable")
    for mcs in (2, 4, 5, 6):
        ref, kr = lib_flat(pkg, va[d], vb[d], w[d], n, mcs)
        got, kg = dev_flat(pkg, ctx, va[d], vb[d], w[d], n, mcs)
        assert kg == kr and np.array_equal(got, ref), (teeth, tie, mcs)


@pytest.mark.parametrize("shape", ["tied_path", "shedding_path", "comb200k"])
def test_device_long_chains_equal_host(pkg, ctx, shape):
    """chains far longer than the ~3k of the tests above: every pointer-jumping pass (tie tops,
    cluster starts, the FOSC heavy paths and the selection) must converge within its launch
    budget, which is sized from the reach a launch guarantees under stale reads
    and checked on the device (HDB_EDEVICE otherwise).
    tied_path: 1M points on a path, every edge weight equal (one tie node of depth ~1M);
    shedding_path: 1M-point path with increasing weights (one cluster shedding a point per
    level: a cluster-start chain ~1M long); comb200k: 200k teeth of 5 points on a spine of
    increasing weights (a 200k-cluster caterpillar: heavy path and selection chains ~200k)"""
    rng = np.random.default_rng(11)
    if shape == "comb200k":
        teeth, tooth = 200_000, 5
        base = np.arange(teeth, dtype=np.int64) * tooth
        ta = np.repeat(base, tooth - 1)
        tb = (base[:, None] + np.arange(1, tooth)[None, :]).ravel()
        tw = rng.random(ta.shape[0]) * 0.5
        sa, sb = base[:-1], base[1:]
        sw = 1.0 + np.arange(teeth - 1, dtype=np.float64)
        va, vb, w = np.r_[ta, sa], np.r_[tb, sb], np.r_[tw, sw]
        n = teeth * tooth
    else:
        n = 1_000_000
        va, vb = np.arange(n - 1), np.arange(1, n)
        w = np.ones(n - 1) if shape == "tied_path" else np.arange(n - 1, dtype=np.float64)
    perm = rng.permutation(n)
    va, vb = perm[va].astype(np.int32), perm[vb].astype(np.int32)
    d = np.argsort(-w, kind="stable")
    for mcs in (2, 5):
        ref, kr = lib_flat(pkg, va[d], vb[d], w[d], n, mcs)
        got, kg = dev_flat(pkg, ctx, va[d], vb[d], w[d], n, mcs)
        assert kg == kr and np.array_equal(got, ref), (shape, mcs)


@pytest.mark.parametrize("relabel", [0, 1])
@pytest.mark.parametrize("n,wmax", [(5000, 3), (200_000, None)])
def test_device_vertex_relabel_either_way(pkg, ctx, relabel, n, wmax):
    """the divide and conquer's rank-ordered vertex labels (flat_relabel, default on) and the
    point-id labels give the host algorithm's labels"""
    rng = np.random.default_rng(n + 1)
    par = (rng.random(n - 1) * np.arange(1, n)).astype(np.int64)
    va, vb = par.astype(np.int32), np.arange(1, n, dtype=np.int32)
    w = rng.random(n - 1) if wmax is None else rng.integers(0, wmax + 1, n - 1).astype(np.float64)
    perm = rng.permutation(n).astype(np.int32)
    va, vb = perm[va], perm[vb]
    d = np.argsort(-w, kind="stable")
    ctx.set_option("flat_relabel", relabel)
    try:
        for mcs in (2, 5):
            ref, kr = lib_flat(pkg, va[d], vb[d], w[d], n, mcs)
            got, kg = dev_flat(pkg, ctx, va[d], vb[d], w[d], n, mcs)
            assert kg == kr and np.array_equal(got, ref), (n, wmax, mcs, relabel)
    finally:
        ctx.set_option("flat_relabel", 1)
