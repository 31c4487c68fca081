"""Sample sort (csrc/ssort.hpp) parity: every order it produces must equal the rocPRIM radix
path it replaces (ctx option ssort=0) and the oracle, bit for bit.

* hdb_sort_edges_desc (the reducers' stable descending merge, SortMST.java:9-17 over
  UnionFindReducer.java:19-69) against oracle.merge_edges: sizes on both sides of every
  plan boundary (one workgroup, 2..4096 buckets), heavy and total ties, -0.0 next to +0.0,
  presorted and reversed inputs, +-inf and huge magnitudes, and the forced chunked-merge path (ssort_cap);
* hdb_exact_mst (the Morton order of the index, the tree/self edge orders of both output
  modes) and K6 flat labels (the stability terms' order) with ssort on and off: identical.
"""
import contextlib

import numpy as np
import pytest
import torch

from conftest import blobs, load_skin

pytestmark = pytest.mark.gpu


def eq(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(0)
    c.use_torch_stream()
    return c


@pytest.fixture(scope="module")
def star(pkg, ctx):
    return pkg.HDBSCANStar(ctx)


@contextlib.contextmanager
def opts(ctx, ssort=1, cap=0):
    ctx.set_option("ssort", ssort)
    ctx.set_option("ssort_cap", cap)
    try:
        yield
    finally:
        ctx.set_option("ssort", 1)
        ctx.set_option("ssort_cap", 0)


def edges(n, kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "uniform":
        w = rng.uniform(0, 50, n)
    elif kind == "ties":  # a few levels, -0.0 beside +0.0
        w = rng.integers(0, 7, n) * 0.5
        z = w == 0
        w[z] = np.where(rng.random(z.sum()) < 0.5, -0.0, 0.0)
    elif kind == "equal":
        w = np.full(n, 3.25)
    elif kind == "asc":
        w = np.sort(rng.uniform(0, 50, n))
    elif kind == "desc":
        w = np.sort(rng.uniform(0, 50, n))[::-1].copy()
    elif kind == "special":  # inf, huge/tiny magnitudes, negative values (NaN has no order: the
        w = rng.uniform(-5, 5, n) * 10.0 ** rng.integers(-300, 300, n)  # oracle's merge is undefined)
        w[rng.integers(0, n, max(1, n // 100))] = np.inf
        w[rng.integers(0, n, max(1, n // 100))] = -np.inf
    else:
        raise ValueError(kind)
    a = rng.integers(0, 1 << 30, n).astype(np.int32)
    b = rng.integers(0, 1 << 30, n).astype(np.int32)
    return a, b, w


def dev_sort(pkg, ctx, a, b, w):
    t = [torch.from_numpy(x.copy()).cuda() for x in (a, b, w)]
    ga, gb, gw = pkg.sort_edges_desc(*t, ctx)
    return ga.cpu().numpy(), gb.cpu().numpy(), gw.cpu().numpy()


@pytest.mark.parametrize("n", [2, 3, 1000, 4096, 4097, 5000, 70_000, 1_048_577, 2_500_000])
@pytest.mark.parametrize("kind", ["uniform", "ties"])
def test_sort_desc_vs_oracle_and_radix(pkg, oracle, ctx, n, kind):
    a, b, w = edges(n, kind, n)
    ra, rb, rw = oracle.merge_edges([(a, b, w)])
    with opts(ctx, ssort=1):
        s = dev_sort(pkg, ctx, a, b, w)
    assert eq(s[0], ra) and eq(s[1], rb) and eq(s[2], rw)
    if n >= 1_000_000:
        with opts(ctx, ssort=0):
            r = dev_sort(pkg, ctx, a, b, w)
        assert eq(s[0], r[0]) and eq(s[1], r[1]) and eq(s[2], r[2])


@pytest.mark.parametrize("kind", ["equal", "asc", "desc", "special"])
@pytest.mark.parametrize("n", [4000, 300_000])
def test_sort_desc_adversarial(pkg, oracle, ctx, kind, n):
    a, b, w = edges(n, kind, 7 * n)
    ra, rb, rw = oracle.merge_edges([(a, b, w)])
    with opts(ctx, ssort=1):
        s = dev_sort(pkg, ctx, a, b, w)
    assert eq(s[0], ra) and eq(s[1], rb) and eq(s[2], rw)


@pytest.mark.parametrize("cap,n", [(2, 5000), (64, 70_000), (1000, 300_000), (4095, 4096)])
def test_sort_desc_chunked_merge_path(pkg, oracle, ctx, cap, n):
    """buckets above the LDS capacity: chunks sorted in LDS, merged pairwise in global memory"""
    a, b, w = edges(n, "ties", cap + n)
    ra, rb, rw = oracle.merge_edges([(a, b, w)])
    with opts(ctx, ssort=1, cap=cap):
        s = dev_sort(pkg, ctx, a, b, w)
    assert eq(s[0], ra) and eq(s[1], rb) and eq(s[2], rw)


def _mst(star, X, merged, self_edges=True):
    Xd = torch.from_numpy(X).cuda()
    core, g = star.exactMST(Xd, 4, None, 2, self_edges, merged=merged)
    return [x.cpu().numpy() for x in (core, g.getVerticeA(), g.getVericeB(), g.getEges())]


@pytest.mark.parametrize("merged", [True, False])
@pytest.mark.parametrize("src", ["blobs20k", "blobs1m", "skin", "d8"])
def test_exact_mst_ssort_equals_radix(ctx, star, merged, src):
    X = {"blobs20k": lambda: blobs(20_000, 3, 8, 11), "blobs1m": lambda: blobs(1_000_000, 3, 20, 1),
         "skin": load_skin, "d8": lambda: blobs(150_000, 8, 30, 5)}[src]()
    with opts(ctx, ssort=0):
        r = _mst(star, X, merged)
    with opts(ctx, ssort=1):
        s = _mst(star, X, merged)
    assert all(eq(x, y) for x, y in zip(r, s))
    with opts(ctx, ssort=1, cap=256):  # the same orders through the chunked merge path
        c = _mst(star, X, merged)
    assert all(eq(x, y) for x, y in zip(r, c))


def test_exact_mst_merged_no_self_ssort(ctx, star):
    X = blobs(50_000, 2, 6, 3)
    with opts(ctx, ssort=0):
        r = _mst(star, X, True, self_edges=False)
    with opts(ctx, ssort=1):
        s = _mst(star, X, True, self_edges=False)
    assert all(eq(x, y) for x, y in zip(r, s))


@pytest.mark.parametrize("src", ["blobs1m", "skin"])
def test_flat_labels_ssort_equals_radix(pkg, ctx, star, src):
    X = blobs(1_000_000, 3, 20, 1) if src == "blobs1m" else load_skin()
    n = X.shape[0]
    _, va, vb, w = [torch.from_numpy(x).cuda() for x in _mst(star, X, True)]
    out = []
    for ss in (0, 1):
        with opts(ctx, ssort=ss):
            lab, k = pkg.flat_labels(va, vb, w, n, 4, ctx=ctx)
            out.append((lab.cpu().numpy(), k))
    assert eq(out[0][0], out[1][0]) and out[0][1] == out[1][1]
