"""K1m (csrc/knn_mfma.hip) parity: k-NN lists and core distances of high-dimensional
euclidean data screened on bf16 MFMA must equal the exact FP64 scan (K1) and the oracle
bit for bit -- the screen only skips pairs whose exact value provably exceeds the current
KC-th smallest (HDBSCANStar.java:84-97 strict insertion), so any difference is a bug.
"""
import contextlib

import numpy as np
import pytest

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
    defaults = {"knn_mfma": 1, "knn_mfma_min_n": 2048, "count_evals": 0}
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
    c.use_torch_stream()
    return c


@pytest.fixture(scope="module")
def star(pkg, ctx):
    return pkg.HDBSCANStar(ctx)


def embeddings(n, d, centers, seed, noise=0.1, normalise=True, offset=0.0):
    """C4's generator shape: centers ~ N(0, I), points = center + noise N(0, I), L2-normalised."""
    rng = np.random.default_rng(seed)
    C = rng.normal(size=(centers, d))
    X = C[rng.integers(0, centers, size=n)] + noise * rng.normal(size=(n, d))
    if normalise:
        X /= np.linalg.norm(X, axis=1, keepdims=True)
    return X + offset


def lists(ctx, star, X, k, mfma):
    with options(ctx, knn_mfma=int(mfma), knn_mfma_min_n=0):
        return star.knn(X, k, None, exclSelf=True)


@pytest.mark.parametrize("d", [17, 32, 64, 100, 128, 200, 256])
@pytest.mark.parametrize("k", [1, 3, 15, 31])
def test_mfma_lists_equal_fp64(ctx, star, d, k):
    X = embeddings(3000, d, 20, d * 7 + k)
    assert eq(lists(ctx, star, X, k, True), lists(ctx, star, X, k, False)), (d, k)


@pytest.mark.parametrize("sem", [0, 1, 2])
def test_mfma_cores_vs_oracle(ctx, star, oracle, sem):
    X = embeddings(2500, 128, 30, 11)
    with options(ctx, knn_mfma=1, knn_mfma_min_n=0):
        got = star.calculateCoreDistances(X, 16, None, sem)
    assert eq(got, oracle.core_distances(X, 16, semantics=sem)), sem


def test_mfma_offset_unnormalised_and_duplicates(ctx, star):
    """Far from the origin (the centring keeps the screen tight), unnormalised, with exact
    duplicates and ties (zero distances)."""
    X = embeddings(3000, 64, 10, 5, noise=1.0, normalise=False, offset=1e6)
    X[100:140] = X[99]
    X[2000:2100] = np.round(X[2000:2100], 1)
    for k in (3, 15):
        assert eq(lists(ctx, star, X, k, True), lists(ctx, star, X, k, False)), k


def test_mfma_scales_and_ragged(ctx, star):
    rng = np.random.default_rng(2)
    for scale in (1e-12, 1e-3, 1.0, 1e9):
        for n in (65, 127, 1000):
            X = rng.normal(size=(n, 40)) * scale
            assert eq(lists(ctx, star, X, 7, True), lists(ctx, star, X, 7, False)), (scale, n)


def test_mfma_nonfinite_falls_back(ctx, star):
    X = embeddings(1000, 32, 5, 3)
    X[5, 3] = np.nan
    X[6, 0] = np.inf
    assert eq(lists(ctx, star, X, 3, True), lists(ctx, star, X, 3, False))


def test_mfma_rechecks_few(ctx, star):
    """The screen is tight: at 20k C4-shaped points the exact re-checks are a tiny fraction
    of n^2 (diagnostic counter)."""
    import torch
    X = torch.from_numpy(embeddings(20000, 128, 50, 4)).cuda()
    with options(ctx, knn_mfma=1, knn_mfma_min_n=0, count_evals=1):
        star.knn(X, 15, None, exclSelf=True)
        re = ctx.get_stat("knn_mfma_rechecks")
    assert 0 < re < 0.05 * 20000 ** 2


def test_mfma_lists_equal_fp64_200k_x_128(pkg, ctx, star):
    """C4's shape at 200k rows (BASELINE config 4: 2M x 128 embeddings, minPts 16): the MFMA
    screen + FP64 re-check must return the same 15-NN lists, bit for bit, as the all-pairs FP64
    scan (K1) over all 200k x 200k pairs.  Data generated on the device (seeded)."""
    import torch
    n, d, k = 200_000, 128, 15
    g = torch.Generator(device="cuda").manual_seed(44)
    C = torch.randn(200, d, dtype=torch.float64, device="cuda", generator=g)
    lab = torch.randint(0, 200, (n,), device="cuda", generator=g)
    X = C[lab] + 0.1 * torch.randn(n, d, dtype=torch.float64, device="cuda", generator=g)
    X = (X / torch.linalg.norm(X, dim=1, keepdim=True)).contiguous()
    got = lists(ctx, star, X, k, True)
    ref = lists(ctx, star, X, k, False)
    assert got.shape == (n, k)
    assert torch.equal(got.view(torch.int64), ref.view(torch.int64))


def test_mfma_cores_full_size_c4_rows(pkg, ctx, star):
    """BASELINE config 4 at full size: 2M x 128 L2-normalised embeddings (bench.py's seeded
    generator), minPts 16, EXCL_SELF core distances through the default path (the MFMA screen
    + FP64 re-check).  64 sampled rows must equal, bit for bit, the (minPts-1)-th smallest
    Java-order distance over all 2M rows (CreateLocalMST.java:138-185: sequential sum of
    (a-b)*(a-b) in dimension order, no FMA -- every step here is its own elementwise kernel,
    so each sub, mul and add rounds once) with the query itself excluded."""
    import torch
    n, d, mp, centers = 2_000_000, 128, 16, 200
    g = torch.Generator(device="cuda").manual_seed(4)
    C = torch.randn(centers, d, dtype=torch.float64, device="cuda", generator=g)
    lab = torch.randint(0, centers, (n,), device="cuda", generator=g)
    X = C[lab] + 0.1 * torch.randn(n, d, dtype=torch.float64, device="cuda", generator=g)
    X = (X / torch.linalg.norm(X, dim=1, keepdim=True)).contiguous()
    del C, lab
    got = star.calculateCoreDistances(X, mp, None, pkg.CORE_EXCL_SELF)
    torch.cuda.synchronize()
    assert ctx.get_stat("knn_mfma_blocks") > 0  # the MFMA path ran (not the FP64 fallback)
    rows = torch.from_numpy(np.random.default_rng(44).choice(n, 64, replace=False)).cuda()
    Q = X[rows]                                  # 64 x 128
    s = torch.zeros(64, n, dtype=torch.float64, device="cuda")
    for j in range(d):
        t = Q[:, j:j + 1] - X[:, j].unsqueeze(0)  # 64 x n
        s += t * t
        del t
    s[torch.arange(64, device="cuda"), rows] = float("inf")
    ref = torch.sqrt(torch.kthvalue(s, mp - 1, dim=1).values)
    assert torch.equal(got[rows].view(torch.int64), ref.view(torch.int64)), \
        (got[rows] - ref).abs().max().item()
    assert bool(torch.isfinite(got).all()) and bool((got >= 0).all())
