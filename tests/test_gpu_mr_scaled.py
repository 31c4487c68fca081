"""The partitioned configs through the HIP driver:

* a SCALED config C5 (300k x 8 blobs, 100 centres, samples_per_subset 2,048, processing_units
  8,192; tests/golden/make_c5s.py) against the CPU oracle's MR-HDBSCAN* (oracle/mr_driver.py,
  Main.java:103-347): with reference-Prim leaves the merged edge list is bit-identical
  (SHA-256 of va, vb, w), and the default driver (K2b for forced leaves above 65,536 points)
  gives the same levels, bubble labels, induced keys, leaf of every point and weight
  multiset; the device flat labels (K6) equal the host algorithm's (csrc/flat.cpp) on the
  merged list (the oracle's top-down flat labels are O(levels x n): hours at this size);
* FULL-SIZE C3 (4M x 16) and C5 (16M x 8) exactly as bench.py runs them: property checks
  (2n - 1 edges, descending, the n - 1 tree edges span the points, one self edge per point,
  every point processed by exactly one leaf, labels in 0..K) and the driver default, which
  the bench runs (prim_leaf_max 65,536: forced leaves up to 65,536 points take the reference
  Prim, larger ones K2b), against prim_leaf_max 4,096 (K2b from 4,097 points; same levels,
  labels, weight multiset)."""
import hashlib

import numpy as np
import pytest

from conftest import blobs, check_driver_structure, golden

pytestmark = pytest.mark.gpu


def _scaled(pkg, **kw):
    G = golden("c5s")
    n, d, centers, seed = (int(x) for x in G["shape"])
    mp, mcl, pu, sps, s2 = (int(x) for x in G["args"])
    X = blobs(n, d, centers, seed, spread=100.0)
    got = pkg.MRHDBSCANStar(minPts=mp, minClSize=mcl, processing_units=pu, samples_per_subset=sps, seed=s2,
                            bubble_slices=1, **kw).run(X)  # the fixture was made with one CombineStep fold
    return G, got


def _digest(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def test_c5_scaled_reference_prim_leaves_bit_exact(pkg):
    G, got = _scaled(pkg, exact_prim_leaves=True)
    check_driver_structure(G, got)
    va, vb, w = (x.cpu().numpy() for x in got["edges"])
    assert w.shape[0] == int(G["n_edges"])
    assert np.array_equal(va[:64], G["head_va"]) and np.array_equal(w[:64], G["head_w"])
    assert np.array_equal(va[-64:], G["tail_va"]) and np.array_equal(w[-64:], G["tail_w"])
    assert _digest(va.astype(np.int32), vb.astype(np.int32), w.astype(np.float64)) == str(G["digest"])
    host, k = pkg.flat_labels(va, vb, w, va.shape[0] // 2 + 1, int(G["args"][1]))  # host arrays, no ctx
    assert got["n_clusters"] == k and np.array_equal(got["labels"].cpu().numpy(), host)


def test_c5_scaled_default_driver(pkg):
    G, got = _scaled(pkg)
    check_driver_structure(G, got)
    w = got["edges"][2].cpu().numpy()
    assert _digest(w.astype(np.float64)) == str(G["digest_w"])  # sorted descending: the multiset
    va, vb = (x.cpu().numpy() for x in got["edges"][:2])
    host, k = pkg.flat_labels(va, vb, w, va.shape[0] // 2 + 1, int(G["args"][1]))
    assert got["n_clusters"] == k and np.array_equal(got["labels"].cpu().numpy(), host)


FULL = {  # bench.py PARTITIONED
    "c3": dict(n=4_000_000, d=16, centers=50, spread=50.0, seed=3, samples_per_subset=4096, processing_units=65536),
    "c5": dict(n=16_000_000, d=8, centers=100, spread=100.0, seed=5, samples_per_subset=16384, processing_units=65536),
}


def _full_data(cfg):
    rng = np.random.default_rng(cfg["seed"])  # bench.py run_partitioned's generator
    C = rng.uniform(-cfg["spread"], cfg["spread"], size=(cfg["centers"], cfg["d"]))
    return C[rng.integers(0, cfg["centers"], size=cfg["n"])] + rng.normal(0, 1.0, size=(cfg["n"], cfg["d"]))


def _check_properties(n, got):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    va, vb, w = (x.cpu().numpy() for x in got["edges"])
    assert w.shape[0] == 2 * n - 1 and np.all(w[:-1] >= w[1:]) and np.all(np.isfinite(w)) and np.all(w >= 0)
    self_e = va == vb
    assert int(self_e.sum()) == n and np.array_equal(np.sort(va[self_e]), np.arange(n))  # one self edge per point
    t = ~self_e
    k, _ = connected_components(coo_matrix((np.ones(n - 1, np.int8), (va[t], vb[t])), shape=(n, n)), directed=False)
    assert k == 1, "the n - 1 tree edges do not span the points"
    leaf_of = got["leaf_of"].cpu().numpy()
    assert np.all(leaf_of >= 0)
    assert sum(c for L in got["levels"] for c in L["leaves"].values()) == n  # each point in exactly one leaf
    lab = got["labels"].cpu().numpy()
    assert lab.min() >= 0 and lab.max() == got["n_clusters"] and got["n_clusters"] >= 1
    return w


@pytest.mark.parametrize("name", ["c3", "c5"])
def test_full_size_partitioned_config(pkg, name):
    cfg = FULL[name]
    X = _full_data(cfg)
    kw = dict(minPts=4, minClSize=4, processing_units=cfg["processing_units"],
              samples_per_subset=cfg["samples_per_subset"])
    got = pkg.MRHDBSCANStar(**kw).run(X)
    w = _check_properties(cfg["n"], got)
    lv = [(L["iteration"], sorted(L["leaves"].items()), sorted(L["big"].items()), L["new_keys"]) for L in got["levels"]]
    lab = got["labels"].cpu().numpy()
    del got
    alt = pkg.MRHDBSCANStar(prim_leaf_max=4096, **kw).run(X)  # more leaves on K2b
    assert [(L["iteration"], sorted(L["leaves"].items()), sorted(L["big"].items()), L["new_keys"])
            for L in alt["levels"]] == lv
    assert np.array_equal(alt["edges"][2].cpu().numpy(), w)
    assert np.array_equal(alt["labels"].cpu().numpy(), lab)
