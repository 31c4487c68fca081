"""End-to-end MR-HDBSCAN* (Main.java:103-347 with D1-D10) on the device: the product driver
(driver.py, HIP operators) against the CPU oracle's restatement of the same loop
(oracle/mr_driver.py).  Every level's subsets, bubble labels, induced keys, the leaf that
processed each point and the merged edge list must match exactly."""
import numpy as np
import pytest

from conftest import blobs, load_iris, load_skin

pytestmark = pytest.mark.gpu


def run_both(pkg, X, **kw):
    """oracle and device on the same input; both fold CombineStep over the same slices (D11:
    the driver's default, or bubble_slices given)"""
    from oracle import mr_driver as M
    kw.setdefault("bubble_slices", pkg.driver.BUBBLE_SLICES)
    ref = M.run(X, **kw)
    got = pkg.MRHDBSCANStar(minPts=kw.get("min_pts", 4), minClSize=kw.get("min_cl_size", 4),
                            processing_units=kw["processing_units"], k=kw.get("k", 0.2),
                            samples_per_subset=kw.get("samples_per_subset"),
                            all_inter_edges=kw.get("all_inter_edges", True),
                            distanceFunction=kw.get("metric"), bubble_slices=kw["bubble_slices"]).run(X)
    return ref, got


def check(ref, got):
    assert got["iterations"] == ref["iterations"]
    assert len(got["levels"]) == len(ref["levels"])
    for a, b in zip(got["levels"], ref["levels"]):
        assert a["leaves"] == b["leaves"] and a["big"] == b["big"]
        assert a["new_keys"] == b["new_keys"]
        assert a.get("model_errors") == b.get("model_errors")
        for k in b["labels"]:
            assert np.array_equal(a["labels"][k], b["labels"][k]), k
    assert np.array_equal(got["leaf_of"].cpu().numpy(), ref["leaf_of"])
    for x, y in zip(got["edges"], ref["edges"]):
        assert np.array_equal(x.cpu().numpy(), y)
    if "labels" in ref:  # D6 global flat labels
        assert got["n_clusters"] == ref["n_clusters"]
        assert np.array_equal(got["labels"].cpu().numpy(), ref["labels"])


@pytest.mark.parametrize("name,pu,k", [("iris", 50, 0.2), ("blobs3k", 300, 0.1), ("blobs3k", 1000, 0.05),
                                       ("skin3k", 300, 0.1), ("blobs8k_d8", 1500, 0.02)])
def test_driver_matches_oracle(pkg, name, pu, k):
    X = {"iris": lambda: load_iris(), "blobs3k": lambda: blobs(3000, 3, 6, 1),
         "skin3k": lambda: load_skin(3000), "blobs8k_d8": lambda: blobs(8000, 8, 10, 2, spread=30.0)}[name]()
    ref, got = run_both(pkg, X, processing_units=pu, k=k)
    check(ref, got)


def test_driver_literal_first_inter_edge(pkg):
    X = blobs(3000, 3, 6, 1)
    ref, got = run_both(pkg, X, processing_units=300, k=0.1, all_inter_edges=False)
    check(ref, got)


def test_driver_samples_per_subset(pkg):
    X = blobs(6000, 2, 8, 4)
    ref, got = run_both(pkg, X, processing_units=800, samples_per_subset=200)
    check(ref, got)


@pytest.mark.parametrize("n,pu,k", [(6000, 6000, 0.2), (20000, 9000, 0.05)])
def test_driver_cosine_forced_leaf_above_4096(pkg, n, pu, k):
    """a non-Euclidean metric (CosineSimilarity.java:28-40) with d = 5 and leaves of
    4,096-65,536 points: K2b does not apply (driver.py boruvka_ok), so those leaves run the
    reference Prim (cooperative launch) -- the whole run must equal the oracle's loop."""
    X = blobs(n, 5, 7, n, spread=20.0) + 25.0  # off the origin: cosine distances spread out
    ref, got = run_both(pkg, X, processing_units=pu, k=k, metric="cosine")
    check(ref, got)
    assert max(max(L["leaves"].values(), default=0) for L in got["levels"]) > 4096


def test_flat_labels_device_inputs(pkg, oracle):
    """hdb_flat_labels on HBM-resident edges (staged once) equals the oracle."""
    import torch
    from oracle.flat_labels import flat_labels
    X = blobs(20000, 3, 12, 3)
    core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    star = pkg.HDBSCANStar()
    mst = star.constructMSTBoruvka(torch.from_numpy(X).cuda(), torch.from_numpy(core).cuda(), True)
    va, vb, w = mst.getVerticeA(), mst.getVericeB(), mst.getEges()
    lab, k = pkg.flat_labels(va, vb, w, X.shape[0], 10)
    ref, kr = flat_labels(X.shape[0], va.cpu().numpy(), vb.cpu().numpy(), w.cpu().numpy(), 10)
    assert k == kr and np.array_equal(lab.cpu().numpy(), ref)


@pytest.mark.parametrize("name,pu,k", [("blobs8k_d8", 1500, 0.02), ("skin3k", 300, 0.1)])
def test_deferred_leaves_equal_per_level_leaves(pkg, name, pu, k):
    """defer_leaves (the default: every level's leaves in one batch after the level loop, one
    LPT over the job) places the same blocks as the per-level leaf batches (Main.java:133-138
    runs a level's leaves inside the level; nothing later reads their edges)."""
    X = {"skin3k": lambda: load_skin(3000), "blobs8k_d8": lambda: blobs(8000, 8, 10, 2, spread=30.0)}[name]()
    kw = dict(processing_units=pu, k=k)
    a = pkg.MRHDBSCANStar(**kw, defer_leaves=True).run(X)
    b = pkg.MRHDBSCANStar(**kw, defer_leaves=False).run(X)
    assert a["iterations"] == b["iterations"]
    assert np.array_equal(a["leaf_of"].cpu().numpy(), b["leaf_of"].cpu().numpy())
    for x, y in zip(a["edges"], b["edges"]):
        assert np.array_equal(x.cpu().numpy(), y.cpu().numpy())
    assert np.array_equal(a["labels"].cpu().numpy(), b["labels"].cpu().numpy())
