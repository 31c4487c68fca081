"""CPU-side checks of the drop-in boundary: the HIP library builds/loads and exports every
entry point include/hdbmi.h declares; the host-side (no device) logic behaves like the
reference.  No compute call needs a GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden


def header_symbols():
    src = open(os.path.join(ROOT, "include", "hdbmi.h")).read()
    return sorted(set(re.findall(r"\b(hdb_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_header_symbol(pkg):
    L = pkg.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(syms) == set(pkg._capi.EXPORTED)


def test_no_device_raises_loudly(pkg):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a device is present")
    except ImportError:
        pass
    with pytest.raises(pkg.HdbError):
        pkg.Context(0)


def test_quicksort_is_host_side_and_matches_oracle(pkg, oracle):
    """UndirectedGraph.quicksortByEdgeWeight has no device part (tie order quirk)."""
    g = golden("merge")
    ug = pkg.UndirectedGraph(g["in_va"].copy(), g["in_vb"].copy(), g["in_w"].copy())
    ug.quicksortByEdgeWeight()
    assert np.array_equal(ug.getVerticeA(), g["qs_va"])
    assert np.array_equal(ug.getVericeB(), g["qs_vb"])
    assert np.array_equal(ug.getEges(), g["qs_w"])


def test_quicksort_random_vs_oracle(pkg, oracle):
    rng = np.random.default_rng(3)
    for n in (1, 2, 3, 17, 301):
        w = np.round(rng.uniform(0, 3, n), 1)
        a = rng.integers(0, 50, n).astype(np.int32)
        b = rng.integers(0, 50, n).astype(np.int32)
        ug = pkg.UndirectedGraph(a.copy(), b.copy(), w.copy())
        ug.quicksortByEdgeWeight()
        oa, ob, ow = oracle.quicksort_edges(a, b, w)
        assert np.array_equal(ug.getVerticeA(), oa) and np.array_equal(ug.getEges(), ow)


def test_quicksort_ties_nan_large_vs_oracle(pkg, oracle):
    """The branch-free partition (round 6) keeps the reference's swaps: heavy ties, NaN weights
    (never '<' the pivot), already-sorted and reversed runs, bit-equal to the oracle."""
    rng = np.random.default_rng(11)
    for n, kind in ((4000, "ties"), (3001, "nan"), (2048, "sorted"), (2049, "reversed")):
        w = np.round(rng.uniform(0, 2, n), 1)
        if kind == "nan":
            w[rng.integers(0, n, 40)] = np.nan
        elif kind == "sorted":
            w = np.sort(w)
        elif kind == "reversed":
            w = np.sort(w)[::-1].copy()
        a = rng.integers(0, 500, n).astype(np.int32)
        b = rng.integers(0, 500, n).astype(np.int32)
        ug = pkg.UndirectedGraph(a.copy(), b.copy(), w.copy())
        ug.quicksortByEdgeWeight()
        oa, ob, ow = oracle.quicksort_edges(a, b, w)
        assert np.array_equal(ug.getVerticeA(), oa) and np.array_equal(ug.getVericeB(), ob), kind
        assert np.array_equal(ug.getEges().view(np.uint64), np.asarray(ow).view(np.uint64)), kind


def test_distance_names(pkg):
    assert pkg.EuclideanDistance().getName() == "euclidean"
    assert pkg.CosineSimilarity().getName() == "cosine"
    assert pkg.PearsonCorrelation().getName() == "pearson"
    assert pkg.ManhattanDistance().getName() == "manhattan"
    assert pkg.SupremumDistance().getName() == "supremum"
