import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
PKG_NAME = "232-hierarchical-density-based-clustering-using-mapreduce_amd"
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module(PKG_NAME)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


def load_iris():
    return np.loadtxt(os.path.join(GOLDEN, "iris_dataset.txt"))


def load_skin(n=None):
    import lzma
    with lzma.open(os.path.join(GOLDEN, "Skin_NonSkin.txt.xz"), "rt") as fh:
        rows = []
        for i, line in enumerate(fh):
            if n is not None and i >= n:
                break
            rows.append(line.split()[:3])  # D1: whitespace split, label column dropped
    return np.asarray(rows, dtype=np.float64)


def blobs(n, d, centers, seed, spread=100.0, sigma=1.0):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-spread, spread, size=(centers, d))
    lab = rng.integers(0, centers, size=n)
    return C[lab] + rng.normal(0, sigma, size=(n, d))


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def driver_levels(got):
    """A driver run's levels packed like tests/golden/make_c1.py / make_c5s.py store them."""
    lv, labels, new_keys, errs = [], {}, {}, []
    for L in got["levels"]:
        for k, c in sorted(L["leaves"].items()):
            lv.append((L["iteration"], k, 0, c))
        for k, c in sorted(L["big"].items()):
            lv.append((L["iteration"], k, 1, c))
        for k in L["labels"]:
            labels[(L["iteration"], k)] = np.asarray(L["labels"][k], np.int32)
        for k in L["new_keys"]:
            new_keys[(L["iteration"], k)] = list(L["new_keys"][k])
        for k, code in sorted(L.get("model_errors", {}).items()):
            errs.append((L["iteration"], k, code))
    return np.asarray(lv, np.int64).reshape(-1, 4), labels, new_keys, np.asarray(errs, np.int64).reshape(-1, 3)


def check_driver_structure(G, got):
    """levels, bubble labels of every local model, induced keys, model exceptions and the
    leaf of every point equal the oracle fixture G"""
    lv, labels, new_keys, errs = driver_levels(got)
    assert got["iterations"] == int(G["iterations"])
    assert np.array_equal(errs, G["model_errors"])
    assert np.array_equal(lv, G["levels"])
    assert len(labels) == G["label_keys"].shape[0]
    for i, (it, k) in enumerate(G["label_keys"].tolist()):
        ref = G["label_vals"][G["label_off"][i]:G["label_off"][i + 1]]
        assert np.array_equal(labels[(it, k)], ref), (it, k)
    for i, (it, k) in enumerate(G["newkey_keys"].tolist()):
        assert new_keys[(it, k)] == G["newkey_vals"][G["newkey_off"][i]:G["newkey_off"][i + 1]].tolist()
    assert np.array_equal(np.asarray(got["leaf_of"].cpu().numpy(), np.int64), np.asarray(G["leaf_of"], np.int64))
