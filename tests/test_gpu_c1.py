"""Config C1 at full size -- the north-star parity target: MR-HDBSCAN* with data bubbles on
ALL 245,057 rows of the reference's Skin_NonSkin.txt with the reference's hard-coded my_args
(Main.java:71: minPts 4, minClSize 4, processing_units 50, k 0.2; D2 sample seed 20210101).

The expected outputs are the CPU oracle's (oracle/mr_driver.py over hdb_oracle.c, the line
restatement of Main.java:103-347 with the deviations D1-D10), committed as
tests/golden/c1_skin_full.npz by tests/golden/make_c1.py.  Level 0 samples 49,012 points;
the bubble model raises the reference's own Clusters.java:45-46 exception on them (D10 records
it, HDB_EREF_NEGATIVE_CLUSTER), so the whole file becomes one forced leaf: the leaf runs the reference Prim on 245,057 points (exact_prim_leaves), and the
edge list must equal the oracle's bit for bit, ties included."""
import time

import numpy as np
import pytest

from conftest import golden, load_skin

pytestmark = pytest.mark.gpu


def _levels(got):
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


def _check_structure(G, got):
    lv, labels, new_keys, errs = _levels(got)
    assert got["iterations"] == int(G["iterations"])
    assert np.array_equal(errs, G["model_errors"])  # D10: the reference's exception, same level
    assert np.array_equal(lv, G["levels"])
    assert len(labels) == G["label_keys"].shape[0]
    for i, (it, k) in enumerate(G["label_keys"].tolist()):
        ref = G["label_vals"][G["label_off"][i]:G["label_off"][i + 1]]
        assert np.array_equal(labels[(it, k)], ref), (it, k)
    for i, (it, k) in enumerate(G["newkey_keys"].tolist()):
        assert new_keys[(it, k)] == G["newkey_vals"][G["newkey_off"][i]:G["newkey_off"][i + 1]].tolist()
    assert np.array_equal(got["leaf_of"].cpu().numpy(), G["leaf_of"])


@pytest.fixture(scope="module")
def skin():
    return load_skin()


def test_c1_full_skin_bit_exact(pkg, skin):
    G = golden("c1_skin_full")
    assert skin.shape == (245057, 3)
    t0 = time.perf_counter()
    got = pkg.MRHDBSCANStar(minPts=4, minClSize=4, processing_units=50, k=0.2, seed=20210101,
                            exact_prim_leaves=True, bubble_slices=1).run(skin)  # the fixture's one fold
    va, vb, w = (x.cpu().numpy() for x in got["edges"])
    print(f"C1 full Skin (exact Prim leaves): {time.perf_counter() - t0:.2f} s")
    _check_structure(G, got)
    assert np.array_equal(w, G["w"]) and np.array_equal(va, G["va"]) and np.array_equal(vb, G["vb"])
    assert got["n_clusters"] == int(G["n_clusters"])
    assert np.array_equal(got["labels"].cpu().numpy(), G["labels"])


def test_c1_full_skin_boruvka_leaf(pkg, skin):
    """Default driver: the 245,057-point forced leaf runs K2b (hdb_exact_mst).  Same levels,
    same sorted weight multiset and the same flat labels as the reference Prim's tree (the
    hierarchy removes a tie group at once, so it does not depend on which MST is used)."""
    G = golden("c1_skin_full")
    t0 = time.perf_counter()
    got = pkg.MRHDBSCANStar(minPts=4, minClSize=4, processing_units=50, k=0.2, seed=20210101,
                            bubble_slices=1).run(skin)
    print(f"C1 full Skin (Boruvka leaf): {time.perf_counter() - t0:.2f} s")
    _check_structure(G, got)
    va, vb, w = (x.cpu().numpy() for x in got["edges"])
    assert np.array_equal(w, G["w"])  # merged list is sorted descending: multiset equality
    assert got["n_clusters"] == int(G["n_clusters"])
    assert np.array_equal(got["labels"].cpu().numpy(), G["labels"])


def test_c1_level0_model_raises_where_the_transcriptions_do(pkg):
    """C1's level-0 model (18,135 Skin bubbles; tests/golden/make_c1_level0.py): the product's
    local model raises the reference's exception at the cluster label, level and point count
    where both independent transcriptions (pure Python, C oracle) throw."""
    z = golden("c1_level0_model")
    with pytest.raises(pkg.IllegalStateException) as ei:
        pkg.LocalModelReduceByKey(int(z["min_pts"]), int(z["mcl"])).call(z["rep"], z["info"])
    import re
    m = re.search(r"\(label (-?\d+), level ([^,]+), numPoints (-?\d+)\)", str(ei.value))
    assert m, str(ei.value)
    assert (int(m.group(1)), float(m.group(2)), int(m.group(3))) == \
        (int(z["label"]), float(z["level"]), int(z["num_points"]))
