"""The second, independent transcription of the bubble local model (oracle/java_transcription.py:
pure Python from the Java, its own JDK 8 HashMap/TreeSet emulation) against the C oracle
(hdb_oracle.c) -- the pin of the Java-collection quirks C1 hinges on:

  * HashMap<Integer, ...> iteration order: bucket spreading, resize splits, the resize that
    treeifyBin performs below 64 buckets, and a hard failure where a tree bin would form;
  * every local-model golden, the 24 tie-heavy stress cases and a ~5k-bubble model:
    identical labels, quicksorted MST, inter-cluster edges -- or the same exception at the
    same cluster label, level and point count (Clusters.java:45-46);
  * C1's level-0 model (18,135 Skin bubbles): the transcription's recorded exception
    (tests/golden/make_c1_level0.py) is reproduced by the C oracle, and is the D10 event of
    the full-Skin golden."""
import numpy as np
import pytest

from conftest import blobs, golden, load_skin
from oracle import java_transcription as J


# ------------------------------------------------------------------ JDK 8 collections
def test_hashmap_order_spreading_and_resize():
    m = J.JavaHashMap()
    for k in (100, 3):
        m.put(k, None)
    assert m.key_set() == [3, 100]  # buckets 3, 4
    m = J.JavaHashMap()
    for k in (65536, 1, 17):  # spread(65536) = 65537 -> bucket 1 with 1 and 17
        m.put(k, None)
    assert m.key_set() == [65536, 1, 17]
    m = J.JavaHashMap()
    keys = list(range(40, 0, -1))  # 13th put resizes to 32, 25th to 64
    for k in keys:
        m.put(k, None)
    assert len(m.table) == 64 and m.key_set() == sorted(keys)
    m.put(7, "again")  # existing key: no structural change
    assert m.size == 40 and m.get(7) == "again"


def test_hashmap_treeify_resizes_small_tables_and_refuses_tree_bins():
    m = J.JavaHashMap()
    keys = [16 * i for i in range(1, 10)]  # nine keys in bucket 0 of a 16-bucket table
    for k in keys:
        m.put(k, None)
    assert len(m.table) == 32  # treeifyBin resized instead (MIN_TREEIFY_CAPACITY = 64)
    assert m.key_set() == [32, 64, 96, 128, 16, 48, 80, 112, 144]
    m = J.JavaHashMap()
    for k in range(1, 26):
        m.put(k, None)
    assert len(m.table) == 64
    with pytest.raises(J.JavaTreeifyError):
        for i in range(1, 10):
            m.put(64 * i, None)


def test_treeset_poll_first_and_lazy_remove():
    s = J.JavaTreeSet([5, 3, 9, 3])
    s.remove(3)
    s.add(1)
    s.add(3)
    assert list(s) == [1, 3, 5, 9]
    assert [s.poll_first() for _ in range(4)] == [1, 3, 5, 9] and s.is_empty()


def test_quicksort_transcription_vs_oracle(oracle):
    rng = np.random.default_rng(3)
    for n in (2, 3, 17, 500, 3000):
        w = np.round(rng.uniform(0, 4, n), 1)  # ties: the unstable order matters
        a = rng.integers(0, 1000, n)
        b = rng.integers(0, 1000, n)
        g = J.UndirectedGraph(1000, a.tolist(), b.tolist(), w.tolist())
        g.quicksort_by_edge_weight()
        ra, rb, rw = oracle.quicksort_edges(a, b, w)
        assert g.va == ra.tolist() and g.vb == rb.tolist() and g.w == rw.tolist(), n
    # long equal-weight runs (Skin's zero ties): the Lomuto partition's degenerate case
    w = np.zeros(2000)
    w[::7] = 1.0
    a = np.arange(2000)
    g = J.UndirectedGraph(2000, a.tolist(), a[::-1].tolist(), w.tolist())
    g.quicksort_by_edge_weight()
    ra, rb, rw = oracle.quicksort_edges(a, a[::-1], w)
    assert g.va == ra.tolist() and g.vb == rb.tolist() and g.w == rw.tolist()


# ------------------------------------------------------------------ local model
def _same(r, ref):
    return (np.array_equal(r["labels"], ref["labels"]) and all(np.array_equal(a, b) for a, b in zip(r["mst"], ref["mst"]))
            and all(np.array_equal(a, b) for a, b in zip(r["inter"], ref["inter"])))


def _cross_check(oracle, rep, info, min_pts, mcl):
    try:
        ref, oerr = oracle.local_model(rep, info, min_pts, mcl), None
    except oracle.OracleError as e:
        ref, oerr = None, (e.code, oracle.last_negative_cluster() if e.code == -12 else None)
    try:
        r, jerr = J.local_model(rep, info, min_pts, mcl), None
    except J.JavaException as e:
        r, jerr = None, (e.code, e.detail if e.code == -12 else None)
    assert oerr == jerr
    if ref is not None:
        assert _same(r, ref)
        assert np.array_equal(r["core"], oracle.bubble_core_distances(rep, info[:, 2].astype(np.int32), info[:, 0],
                                                                     info[:, 1], min_pts))
    return oerr


@pytest.mark.parametrize("name", ["iris", "skin_bubbles2k", "blobs2k"])
def test_transcription_local_model_golden(oracle, name):
    g = golden(name)
    r = J.local_model(g["b_rep"], g["b_info"], 4, 4)
    assert np.array_equal(r["labels"], g["b_labels"])
    assert np.array_equal(r["mst"][0], g["b_mst_va"]) and np.array_equal(r["mst"][2], g["b_mst_w"])
    assert np.array_equal(r["inter"][0], g["b_ic_va"]) and np.array_equal(r["inter"][2], g["b_ic_w"])
    _cross_check(oracle, g["b_rep"], g["b_info"], 4, 4)


def _stress_inputs(oracle, case):
    """the same generator as tests/test_gpu_parity.py::test_local_model_stress_vs_oracle"""
    rng = np.random.default_rng(1000 + case)
    kind = case % 3
    n = int(rng.integers(300, 6000))
    if kind == 0:
        X = rng.integers(0, 6, size=(n, 2)).astype(np.float64)
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
    return st["rep"], st["info"], int(rng.choice([2, 4, 8])), int(rng.choice([2, 4, 16, 64]))


def test_transcription_stress_cases_vs_oracle(oracle):
    errors = 0
    for case in range(24):
        rep, info, mp, mcl = _stress_inputs(oracle, case)
        errors += _cross_check(oracle, rep, info, mp, mcl) is not None
    assert errors >= 3  # the exception path is exercised, not only the normal one


def test_transcription_5k_model_vs_oracle(oracle):
    X = blobs(30000, 3, 8, 12)
    rng = np.random.default_rng(12)
    sids = np.sort(rng.choice(30000, 5000, replace=False))
    near, _ = oracle.nearest_sample(X, X[sids])
    used = np.unique(near)
    remap = -np.ones(5000, np.int32)
    remap[used] = np.arange(used.shape[0], dtype=np.int32)
    st = oracle.bubble_stats(X, remap[near], used.shape[0])
    err = _cross_check(oracle, st["rep"], st["info"], 4, 4)
    assert err is not None and err[0] == -12 and err[1]["num_points"] < 0


def test_c1_level0_model_exception_pinned(oracle):
    """C1 (Skin, my_args) level 0: the independent transcription threw at (label, level,
    numPoints) when the fixture was made; the C oracle must throw at exactly that point, and
    that is the D10 event the full-Skin golden records (iteration 0, key 0)."""
    z = np.load(__import__("os").path.join(__import__("conftest").GOLDEN, "c1_level0_model.npz"))
    assert int(z["code"]) == -12
    with pytest.raises(oracle.OracleError) as ei:
        oracle.local_model(z["rep"], z["info"], int(z["min_pts"]), int(z["mcl"]))
    assert ei.value.code == -12
    d = oracle.last_negative_cluster()
    assert (d["label"], d["level"], d["num_points"]) == (int(z["label"]), float(z["level"]), int(z["num_points"]))
    c1 = golden("c1_skin_full")
    assert c1["model_errors"].tolist() == [[0, 0, -12]]
    assert c1["label_off"][1] == z["rep"].shape[0]  # the model the driver ran had these bubbles
