"""Record formats through the C-ABI (host code, runs without a GPU):
MapperDataset_github.java:12-20 (dataset lines), CreateLocalMST.java:110-123 (local-MST
text with Double.toString weights), UnionFindReducer.java:22-45 (its parse).  Checked against
oracle/formats.py and the javadoc-stated Double.toString values."""
import lzma
import os
import struct

import numpy as np
import pytest

from conftest import GOLDEN, load_iris, load_skin
from oracle import formats as OF

# java.lang.Double javadoc / JLS values
JAVA_KAT = [
    (0.0, "0.0"), (-0.0, "-0.0"), (1.0, "1.0"), (-1.0, "-1.0"), (100.0, "100.0"), (0.1, "0.1"),
    (1e7, "1.0E7"), (9999999.0, "9999999.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1.5e-5, "1.5E-5"),
    (1e23, "1.0E23"), (1.0e21, "1.0E21"), (5e-324, "4.9E-324"), (1.7976931348623157e308, "1.7976931348623157E308"),
    (2.2250738585072014e-308, "2.2250738585072014E-308"), (123456.789, "123456.789"),
    (12345678.0, "1.2345678E7"), (float("nan"), "NaN"), (float("inf"), "Infinity"), (float("-inf"), "-Infinity"),
    (2.0 / 3.0, "0.6666666666666666"), (43.56520099453603, "43.56520099453603"),
    (0.09999999999999998, "0.09999999999999998"), (1.0e-3 * 0.5, "5.0E-4"), (3.0e10, "3.0E10"),
]


def test_double_to_string_java_kat(pkg):
    for v, s in JAVA_KAT:
        assert pkg.double_to_string(v) == s, (v, s)
        assert OF.double_to_string(v) == s, (v, s)


def test_double_to_string_random_equals_oracle_and_round_trips(pkg):
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 2**63 - 1, size=4000, dtype=np.int64)
    vals = [struct.unpack("<d", struct.pack("<q", int(b)))[0] for b in bits]
    vals += list(rng.normal(size=3000) * 10.0 ** rng.integers(-8, 12, size=3000))
    vals += [float(v) for v in np.round(rng.normal(size=1000) * 100, 2)]
    for v in vals:
        if not np.isfinite(v):
            continue
        s = pkg.double_to_string(v)
        assert s == OF.double_to_string(v), v
        assert OF.parse_double(s) == v  # Double.parseDouble(Double.toString(v)) == v


def test_parse_double_java_grammar(pkg):
    good = ["1", "-1.5", "+.5", "5.", "1e3", "1E-3", "1.5d", "2F", "0x1.8p1", "NaN", "-Infinity", "1e+2D"]
    for s in good:
        X = pkg.read_dataset(s + "\n", strict=True)
        ref = OF.parse_double(s)
        assert X.shape == (1, 1)
        assert (np.isnan(ref) and np.isnan(X[0, 0])) or X[0, 0] == ref, s
    for s in ["", "abc", "1e", "0x1.8", "inf", "nan", "1.2.3", "--1", "1e5x", "0x"]:
        with pytest.raises(OF.NumberFormatException):
            OF.parse_double(s)
        with pytest.raises(pkg.NumberFormatException):
            pkg.read_dataset(("1 " + s) if s else "1  2", strict=True)


def test_parse_double_ignores_type_suffix(pkg):
    """Double.parseDouble's javadoc: trailing type specifiers (1.0f, 1.0d) do not influence the
    result -- "0.1f" is the double 0.1, not the float 0.1f widened."""
    for s, v in [("0.1f", 0.1), ("0.1F", 0.1), ("0x1.999999999999ap-4F", 0.1), ("0.1d", 0.1),
                 ("1.1f", 1.1), ("3.3e-3F", 3.3e-3)]:
        assert OF.parse_double(s) == v, s
        assert pkg.read_dataset(s + "\n", strict=True)[0, 0] == v, s


def test_double_to_string_powers_of_two(pkg):
    """At a power of two the rounding interval is asymmetric; the shortest digits can be a
    decimal farther than the nearest one of that length (Python's repr finds them)."""
    import math
    for k in range(-1074, 1024):
        v = math.ldexp(1.0, k)
        s = pkg.double_to_string(v)
        assert s == OF.double_to_string(v), (k, s)
        assert OF.parse_double(s) == v


def test_strict_split_semantics(pkg):
    """s.split(" "): trailing empty fields vanish, a doubled space is an empty field, tabs are
    not separators (-> NumberFormatException on Skin's TAB lines without D1)."""
    X = pkg.read_dataset("1 2 3   \n4 5 6\n", strict=True)
    assert X.tolist() == [[1, 2, 3], [4, 5, 6]] == OF.read_dataset("1 2 3   \n4 5 6\n")
    with pytest.raises(pkg.NumberFormatException):
        pkg.read_dataset("74\t85\t123\t1\n", strict=True)
    with pytest.raises(pkg.NumberFormatException):
        pkg.read_dataset("1 2\n\n3 4\n", strict=True)  # empty line: parseDouble("")
    with pytest.raises(pkg.NumberFormatException):
        pkg.read_dataset(" 1 2\n", strict=True)  # leading "" field
    assert OF.parse_double(" 7\t") == 7.0  # parseDouble itself trims
    with pytest.raises(pkg.ArrayIndexOutOfBoundsException):
        pkg.read_dataset("1 2 3\n4 5\n", strict=True)  # ragged


def test_mapper_dataset_github_ids(pkg):
    m = pkg.MapperDataset_github()
    out = [m.call(s) for s in ("5.1 3.5 1.4 0.2", "4.9 3.0 1.4 0.2")]
    assert [o[0] for o in out] == [0, 0] and [o[1][0] for o in out] == [0, 1]
    assert out[1][1][1].tolist() == [4.9, 3.0, 1.4, 0.2]


def test_read_reference_datasets(pkg):
    """The reference's own data files: 数据集/dataset.txt (copied as iris_dataset.txt, space
    separated, strict split) and Skin_NonSkin.txt (TAB + label column, D1 with d = 3)."""
    X = pkg.read_dataset(os.path.join(GOLDEN, "iris_dataset.txt"), strict=True)
    assert np.array_equal(X, load_iris())
    with lzma.open(os.path.join(GOLDEN, "Skin_NonSkin.txt.xz"), "rb") as fh:
        raw = fh.read()
    S = pkg.read_dataset(raw, d=3, strict=False)
    assert S.shape == (245057, 3)
    assert np.array_equal(S[:5000], load_skin(5000))
    assert np.array_equal(S, np.asarray(OF.read_dataset(raw.decode(), d=3, strict=False)))


def test_local_mst_text_round_trip(pkg, oracle):
    X = load_iris()
    core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    va, vb, w = oracle.prim_mst(X, core, self_edges=True)
    rng = np.random.default_rng(3)
    f1, f2, nd = (rng.integers(-5, 1000, size=va.shape[0]).astype(np.int32) for _ in range(3))
    t = pkg.format_local_mst(va, vb, w, f1, f2, nd)
    assert t == OF.format_local_mst(va, vb, w, f1, f2, nd)
    assert not t.endswith("\n") and t.count("\n") == va.shape[0] - 1
    got = pkg.parse_local_mst(t)
    for a, b in zip(got, (va, vb, w, f1, f2, nd)):
        assert np.array_equal(a, b)
    assert list(zip(*[g.tolist() for g in got])) == OF.parse_local_mst(t)
    assert pkg.format_local_mst(va[:1], vb[:1], w[:1]).endswith(" 0 0 0")


def test_local_mst_parse_errors(pkg):
    with pytest.raises(pkg.ArrayIndexOutOfBoundsException):
        pkg.parse_local_mst("1 2 0.5 0 0")
    with pytest.raises(pkg.NumberFormatException):
        pkg.parse_local_mst("1 2 0.5 0 0 x")
    with pytest.raises(pkg.NumberFormatException):
        pkg.parse_local_mst("1 2 0.5 0 0 2147483648")
    # UnionFindReducer.java:26-31 parses data[0..5] in order: a bad early field throws
    # NumberFormatException before a missing index is reached
    with pytest.raises(pkg.NumberFormatException):
        pkg.parse_local_mst("")  # "".split("\n") == [""] -> Integer.parseInt("") throws
    with pytest.raises(OF.NumberFormatException):
        OF.parse_local_mst("")
    with pytest.raises(pkg.NumberFormatException):
        pkg.parse_local_mst("1 2 x")  # data[2] throws before data[3] is read
    with pytest.raises(OF.NumberFormatException):
        OF.parse_local_mst("1 2 x")
    with pytest.raises(pkg.ArrayIndexOutOfBoundsException):
        pkg.parse_local_mst("1 2 0.5")
    with pytest.raises(IndexError):
        OF.parse_local_mst("1 2 0.5")
    va, vb, w, *_ = pkg.parse_local_mst("1 2 1.0E-5 0 0 0\n3 4 5.0 0 0 1\n\n")
    assert va.tolist() == [1, 3] and w.tolist() == [1e-5, 5.0]


@pytest.mark.gpu
def test_dataset_to_local_mst_text_on_device(pkg, oracle):
    """The reference's own data path end to end: dataset.txt -> MapperDataset_github points
    -> exact leaf MST on the GPU -> CreateLocalMST text -> UnionFindReducer parse: the
    parsed records equal the MST (and the oracle's Prim weights)."""
    X = pkg.read_dataset(os.path.join(GOLDEN, "iris_dataset.txt"), strict=True)
    core, mst = pkg.HDBSCANStar().exactMST(X, 4, None, pkg.CORE_EXCL_SELF, True)
    va, vb, w = (np.asarray(a) for a in (mst.getVerticeA(), mst.getVericeB(), mst.getEges()))
    text = pkg.format_local_mst(va, vb, w)
    assert text == OF.format_local_mst(va, vb, w)
    pa, pb, pw, *_ = pkg.parse_local_mst(text)
    assert np.array_equal(pa, va) and np.array_equal(pb, vb) and np.array_equal(pw, w)
    ref_core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
    _, _, rw = oracle.prim_mst(X, ref_core, self_edges=False)
    assert np.array_equal(np.sort(pw[: X.shape[0] - 1]), np.sort(rw))


@pytest.mark.gpu
def test_create_local_mst_unrelaxed_vertices(pkg, oracle):
    """rows at infinity / NaN: their mutual-reachability distances are inf or NaN, never below
    Double.MAX_VALUE, so Prim never relaxes them and the reference keeps the Java defaults
    (nearestMRDNeighbors = 0, nearestneighborsID = 0, weight MAX_VALUE; CreateLocalMST.java:
    203,242) -- the record fields must say 0 there, not the local index of global id 0"""
    from conftest import load_iris
    X = load_iris()[:40].copy()
    X[7] = np.inf
    X[23, 1] = np.nan
    n = X.shape[0]
    # global id 0 absent, and present at the last local position
    for ids in (np.arange(100, 100 + n, dtype=np.int32), np.r_[np.arange(5, 5 + n - 1), 0].astype(np.int32)):
        star = pkg.HDBSCANStar()
        core = oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF)
        got = star.constructLocalMST(X, ids, core, True, None, 3)
        ref = oracle.create_local_mst(X, core, ids, 3)
        assert np.any(ref[2][: n - 1] == np.finfo(np.float64).max)  # some vertex was never relaxed
        for g, r in zip(got, ref):
            assert np.array_equal(np.asarray(g), r)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["iris", "skin"])
def test_create_local_mst_text_byte_exact(pkg, oracle, which):
    """CreateLocalMST end to end on the device: EXCL_SELF cores (CreateLocalMST.java:138-185),
    reference Prim with global ids, the record fields fake1/fake2/node (hdb_local_mst_ids) and
    the text (hdb_format_mst_records) equal the oracle's restatement byte for byte."""
    from conftest import load_iris, load_skin
    X = load_iris() if which == "iris" else load_skin(2000)
    n = X.shape[0]
    rng = np.random.default_rng(7)
    ids = np.sort(rng.choice(10 * n, size=n, replace=False)).astype(np.int32)  # the subset's global ids
    node = 37
    star = pkg.HDBSCANStar()
    core = star.calculateCoreDistances(X, 4, None, pkg.CORE_EXCL_SELF)
    got = star.constructLocalMST(X, ids, core, True, None, node)
    ref = oracle.create_local_mst(X, oracle.core_distances(X, 4, semantics=oracle.EXCL_SELF), ids, node)
    for g, r in zip(got, ref):
        assert np.array_equal(np.asarray(g), r)
    assert pkg.format_local_mst(*got) == OF.format_local_mst(*ref)
    # the record fields of another edge order (K2b) are the local indices of its vertices
    va, vb = ref[0][::-1].copy(), ref[1][::-1].copy()
    f1, f2, nd = (np.zeros(va.shape[0], np.int32) for _ in range(3))
    ctx = pkg.Context.get(0)
    A = pkg._capi
    A.check(A.lib().hdb_local_mst_ids(ctx.h, A.ptr(ids), n, A.ptr(va), A.ptr(vb), None, va.shape[0], 5, A.ptr(f1),
                                      A.ptr(f2), A.ptr(nd)), "local ids")
    assert np.array_equal(ids[f1], va) and np.array_equal(ids[f2], vb) and np.all(nd == 5)
    bad = va.copy()
    bad[0] = 10 * n + 1
    with pytest.raises(pkg.HdbError):
        A.check(A.lib().hdb_local_mst_ids(ctx.h, A.ptr(ids), n, A.ptr(bad), A.ptr(vb), None, va.shape[0], 5,
                                          A.ptr(f1), A.ptr(f2), A.ptr(nd)), "local ids")
