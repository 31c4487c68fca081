"""Generates the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference (Java/Spark) cannot execute in this container (no JVM, no Spark jars), so
the vectors are produced by oracle/hdb_oracle.c -- the line-faithful restatement -- whose
own pinning is in tests/test_oracle.py (KATs from the Java source, scipy/sklearn
cross-checks).  Inputs are the reference's own data files (数据集/dataset.txt, the
Skin_NonSkin prefix) and seeded synthetic blobs.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as O  # noqa: E402
from conftest import blobs, load_iris, load_skin  # noqa: E402


def sample_ids(n, frac, seed):
    """D2: seeded exact-size sample (ceil(frac*n)), ascending global id order."""
    m = int(math.ceil(frac * n))
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n, size=m, replace=False)).astype(np.int32)


def bubble_slice(X, frac, seed, min_pts, min_cl, variant="combine"):
    """Iteration-0 slice of the driver (Main.java:132-299) with D2-D5:
    sample -> nearest sample (FirstStep) -> non-empty bubbles compacted in sample order ->
    bubble stats (CombineStep) -> local model (LocalModelReduceByKey)."""
    sids = sample_ids(X.shape[0], frac, seed)
    S = X[sids]
    near, _ = O.nearest_sample(X, S)
    used = np.unique(near)
    remap = -np.ones(S.shape[0], np.int32)
    remap[used] = np.arange(used.shape[0], dtype=np.int32)
    bo = remap[near]
    st = O.bubble_stats(X, bo, used.shape[0], variant)
    lm = O.local_model(st["rep"], st["info"], min_pts, min_cl)
    return dict(sids=sids, near=near, bubble_of=bo, used=used.astype(np.int32), ls=st["ls"], ss=st["ss"],
                rep=st["rep"], info=st["info"], labels=lm["labels"], mst_va=lm["mst"][0], mst_vb=lm["mst"][1],
                mst_w=lm["mst"][2], ic_va=lm["inter"][0], ic_vb=lm["inter"][1], ic_w=lm["inter"][2])


def point_case(X, min_pts, ids_offset=0):
    out = dict(X=X)
    n = X.shape[0]
    ids = (np.arange(n) + ids_offset).astype(np.int32)
    out["ids"] = ids
    for sem, tag in [(O.INCL_SELF_CUMULATIVE, "cum"), (O.INCL_SELF, "incl"), (O.EXCL_SELF, "excl")]:
        core = O.core_distances(X, min_pts, semantics=sem)
        out[f"core_{tag}"] = core
        va, vb, w = O.prim_mst(X, core, ids, self_edges=True)
        out[f"prim_{tag}_va"], out[f"prim_{tag}_vb"], out[f"prim_{tag}_w"] = va, vb, w
    out["knn_incl"] = O.knn_lists(X, min_pts, excl_self=False)
    out["knn_excl"] = O.knn_lists(X, min_pts, excl_self=True)
    return out


def save(name, d):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **d)
    print(f"{name}: {os.path.getsize(path)} bytes")


def main():
    O.build()
    # ---------------------------------------------------------------- Iris
    X = load_iris()
    d = point_case(X, 4, ids_offset=1000)
    d.update({"b_" + k: v for k, v in bubble_slice(X, 0.2, 7, 4, 4).items()})
    S = X[sample_ids(X.shape[0], 0.2, 7)]
    d["ns_S"] = S
    d["ns_idx"], d["ns_dist"] = O.nearest_sample(X, S)
    save("iris", d)
    # --------------------------------------------------- Skin prefix (ties)
    Xs = load_skin(3000)
    d = point_case(Xs, 4)
    S = Xs[sample_ids(Xs.shape[0], 0.2, 11)]
    d["ns_S"] = S
    d["ns_idx"], d["ns_dist"] = O.nearest_sample(Xs, S)
    save("skin3k", d)
    # Skin: a spread sample (rows across both classes) for the bubble slice
    import lzma
    Xall = load_skin()
    rng = np.random.default_rng(20210101)
    pick = np.sort(rng.choice(Xall.shape[0], size=2000, replace=False))
    Xb = Xall[pick]
    d = {"X": Xb, "pick": pick.astype(np.int64)}
    d.update({"b_" + k: v for k, v in bubble_slice(Xb, 0.2, 20210101, 4, 4).items()})
    save("skin_bubbles2k", d)
    # --------------------------------------------------------------- blobs
    Xb = blobs(2000, 3, 6, 5)
    d = point_case(Xb, 4)
    d.update({"b_" + k: v for k, v in bubble_slice(Xb, 0.2, 3, 4, 4).items()})
    cf = O.bubble_stats(Xb, d["b_bubble_of"], d["b_used"].shape[0], "cf")
    d["cf_rep"], d["cf_info"], d["cf_ls"], d["cf_ss"] = cf["rep"], cf["info"], cf["ls"], cf["ss"]
    save("blobs2k", d)
    # ---------------------------------------------- other metrics (a2)
    rng = np.random.default_rng(42)
    Xm = rng.normal(size=(300, 5))
    d = {"X": Xm}
    Sm = Xm[sample_ids(300, 0.2, 1)]
    d["S"] = Sm
    for name in ["euclidean", "cosine", "pearson", "manhattan", "supremum"]:
        core = O.core_distances(Xm, 5, name, O.INCL_SELF)
        d[f"{name}_core_incl"] = core
        d[f"{name}_core_excl"] = O.core_distances(Xm, 5, name, O.EXCL_SELF)
        d[f"{name}_core_cum"] = O.core_distances(Xm, 5, name, O.INCL_SELF_CUMULATIVE)
        va, vb, w = O.prim_mst(Xm, core, None, name, True)
        d[f"{name}_va"], d[f"{name}_vb"], d[f"{name}_w"] = va, vb, w
        d[f"{name}_ns_idx"], d[f"{name}_ns_dist"] = O.nearest_sample(Xm, Sm, name)
    save("metrics300", d)
    # ------------------------------------------------------------- merge
    rng = np.random.default_rng(9)
    lists = []
    for r in range(4):
        ne = int(rng.integers(50, 120))
        w = np.round(rng.uniform(0, 5, ne), 1)  # many ties
        lists.append((rng.integers(0, 1000, ne).astype(np.int32), rng.integers(0, 1000, ne).astype(np.int32), w))
    va, vb, w = O.merge_edges(lists)
    d = {"in_va": np.concatenate([l[0] for l in lists]), "in_vb": np.concatenate([l[1] for l in lists]),
         "in_w": np.concatenate([l[2] for l in lists]), "va": va, "vb": vb, "w": w}
    qa, qb, qw = O.quicksort_edges(d["in_va"], d["in_vb"], d["in_w"])
    d["qs_va"], d["qs_vb"], d["qs_w"] = qa, qb, qw
    save("merge", d)


if __name__ == "__main__":
    main()
