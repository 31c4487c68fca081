"""Generates tests/golden/c1_skin_full.npz: the CPU oracle's MR-HDBSCAN* (oracle/mr_driver.py,
the line restatement of Main.java:103-347 with the deviations D1-D10) on ALL 245,057 rows of
the reference's Skin_NonSkin.txt with the reference's hard-coded my_args (Main.java:71:
minPts=4, minClSize=4, processing_units=50, k=0.2) and the D2 sample seed 20210101.
Level 0's bubble model (49,012 bubbles) raises the reference's own exception
(Clusters.java:45-46, HDB_EREF_NEGATIVE_CLUSTER); D10 records it and the subset becomes one
forced leaf, so the whole file runs the exact leaf MST (~20 min of oracle Prim).

Run in the build container (the oracle is test infrastructure; takes minutes):
    python tests/golden/make_c1.py
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import load_skin  # noqa: E402
from oracle import mr_driver as M  # noqa: E402

ARGS = dict(min_pts=4, min_cl_size=4, processing_units=50, k=0.2, seed=20210101)


def main(out=os.path.join(HERE, "c1_skin_full.npz")):
    X = load_skin()
    t0 = time.time()
    r = M.run(X, log=lambda s: print(f"[{time.time() - t0:8.1f}s] {s}", flush=True), **ARGS)
    print(f"oracle run {time.time() - t0:.1f} s, iterations {r['iterations']}", flush=True)
    va, vb, w = r["edges"]
    lv = []  # per level: (iteration, key, kind, count) rows; kind 0 leaf, 1 big
    lab_keys, lab_off, lab_vals, nk_keys, nk_off, nk_vals = [], [0], [], [], [0], []
    errs = []  # D10: (iteration, key, code) of local models that raise the reference's exception
    for L in r["levels"]:
        for k, c in sorted(L["leaves"].items()):
            lv.append((L["iteration"], k, 0, c))
        for k, c in sorted(L["big"].items()):
            lv.append((L["iteration"], k, 1, c))
        for k in sorted(L["labels"]):
            lab_keys.append((L["iteration"], k))
            lab_vals.append(np.asarray(L["labels"][k], np.int32))
            lab_off.append(lab_off[-1] + len(L["labels"][k]))
        for k in sorted(L["new_keys"]):
            nk_keys.append((L["iteration"], k))
            nk_vals.append(np.asarray(L["new_keys"][k], np.int64))
            nk_off.append(nk_off[-1] + len(L["new_keys"][k]))
        for k, code in sorted(L.get("model_errors", {}).items()):
            errs.append((L["iteration"], k, code))
    cat = lambda a, t: np.concatenate(a).astype(t) if a else np.zeros(0, t)
    np.savez_compressed(
        out, va=va, vb=vb, w=w, leaf_of=r["leaf_of"], labels=r["labels"], n_clusters=r["n_clusters"],
        iterations=r["iterations"], levels=np.asarray(lv, np.int64).reshape(-1, 4),
        label_keys=np.asarray(lab_keys, np.int64).reshape(-1, 2), label_off=np.asarray(lab_off, np.int64),
        label_vals=cat(lab_vals, np.int32), newkey_keys=np.asarray(nk_keys, np.int64).reshape(-1, 2),
        newkey_off=np.asarray(nk_off, np.int64), newkey_vals=cat(nk_vals, np.int64),
        model_errors=np.asarray(errs, np.int64).reshape(-1, 3),
        args=np.asarray([ARGS["min_pts"], ARGS["min_cl_size"], ARGS["processing_units"], ARGS["seed"]], np.int64),
        k=ARGS["k"])
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main(*sys.argv[1:])
