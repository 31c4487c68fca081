"""Generates tests/golden/c5s.npz: the CPU oracle's MR-HDBSCAN* (oracle/mr_driver.py, the line
restatement of Main.java:103-347 with the deviations D1-D10) on a SCALED config C5 -- the
same generator family and recursion shape (blobs in d = 8, 100 centres U[-100, 100]^8,
sigma 1, seed 5; an explicit per-subset sample count; data bubbles) at a size the oracle
finishes in minutes: 300,000 points, samples_per_subset 2,048, processing_units 8,192.

The merged edge list (2n - 1 = 599,999 edges of random doubles) is not stored: its SHA-256
(va, vb, w bytes) and that of the weights alone (the sorted multiset, which any exact MST
shares) are, with its first/last 64 edges; the levels, the bubble labels of every
local model and the subset of every point are stored in full.  Flat labels are not: the
oracle's top-down restatement (oracle/flat_labels.py) is O(levels x n), hours at 600k distinct
levels; the test checks the device labels against the product's host algorithm instead
(csrc/flat.cpp, itself pinned to oracle/flat_labels.py on smaller inputs).
tests/test_gpu_mr_scaled.py runs the HIP driver on the same input and compares.

Run in the build container (CPU only):  python tests/golden/make_c5s.py
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import blobs  # noqa: E402
from oracle import mr_driver as M  # noqa: E402

N, D, CENTERS, SEED = 300_000, 8, 100, 5
ARGS = dict(min_pts=4, min_cl_size=4, processing_units=8192, samples_per_subset=2048, seed=20210101)


def data():
    return blobs(N, D, CENTERS, SEED, spread=100.0)


def edge_digest(va, vb, w):
    h = hashlib.sha256()
    for a, t in ((va, np.int32), (vb, np.int32), (w, np.float64)):
        h.update(np.ascontiguousarray(a, t).tobytes())
    return h.hexdigest()


def pack_levels(levels):
    lv, lab_keys, lab_off, lab_vals, nk_keys, nk_off, nk_vals, errs = [], [], [0], [], [], [0], [], []
    for L in levels:
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
    return dict(levels=np.asarray(lv, np.int64).reshape(-1, 4), label_keys=np.asarray(lab_keys, np.int64).reshape(-1, 2),
                label_off=np.asarray(lab_off, np.int64), label_vals=cat(lab_vals, np.int32),
                newkey_keys=np.asarray(nk_keys, np.int64).reshape(-1, 2), newkey_off=np.asarray(nk_off, np.int64),
                newkey_vals=cat(nk_vals, np.int64), model_errors=np.asarray(errs, np.int64).reshape(-1, 3))


def main(out=os.path.join(HERE, "c5s.npz")):
    X = data()
    t0 = time.time()
    r = M.run(X, log=lambda s: print(f"[{time.time() - t0:8.1f}s] {s}", flush=True), flat=False, **ARGS)
    print(f"oracle run {time.time() - t0:.1f} s, iterations {r['iterations']}", flush=True)
    va, vb, w = r["edges"]
    np.savez_compressed(
        out, digest=np.asarray(edge_digest(va, vb, w)), digest_w=np.asarray(hashlib.sha256(w.tobytes()).hexdigest()),
        n_edges=w.shape[0], head_va=va[:64], head_vb=vb[:64],
        head_w=w[:64], tail_va=va[-64:], tail_vb=vb[-64:], tail_w=w[-64:], w_sum=np.sum(np.sort(w)),
        leaf_of=r["leaf_of"].astype(np.int32),
        iterations=r["iterations"], args=np.asarray([ARGS["min_pts"], ARGS["min_cl_size"], ARGS["processing_units"],
                                                     ARGS["samples_per_subset"], ARGS["seed"]], np.int64),
        shape=np.asarray([N, D, CENTERS, SEED], np.int64), **pack_levels(r["levels"]))
    print("wrote", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main(*sys.argv[1:])
