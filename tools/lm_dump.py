"""Dumps one C5-shaped local model's host inputs (the tools/lm_bench.py model: bubble reps,
extents, nnDist, counts, and its bubble Prim MST + self edges in Prim order) as raw files, for the
CPU benchmark of the host half (tools/lm_host_bench.cpp).  usage: python tools/lm_dump.py outdir [b] [d]"""
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_blobs  # noqa: E402

pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
A = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd._capi")
out = sys.argv[1]
b = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
d = int(sys.argv[3]) if len(sys.argv) > 3 else 8
os.makedirs(out, exist_ok=True)
rep = make_blobs(b, d, 100, 5)
rng = np.random.default_rng(1)
eB, nnB, nB = rng.uniform(0.5, 1.5, b), rng.uniform(0.1, 0.5, b), rng.integers(500, 1500, b).astype(np.int32)
ctx = pkg.Context.get(0)
core = np.zeros(b)
rc = A.lib().hdb_bubble_core_distances(ctx.h, A.ptr(rep), A.ptr(nB), A.ptr(eB), A.ptr(nnB), b, d, 4,
                                       A.METRIC["euclidean"], A.ptr(core))
assert rc == 0, rc
ne = 2 * b - 1
va, vb, w = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
ids = np.arange(b, dtype=np.int32)
rc = A.lib().hdb_bubble_prim_mst(ctx.h, A.ptr(rep), A.ptr(eB), A.ptr(nnB), A.ptr(ids), A.ptr(core), b, d,
                                 A.METRIC["euclidean"], 1, A.ptr(va), A.ptr(vb), A.ptr(w))
assert rc == 0, rc
for k, v in (("rep", rep), ("eB", eB), ("nnB", nnB), ("nB", nB), ("va", va), ("vb", vb), ("w", w)):
    np.ascontiguousarray(v).tofile(os.path.join(out, k + ".bin"))
json.dump({"b": b, "d": d, "ne": ne}, open(os.path.join(out, "meta.json"), "w"))
print("dumped", b, d, ne)
