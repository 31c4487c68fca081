"""One C5-shaped local model (LocalModelReduceByKey: bubble cores, bubble Prim, cluster tree,
FOSC) with its phase times.  usage: python tools/lm_bench.py [b] [d] [reps]"""
import importlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_blobs  # noqa: E402

pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
A = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd._capi")
b = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rep = make_blobs(b, d, 100, 5)
rng = np.random.default_rng(1)
info = np.stack([rng.uniform(0.5, 1.5, b), rng.uniform(0.1, 0.5, b), rng.integers(500, 1500, b).astype(float)], 1)
ctx = pkg.Context.get(0)
ne = 2 * b - 1
out = {k: np.zeros(ne, t) for k, t in (("va", np.int32), ("vb", np.int32), ("w", np.float64),
                                          ("iva", np.int32), ("ivb", np.int32), ("iw", np.float64))}
labels = np.zeros(b, np.int32)
nic = np.zeros(1, np.int64)


def call():
    return A.lib().hdb_local_model(ctx.h, A.ptr(rep), A.ptr(info), b, d, 4, 4, A.METRIC["euclidean"], A.ptr(labels),
                                   A.ptr(out["va"]), A.ptr(out["vb"]), A.ptr(out["w"]), A.ptr(out["iva"]),
                                   A.ptr(out["ivb"]), A.ptr(out["iw"]), A.ptr(nic))


call()
keys = ("lm_core_us", "lm_prim_us", "lm_quicksort_us", "lm_tree_us", "lm_fosc_us", "lm_calls")
base = {k: ctx.get_stat(k) for k in keys}
t0 = time.perf_counter()
rcs = [call() for _ in range(reps)]
dt = (time.perf_counter() - t0) / reps
res = {k: (ctx.get_stat(k) - base[k]) / reps / 1e3 for k in keys[:-1]}
print(json.dumps({"b": b, "d": d, "rc": rcs[-1], "ms_per_model": dt * 1e3, "phases_ms": res,
                  "clusters": int(labels.max())}))
