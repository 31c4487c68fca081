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

# concurrency: T threads each running `reps` models on their own context (driver's model pool)
import threading  # noqa: E402

for T in (1, 2, 4):
    ctxs = []

    def worker():
        c = pkg.Context.get(0)
        ctxs.append(c)
        o = {k: np.zeros(ne, t) for k, t in (("va", np.int32), ("vb", np.int32), ("w", np.float64),
                                              ("iva", np.int32), ("ivb", np.int32), ("iw", np.float64))}
        lab = np.zeros(b, np.int32)
        nn = np.zeros(1, np.int64)
        for _ in range(reps):
            A.lib().hdb_local_model(c.h, A.ptr(rep), A.ptr(info), b, d, 4, 4, A.METRIC["euclidean"], A.ptr(lab),
                                    A.ptr(o["va"]), A.ptr(o["vb"]), A.ptr(o["w"]), A.ptr(o["iva"]), A.ptr(o["ivb"]),
                                    A.ptr(o["iw"]), A.ptr(nn))

    base_p = pkg.Context.stat_total("lm_prim_us") if hasattr(pkg.Context, "stat_total") else 0
    base_c = pkg.Context.stat_total("lm_core_us") if hasattr(pkg.Context, "stat_total") else 0
    th = [threading.Thread(target=worker) for _ in range(T)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    prim = (pkg.Context.stat_total("lm_prim_us") - base_p) / (T * reps) / 1e3
    core = (pkg.Context.stat_total("lm_core_us") - base_c) / (T * reps) / 1e3
    print(json.dumps({"threads": T, "models": T * reps, "wall_s": wall, "prim_ms_per_model": prim,
                      "core_ms_per_model": core}))
