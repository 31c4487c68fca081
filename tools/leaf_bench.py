"""Cost of one forced leaf (hdb_exact_mst: cumulative cores + exact MST) at the C3/C5 leaf
shapes, split by kernel timer.  usage: python tools/leaf_bench.py [n d] ..."""
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
A = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd._capi")
args = [int(a) for a in sys.argv[1:]] or [40000, 8, 80000, 16]
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
NAMES = ["exact_leaf_total", "knn_tree", "knn_generic", "knn_mfma", "leaf_core", "boruvka_total", "boruvka_scan",
         "boruvka_r0", "boruvka_r1", "boruvka_r2", "boruvka_r3", "boruvka_r4", "boruvka_r5", "boruvka_r6",
         "boruvka_r7", "boruvka_r8+", "merge_sort"]
for n, d in zip(args[0::2], args[1::2]):
    rng = np.random.default_rng(n + d)
    X = torch.from_numpy(rng.normal(size=(n, d))).cuda()
    va = torch.empty(2 * n - 1, dtype=torch.int32, device="cuda")
    vb = torch.empty_like(va)
    w = torch.empty(2 * n - 1, dtype=torch.float64, device="cuda")
    run = lambda: A.check(A.lib().hdb_exact_mst(ctx.h, X.data_ptr(), n, d, 4, 0, A.CORE_INCL_SELF_CUMULATIVE, 1, None,
                                                 va.data_ptr(), vb.data_ptr(), w.data_ptr()), "exact")
    run()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    for nm in NAMES:
        ctx.kernel_time(nm)
    t = time.perf_counter()
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / 3
    ctx.set_timing(False)
    parts = {nm: round(ctx.kernel_time(nm)[0] / 3, 3) for nm in NAMES}
    print(f"n={n} d={d}: {wall * 1e3:.2f} ms/leaf;", {k: v for k, v in parts.items() if v})
