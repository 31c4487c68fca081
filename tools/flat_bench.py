"""K6 timing: the C2 merged list (1M blobs, exact MST + self edges, stable descending sort) ->
device flat labels, warm, repeated.  Usage: python tools/flat_bench.py [n] [reps]"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import make_blobs  # noqa: E402

pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
X = torch.from_numpy(make_blobs(n, 3, 20, 1)).cuda()
_, g = star.exactMST(X, 4, None, pkg.CORE_EXCL_SELF, True)
va, vb, w = pkg.sort_edges_desc(g.getVerticeA(), g.getVericeB(), g.getEges(), ctx)
lab, k = pkg.flat_labels(va, vb, w, n, 4, ctx=ctx)
torch.cuda.synchronize()
ctx.set_timing(True)
ctx.kernel_time("flat_labels")
t0 = time.perf_counter()
for _ in range(reps):
    lab, k = pkg.flat_labels(va, vb, w, n, 4, ctx=ctx)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
ms, cnt = ctx.kernel_time("flat_labels")
print(f"flat labels n={n}: {dt * 1e3:.3f} ms/call wall, {ms / max(cnt, 1):.3f} ms device span, K={k}, clusters {ctx.get_stat('flat_clusters_total')}, FOSC on the device")
