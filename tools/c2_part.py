"""One C2 partition at a time (1M x 3 blobs, minPts 4, EXCL_SELF): exact MST in the merge order
(hdb_exact_mst, HDB_EDGES_MERGED) then K6 flat labels, each call alone on one stream.  Prints
the wall time per partition and the library's kernel timers; run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel split (every kernel alone, no overlap).
usage: python tools/c2_part.py [reps] [n]"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "232-hierarchical-density-based-clustering-using-mapreduce_amd"
pkg = importlib.import_module(PKG)
bench = importlib.import_module("bench")

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
X = torch.from_numpy(bench.make_blobs(n, 3, 20, seed=1)).cuda()
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
NAMES = ["knn_tree", "boruvka_total", "boruvka_scan", "flat_labels"]


def part():
    _, mst = star.exactMST(X, 4, None, pkg.CORE_EXCL_SELF, True, merged=True)
    own = (mst.getVerticeA(), mst.getVericeB(), mst.getEges())
    return own, pkg.flat_labels(*own, n, 4, ctx=ctx)


own, (lab, k) = part()
torch.cuda.synchronize()
ctx.set_timing(True)
for nm in NAMES:
    ctx.kernel_time(nm)
t0 = time.perf_counter()
for _ in range(reps):
    own, (lab, k) = part()
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / reps
ctx.set_timing(False)
parts = {nm: round(ctx.kernel_time(nm)[0] / reps, 3) for nm in NAMES}
w = own[2].cpu().numpy()
assert np.all(w[:-1] >= w[1:]), "merged list not descending"
print(f"n={n}: {wall * 1e3:.3f} ms/partition, clusters {k};", parts, flush=True)
