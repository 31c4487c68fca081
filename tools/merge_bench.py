"""The N>1 C2 merge on one device: R presorted runs of 2n-1 edges (per-rank C2-like lists) ->
merged list, hdb_merge_sorted_runs vs a re-sort of the concatenation (hdb_sort_edges_desc).
Usage: python tools/merge_bench.py [runs] [edges_per_run] [reps]"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
R = int(sys.argv[1]) if len(sys.argv) > 1 else 8
E = int(sys.argv[2]) if len(sys.argv) > 2 else 1_999_999
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
g = torch.Generator(device="cuda").manual_seed(3)
runs = []
for r in range(R):
    w = torch.rand(E, dtype=torch.float64, device="cuda", generator=g) * 4
    w[: E // 2] = 0.0  # the self edges' zero weights: one long tie block per run
    va = torch.randint(0, 10**6, (E,), dtype=torch.int32, device="cuda", generator=g)
    vb = torch.randint(0, 10**6, (E,), dtype=torch.int32, device="cuda", generator=g)
    runs.append(pkg.sort_edges_desc(va, vb, w, ctx))
cat = [torch.cat([x[i] for x in runs]) for i in range(3)]
off = np.arange(R + 1, dtype=np.int64) * E


def t_of(f):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, out


ms_m, m = t_of(lambda: pkg.merge_sorted_runs(*cat, off, ctx=ctx))
ms_s, s = t_of(lambda: pkg.sort_edges_desc(*(x.clone() for x in cat), ctx))
same = all(torch.equal(a, b) for a, b in zip(m, s))
print(f"R={R} x {E} edges: merge of presorted runs {ms_m:.3f} ms, re-sort (incl. clone) {ms_s:.3f} ms, identical={same}")
