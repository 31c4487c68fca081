"""Micro-benchmark of K1 (and Boruvka) at config-2 size: prints kernel times, both K1 paths."""
import importlib, sys, time, json, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
from bench import make_blobs
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X = torch.from_numpy(make_blobs(n, 3, 20, 1)).cuda()
ctx = pkg.Context.get(0); ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
res = {}
for screen in (1, 0):
    ctx.set_option("knn_fp32_screen", screen)
    core = star.calculateCoreDistances(X, 4, None, 2); torch.cuda.synchronize()
    ctx.set_timing(True); ctx.kernel_time("knn_sq")
    for _ in range(3):
        core = star.calculateCoreDistances(X, 4, None, 2)
    torch.cuda.synchronize()
    ms, cnt = ctx.kernel_time("knn_sq"); ctx.set_timing(False)
    res[f"knn_screen{screen}_ms"] = ms / cnt
ctx.set_option("knn_fp32_screen", 1)
ctx.set_timing(True); ctx.kernel_time("boruvka_total"); ctx.kernel_time("boruvka_scan")
mst = star.constructMSTBoruvka(X, core, True); torch.cuda.synchronize()
res["boruvka_total_ms"] = ctx.kernel_time("boruvka_total")[0]
res["boruvka_scan_ms"], res["boruvka_rounds"] = ctx.kernel_time("boruvka_scan")
print(json.dumps(res))
