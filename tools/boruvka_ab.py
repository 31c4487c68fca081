"""A/B of K2b scan knobs at C2 (1M x 3, minPts 4): exact-leaf time (HIP events) per setting,
interleaved repeats.  usage: python tools/boruvka_ab.py "k=v,k=v" "k=v" ..."""
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_blobs  # noqa: E402

pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
X = torch.from_numpy(make_blobs(1_000_000, 3, 20, 1)).cuda()
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
confs = [dict(kv.split("=") for kv in a.split(",")) if a else {} for a in (sys.argv[1:] or [""])]
defaults = {"boruvka_early_pts": 0, "boruvka_early_rounds": 5, "boruvka_wave_pts": 64}
ref = None
res = {i: [] for i in range(len(confs))}
for rep in range(6):
    for i, c in enumerate(confs):
        for k, v in defaults.items():
            ctx.set_option(k, v)
        for k, v in c.items():
            ctx.set_option(k, int(v))
        star.exactMST(X, 4, None, 2, True)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        ctx.kernel_time("exact_leaf_total")
        ctx.kernel_time("boruvka_scan")
        _, g = star.exactMST(X, 4, None, 2, True)
        torch.cuda.synchronize()
        ms, _ = ctx.kernel_time("exact_leaf_total")
        sc, _ = ctx.kernel_time("boruvka_scan")
        ctx.set_timing(False)
        w = torch.sort(g.getEges())[0]
        if ref is None:
            ref = w
        assert torch.equal(w, ref), c
        res[i].append((ms, sc))
for i, c in enumerate(confs):
    a = np.array(res[i])
    print(f"{c or 'default'}: leaf {np.median(a[:, 0]):.3f} ms (min {a[:, 0].min():.3f}), scan {np.median(a[:, 1]):.3f} ms")
