"""K4 bubble statistics at C5's level-0 shape (16M x 8 points, 16,384 bubbles): the fold with
one lane per (bubble, dimension) against one lane per bubble (option bubble_fold_dim), identical
outputs.  usage: python tools/bubble_stats_bench.py [n] [d] [nb]"""
import importlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
A = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd._capi")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 8
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
g = torch.Generator(device="cuda").manual_seed(5)
X = torch.randn(n, d, dtype=torch.float64, device="cuda", generator=g) * 30
bo = torch.randint(0, nb, (n,), dtype=torch.int32, device="cuda", generator=g)
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
out = {}
for rep in range(2):
    for mode in (1, 0):
        ctx.set_option("bubble_fold_dim", mode)
        ls = torch.empty((nb, d), dtype=torch.float64, device="cuda")
        ss, rp = torch.empty_like(ls), torch.empty_like(ls)
        info = torch.empty((nb, 3), dtype=torch.float64, device="cuda")
        call = lambda: A.check(A.lib().hdb_bubble_stats(ctx.h, X.data_ptr(), n, d, bo.data_ptr(), nb,
                                                        A.BUBBLE_COMBINESTEP, ls.data_ptr(), ss.data_ptr(),
                                                        rp.data_ptr(), info.data_ptr()), "bubble_stats")
        call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        r = tuple(x.cpu().numpy().copy() for x in (ls, ss, rp, info))
        if rep == 0 and mode in out:
            pass
        if 1 - mode in out:
            assert all(np.array_equal(a.view(np.int64), b.view(np.int64)) for a, b in zip(r, out[1 - mode])), "differ"
        out[mode] = r
        print(f"bubble_fold_dim={mode}: {dt * 1e3:.2f} ms per call (n={n} d={d} nb={nb})", flush=True)
print("identical outputs")
