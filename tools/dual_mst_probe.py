"""Probe: do two partitions' exact MSTs (K1t cores -> K2b Boruvka -> sort) overlap on one GPU?
T threads, each with its own library context and HIP stream, each running S steps of
hdb_exact_mst + sort_edges_desc on a 1M x 3 partition; prints ms per partition.
usage: python tools/dual_mst_probe.py [T] [S]"""
import importlib
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

pkg = importlib.import_module(bench.PKG)
T = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = int(sys.argv[2]) if len(sys.argv) > 2 else 10
X = torch.from_numpy(bench.make_blobs(bench.N_POINTS, bench.D, bench.CENTERS, seed=1)).cuda()


def worker(steps, out, idx, barrier):
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ctx = pkg.Context.get(0)
        ctx.use_torch_stream()
        star = pkg.HDBSCANStar(ctx)
        _, mst = star.exactMST(X, bench.MIN_PTS, None, pkg.CORE_EXCL_SELF, True)  # warm
        s.synchronize()
        barrier.wait()
        t0 = time.perf_counter()
        for _ in range(steps):
            _, mst = star.exactMST(X, bench.MIN_PTS, None, pkg.CORE_EXCL_SELF, True)
            pkg.sort_edges_desc(mst.getVerticeA(), mst.getVericeB(), mst.getEges(), ctx)
        s.synchronize()
        out[idx] = time.perf_counter() - t0


res = {}
for t in sorted({1, T}):
    out = [0.0] * t
    b = threading.Barrier(t)
    th = [threading.Thread(target=worker, args=(S, out, i, b)) for i in range(t)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    res[t] = max(out) * 1e3 / (S * t)
print(json.dumps({"ms_per_partition": res, "steps_per_thread": S}))
