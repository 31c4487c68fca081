"""Per-round Boruvka diagnostics of hdb_exact_mst at config-2 size (1M x 3, minPts 4):
round time (HIP events), lanes/waves searching at the start of the scan, node/leaf visits,
pair evals.  Usage: python tools/boruvka_stats.py [n] [option=value ...]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
from bench import make_blobs  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 and "=" not in sys.argv[1] else 1_000_000
X = torch.from_numpy(make_blobs(n, 3, 20, 1)).cuda()
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
for a in sys.argv[1:]:
    if "=" in a:
        k, v = a.split("=")
        ctx.set_option(k, int(v))
star = pkg.HDBSCANStar(ctx)
star.exactMST(X, 4, None, 2, True)
torch.cuda.synchronize()
ctx.set_timing(True)
names = [f"boruvka_r{r}" for r in range(8)] + ["boruvka_r8+", "knn_tree", "boruvka_total", "exact_leaf_total"]
for k in names:
    ctx.kernel_time(k)
star.exactMST(X, 4, None, 2, True)
torch.cuda.synchronize()
for k in names:
    ms, c = ctx.kernel_time(k)
    print(f"{k:18s} {ms:8.3f} ms  x{c}")
ctx.set_timing(False)
ctx.set_option("count_evals", 1)
star.exactMST(X, 4, None, 2, True)
for r in range(12):
    p = f"boruvka_r{r}"
    try:
        vals = [ctx.get_stat(p + s) for s in ("_active_lanes", "_active_waves", "_nodes", "_leaves", "_evals")]
    except Exception:
        break
    cyc = [ctx.get_stat(p + "_wave_cyc_" + s) for s in ("mean", "p50", "p99", "max")]
    print(f"r{r}: active lanes {vals[0]:>8d}  waves {vals[1]:>6d}  nodes {vals[2]:>9d}  leaves {vals[3]:>8d}  evals {vals[4]:>11d}  wave cyc mean/p50/p99/max {cyc}")
    try:  # HDB_BOR_PROF build: cycle split summed over the round's waves, per node visit
        pn = ("setup", "pop", "stage", "test", "push", "leaf_load", "leaf_mask", "leaf_eval", "publish", "tail")
        pr = [ctx.get_stat(p + "_prof_" + s) for s in pn]
        tot = sum(pr) or 1
        print("    cycles/visit " + "  ".join(f"{s} {v / max(vals[2], 1):.0f}" for s, v in zip(pn, pr)) +
              f"  | share " + " ".join(f"{s} {100 * v / tot:.0f}%" for s, v in zip(pn, pr)))
    except Exception:
        pass
