"""Micro-benchmark at config-2 size (1M x 3): K1t (tree) and optionally K1 (dense) kernel
times, K1t evaluated pairs, and the Boruvka total / per-round scan times.

usage: python tools/knn_bench.py [n] [--dense]
"""
import importlib, sys, json, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
from bench import make_blobs

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 1_000_000
d = int(args[1]) if len(args) > 1 else 3
X = torch.from_numpy(make_blobs(n, d, 20, 1)).cuda()
ctx = pkg.Context.get(0); ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
res = {"n": n, "d": d}
for opt in os.environ.get("HDB_OPTS", "").split(","):
    if opt:
        k, v = opt.split("=")
        ctx.set_option(k, int(v))
        res[k] = int(v)


def timed(name, fn, reps=3):
    fn(); torch.cuda.synchronize()
    ctx.set_timing(True); ctx.kernel_time(name)
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    ms, cnt = ctx.kernel_time(name); ctx.set_timing(False)
    return out, ms / max(cnt, 1)


core, res["knn_tree_ms"] = timed("knn_tree", lambda: star.calculateCoreDistances(X, 4, None, 2))
ctx.set_option("count_evals", 1)
star.calculateCoreDistances(X, 4, None, 2)
for k in ("knn_tree_evals", "knn_tree_leaves", "knn_tree_nodes"):
    res[k] = ctx.get_stat(k)
ctx.set_option("count_evals", 0)
if "--dense" in sys.argv:
    ctx.set_option("knn_tree", 0)
    core2, res["knn_dense_ms"] = timed("knn_sq", lambda: star.calculateCoreDistances(X, 4, None, 2), reps=1)
    ctx.set_option("knn_tree", 1)
    res["tree_equals_dense"] = bool(torch.equal(core, core2))
names = ["boruvka_total", "boruvka_scan"] + [f"boruvka_r{i}" for i in range(8)] + ["boruvka_r8+"]
star.constructMSTBoruvka(X, core, True); torch.cuda.synchronize()
ctx.set_timing(True)
for k in names:
    ctx.kernel_time(k)
star.constructMSTBoruvka(X, core, True); torch.cuda.synchronize()
for k in names:
    ms, c = ctx.kernel_time(k)
    if c:
        res[k + "_ms"] = round(ms, 3)
ctx.set_timing(False)
ctx.set_option("count_evals", 1)
star.constructMSTBoruvka(X, core, True)
res["boruvka_evals"] = ctx.get_stat("last_evals")
for r in range(12):
    try:
        res[f"r{r}"] = [ctx.get_stat(f"boruvka_r{r}_{k}") for k in ("evals", "leaves", "nodes")]
    except Exception:
        break
ctx.set_option("count_evals", 0)
print(json.dumps(res))
