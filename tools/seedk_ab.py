"""A/B of the exact leaf's k-NN list length (ctx option leaf_seed_k) at BASELINE config 2
(1M x 3 blobs, minPts 4): ms per hdb_exact_mst and the kernel split.  usage:
python tools/seedk_ab.py [n]"""
import importlib, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
pkg = importlib.import_module(bench.PKG)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
X = torch.from_numpy(bench.make_blobs(n, 3, 20, seed=1)).cuda()
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
star = pkg.HDBSCANStar(ctx)
ref = None
for k, lr in ((0, 64), (-1, 64), (-1, 2), (-1, 3), (-1, 5), (0, 3)):
    ctx.set_option("leaf_seed_k", k)
    ctx.set_option("leaf_list_rounds", lr)
    for _ in range(2):
        star.exactMST(X, 4, None, pkg.CORE_EXCL_SELF, True)
    torch.cuda.synchronize()
    ctx.set_timing(True)
    for nm in ("knn_tree", "boruvka_total", "boruvka_scan"):
        ctx.kernel_time(nm)
    t0 = time.perf_counter()
    for _ in range(5):
        core, mst = star.exactMST(X, 4, None, pkg.CORE_EXCL_SELF, True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5 * 1e3
    kt = {nm: ctx.kernel_time(nm)[0] / 5 for nm in ("knn_tree", "boruvka_total", "boruvka_scan")}
    ctx.set_timing(False)
    w = torch.sort(torch.as_tensor(mst.getEges()).cpu())[0]
    same = True if ref is None else bool(torch.equal(w, ref))
    ref = w if ref is None else ref
    print(json.dumps({"leaf_seed_k": k, "list_rounds": lr, "ms": dt, **kt, "weights_equal": same}), flush=True)
