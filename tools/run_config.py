"""End-to-end MR-HDBSCAN* runs of BASELINE.json's configs on one device (driver.py), with
per-phase wall times and per-level shape.  usage: python tools/run_config.py c1|c3|c5 [n]"""
import importlib, json, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")

cfg = sys.argv[1]
if cfg == "c1":
    from conftest import load_skin
    X = load_skin()
    kw = dict(minPts=4, minClSize=4, processing_units=50, k=0.2)
elif cfg == "c3":
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
    rng = np.random.default_rng(3)
    C = rng.uniform(-50, 50, size=(50, 16))
    X = C[rng.integers(0, 50, size=n)] + rng.normal(0, 1.0, size=(n, 16))
    kw = dict(minPts=4, minClSize=4, processing_units=65536, samples_per_subset=4096)
elif cfg == "c5":
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16_000_000
    rng = np.random.default_rng(5)
    C = rng.uniform(-100, 100, size=(100, 8))
    X = C[rng.integers(0, 100, size=n)] + rng.normal(0, 1.0, size=(n, 8))
    kw = dict(minPts=4, minClSize=4, processing_units=65536, samples_per_subset=16384)
else:
    raise SystemExit("c1|c3|c5")
Xd = torch.from_numpy(X).cuda()
drv = pkg.MRHDBSCANStar(profile=True, prim_leaf_max=4096, model_threads=int(os.environ.get("MODEL_THREADS", "4")), **kw)
t = time.perf_counter()
r = drv.run(Xd)
torch.cuda.synchronize()
dt = time.perf_counter() - t
lv = [dict(it=l["iteration"], leaves=len(l["leaves"]), leaf_pts=int(sum(l["leaves"].values())),
           big=len(l["big"]), big_pts=int(sum(l["big"].values())), errors=l.get("model_errors"))
      for l in r["levels"]]
lm = {}
for k in ("lm_calls", "lm_core_us", "lm_prim_us", "lm_quicksort_us", "lm_tree_us", "lm_fosc_us"):
    try:
        lm[k] = drv.ctx.get_stat(k)
    except Exception:
        pass
print(json.dumps(dict(local_model=lm, config=cfg, n=int(X.shape[0]), d=int(X.shape[1]), seconds=dt, points_per_s=X.shape[0] / dt,
                      iterations=r["iterations"], n_clusters=r.get("n_clusters"),
                      timings={k: round(v, 4) for k, v in drv.timings.items()}, levels=lv)))
