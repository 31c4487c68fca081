"""K1m at BASELINE config 4 (2M x 128 L2-normalised embeddings, 200 centers, minPts 16):
time of the exact k-NN lists on MFMA, re-check count, MFMA rate, and an exact spot check
of sampled rows against a Java-order FP64 scan done with torch (one op per dimension, no
fusion).  usage: python tools/k1m_bench.py [n] [d]"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("232-hierarchical-density-based-clustering-using-mapreduce_amd")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 128
MIN_PTS = 16
g = torch.Generator(device="cuda").manual_seed(4)
C = torch.randn(200, d, dtype=torch.float64, device="cuda", generator=g)
lab = torch.randint(0, 200, (n,), device="cuda", generator=g)
X = C[lab] + 0.1 * torch.randn(n, d, dtype=torch.float64, device="cuda", generator=g)
X = X / torch.linalg.norm(X, dim=1, keepdim=True)
X = X.contiguous()
ctx = pkg.Context.get(0)
ctx.use_torch_stream()
SINGLE = int(os.environ.get("K1M_SINGLE", "1"))
ctx.set_option("knn_mfma_single", SINGLE)
star = pkg.HDBSCANStar(ctx)
k = MIN_PTS - 1
star.knn(X[:4096].contiguous(), k, None, exclSelf=True)  # warm
torch.cuda.synchronize()
ctx.set_timing(True)
ctx.kernel_time("knn_mfma")
ctx.kernel_time("knn_mfma_final")
ctx.kernel_time("knn_mfma_order")
t0 = time.perf_counter()
L = star.knn(X, k, None, exclSelf=True)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
ms, _ = ctx.kernel_time("knn_mfma")
ms_final, _ = ctx.kernel_time("knn_mfma_final")
ms_order, _ = ctx.kernel_time("knn_mfma_order")
ovf = ctx.get_stat("knn_mfma_log_overflow") if SINGLE else 0
ctx.set_timing(False)
if os.environ.get("K1M_QUICK"):
    nb = ctx.get_stat("knn_mfma_blocks")
    rows = ctx.get_stat("knn_mfma_group_rows")
    n_pad = -(-n // 512) * 512
    out = {"n": n, "d": d, "lib": os.environ.get("HDBMI_LIB", "default"), "wall_s": dt, "knn_mfma_ms": ms,
           "knn_mfma_final_ms": ms_final, "knn_mfma_order_ms": ms_order, "blocks": nb,
           "block_frac": nb * rows * 32 / (n * n_pad)}
    if os.environ.get("K1M_PROF"):  # a HDB_K1S_PROF=1 build: per-wave cycle split of the screen
        for key in ("wait", "mfma", "hit", "hitsteps", "setup", "wavesteps", "hits"):
            out["prof_" + key] = ctx.get_stat("k1s_prof_" + key)
    if os.environ.get("K1M_DIAG"):
        ctx.set_option("count_evals", 1)
        star.knn(X, k, None, exclSelf=True)
        ctx.set_option("count_evals", 0)
        for key in ("knn_mfma_qrad_med_e6", "knn_mfma_sbrad_med_e6", "knn_mfma_nsb", "knn_mfma_rechecks",
                    "knn_mfma_layout_rows"):
            out[key] = ctx.get_stat(key)
        import math
        mu = X.mean(0)
        sc = 2.0 ** -math.frexp(float((X - mu).abs().max()))[1]
        out["scale"] = sc
        out["kth_dist_scaled_med"] = float(L[:, -1].median()) * sc
    print(json.dumps(out))
    sys.exit(0)
ctx.set_option("count_evals", 1)
star.knn(X[: min(n, 200_000)].contiguous(), k, None, exclSelf=True)
re_sub = ctx.get_stat("knn_mfma_rechecks")
ctx.set_option("count_evals", 0)
n_pad = -(-n // 256) * 256
DP = 32 if d <= 32 else 64 if d <= 64 else 128 if d <= 128 else 256
passes = 1 if SINGLE else 2  # single pass (screen + log) or upper-bound pass + exact pass
flops = passes * 3 * 2.0 * n_pad * n_pad * DP  # bf16 split: 3 MFMA products per pass
# exact spot check (Java order): 16 sampled rows
rows = torch.randint(0, n, (16,), device="cuda", generator=g)
bad = 0
for r in rows.tolist():
    s = (X[:, 0] - X[r, 0]) * (X[:, 0] - X[r, 0])
    for j in range(1, d):
        t = X[:, j] - X[r, j]
        s = s + t * t
    s[r] = float("inf")
    ref = torch.sqrt(torch.topk(s, k, largest=False).values)
    bad += int(not torch.equal(ref, L[r]))
print(json.dumps({"n": n, "d": d, "k": k, "single": SINGLE, "wall_s": dt, "knn_mfma_ms": ms,
                  "knn_mfma_final_ms": ms_final, "log_overflow": ovf, "mfma_tflops": flops / (ms / 1e3) / 1e12,
                  "mfma_peak_tflops": 2500.0, "logged_per_query_200k" if SINGLE else "rechecks_per_query_200k": re_sub / min(n, 200_000),
                  "spot_rows": 16, "spot_mismatch": bad}))
