"""bench.py -- BASELINE.json's metric on its config 2 (the largest single-GPU config):

    "Synthetic Gaussian blobs 1M x 3, exact HDBSCAN* (no sampling) on one MI355X, FP64"

One step = the exact MR-HDBSCAN* leaf path over one 1M x 3 partition already resident in
HBM: core distances (K1t: exact k-NN over minPts = 4 on the Morton/BVH index -- the lists
are bit-identical to the all-pairs scan) -> mutual-reachability MST (K2b Boruvka; n-1 tree
edges + n self edges as FirstStep emits them) -> the reducers' merge (stable descending
sort, SortMST).  With N GPUs (torchrun, one process per GPU) every
rank owns its own 1M-point partition (weak scaling, as MR-HDBSCAN* shards partitions) and the
merge all-gathers every rank's edge list over RCCL before the sort.

Prints ONE JSON line (rank 0).  value = points/s over all ranks.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "232-hierarchical-density-based-clustering-using-mapreduce_amd"

N_POINTS = 1_000_000
D = 3
MIN_PTS = 4
CENTERS = 20
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, FMA counted as 2 flops (spec)
FP64_NOFMA_TOPS = 39.3   # non-FMA issue ceiling (256 CU x 2.4 GHz x 64 lanes)


def make_blobs(n, d, centers, seed):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-100, 100, size=(centers, d))
    lab = rng.integers(0, centers, size=n)
    return C[lab] + rng.normal(0, 1.0, size=(n, d))


def cpu_baseline(X, budget_s=20.0):
    """Oracle (line-faithful C restatement, -O2, 1 thread) on a bounded sample of the same
    workload: k-NN core distances for R query rows against all n rows (n^2 work per
    point, extrapolated linearly in rows) + reference Prim on an m-point prefix
    (extrapolated by (n/m)^2).  points/s = n / (t_knn_full + t_prim_full)."""
    from oracle import oracle as O
    O.lib()
    n = X.shape[0]
    rows = np.arange(0, n, max(1, n // 64))[:64]
    t0 = time.perf_counter()
    O.core_rows(X, rows, MIN_PTS, excl_self=True)
    t_rows = time.perf_counter() - t0
    # grow the row sample to ~half the budget
    r2 = int(min(n, max(len(rows), len(rows) * (0.5 * budget_s) / max(t_rows, 1e-3))))
    rows2 = np.linspace(0, n - 1, r2).astype(np.int64)
    t0 = time.perf_counter()
    O.core_rows(X, rows2, MIN_PTS, excl_self=True)
    t_knn = (time.perf_counter() - t0) * (n / len(rows2))
    m = 4000
    Xm = X[:m]
    core = O.core_distances(Xm, MIN_PTS, semantics=O.EXCL_SELF)
    t0 = time.perf_counter()
    O.prim_mst(Xm, core)
    t_p = time.perf_counter() - t0
    m2 = int(min(40000, m * max(1.0, (0.4 * budget_s / max(t_p, 1e-3)) ** 0.5)))
    Xm = X[:m2]
    core = O.core_rows(Xm, np.arange(m2), MIN_PTS, excl_self=True)
    t0 = time.perf_counter()
    O.prim_mst(Xm, core)
    t_prim = (time.perf_counter() - t0) * (n / m2) ** 2
    total = t_knn + t_prim
    return {"value": n / total, "unit": "points/s", "cores": 1, "kind": "port",
            "sample": f"oracle C -O2 1 thread: kNN of {len(rows2)} query rows vs all {n} rows "
                      f"(x{n / len(rows2):.0f}) + reference Prim on a {m2}-point prefix "
                      f"(x{(n / m2) ** 2:.0f}); extrapolated full step {total:.0f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=N_POINTS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split", action="store_true",
                    help="two calls (core distances, then Boruvka on a second index) instead of the fused leaf")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    pkg = importlib.import_module(PKG)
    from importlib import import_module
    par = import_module(PKG + ".parallel")

    n = args.n
    X_host = make_blobs(n, D, CENTERS, seed=1 + rank)
    X = torch.from_numpy(X_host).cuda()
    ctx = pkg.Context.get(local)
    ctx.use_torch_stream()
    star = pkg.HDBSCANStar(ctx)

    def leaf():
        if args.split:
            core = star.calculateCoreDistances(X, MIN_PTS, None, pkg.CORE_EXCL_SELF)
            return core, star.constructMSTBoruvka(X, core, True)
        return star.exactMST(X, MIN_PTS, None, pkg.CORE_EXCL_SELF, True)

    def step():
        _, mst = leaf()
        va, vb, w = mst.getVerticeA(), mst.getVericeB(), mst.getEges()
        if world > 1:
            return par.merge_local_msts(va, vb, w)
        return pkg.sort_edges_desc(va, vb, w, ctx)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    # per-kernel device times: HIP events recorded on the launch stream inside the timed
    # region (measured cost of the records: ~1% of a step)
    ctx.set_timing(True)
    for k in ("knn_tree", "knn_sq", "boruvka_total", "boruvka_scan", "merge_sort", "exact_leaf_total"):
        ctx.kernel_time(k)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    barrier()
    dt = time.perf_counter() - t0
    ctx.set_timing(False)
    tsteps = args.steps
    knn_ms, knn_n = ctx.kernel_time("knn_tree")
    bor_ms, bor_n = ctx.kernel_time("boruvka_total")
    scan_ms, scan_n = ctx.kernel_time("boruvka_scan")
    srt_ms, srt_n = ctx.kernel_time("merge_sort")
    t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms_step = dt * 1e3 / args.steps
    # executed work (diagnostic pass outside the timed region): pairs each traversal evaluated
    ctx.set_option("count_evals", 1)
    leaf()
    knn_evals = ctx.get_stat("knn_tree_evals")
    bor_evals = ctx.get_stat("boruvka_evals")
    ctx.set_option("count_evals", 0)

    # sanity: the merged list is sorted descending and has N*(2n-1) edges
    w_out = out[2]
    assert w_out.shape[0] == world * (2 * n - 1)
    total_points = world * n
    value = total_points * args.steps / dt
    evals = world * (n * n + n * (n - 1) / 2)  # kNN n^2 + MST n(n-1)/2
    # roofline of the dominant kernel (per launch, HIP events on the launch stream)
    kern = {"knn_tree": (knn_ms, knn_n, knn_evals * tsteps), "boruvka_scan": (scan_ms, scan_n, bor_evals * tsteps)}
    dom = max(kern, key=lambda k: kern[k][0])
    k_ms, k_n, k_ev = kern[dom]
    avg_s = k_ms / max(k_n, 1) / 1e3
    flops_per_launch = 3 * D * (k_ev / max(k_n, 1))  # executed pair evals x 3d flops
    achieved = flops_per_launch / avg_s / 1e12 if avg_s > 0 else 0.0
    algo_flops = 3 * D * (n * n if dom == "knn_tree" else n * (n - 1) / 2) / max(k_n / tsteps, 1)
    traffic = None
    # HBM bytes per launch from the committed rocprofv3 PMC passes (tools/profile_bench.sh,
    # FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md), keyed by kernel symbol
    pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
    sym = {"knn_tree": "knn_tree_kernel", "boruvka_scan": "boruvka_bvh_kernel"}[dom]
    if os.path.exists(pmc):
        with open(pmc) as fh:
            traffic = json.load(fh).get(sym, {}).get("hbm_bytes_per_launch")
    line = {
        "metric": "points/sec end-to-end + mutual-reach distance evals/sec at 1/2/4/8 GPUs",
        "value": value,
        "unit": "points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded Gaussian blobs, 20 centers ~U[-100,100]^3, sigma 1, seed 1+rank)",
        "config": {"workload": "config 2: blobs 1M x 3 exact HDBSCAN* (no sampling), minPts 4",
                   "points_per_gpu": n, "d": D, "min_pts": MIN_PTS, "core": "EXCL_SELF",
                   "mst": "boruvka (exact; Prim-identical sorted weights)"
                   + (" on a second index" if args.split else ", kNN-seeded round 0 on the K1t index"), "merge": "stable desc sort",
                   "parallelism": f"partition-sharded x{world}"},
        "mrd_evals_per_s": evals * args.steps / dt,
        "kernels_ms_per_step": {"knn_tree": knn_ms / tsteps, "boruvka_total": bor_ms / tsteps,
                                "boruvka_scan": scan_ms / tsteps, "merge_sort": srt_ms / tsteps},
        "executed_pair_evals_per_step": {"knn_tree": knn_evals, "boruvka_scan": bor_evals,
                                         "algorithmic": n * n + n * (n - 1) // 2},
        "roofline": {"bound": "fp64-valu", "kernel": dom, "achieved": achieved,
                     "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                     "traffic": traffic, "work": "executed pair evals x 3d flops (pruned traversal)",
                     "flops_per_launch": flops_per_launch, "avg_launch_ms": avg_s * 1e3,
                     "launches_per_step": k_n / tsteps,
                     "algorithmic_equiv_tflops": algo_flops / avg_s / 1e12},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(X_host)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
