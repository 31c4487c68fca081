"""bench.py -- BASELINE.json's metric on its config 2 (the largest single-GPU config):

    "Synthetic Gaussian blobs 1M x 3, exact HDBSCAN* (no sampling) on one MI355X, FP64"

One step = the whole job for one 1M x 3 partition, end to end as SURVEY.md §8(d) defines it:
parsed points resident in HBM -> core distances (K1t: exact k-NN over minPts =
4 on the Morton/BVH index, bit-identical to the all-pairs scan) -> mutual-reachability MST (K2b
Boruvka; n-1 tree edges + n self edges as FirstStep emits them) -> the reducers' merge (stable
descending sort, SortMST) -> global HDBSCAN* hierarchy + flat labels (K6, minClSize 4) ->
merged edge list and labels back in host memory.  With N GPUs (torchrun, one process per GPU)
every rank owns its own 1M-point partition (weak scaling, as MR-HDBSCAN* shards partitions):
each rank labels its partition, and the merge all-gathers every rank's edge list over RCCL
before the sort (rank 0 copies the merged list out).

Several partitions are in flight on one GPU (MR-HDBSCAN* maps over independent partitions):
--mst-workers stage-1 threads (exact MST + sort, own context and stream each; default 5) and
--label-workers label stages (default 2), so one partition's latency-bound Boruvka rounds and
flat-label kernels overlap the next partitions' work.  Every step still does all of its work.

Prints ONE JSON line (rank 0).  value = points/s over all ranks, end to end from parsed points
in pinned host memory (every step uploads its points inside the timed region) to the merged
list and labels back in host memory; hbm_resident_points_per_s = the same pipeline from points
already in HBM; device_resident_points_per_s = MST + merge only (HBM to HBM, no labels).
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import queue
import sys
import threading
import time

import numpy as np

# Hardware queues for this process (read by the HIP runtime when it initialises, after this
# module is imported).  The C2 pipeline keeps 5 stage-1 + 2 label streams busy and the C3/C5
# driver runs concurrent local-model threads; with HIP's default of 4 queues several streams
# share one queue and their kernels serialise (C2: 6.63 -> 6.1 ms/step with 8,
# profiles/r05/hwq/).  Never above the pool's limit of 32.
# HDB_HW_QUEUES (> 0) is the explicit knob and wins in both directions.  Without it,
# GPU_MAX_HW_QUEUES is raised to 8 but never lowered: the GPU pool exports
# GPU_MAX_HW_QUEUES=4 (HIP's own default) into every job, so a value of 4 there is the
# environment's, not a request for fewer queues.
_hwq_req = int(os.environ.get("HDB_HW_QUEUES", "0") or 0)
_hwq_env = int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)
HW_QUEUES = min(32, _hwq_req if _hwq_req > 0 else max(8, _hwq_env))
os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "232-hierarchical-density-based-clustering-using-mapreduce_amd"

N_POINTS = 1_000_000
D = 3
MIN_PTS = 4
MIN_CL_SIZE = 4
CENTERS = 20
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, FMA counted as 2 flops (spec)
FP64_NOFMA_TOPS = 39.3   # non-FMA issue ceiling (256 CU x 2.4 GHz x 64 lanes)
HBM_PEAK_GBS = 8000.0
MALL_HIT_NS = 227.0      # MI355X_MICROARCH.md: global_load Infinity Cache hit latency (one lane, idle)
WAVE_SLOTS = 256 * 4 * 4  # resident waves of the K2b scan: 256 CUs x 4 SIMDs x 4 waves (127 VGPRs)


def make_blobs(n, d, centers, seed):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-100, 100, size=(centers, d))
    lab = rng.integers(0, centers, size=n)
    return C[lab] + rng.normal(0, 1.0, size=(n, d))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def thread_cap():
    """How the CPU-all legs' thread count was set (reported in cpu_baseline: the GPU box exports
    OMP_NUM_THREADS=16, so the legs run 16 threads there although the affinity mask is larger)."""
    omp = os.environ.get("OMP_NUM_THREADS")
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    return {"affinity_cpus": aff, "omp_num_threads": int(omp) if omp and omp.isdigit() else None,
            "threads_used": host_threads(),
            "cap": (f"OMP_NUM_THREADS={omp} (set by the environment) caps the {aff}-CPU affinity mask"
                    if omp and omp.isdigit() and int(omp) < aff else f"the whole {aff}-CPU affinity mask")}


def host_threads():
    """CPU threads this process may run on (the affinity mask, not the machine's CPU count),
    capped by OMP_NUM_THREADS when set."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(aff, omp) if omp > 0 else aff


def cpu_baseline(X, budget_s=10.0):
    """Oracle (line-faithful C restatement, -O2) on a bounded sample of the same workload:
    k-NN core distances for R query rows against all n rows (n^2 work per point,
    extrapolated linearly in rows) + reference Prim on an m-point prefix (extrapolated by
    (n/m)^2); points/s = n / (t_knn_full + t_prim_full).  Timed twice: CPU-all (OpenMP over
    query rows and over each Prim step's scan, OMP_NUM_THREADS threads -- Spark local[*]'s
    stand-in) and one thread (what the reference runs at level 0).  The
    labels step (O(n log n)) is left out of both: < 0.01 % of the O(n^2) work."""
    from oracle import oracle as O
    O.lib()
    n = X.shape[0]
    threads = host_threads()

    def sample(T, budget):
        core_rows = (lambda Xs, r: O.core_rows(Xs, r, MIN_PTS)) if T == 1 else \
            (lambda Xs, r: O.core_rows_par(Xs, r, MIN_PTS, T))
        rows = np.arange(0, n, max(1, n // (64 * T)))[:64 * T]
        t0 = time.perf_counter()
        core_rows(X, rows)
        t_rows = time.perf_counter() - t0
        r2 = int(min(n, max(len(rows), len(rows) * (0.5 * budget) / max(t_rows, 1e-3))))
        rows2 = np.linspace(0, n - 1, r2).astype(np.int64)
        t0 = time.perf_counter()
        core_rows(X, rows2)
        t_knn = (time.perf_counter() - t0) * (n / len(rows2))
        prim = (lambda Xs, c: O.prim_mst(Xs, c, self_edges=False)) if T == 1 else \
            (lambda Xs, c: O.prim_mst_par(Xs, c, T))
        m = 4000
        core = O.core_rows(X[:m], np.arange(m), MIN_PTS)
        t0 = time.perf_counter()
        prim(X[:m], core)
        t_p = time.perf_counter() - t0
        m2 = int(min(60000, m * max(1.0, (0.4 * budget / max(t_p, 1e-3)) ** 0.5)))
        Xm = X[:m2]
        core = O.core_rows_par(Xm, np.arange(m2), MIN_PTS, threads)
        t0 = time.perf_counter()
        prim(Xm, core)
        t_prim = (time.perf_counter() - t0) * (n / m2) ** 2
        total = t_knn + t_prim
        return total, len(rows2), m2

    tot_all, r_all, m_all = sample(threads, budget_s)
    tot_1, r_1, m_1 = sample(1, budget_s)
    return {"value": n / tot_all, "unit": "points/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "thread_cap": thread_cap(),
            "sample": f"oracle C -O2, OpenMP {threads} threads: kNN of {r_all} query rows vs all {n} rows "
                      f"(x{n / r_all:.0f}) + reference Prim (parallel scan per step) on a {m_all}-point prefix "
                      f"(x{(n / m_all) ** 2:.0f}); extrapolated full step {tot_all:.0f} s",
            "single_thread": {"value": n / tot_1, "cores": 1,
                              "sample": f"kNN of {r_1} rows (x{n / r_1:.0f}) + Prim on a {m_1}-point prefix "
                                        f"(x{(n / m_1) ** 2:.0f}); extrapolated full step {tot_1:.0f} s"}}


C4 = dict(n=2_000_000, d=128, centers=200, noise=0.1, seed=4, min_pts=16)
MFMA_BF16_DENSE_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (no sparsity)
# HBM bytes per launch from the PMC passes of this build (FETCH_SIZE / WRITE_SIZE runs of their
# own, corrected by tools/pmc_summary.py): tools/profile_bench.sh (C2), tools/profile_c4.sh (C4)
PMC_C2 = next((p for p in (os.path.join(ROOT, "profiles", r, "final", "prof_c2", "pmc_summary.json")
                            for r in ("r06", "r05", "r04", "r03", "r02")) if os.path.exists(p)),
              os.path.join(ROOT, "profiles", "r02", "final", "prof_c2", "pmc_summary.json"))
PMC_C4 = next((p for p in (os.path.join(ROOT, "profiles", r, "c4_final", "pmc_summary.json")
                            for r in ("r06", "r05", "r04", "r03", "r02")) if os.path.exists(p)),
              os.path.join(ROOT, "profiles", "r02", "c4_final", "pmc_summary.json"))


def _pmc_bytes(path, kernel):
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh).get(kernel, {}).get("hbm_bytes_per_launch")


def run_c4(args):
    """BASELINE config 4: 2M x 128 L2-normalised embeddings, core distances over minPts = 16
    (EXCL_SELF) on the MFMA path (K1m: k-means layout, bf16-split norm-expansion screen on MFMA
    over the (query group, candidate block) pairs the FP64 balls cannot exclude, candidate log,
    exact FP64 re-check of the log; lists bit-identical to the FP64 scan).  Timed region: X in
    pinned host memory -> H2D -> core distances -> D2H of the cores (the HBM-resident rate rides
    along).  One GPU (the core distances of one
    partition; C4 names no sharding).  Roofline of the screen kernel: the MFMA flops it issues
    (3 bf16 products per pair of every computed block pair) / its time vs the dense bf16 peak;
    the all-pairs-equivalent 2 n^2 d rate rides along."""
    import torch
    pkg = importlib.import_module(PKG)
    A = importlib.import_module(PKG + "._capi")
    n = args.n if args.n != N_POINTS else C4["n"]
    d, mp = C4["d"], C4["min_pts"]
    g = torch.Generator(device="cuda").manual_seed(C4["seed"])
    C = torch.randn(C4["centers"], d, dtype=torch.float64, device="cuda", generator=g)
    lab = torch.randint(0, C4["centers"], (n,), device="cuda", generator=g)
    X = C[lab] + C4["noise"] * torch.randn(n, d, dtype=torch.float64, device="cuda", generator=g)
    X_pin = (X / torch.linalg.norm(X, dim=1, keepdim=True)).cpu().pin_memory()
    del X, C, lab
    torch.cuda.empty_cache()
    ctx = pkg.Context.get(0)
    ctx.use_torch_stream()
    core_h = torch.empty(n, dtype=torch.float64).pin_memory()
    X_res = X_pin.cuda()  # the input resident in HBM (the value's timed region starts there)

    X_bufs = [X_res, torch.empty_like(X_res)]
    h2d_s = torch.cuda.Stream()
    h2d_ev = [None, None]

    def prefetch(j):
        """step j's points from pinned host memory into buffer j % 2 on the copy stream (its
        last reader, step j - 2, is queued on the compute stream before this wait)"""
        h2d_s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(h2d_s):
            X_bufs[j % 2].copy_(X_pin, non_blocking=True)
            h2d_ev[j % 2] = torch.cuda.Event()
            h2d_ev[j % 2].record()

    def run(steps, resident):
        """steps back to back; not resident: every step uploads its 2 GB of points from pinned
        host memory (prefetched one step ahead on a copy stream, double-buffered)"""
        if not resident:
            prefetch(0)
        for i in range(steps):
            if resident:
                Xd = X_res
            else:
                torch.cuda.current_stream().wait_event(h2d_ev[i % 2])
                Xd = X_bufs[i % 2]
                if i + 1 < steps:
                    prefetch(i + 1)
            core = torch.empty(n, dtype=torch.float64, device="cuda")
            A.check(A.lib().hdb_core_distances(ctx.h, Xd.data_ptr(), n, d, mp, A.METRIC["euclidean"],
                                               A.CORE_EXCL_SELF, core.data_ptr()), "core distances")
            core_h.copy_(core, non_blocking=True)
            torch.cuda.current_stream().synchronize()  # the step's cores are on the host
        torch.cuda.synchronize()

    run(args.warmup, resident=False)
    run(1, resident=True)
    # the value: points in pinned host memory -> H2D -> K1m -> D2H of the cores
    t0 = time.perf_counter()
    run(args.steps, resident=False)
    dt = (time.perf_counter() - t0) / args.steps
    # X already resident in HBM (beside the value, never as it); its HIP events time the kernels
    ctx.set_timing(True)
    for name in ("knn_mfma", "knn_mfma_final", "knn_mfma_order"):
        ctx.kernel_time(name)
    t0 = time.perf_counter()
    run(args.steps, resident=True)
    dt_hbm = (time.perf_counter() - t0) / args.steps
    k_ms, k_calls = ctx.kernel_time("knn_mfma")
    f_ms, _ = ctx.kernel_time("knn_mfma_final")
    o_ms, _ = ctx.kernel_time("knn_mfma_order")
    ctx.set_timing(False)
    k_s = k_ms / 1e3 / args.steps  # K1m screen kernel time of one step (HIP events on its stream)
    blocks = ctx.get_stat("knn_mfma_blocks")  # (query group, 32-candidate block) pairs of the last call
    rows = ctx.get_stat("knn_mfma_group_rows")
    DP = 32 if d <= 32 else 64 if d <= 64 else 128 if d <= 128 else 256
    pairs = blocks * rows * 32
    alg = 2.0 * n * n * d
    issued = 3 * 2.0 * pairs * DP  # 3 bf16 products per computed pair (split operands)
    c = core_h.numpy()
    assert np.all(np.isfinite(c)) and np.all(c >= 0)
    line = {"metric": "points/sec end-to-end + mutual-reach distance evals/sec at 1/2/4/8 GPUs",
            "value": n / dt, "unit": "points/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64 (bf16-split MFMA screen + f64 re-check)",
            "data": f"synthetic (L2-normalised embeddings, {C4['centers']} centers + N(0, {C4['noise']}^2), seed {C4['seed']})",
            "config": {"workload": "config 4: 2M x 128 embeddings, core distances minPts 16 (EXCL_SELF) on the MFMA path",
                       "points": n, "d": d, "min_pts": mp,
                       "timed": "X in pinned host memory -> H2D (2 GB, prefetched one step ahead on a copy "
                                "stream) -> K1m core distances -> D2H of the cores"},
            "hbm_resident_points_per_s": n / dt_hbm, "hbm_resident_ms_per_step": dt_hbm * 1e3,
            "hbm_resident_kind": "the same steps from X already resident in HBM (no H2D; not the value)",
            "mrd_evals_per_s": pairs / dt,
            "mrd_evals_per_s_kind": "executed: (query, candidate) pairs the MFMA screen computes, over the step time",
            "all_pairs_equivalent_evals_per_s": n * (n - 1) / dt,
            "roofline": {"bound": "mfma", "kernel": "knn_mfma_screen_kernel (K1m)", "achieved": issued / k_s / 1e12,
                         "peak": MFMA_BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                         "frac": issued / k_s / 1e12 / MFMA_BF16_DENSE_TFLOPS,
                         "traffic": _pmc_bytes(PMC_C4, "knn_mfma_screen_kernel"),
                         "traffic_source": os.path.relpath(PMC_C4, ROOT),
                         "hbm": {"achieved_gbs": (_pmc_bytes(PMC_C4, "knn_mfma_screen_kernel") or 0.0)
                                 / (k_s / max(k_calls / args.steps, 1)) / 1e9, "peak": 8000.0},
                         "work": "issued: 3 bf16 MFMA products x 2 DP flops per computed (query, candidate) pair",
                         "computed_pair_frac": pairs / (n * n), "all_pairs_equivalent_tflops": alg / k_s / 1e12,
                         "kernel_s_per_step": k_s, "launches_per_step": k_calls / args.steps,
                         "order_s_per_step": o_ms / 1e3 / args.steps, "recheck_s_per_step": f_ms / 1e3 / args.steps}}
    if not args.no_cpu_baseline:
        from oracle import oracle as O
        O.lib()
        threads = host_threads()
        Xh = X_pin.numpy()
        rows = np.linspace(0, n - 1, 16 * threads).astype(np.int64)
        t0 = time.perf_counter()
        O.core_rows_par(Xh, rows, mp, threads)
        t_r = time.perf_counter() - t0
        full = t_r * n / rows.shape[0]
        line["cpu_baseline"] = {"value": n / full, "unit": "points/s", "cores": threads, "kind": "port",
                                "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
                                "sample": f"oracle C -O2, OpenMP {threads} threads: core distances of {rows.shape[0]} "
                                          f"query rows vs all {n} rows (x{n / rows.shape[0]:.0f}); "
                                          f"extrapolated full step {full:.0f} s"}
    emit(line)


PARTITIONED = {  # SURVEY.md §8(d) C3 / C5 (recursive sampling, data bubbles), strong scaling
    "c3": dict(n=4_000_000, d=16, centers=50, spread=50.0, seed=3, samples_per_subset=4096, processing_units=65536,
               desc="config 3: blobs 4M x 16, recursive sampling (4,096 samples/subset, pu 65,536)"),
    "c5": dict(n=16_000_000, d=8, centers=100, spread=100.0, seed=5, samples_per_subset=16384,
               processing_units=65536,
               desc="config 5: blobs 16M x 8, data bubbles (16,384 samples/subset, pu 65,536), RCCL merge"),
}


TIMED_KERNELS = ("prim_coop", "prim_block", "prim_step_total", "knn_tree", "boruvka_scan", "boruvka_total",
                 "leaf_core", "knn_generic", "nearest_grouped", "nearest_sq", "nearest_generic", "bubble_knn",
                 "bubble_stats", "merge_sort", "merge_edges", "flat_labels")
# K2b's launches sit inside boruvka_total; exact_leaf_total / boruvka_total nest other timers
NESTED = {"boruvka_scan"}


def boruvka_roofline(scan_s, bound_s, evals, d):
    """The K2b scan (boruvka_bvh_kernel) on the job's forced leaves above prim_leaf_max: the C2
    line's latency model -- per round, visits x 227 ns (one dependent Infinity-Cache round trip
    per node or leaf visit) / min(waves, resident wave slots) -- summed over every round of every
    leaf in a count_evals pass of the same job (boruvka_bound_ns_sum), over the scan's HIP-event
    time in the timed jobs; the FP64 fraction of the executed pair evals rides along."""
    fp64 = 3 * d * evals / scan_s / 1e12 if scan_s > 0 else 0.0
    return {"bound": "latency", "kernel": "boruvka_bvh_kernel (K2b scan, forced leaves)", "unit": "s",
            "achieved": scan_s, "peak": bound_s, "frac": bound_s / scan_s if scan_s > 0 else 0.0, "traffic": None,
            "model": f"per round: visits x {MALL_HIT_NS:.0f} ns / min(waves, {WAVE_SLOTS} resident wave slots), "
                     "summed over every round of every forced leaf (count_evals pass)",
            "fp64": {"achieved_tflops": fp64, "peak": FP64_PEAK_TFLOPS, "frac": fp64 / FP64_PEAK_TFLOPS,
                     "work": "executed pair evals x 3d flops"}}


def partitioned_roofline(kt, coop_steps, coop_launches, steps):
    """Latency roofline of the cooperative Prim (prim_coop: the bubble models' and the big
    leaves' reference Prim, the level loop's critical path): every Prim step needs at least
    one inter-workgroup exchange through the device-coherent cache -- the winner's key
    published by a store and observed by a load of every workgroup, two dependent
    Infinity-Cache round trips (MI355X_MICROARCH.md: 227 ns each).  Lower bound = steps x
    2 x 227 ns; frac = bound / measured prim_coop time."""
    t = kt.get("prim_coop", [0.0, 0])[0] / steps
    s = coop_steps / steps
    bound = s * 2 * MALL_HIT_NS * 1e-9
    top = max(((k, v[0]) for k, v in kt.items() if k not in NESTED), key=lambda x: x[1], default=(None, 0.0))
    return {"bound": "latency", "kernel": "prim_coop4_kernel (cooperative reference Prim, HdbscanDataBubbles.java:"
                                          "165-254 / HDBSCANStar.java:124-205)",
            "unit": "Prim steps/s", "achieved": s / t if t > 0 else 0.0,
            "peak": 1.0 / (2 * MALL_HIT_NS * 1e-9), "frac": bound / t if t > 0 else 0.0, "traffic": None,
            "model": "per step: 2 dependent Infinity-Cache round trips (publish the workgroup minimum, observe "
                     f"every workgroup's) x {MALL_HIT_NS:.0f} ns",
            "steps_per_job": s, "launches_per_job": coop_launches / steps, "kernel_s_per_job": t,
            "us_per_step": t / s * 1e6 if s else None,
            "dominant_kernel": top[0], "dominant_kernel_s": top[1] / steps}


CPU_SAMPLES = {  # the partitioned configs' family at a size the serial oracle runs in ~10-30 s
    "c3": dict(n=50_000, d=16, centers=50, spread=50.0, seed=3, samples_per_subset=512, processing_units=4096),
    "c5": dict(n=50_000, d=8, centers=100, spread=100.0, seed=5, samples_per_subset=1024, processing_units=4096),
}


def cpu_sample_instance(workload):
    cs = CPU_SAMPLES[workload]
    rng = np.random.default_rng(cs["seed"])
    C = rng.uniform(-cs["spread"], cs["spread"], size=(cs["centers"], cs["d"]))
    return cs, C[rng.integers(0, cs["centers"], size=cs["n"])] + rng.normal(0, 1.0, size=(cs["n"], cs["d"]))


def partitioned_cpu_baseline(workload, gpu_run=None):
    """The oracle's MR-HDBSCAN* loop (oracle/mr_driver.py over hdb_oracle.c, -O2) on a 50k-point
    instance of the config's family (samples per subset and processing_units scaled down with
    it; flat labels left out: the reference never computes them), timed twice on the same
    instance: CPU-all -- a thread pool of the affinity mask's threads over each level's
    independent subsets and the nearest-sample row chunks (Spark local[*]'s stand-in, one task
    per subset, Main.java:89,166-169) -- and one thread (setMaster("local"), what the reference
    runs).  gpu_run(X, cs) -> seconds: the device driver on the same instance, so the three
    rates compare like for like (the loop is superlinear in n: the full-size CPU rate would be
    lower still)."""
    from oracle import mr_driver as M
    cs, X = cpu_sample_instance(workload)
    threads = host_threads()
    kw = dict(min_pts=MIN_PTS, min_cl_size=MIN_CL_SIZE, processing_units=cs["processing_units"],
              samples_per_subset=cs["samples_per_subset"], flat=False)
    t0 = time.perf_counter()
    r = M.run(X, workers=threads, **kw)
    dt_all = time.perf_counter() - t0
    t0 = time.perf_counter()
    M.run(X, **kw)
    dt_1 = time.perf_counter() - t0
    inst = (f"{cs['n']} x {cs['d']} blobs ({cs['centers']} centres, seed {cs['seed']}), samples/subset "
            f"{cs['samples_per_subset']}, processing_units {cs['processing_units']}, {r['iterations']} levels")
    out = {"value": cs["n"] / dt_all, "unit": "points/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
           "affinity_cpus": len(os.sched_getaffinity(0)), "thread_cap": thread_cap(),
           "sample": f"oracle MR-HDBSCAN* loop (mr_driver, C -O2), thread pool of {threads} over each level's "
                     f"subsets and nearest-sample row chunks, on {inst}: {dt_all:.1f} s",
           "single_thread": {"value": cs["n"] / dt_1, "cores": 1, "sample": f"the same instance, 1 thread: {dt_1:.1f} s"}}
    if gpu_run is not None:
        dt_g = gpu_run(X, cs)
        out["gpu_same_instance"] = {"value": cs["n"] / dt_g, "unit": "points/s",
                                    "sample": f"the device driver on the same instance (1 GPU, flat labels included): "
                                              f"{dt_g * 1e3:.1f} ms"}
    return out


def predicted_scaling(drv, par, ns=(1, 2, 4, 8)):
    """C3/C5 --phases: the sharded driver's critical path at N ranks predicted from the tasks
    measured at N = 1.  Per level: leaves and local models are assigned to ranks by the
    driver's own LPT on its own weights (n^2, b^2); a rank's phase time = the summed measured
    durations of its tasks x (phase wall time / summed task time at N = 1: the concurrency the
    model threads reach on one GPU), the phase = its slowest rank; the point-chunked nearest
    sample scales as 1/N, so do the bubble statistics' slice partials (D11: bubble_slices
    slices, a rank folds its own); their merge, bookkeeping, the merge of the edge lists and the
    flat labels do not scale.  The driver's deferred leaves (every level's leaves in one
    batch after the level loop) are one more "level" holding only leaves, so their LPT runs
    over the whole job.  Not modelled: the all-gathers and the RCCL merge exchange."""
    fixed = sum(v for k, v in drv.timings.items() if k in ("bookkeeping", "merge", "flat_labels"))
    out, per, lpt_model = {}, {}, {}
    for N in ns:
        tot = {"leaves": 0.0, "local_models": 0.0, "nearest_sample": 0.0, "bubbles": 0.0}
        lpt_tot = 0.0  # round 3-5's estimate, kept beside: N = 1 task times x the one-device concurrency
        for L in drv.level_tasks:
            ph = L["phase_s"]
            for kind in ("leaves", "local_models"):
                tasks = L.get(kind, [])
                wall = ph.get(kind, 0.0)
                work = sum(t for _, t in tasks)
                em = L.get("emulated_" + kind, {})
                if not tasks or work <= 0:
                    est = wall
                else:
                    owner = par.lpt([w for w, _ in tasks], N)
                    load = np.zeros(N)
                    for (w, t), o in zip(tasks, owner):
                        load[o] += t
                    est = float(load.max()) * wall / work
                lpt_tot += est
                # emulated: every rank's LPT share run on its own (driver emulate_ranks)
                tot[kind] += wall if N == 1 else em.get(N, est)
            tot["nearest_sample"] += ph.get("nearest_sample", 0.0) / N
            # D11: the slice partials shard over the ranks (a rank folds its slices); the merge
            # of the gathered partials and the host copy of rep / info do not
            tot["bubbles"] += (ph.get("bubble_partials", 0.0) / min(N, getattr(drv, "bubble_slices", 1))
                               + ph.get("bubbles", 0.0))
        per[N] = {k: round(v, 3) for k, v in tot.items()} | {"fixed": round(fixed, 3)}
        out[N] = sum(tot.values()) + fixed
        lpt_model[N] = out[N] - tot["leaves"] - tot["local_models"] + lpt_tot
    emulated = any("emulated_local_models" in L for L in drv.level_tasks)
    return {"model": ("local models and leaves EMULATED per level: each of the N ranks' LPT share run on its "
                      "own on this GPU, the slowest rank counted (driver emulate_ranks); " if emulated else
                      "LPT makespan of the measured N=1 task durations x the one-device concurrency per level; ") +
                     "nearest sample / N, bubble slice partials / min(N, slices), their merge + "
                     "bookkeeping + merge + flat labels unscaled; "
                     "all-gathers and the RCCL merge exchange not modelled",
            "seconds": {str(N): round(v, 3) for N, v in out.items()},
            "speedup": {str(N): round(out[1] / v, 2) for N, v in out.items()},
            "phases": {str(N): v for N, v in per.items()},
            "lpt_concurrency_estimate": {"speedup": {str(N): round(out[1] / v, 2) for N, v in lpt_model.items()},
                                         "note": "rounds 3-5's model: N = 1 task durations (measured while the "
                                                 "model pool shares the GPU) x that level's one-device concurrency "
                                                 "factor -- optimistic when a rank holds one or two models, which "
                                                 "then run at their own latency-bound speed"}}


def run_partitioned(args, workload):
    """C3 / C5: the whole MR-HDBSCAN* job (every level, the merge, the flat labels) on N GPUs
    with the sharded driver; every rank holds the parsed points (pinned host memory), the
    timed region covers H2D, the job and the D2H of the merged list and labels.  Strong
    scaling: the same job at every N; value = points / job time."""
    import torch
    import torch.distributed as dist
    os.environ.setdefault("HDB_KERNEL_TIMING", "1")  # every context (model threads too) times its kernels
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    pkg = importlib.import_module(PKG)
    A = importlib.import_module(PKG + "._capi")
    cfg = PARTITIONED[workload]
    n = args.n if args.n != N_POINTS else cfg["n"]
    rng = np.random.default_rng(cfg["seed"])
    C = rng.uniform(-cfg["spread"], cfg["spread"], size=(cfg["centers"], cfg["d"]))
    X_pin = torch.from_numpy(C[rng.integers(0, cfg["centers"], size=n)] +
                             rng.normal(0, 1.0, size=(n, cfg["d"]))).pin_memory()
    drv = pkg.MRHDBSCANStar(minPts=MIN_PTS, minClSize=MIN_CL_SIZE, processing_units=cfg["processing_units"],
                            samples_per_subset=cfg["samples_per_subset"], profile=args.phases)
    out = {}

    if os.environ.get("HDB_WATCHDOG"):  # diagnosis: every thread's Python stack every N s
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["HDB_WATCHDOG"]))  # re-armed per level

    def job():
        Xd = X_pin.to("cuda", non_blocking=True)
        r = drv.run(Xd)
        if rank == 0:
            out["edges"] = [x.to("cpu") for x in r["edges"]]
            out["labels"] = r["labels"].to("cpu")
        out["r"] = r
        torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def kernel_totals(reset=True):
        """summed device time (s) and launches per timed kernel over every context (driver
        thread + model threads), HIP events on each context's stream"""
        tot = {}
        for c in list(A.Context._all):
            for k in TIMED_KERNELS:
                ms, calls = c.kernel_time(k, reset)
                if calls:
                    a = tot.setdefault(k, [0.0, 0])
                    a[0] += ms / 1e3
                    a[1] += calls
        return tot

    def stat_total(name, reset_to=None):
        return sum(c.get_stat(name) for c in list(A.Context._all))

    for _ in range(args.warmup):
        job()
    barrier()
    kernel_totals()
    steps0 = stat_total("prim_coop_steps")
    launches0 = stat_total("prim_coop_launches")
    retries0 = stat_total("prim_coop_plain_retries")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job()
    barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    r = out["r"]
    kt = kernel_totals()
    coop_steps = stat_total("prim_coop_steps") - steps0
    coop_launches = stat_total("prim_coop_launches") - launches0
    coop_retries = stat_total("prim_coop_plain_retries") - retries0
    # diagnostic pass (outside the timed region): per-round visits / waves of every K2b scan
    for c in list(A.Context._all):
        c.set_option("count_evals", 1)
    b0 = {k: stat_total(k) for k in ("boruvka_bound_ns_sum", "boruvka_evals_sum")}
    job()
    barrier()
    for c in list(A.Context._all):
        c.set_option("count_evals", 0)
    if args.phases and world == 1:
        # one more untimed job for predicted_scaling: the real phases plus every level's local
        # models and the deferred leaves re-run as 2, 4 and 8 ranks would run them (emulate_ranks)
        drv.emulate_ranks = (2, 4, 8)
        job()
        barrier()
        drv.emulate_ranks = ()
    k2b_roof = boruvka_roofline(kt.get("boruvka_scan", [0.0, 0])[0] / args.steps,
                                (stat_total("boruvka_bound_ns_sum") - b0["boruvka_bound_ns_sum"]) * 1e-9,
                                stat_total("boruvka_evals_sum") - b0["boruvka_evals_sum"], cfg["d"])
    if rank == 0:
        w = out["edges"][2].numpy()
        assert w.shape[0] == 2 * n - 1 and np.all(w[:-1] >= w[1:])
        lv = r["levels"]
        line = {"metric": "points/sec end-to-end + mutual-reach distance evals/sec at 1/2/4/8 GPUs",
                "value": n * args.steps / dt, "unit": "points/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "f64",
                "data": f"synthetic (seeded Gaussian blobs, seed {cfg['seed']})",
                "config": {"workload": cfg["desc"], "points": n, "d": cfg["d"], "min_pts": MIN_PTS,
                           "min_cl_size": MIN_CL_SIZE, "prim_leaf_max": drv.prim_leaf_max,
                           "model_threads": drv.model_threads, "bubble_slices": drv.bubble_slices,
                           "parallelism": f"sharded driver x{world} (leaves/local models by LPT, "
                                          f"point-chunked nearest sample, sliced bubble partials, RCCL merge)"},
                "iterations": r["iterations"], "n_clusters": r["n_clusters"],
                "levels": len(lv), "leaves": int(sum(len(L["leaves"]) for L in lv)),
                "model_errors": int(sum(len(L.get("model_errors", {})) for L in lv)),
                "phases_s": {k: round(v, 4) for k, v in drv.timings.items()} if args.phases else None,
                "local_model_s": ({k: round(A.Context.stat_total("lm_" + k + "_us") / 1e6, 3) for k in
                                   ("core", "prim", "quicksort", "tree", "fosc", "fosc_select", "fosc_label",
                                    "fosc_noise")} |
                                  {"calls": A.Context.stat_total("lm_calls")}) if args.phases else None,
                "kernels_s": {k: round(v[0] / args.steps, 4) for k, v in sorted(kt.items(), key=lambda x: -x[1][0])},
                "kernel_launches": {k: v[1] // args.steps for k, v in kt.items()},
                "prim_coop_plain_retries": coop_retries,
                "bubble_knn_replay_overflows": stat_total("bubble_knn_replay_overflows"),
                "predicted_scaling": predicted_scaling(drv, importlib.import_module(PKG + ".parallel"))
                if args.phases and world == 1 else None,
                "roofline": partitioned_roofline(kt, coop_steps, coop_launches, args.steps)}
        line["roofline"]["boruvka"] = k2b_roof
        dom = line["roofline"]["dominant_kernel"]
        if dom in ("boruvka_total", "boruvka_scan", "exact_leaf_total") and k2b_roof["achieved"] > 0:
            # the dominant kernel is K2b: the line's top-level roofline is K2b's, the Prim's rides along
            prim_roof = {k: v for k, v in line["roofline"].items() if k != "boruvka"}
            line["roofline"] = dict(k2b_roof) | {"dominant_kernel": dom, "dominant_kernel_s": prim_roof["dominant_kernel_s"],
                                                 "prim_coop": prim_roof}
        if world == 1 and not args.no_cpu_baseline:
            def gpu_run(Xs, cs):
                d2 = pkg.MRHDBSCANStar(minPts=MIN_PTS, minClSize=MIN_CL_SIZE, processing_units=cs["processing_units"],
                                       samples_per_subset=cs["samples_per_subset"])
                Xp = torch.from_numpy(Xs).pin_memory()
                best = None
                for i in range(3):  # the first run warms the instance's kernels; best of the other two
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    r2 = d2.run(Xp.to("cuda", non_blocking=True))
                    [x.to("cpu") for x in r2["edges"]]
                    r2["labels"].to("cpu")
                    torch.cuda.synchronize()
                    dt2 = time.perf_counter() - t0
                    if i:
                        best = dt2 if best is None else min(best, dt2)
                return best
            line["cpu_baseline"] = partitioned_cpu_baseline(workload, gpu_run)
        emit(line)
    if world > 1:
        dist.destroy_process_group()


# Definitions of the line's keys changed in round 4: `value` includes the
# pinned-host H2D (round 3: HBM-resident inputs), the HBM-resident rate is `hbm_resident_*`
# (round 3's `pcie_inclusive_*` meant the opposite), and C4's `mrd_evals_per_s` counts executed
# screen pairs (the all-pairs-equivalent rate is `all_pairs_equivalent_evals_per_s`).
LINE_SCHEMA = 4
LINE_SCHEMA_NOTE = ("v4 (since round 4): value includes the pinned-host H2D; hbm_resident_* = HBM-resident "
                    "inputs (r03's pcie_inclusive_* meant the opposite); C4 mrd_evals_per_s = executed screen pairs")


def emit(line):
    line = dict(line, schema=LINE_SCHEMA, schema_note=LINE_SCHEMA_NOTE)
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 30 (c2), 5 (c4), 1 (c3/c5)")
    ap.add_argument("--warmup", type=int, default=None, help="default 5 (c2), 2 (c4), 0 (c3/c5)")
    ap.add_argument("--n", type=int, default=N_POINTS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5"], default="c2",
                    help="c2 (default): the per-GPU C2 pipeline (weak scaling); c3/c5: the whole "
                         "partitioned job over the sharded driver (strong scaling)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group for N>1 (gloo: rehearse several ranks on one device)")
    ap.add_argument("--phases", action="store_true", help="c3/c5: per-phase times (synchronising)")
    ap.add_argument("--mst-workers", type=int, default=int(os.environ.get("HDB_BENCH_MST_WORKERS", "5")),
                    help="c2: partitions in flight in stage 1 (one thread, context and stream each)")
    ap.add_argument("--label-workers", type=int, default=int(os.environ.get("HDB_BENCH_LABEL_WORKERS", "2")),
                    help="c2: label stages (0: as many as --mst-workers)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = {"c2": 30, "c4": 5}.get(args.workload, 1)
    if args.warmup is None:
        args.warmup = {"c2": 5, "c4": 2}.get(args.workload, 0)
    if args.workload == "c4":
        return run_c4(args)
    if args.workload != "c2":
        return run_partitioned(args, args.workload)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "gloo":
        local = 0  # rehearsal: every rank on device 0
    if world > 1:
        dist.init_process_group(args.backend, **({"device_id": torch.device("cuda", local)}
                                                 if args.backend == "nccl" else {}))
    torch.cuda.set_device(local)
    pkg = importlib.import_module(PKG)
    par = importlib.import_module(PKG + ".parallel")

    n = args.n
    X_host = make_blobs(n, D, CENTERS, seed=1 + rank)
    X_pin = torch.from_numpy(X_host).pin_memory()      # parsed points in host memory
    X_dev = torch.empty(X_pin.shape, dtype=X_pin.dtype, device="cuda")
    X_res = X_pin.cuda()                               # HBM-resident copy (device-only line)
    ne_local = 2 * n - 1
    ne_out = world * ne_local if rank == 0 else 0
    va_h = torch.empty(ne_out, dtype=torch.int32).pin_memory()
    vb_h = torch.empty(ne_out, dtype=torch.int32).pin_memory()
    w_h = torch.empty(ne_out, dtype=torch.float64).pin_memory()
    lab_h = torch.empty(n, dtype=torch.int32).pin_memory()
    ctx = pkg.Context.get(local)
    ctx.use_torch_stream()
    star = pkg.HDBSCANStar(ctx)
    n_clusters = [0]
    copy_s = torch.cuda.Stream()

    def leaf(X):
        """FirstStep's leaf (cores + exact MST + self edges), its edge list handed over in the
        reducers' merge order (SortMST: stable descending) -- hdb_exact_mst's HDB_EDGES_MERGED,
        identical to sorting the plain list with hdb_sort_edges_desc"""
        _, mst = star.exactMST(X, MIN_PTS, None, pkg.CORE_EXCL_SELF, True, merged=True)
        return mst.getVerticeA(), mst.getVericeB(), mst.getEges()

    def merge(va, vb, w):
        """the reducers' merge: N=1 the leaf's list is already in merge order; N>1 rank 0
        merges every rank's presorted list (hdb_merge_sorted_runs)"""
        if world > 1:
            return (va, vb, w), par.gather_sorted_msts(va, vb, w, dst=0)
        return (va, vb, w), (va, vb, w)

    def step_e2e():
        X_dev.copy_(X_pin, non_blocking=True)                    # H2D
        own, merged = merge(*leaf(X_dev))
        main = torch.cuda.current_stream()
        if rank == 0:  # D2H of the merged list on a copy stream, overlapping the labels
            ma, mb, mw = merged
            copy_s.wait_stream(main)
            with torch.cuda.stream(copy_s):
                va_h.copy_(ma, non_blocking=True)
                vb_h.copy_(mb, non_blocking=True)
                w_h.copy_(mw, non_blocking=True)
        lab, n_clusters[0] = pkg.flat_labels(*own, n, MIN_CL_SIZE, ctx=ctx)  # this partition's labels
        lab_h.copy_(lab, non_blocking=True)
        main.synchronize()
        copy_s.synchronize()

    class LabelStage:
        """Stage 2 of the step pipeline, on its own thread, HIP stream and library context:
        partition i's K6 flat labels and the D2H of its merged list and labels run while the
        main thread runs partition i+1's H2D, MST and merge (the library's ctypes calls release
        the GIL).  Every step still does all of its work; the timer stops after the last
        step's stage 2 has finished."""

        def __init__(self, bufs):
            self.bufs = bufs  # this stage's pinned host buffers (merged va, vb, w; labels)
            self.q = queue.Queue(maxsize=1)
            self.err = None
            self.ready = threading.Event()
            self.t = threading.Thread(target=self._run, daemon=True)
            self.t.start()
            self.ready.wait()

        def _run(self):
            torch.cuda.set_device(local)
            prio = int(os.environ.get("HDB_BENCH_STAGE2_PRIO", "0"))  # A/B knob: -1 = high priority
            s, cs = torch.cuda.Stream(priority=prio), torch.cuda.Stream(priority=prio)
            with torch.cuda.stream(s):
                self.ctx = pkg.Context.get(local)  # thread-local: a second context
                self.ctx.use_torch_stream()
                self.ready.set()
                while True:
                    job = self.q.get()
                    if job is None:
                        self.q.task_done()
                        return
                    try:
                        ev, own, merged = job
                        s.wait_event(ev)
                        if merged is not None:  # rank 0: D2H of the merged list beside the labels
                            cs.wait_event(ev)
                            with torch.cuda.stream(cs):
                                self.bufs[0].copy_(merged[0], non_blocking=True)
                                self.bufs[1].copy_(merged[1], non_blocking=True)
                                self.bufs[2].copy_(merged[2], non_blocking=True)
                        lab, k = pkg.flat_labels(*own, n, MIN_CL_SIZE, ctx=self.ctx)
                        self.bufs[3].copy_(lab, non_blocking=True)
                        s.synchronize()
                        cs.synchronize()
                        n_clusters[0] = k
                    except BaseException as e:  # re-raised on the main thread
                        self.err = e
                    finally:
                        job = own = merged = lab = None
                        self.q.task_done()

        def submit(self, own, merged):
            if self.err is not None:
                raise self.err
            ev = torch.cuda.Event()
            ev.record()  # the main stream's MST + merge of this partition
            self.q.put((ev, own, merged))

        def drain(self):
            self.q.join()
            if self.err is not None:
                raise self.err

        def close(self):
            self.q.put(None)
            self.t.join()

    class MstWorkers:
        """Stage 1 on M threads (own library context and HIP stream each): partition i's exact
        MST (K1t cores -> K2b Boruvka + self edges) and its sort run on worker i % M, so one
        partition's latency-bound Boruvka rounds overlap the next partition's k-NN.  Results
        are taken in step order; the N>1 gather (a collective) stays on the main thread, in step
        order on every rank."""

        def __init__(self, m):
            self.m = m
            self.qs = [queue.Queue() for _ in range(m)]
            self.res = {}
            self.cv = threading.Condition()
            self.ctxs = [None] * m
            self.ready = threading.Barrier(m + 1)
            self.ts = [threading.Thread(target=self._run, args=(j,), daemon=True) for j in range(m)]
            for t in self.ts:
                t.start()
            self.ready.wait()

        def _run(self, j):
            torch.cuda.set_device(local)
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                c = pkg.Context.get(local)  # thread-local: this worker's own context
                c.use_torch_stream()
                st = pkg.HDBSCANStar(c)
                self.ctxs[j] = c
                self.ready.wait()
                Xw = torch.empty_like(X_res)  # this worker's point buffer (H2D target)
                while True:
                    job = self.qs[j].get()
                    if job is None:
                        return
                    i, resident = job
                    try:
                        if not resident:  # the step's points uploaded from pinned host memory
                            Xw.copy_(X_pin, non_blocking=True)
                        _, mst = st.exactMST(X_res if resident else Xw, MIN_PTS, None, pkg.CORE_EXCL_SELF, True,
                                             merged=True)
                        own = (mst.getVerticeA(), mst.getVericeB(), mst.getEges())
                        ev = torch.cuda.Event()
                        ev.record()
                        out = (ev, own)
                    except BaseException as e:  # re-raised on the main thread
                        out = e
                    with self.cv:
                        self.res[i] = out
                        self.cv.notify_all()

        def submit(self, i, resident):
            self.qs[i % self.m].put((i, resident))

        def result(self, i):
            with self.cv:
                self.cv.wait_for(lambda: i in self.res)
                out = self.res.pop(i)
            if isinstance(out, BaseException):
                raise out
            return out

        def close(self):
            for q in self.qs:
                q.put(None)
            for t in self.ts:
                t.join()

    M = max(1, args.mst_workers)
    workers = MstWorkers(M) if M > 1 else None

    class LabelStages:
        """L label stages (one thread, context and stream each), steps dealt round-robin: with
        several partitions in flight in stage 1 one label stage becomes the bottleneck.  Stage
        0 writes the host buffers the final checks read; the others have their own."""

        def __init__(self, nl):
            pin = lambda t: t.pin_memory()
            self.st = [LabelStage((va_h, vb_h, w_h, lab_h) if j == 0 else
                                  (pin(torch.empty_like(va_h)), pin(torch.empty_like(vb_h)),
                                   pin(torch.empty_like(w_h)), pin(torch.empty_like(lab_h)))) for j in range(nl)]
            self.ctxs = [x.ctx for x in self.st]
            self.k = 0

        def submit(self, own, merged):
            self.st[self.k % len(self.st)].submit(own, merged)
            self.k += 1

        def drain(self):
            for x in self.st:
                x.drain()

        def close(self):
            for x in self.st:
                x.close()

    L = max(1, args.label_workers if args.label_workers else M)
    stage = LabelStages(L)
    # H2D of step i+1's points on a copy stream during step i's MST (two point buffers)
    X_bufs = [X_dev, torch.empty_like(X_dev)]
    h2d_s = torch.cuda.Stream()
    h2d_ev = [None, None]
    pipe = {"next": 0, "end": 0}

    def prefetch(j):
        h2d_s.wait_stream(torch.cuda.current_stream())  # buffer j % 2's last reader (step j - 2) is queued before
        with torch.cuda.stream(h2d_s):
            X_bufs[j % 2].copy_(X_pin, non_blocking=True)
            h2d_ev[j % 2] = torch.cuda.Event()
            h2d_ev[j % 2].record()

    def pipe_run(steps, resident=False):
        """`steps` pipelined steps; returns when the last one's labels are on the host.
        resident: the points are already in HBM (no H2D: the value's timed region);
        otherwise every step uploads its points from pinned host memory first"""
        i0 = pipe["next"]
        if workers is not None:  # M partitions in flight in stage 1 (each uploads its own points)
            for i in range(i0, min(i0 + M, i0 + steps)):
                workers.submit(i, resident)
            for i in range(i0, i0 + steps):
                ev, own = workers.result(i)
                if i + M < i0 + steps:
                    workers.submit(i + M, resident)
                torch.cuda.current_stream().wait_event(ev)
                merged = par.gather_sorted_msts(*own, dst=0) if world > 1 else own
                stage.submit(own, merged if rank == 0 else None)
            pipe["next"] = i0 + steps
            stage.drain()
            return
        if not resident:
            prefetch(i0)
        for i in range(i0, i0 + steps):
            if not resident:
                torch.cuda.current_stream().wait_event(h2d_ev[i % 2])
                if i + 1 < i0 + steps:
                    prefetch(i + 1)
            own, merged = merge(*leaf(X_res if resident else X_bufs[i % 2]))
            stage.submit(own, merged if rank == 0 else None)
        pipe["next"] = i0 + steps
        stage.drain()

    def step_dev():
        return merge(*leaf(X_res))[1]

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64, device="cuda" if args.backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    pipe_run(args.warmup)
    pipe_run(1, resident=True)  # the HBM-resident path warm too
    barrier()
    # the value: every step's points uploaded from pinned host memory inside the timed region
    # (from parsed points resident in host memory)
    t0 = time.perf_counter()
    pipe_run(args.steps)
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    # the same pipeline from points already resident in HBM (reported beside the value, never as it)
    barrier()
    t0 = time.perf_counter()
    pipe_run(args.steps, resident=True)
    barrier()
    dt_hbm = max_over_ranks(time.perf_counter() - t0)
    stage.close()
    if workers is not None:
        workers.close()
    # latency of one step without the pipeline (each step's stages back to back); its HIP
    # events time the flat labels of one partition alone
    keys = ("knn_tree", "boruvka_total", "boruvka_scan")
    step_e2e()
    barrier()
    ctx.set_timing(True)
    ctx.kernel_time("flat_labels")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_e2e()
    barrier()
    dt_lat = max_over_ranks(time.perf_counter() - t0)
    kt_lab = ctx.kernel_time("flat_labels")
    ctx.set_timing(False)
    # the same pipeline from HBM-resident points to HBM-resident merged edges, one partition at
    # a time: its HIP events time each kernel alone (the roofline's kernel duration; in the
    # pipelined region several partitions overlap and an event pair also spans other streams')
    step_dev()
    barrier()
    ctx.set_timing(True)
    for k in keys:
        ctx.kernel_time(k)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step_dev()
    barrier()
    dt_dev = max_over_ranks(time.perf_counter() - t0)
    kt_seq = {k: ctx.kernel_time(k) for k in keys}
    ctx.set_timing(False)
    tsteps = args.steps

    # checks on the last end-to-end step's host outputs
    if rank == 0:
        w_np = w_h.numpy()
        assert w_np.shape[0] == world * ne_local and np.all(w_np[:-1] >= w_np[1:]), "merged list not descending"
        if world == 1:
            from scipy.sparse import coo_matrix
            from scipy.sparse.csgraph import connected_components
            a, b = va_h.numpy(), vb_h.numpy()
            t = a != b
            assert int(t.sum()) == n - 1, "not n-1 tree edges"
            k, _ = connected_components(coo_matrix((np.ones(n - 1), (a[t], b[t])), shape=(n, n)), directed=False)
            assert k == 1, "tree edges do not span the points"
    lab_np = lab_h.numpy()
    assert lab_np.min() >= 0 and lab_np.max() == n_clusters[0]

    # executed work (diagnostic pass outside the timed region): per-round traversal stats
    ctx.set_option("count_evals", 1)
    leaf(X_res)
    knn_evals = ctx.get_stat("knn_tree_evals")
    bor_evals = ctx.get_stat("boruvka_evals")
    rounds = []
    for r in range(64):
        try:
            visits = ctx.get_stat(f"boruvka_r{r}_nodes") + ctx.get_stat(f"boruvka_r{r}_leaves")
            waves = ctx.get_stat(f"boruvka_r{r}_active_waves")
        except Exception:
            break
        rounds.append((visits, waves))
    ctx.set_option("count_evals", 0)

    total_points = world * n
    value = total_points * tsteps / dt
    # per-partition kernel times, each kernel alone (one partition at a time: the device-resident
    # pass for stage 1, the latency pass for the labels)
    ms = {k: v[0] / tsteps for k, v in kt_seq.items()} | {"flat_labels": kt_lab[0] / tsteps}
    scan_ms, scan_n = kt_seq["boruvka_scan"]
    avg_scan_s = scan_ms / max(scan_n, 1) / 1e3
    # Latency roofline of the dominant kernel (the K2b scan): every node or leaf visit needs
    # at least one dependent round trip to the index (L2/Infinity-Cache resident, MALL-hit
    # latency), and a round can keep at most min(its waves, resident wave slots) of them in
    # flight.  Lower bound per round = visits x latency / min(waves, slots); frac = the sum of
    # those bounds / the measured scan time.
    t_min = sum(v * MALL_HIT_NS * 1e-9 / max(1, min(w, WAVE_SLOTS)) for v, w in rounds if v)
    visits = sum(v for v, _ in rounds)
    scan_s_step = scan_ms / tsteps / 1e3
    achieved = visits / scan_s_step if scan_s_step > 0 else 0.0
    peak = visits / t_min if t_min > 0 else 0.0
    traffic = None
    traffic = _pmc_bytes(PMC_C2, "boruvka_bvh_kernel")
    fp64_tflops = 3 * D * (bor_evals / max(scan_n / tsteps, 1)) / avg_scan_s / 1e12 if avg_scan_s > 0 else 0.0
    evals = world * (n * n + n * (n - 1) / 2)  # kNN n^2 + MST n(n-1)/2
    line = {
        "metric": "points/sec end-to-end + mutual-reach distance evals/sec at 1/2/4/8 GPUs",
        "value": value,
        "unit": "points/s",
        "n_gpus": world,
        "steps": tsteps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / tsteps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded Gaussian blobs, 20 centers ~U[-100,100]^3, sigma 1, seed 1+rank)",
        "config": {"workload": "config 2: blobs 1M x 3 exact HDBSCAN* (no sampling), minPts 4, minClSize 4",
                   "points_per_gpu": n, "d": D, "min_pts": MIN_PTS, "min_cl_size": MIN_CL_SIZE,
                   "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0),
                   "core": "EXCL_SELF", "timed": "X in pinned host memory -> H2D (each stage-1 worker uploads "
                   "its step's points on its own stream) -> K1t cores -> K2b MST + self edges, in the merge "
                   "order (HDB_EDGES_MERGED: tree edges sorted descending, self edges by core, one merge-path pass) "
                   "-> N>1: gather to rank 0, merge of the presorted runs -> "
                   "K6 flat labels of the partition (D2H of the merged list overlapping it on a copy "
                   "stream) -> D2H of the labels; pipelined: step i's labels + D2H (own thread, stream and "
                   "library context) overlap step i+1's MST + merge; the timer stops after the last step's "
                   "labels are on the host",
                   "stage1_partitions_in_flight": M, "label_stages": L,
                   "parallelism": f"partition-sharded x{world}"},
        "n_clusters": n_clusters[0],
        "hbm_resident_points_per_s": total_points * tsteps / dt_hbm,
        "hbm_resident_ms_per_step": dt_hbm * 1e3 / tsteps,
        "hbm_resident_kind": "the same pipeline from points already resident in HBM (no H2D; not the value)",
        "latency_ms_per_step": dt_lat * 1e3 / tsteps,
        "latency_kind": "the same steps without the pipeline: each step's stages back to back",
        "device_resident_points_per_s": total_points * tsteps / dt_dev,
        "device_resident_ms_per_step": dt_dev * 1e3 / tsteps,
        "mrd_evals_per_s": evals * tsteps / dt,
        "mrd_evals_per_s_kind": "algorithmic-equivalent: n^2 (k-NN) + n(n-1)/2 (MST) per partition (SURVEY.md "
                                "8(d)) over the step time; the exact pruned kernels execute ~1/1000 of it "
                                "(executed_pair_evals_per_s)",
        "executed_pair_evals_per_s": world * (knn_evals + bor_evals) * tsteps / dt,
        "kernels_ms_per_partition": ms,
        "kernels_kind": "HIP events on the launch stream, one partition at a time (stage 1: the device-resident "
                        "pass; flat_labels: the latency pass); boruvka_total includes boruvka_scan",
        "executed_pair_evals_per_step": {"knn_tree": knn_evals, "boruvka_scan": bor_evals,
                                         "algorithmic": n * n + n * (n - 1) // 2},
        "roofline": {"bound": "latency", "kernel": "boruvka_scan (boruvka_bvh_kernel)",
                     "unit": "node visits/s", "achieved": achieved, "peak": peak,
                     "frac": achieved / peak if peak else 0.0, "traffic": traffic, "traffic_source": os.path.relpath(PMC_C2, ROOT),
                     "model": f"per round: visits x {MALL_HIT_NS:.0f} ns (one dependent Infinity-Cache "
                              f"round trip per visit) / min(waves, {WAVE_SLOTS} resident wave slots)",
                     "visits_per_step": visits, "rounds": [[v, w] for v, w in rounds],
                     "avg_launch_ms": avg_scan_s * 1e3, "launches_per_step": scan_n / tsteps,
                     "timing": "HIP events on the launch stream over the device-resident pass (one partition "
                               "at a time: each kernel alone); the pipelined value region overlaps several "
                               "partitions, where an event pair also spans the other streams' work",
                     "fp64": {"achieved_tflops": fp64_tflops, "peak": FP64_PEAK_TFLOPS,
                              "frac": fp64_tflops / FP64_PEAK_TFLOPS,
                              "work": "executed pair evals x 3d flops"},
                     "hbm": {"achieved_gbs": (traffic or 0) / avg_scan_s / 1e9 if avg_scan_s > 0 else 0.0,
                             "peak": HBM_PEAK_GBS}},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(X_host)
    if rank == 0:
        emit(line)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
