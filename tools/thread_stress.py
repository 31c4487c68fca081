"""Concurrent local models and leaf MSTs from many host threads: the C3/C5
driver's model pool, reduced to its library calls.

Every thread owns its own context (A.Context.get: thread-local, own stream), exactly as
driver.py's pool threads do, and runs a shuffled list of jobs:
  * hdb_local_model on bubble sets of 600..16,384 bubbles at d = 8 (bubble K5 core distances,
    block / cooperative Prim, host cluster tree + FOSC) -- LocalModelReduceByKey.java:29-114;
  * hdb_exact_mst on 20k..150k-point d = 8 blob leaves (K1t + K2b on one index);
  * hdb_leaf_msts on a batch of small leaves (reference Prim, batched).
Each job's outputs are hashed; the digests must equal a serial pass over the same jobs.  Run
with GPU_MAX_HW_QUEUES / HDB_HW_QUEUES set (HIP reads it at start-up) to put more streams on
more hardware queues, and with -X faulthandler + HDB_NATIVE_BACKTRACE=1 so a crash leaves both
stacks.

usage: python -X faulthandler tools/thread_stress.py [--threads 8] [--rounds 2] [--quick]
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import os
import random
import sys
import threading
import time

_req = int(os.environ.get("HDB_HW_QUEUES", "0") or 0)
if _req > 0:
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, _req))

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "232-hierarchical-density-based-clustering-using-mapreduce_amd"


def blobs(n, d, centers, seed, spread=100.0):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-spread, spread, size=(centers, d))
    return C[rng.integers(0, centers, size=n)] + rng.normal(0, 1.0, size=(n, d))


def digest(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def make_jobs(pkg, quick):
    import torch
    A = pkg._capi
    jobs = []
    sizes = [600, 2000, 4096, 6000] if quick else [600, 2000, 4096, 6000, 9000, 12000, 16384]
    for i, b in enumerate(sizes):  # bubble sets: C5-like (blob points -> samples -> stats)
        X = torch.from_numpy(blobs(8 * b, 8, 12 + i, 100 + i)).cuda()
        S = X[torch.from_numpy(np.sort(np.random.default_rng(i).choice(8 * b, b, replace=False))).cuda()].contiguous()
        near = pkg.nearest_sample(X, S)
        used = torch.unique(near)
        remap = torch.full((b,), -1, dtype=torch.int32, device="cuda")
        remap[used.long()] = torch.arange(used.shape[0], dtype=torch.int32, device="cuda")
        _, _, rep, info = pkg.bubble_stats(X, remap[near.long()], int(used.shape[0]))
        rep, info = rep.cpu().numpy(), info.cpu().numpy()

        def lm(rep=rep, info=info):
            try:
                labels, mst, inter = pkg.LocalModelReduceByKey(4, 4).call(rep, info)
            except pkg.HdbError as e:  # the reference's own exceptions are results too
                return f"exc{e.code}"
            return digest(labels, mst.getVerticeA(), mst.getEges(), *inter)
        jobs.append((f"local_model b={rep.shape[0]}", lm))
    for i, n in enumerate([20000, 60000] if quick else [20000, 60000, 100000, 150000]):
        Xl = torch.from_numpy(blobs(n, 8, 6, 200 + i)).cuda()

        def leaf(Xl=Xl, n=n):
            c = A.Context.get(0)
            va = torch.empty(2 * n - 1, dtype=torch.int32, device="cuda")
            vb, w = torch.empty_like(va), torch.empty(2 * n - 1, dtype=torch.float64, device="cuda")
            A.check(A.lib().hdb_exact_mst(c.h, Xl.data_ptr(), n, 8, 4, 0, A.CORE_INCL_SELF_CUMULATIVE, 1, None,
                                          va.data_ptr(), vb.data_ptr(), w.data_ptr()), "exact MST")
            c.synchronize()
            return digest(va.cpu().numpy(), vb.cpu().numpy(), w.cpu().numpy())
        jobs.append((f"exact_mst n={n}", leaf))
    Xs = blobs(30000, 8, 30, 300)
    offs = np.concatenate([[0], np.cumsum(np.random.default_rng(3).integers(50, 3000, 20))]).astype(np.int64)
    offs = offs[offs <= Xs.shape[0]]

    def small_leaves():
        core, g = pkg.FirstStep(0.2, 50, 4).leaf(Xs[:offs[-1]], np.arange(offs[-1], dtype=np.int32), offs)
        return digest(core, g.getVerticeA(), g.getVericeB(), g.getEges())
    jobs.append(("leaf_msts", small_leaves))
    return jobs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    import torch
    pkg = importlib.import_module(PKG)
    jobs = make_jobs(pkg, a.quick)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ref = {name: f() for name, f in jobs}
    print(f"serial pass: {len(jobs)} jobs in {time.perf_counter() - t0:.2f} s", flush=True)
    errors = []
    for r in range(a.rounds):
        work = [(name, f) for name, f in jobs for _ in range(max(1, a.threads // 2))]
        random.Random(r).shuffle(work)
        lock = threading.Lock()
        got = []

        def worker():
            while True:
                with lock:
                    if not work:
                        return
                    name, f = work.pop()
                try:
                    res = f()
                except Exception as e:  # noqa: BLE001 -- reported below
                    res = f"raised {type(e).__name__}: {e}"
                with lock:
                    got.append((name, res))
        t0 = time.perf_counter()
        th = [threading.Thread(target=worker) for _ in range(a.threads)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        bad = [(n, res, ref[n]) for n, res in got if res != ref[n]]
        errors += bad
        print(f"round {r}: {len(got)} jobs on {a.threads} threads in {time.perf_counter() - t0:.2f} s, "
              f"{len(bad)} mismatches", flush=True)
    for n, res, want in errors[:10]:
        print(f"MISMATCH {n}: {res} != {want}", flush=True)
    print(f"hw_queues {os.environ.get('GPU_MAX_HW_QUEUES')}, contexts {len(pkg._capi.Context._all)}")
    if errors:
        sys.exit(1)
    print("thread stress ok")


if __name__ == "__main__":
    main()
