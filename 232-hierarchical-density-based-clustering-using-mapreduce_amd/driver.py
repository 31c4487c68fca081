"""MR-HDBSCAN* iteration driver over the HIP operators -- the stand-in for the reference's
Spark driver (main/Main.java:103-347) used by the end-to-end tests and benchmarks.

In production the Java/Spark driver stays in place and calls the operators through JNI
(INTEGRATION.md); this module runs the same loop without Spark, device-resident: the points
stay in HBM for the whole run, every level's work is batched over all subsets of the level,
and only per-subset bookkeeping (a few integers per subset, one label per bubble) touches
the host.  Semantics follow Main.java with the deterministic deviations of SURVEY.md
Appendix A.2 (D1-D11, listed in oracle/mr_driver.py, which restates the same loop on the CPU
oracle for the parity tests):

  level loop (Main.java:107)   subsets grouped by key, ascending (D5)
  leaves  (FirstStep.java:104-120)  subsets <= processing_units (or forced, D9): cumulative
          core distances + Prim with self edges over the rows in ascending global id, one
          batched call for all leaves <= LEAF_PRIM_MAX points (and for any size when
          exact_prim_leaves is set or K2b does not apply: other metrics, other d); larger
          forced leaves use hdb_exact_mst: the same cores + Boruvka on one index (exact
          weights; topology differs from Prim only on ties).  Leaves are end points of
          the subset tree, so they are deferred (defer_leaves): every level's leaves run as
          one batch after the level loop (identical blocks, placed by their canonical ids)
  big subsets: D2 samples -> keyed nearest sample (FirstStep.java:74-85, D3) -> bulk
          CombineStep (D5 fold order per slice, D11 merge) -> per subset LocalModelReduceByKey (D4) -> partition
          induction (Main.java:272-289, including the in-place relabel) -> LabelClassification
  merge   UnionFindReducer + SortMST: stable descending sort of the iteration-major edge list

Multi-GPU (one process per GPU, torch.distributed initialised, X given to
every rank): the plan is computed identically on every rank -- leaves go to ranks by LPT on
n_i^2 (over the whole job when deferred, per level otherwise), the big subsets' points are split in contiguous chunks for the nearest-sample scan (the
assignments are all-gathered), bubble statistics are folded per fixed row slice by the rank
that owns the slice and the gathered partials merged in slice order (D11: the same result at
every rank count), local models go to ranks by LPT on b_i^2 (results all-gathered
and applied in subset order), and the merge places every local edge at its position in the
single-device concatenation (hdb_merge_edges over the library's RCCL communicator under
nccl, torch.distributed under gloo) before the stable sort.  Every rank returns the same
result as one device does.
"""
from __future__ import annotations

import math

import os

import numpy as np

from . import _capi as A
from . import parallel as P
from .hdbscanstar import metric_of

LEAF_PRIM_MAX = 65536  # leaves up to this size run the exact reference Prim (batched; one
#                       workgroup per leaf <= 4096 points, one cooperative launch above)
BORUVKA_DIMS = (1, 2, 3, 4, 8, 16)  # d with a K1t/K2b instantiation (csrc/spatial.hip)
BUBBLE_SLICES = 8  # D11: CombineStep partials per fixed row slice (a rank folds only its slices)


def boruvka_ok(metric: int, d: int, min_pts: int) -> bool:
    """hdb_exact_mst's K2b path: Euclidean, d with an instantiation, 2 <= minPts <= 32."""
    return metric == A.METRIC["euclidean"] and d in BORUVKA_DIMS and 2 <= min_pts <= 32


def sample_ids(n_key: int, k: float, samples_per_subset, seed: int, iteration: int, key: int):
    """D2: positions (into the subset's rows, ascending global id) of the subset's samples,
    ascending; size ceil(k * n) (sampleByKeyExact, Main.java:141) or an explicit count."""
    m = samples_per_subset if samples_per_subset else int(math.ceil(k * n_key))
    m = max(1, min(n_key, m))
    rng = np.random.Generator(np.random.PCG64([seed, iteration, key]))
    return np.sort(rng.choice(n_key, size=m, replace=False)).astype(np.int64)


class MRHDBSCANStar:
    """Main.main's MR-HDBSCAN* loop (with data bubbles) on one device."""

    def __init__(self, minPts=4, minClSize=4, processing_units=50, k=0.2, samples_per_subset=None,
                 seed=20210101, distanceFunction=None, all_inter_edges=True, max_levels=64, ctx=None,
                 device=0, flat_labels=True, profile=False, exact_prim_leaves=False, group=None,
                 prim_leaf_max=LEAF_PRIM_MAX, model_threads=4, defer_leaves=True, bubble_slices=BUBBLE_SLICES,
                 emulate_ranks=(), cores_first=False):
        self.minPts = minPts
        self.minClSize = minClSize
        self.processing_units = processing_units
        self.k = k
        self.samples_per_subset = samples_per_subset
        self.seed = seed
        self.metric = metric_of(distanceFunction)
        self.all_inter_edges = all_inter_edges
        self.max_levels = max_levels
        self.device = device
        self.ctx = ctx
        self.flat_labels = flat_labels
        self.profile = profile       # phase wall times (synchronising) in self.timings
        # True: every leaf, however large, runs the reference Prim (the exact edge list of
        # HDBSCANStar.constructMST, ties included; stepwise above 65,536 points).  False:
        # forced leaves above LEAF_PRIM_MAX use Boruvka where it applies (same weights,
        # topology may differ among equal-weight edges)
        self.exact_prim_leaves = exact_prim_leaves
        # leaves up to this size run the reference Prim (exact topology, latency-bound: one
        # step per point); larger ones K2b where it applies (exact weights, ties may differ)
        self.prim_leaf_max = prim_leaf_max
        # a level's local models run concurrently, one host thread (own context and stream)
        # each: a bubble Prim occupies only ceil(b / 1024) CUs
        self.model_threads = int(os.environ.get("HDB_MODEL_THREADS", model_threads))
        # cores_first: a rank holding several models of a level computes all their bubble core
        # distances before any of their Prims (hdb_local_model_cores; same cores, same outputs).
        # Measured on C5 (round 6): no change (emulated N = 8 local models 1.956 vs 1.951 s), so
        # off by default
        self.cores_first = bool(int(os.environ.get("HDB_CORES_FIRST", int(cores_first))))
        # leaves are end points of the subset tree: nothing later in the loop reads their edges,
        # so they can wait until the level loop is done and then run as ONE batch over the
        # whole job (global LPT over the ranks, one batched Prim launch for every small leaf)
        # instead of one synchronising batch per level -- the same blocks, the same result
        self.defer_leaves = defer_leaves
        # D11 (oracle/mr_driver.py): a level's big-subset rows are cut into this many fixed
        # slices; CombineStep folds each slice and merges the partials in slice order (Spark's
        # map-side combine per partition, Main.java:236-237, with the partitions fixed).  A rank
        # folds only its own slices, so the statistics shard; 1 = one sequential fold (the
        # round-1..5 order; the committed C1 / scaled-C5 fixtures were made with it)
        self.bubble_slices = int(bubble_slices)
        if not 1 <= self.bubble_slices <= 64:
            raise ValueError("bubble_slices: 1..64")
        # profile at N = 1 only: after every level's local models (and the deferred leaves) ran
        # for real, run them again once per N in emulate_ranks as the N-rank driver would --
        # each rank's LPT share on its own, one rank after another -- and record the slowest
        # rank's wall time (bench.py predicted_scaling).  A rank then gets the concurrency its
        # own share allows, not the one-device pool's: with ~8 models per level, 8 ranks hold
        # one or two each, and a lone model runs at its own (latency-bound) speed.
        self.emulate_ranks = tuple(int(x) for x in emulate_ranks)
        self._emulating = False
        self._pool = None
        self.group = group      # torch.distributed group (None: the default group, if any)
        self._comm = None       # HdbComm for the merge under nccl
        self.timings = {}
        self.level_tasks = []   # profile: per level, task durations + phase wall times
        self._lvl = None
        self._t0 = None
        self._progress = bool(os.environ.get("HDB_PROGRESS"))  # one stderr line per level
        # a fatal signal in any thread (the model pool drives the library from several) leaves
        # every thread's Python stack on stderr; cheap, so always armed
        import faulthandler
        if not faulthandler.is_enabled():
            faulthandler.enable(all_threads=True)

    def _mark(self, phase):
        """profile: phase wall time since the previous mark (synchronising); returns it"""
        if not self.profile:
            return 0.0
        import time
        import torch
        torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        dt = 0.0
        if self._t0 is not None and phase:
            dt = now - self._t0
            self.timings[phase] = self.timings.get(phase, 0.0) + dt
        self._t0 = now
        return dt

    def _task(self, kind, weight, seconds):
        """profile: one task's duration in the current level (the LPT weight the sharded
        driver assigns it by, and its measured seconds at this world size)"""
        if self.profile and self._lvl is not None and not self._emulating:
            self._lvl.setdefault(kind, []).append((float(weight), float(seconds)))

    # ------------------------------------------------------------------ helpers
    def _c(self):
        if self.ctx is None:
            self.ctx = A.Context.get(self.device)
        self.ctx.use_torch_stream()
        return self.ctx

    def _leaves(self, X, rows_list, keys):
        """FirstStep leaf branch for every leaf subset of the level; returns edge tuples in
        key order."""
        import torch
        out = []
        c = self._c()
        d = X.shape[1]
        prim = lambda n: (n <= self.prim_leaf_max or self.exact_prim_leaves
                          or not boruvka_ok(self.metric, d, self.minPts))
        small = [(k, r) for k, r in zip(keys, rows_list) if prim(r.shape[0])]
        if small:
            rows = torch.cat([r for _, r in small])
            sizes = np.array([r.shape[0] for _, r in small], np.int64)
            offs = np.zeros(len(small) + 1, np.int64)
            offs[1:] = np.cumsum(sizes)
            Xl = X.index_select(0, rows).contiguous()
            ids = rows.to(torch.int32)
            ne = int(np.sum(2 * sizes - 1))
            core = torch.empty(rows.shape[0], dtype=torch.float64, device=X.device)
            va = torch.empty(ne, dtype=torch.int32, device=X.device)
            vb = torch.empty_like(va)
            w = torch.empty(ne, dtype=torch.float64, device=X.device)
            if self.profile:
                import time
                torch.cuda.synchronize(X.device)
                t_small = time.perf_counter()
            A.check(A.lib().hdb_leaf_msts(c.h, Xl.data_ptr(), offs.ctypes.data, len(small), X.shape[1],
                                          ids.data_ptr(), self.minPts, self.metric, core.data_ptr(), va.data_ptr(),
                                          vb.data_ptr(), w.data_ptr()), "FirstStep.leaf")
            if self.profile:  # one batched launch: its time split over the leaves by n^2
                torch.cuda.synchronize(X.device)
                t_small = time.perf_counter() - t_small
                wsum = float(np.sum(sizes.astype(np.float64) ** 2))
                for sz in sizes.tolist():
                    self._task("leaves", float(sz) ** 2, t_small * float(sz) ** 2 / wsum)
            eo = np.zeros(len(small) + 1, np.int64)
            eo[1:] = np.cumsum(2 * sizes - 1)
            by_key = {k: (va[eo[i]:eo[i + 1]], vb[eo[i]:eo[i + 1]], w[eo[i]:eo[i + 1]])
                      for i, (k, _) in enumerate(small)}
        else:
            by_key = {}
        # large forced leaves (D9) where K2b applies: cumulative cores + exact MST (Boruvka:
        # exact weights) in one call sharing one spatial index (hdb_exact_mst).  A leaf of
        # ~1e5 points keeps only part of the chip busy, so several run concurrently, each on a
        # host thread with its own context and stream.
        big = [(k, r) for k, r in zip(keys, rows_list) if k not in by_key]
        jobs = {}
        for k, r in big:
            n = r.shape[0]
            Xl = X.index_select(0, r).contiguous()
            va = torch.empty(2 * n - 1, dtype=torch.int32, device=X.device)
            jobs[k] = (r, Xl, va, torch.empty_like(va), torch.empty(2 * n - 1, dtype=torch.float64, device=X.device))
        if big:
            torch.cuda.current_stream(X.device).synchronize()  # inputs ready for the other streams

        def leaf(k, threaded):
            import time
            t0 = time.perf_counter()
            r, Xl, va, vb, w = jobs[k]
            cc = A.Context.get(self.device) if threaded else c
            A.check(A.lib().hdb_exact_mst(cc.h, Xl.data_ptr(), r.shape[0], X.shape[1], self.minPts, self.metric,
                                          A.CORE_INCL_SELF_CUMULATIVE, 1, None, va.data_ptr(), vb.data_ptr(),
                                          w.data_ptr()), "leaf exact MST")
            if threaded or self.profile:
                cc.synchronize()
            self._task("leaves", float(r.shape[0]) ** 2, time.perf_counter() - t0)

        if len(big) > 1 and self.model_threads > 1:
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._pool = ThreadPoolExecutor(self.model_threads)
            list(self._pool.map(lambda k: leaf(k, True), [k for k, _ in big]))
        else:
            for k, _ in big:
                leaf(k, False)
        for k, r in zip(keys, rows_list):
            if k in by_key:
                out.append(by_key[k])
                continue
            r, _, va, vb, w = jobs[k]
            g = r.to(torch.int32)
            out.append((g[va.long()], g[vb.long()], w))
        return out

    # --------------------------------------------------------------------- run
    def run(self, X):
        """X: n x d float64 (numpy or torch).  Returns dict(edges=(va, vb, w) merged,
        levels=[...], leaf_of=subset key that processed each point, iterations)."""
        import torch
        dev = torch.device("cuda", self.device)
        X = torch.as_tensor(X, dtype=torch.float64).to(dev).contiguous()
        n, d = X.shape
        c = self._c()
        self.timings = {}
        self.level_tasks = []
        self._lvl = None
        self._t0 = None
        self._mark(None)
        import time
        t_run = time.perf_counter()
        world, rank = P.world_rank(self.group)
        key_of = torch.zeros(n, dtype=torch.int64, device=dev)
        alive = torch.arange(n, dtype=torch.int64, device=dev)  # ids in the current _unprocessed_ file
        forced = set()
        leaf_of = torch.full((n,), -1, dtype=torch.int64, device=dev)
        blocks, block_size, levels = [], {}, []  # blocks: (canonical id, edges) computed here
        pending = []  # deferred leaves: (canonical block id, rows)
        iteration, processed, next_id = 0, 0, 2  # Main.java:103-105
        while processed < n:
            # group the alive records by (key, global id) -- D5
            order = torch.argsort(key_of[alive] * (n + 1) + alive)
            alive = alive[order]
            akeys = key_of[alive]
            ukeys, counts = torch.unique_consecutive(akeys, return_counts=True)
            ukeys, counts = ukeys.cpu().numpy(), counts.cpu().numpy()
            starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
            leaf_k, leaf_rows, big = [], [], []
            for kk, s0, cnt in zip(ukeys.tolist(), starts.tolist(), counts.tolist()):  # Main.java:133-138
                rows = alive[s0:s0 + cnt]
                if cnt <= self.processing_units or kk in forced or iteration >= self.max_levels:
                    leaf_k.append(kk)
                    leaf_rows.append(rows)
                    processed += cnt
                else:
                    big.append((kk, s0, cnt))
            level = dict(iteration=iteration, leaves={k: int(r.shape[0]) for k, r in zip(leaf_k, leaf_rows)},
                         big={k: cnt for k, _, cnt in big}, labels={}, new_keys={})
            if self.profile:
                self._lvl = {"phase_s": {}}
                self.level_tasks.append(self._lvl)
            if leaf_k and self.defer_leaves:
                for i, (kk, r) in enumerate(zip(leaf_k, leaf_rows)):
                    block_size[(iteration, 0, i)] = 2 * int(r.shape[0]) - 1
                    leaf_of[r] = kk
                    pending.append(((iteration, 0, i), r))
            elif leaf_k:
                self._mark("bookkeeping")
                owner = P.lpt([int(r.shape[0]) ** 2 for r in leaf_rows], world)
                mine = [i for i in range(len(leaf_k)) if owner[i] == rank]
                if mine:
                    got = self._leaves(X, [leaf_rows[i] for i in mine], [leaf_k[i] for i in mine])
                    blocks.extend(((iteration, 0, i), e) for i, e in zip(mine, got))
                for i, r in enumerate(leaf_rows):
                    block_size[(iteration, 0, i)] = 2 * int(r.shape[0]) - 1
                if self.profile:
                    self._lvl["phase_s"]["leaves"] = self._mark("leaves")
                for kk, r in zip(leaf_k, leaf_rows):
                    leaf_of[r] = kk
            iteration += 1
            if self._progress:
                import sys
                import time
                print(f"[hdb] level {iteration - 1}: {len(leaf_k)} leaves, {len(big)} big subsets, "
                      f"{processed}/{n} points done, {time.perf_counter() - t_run:.2f} s", file=sys.stderr, flush=True)
                if os.environ.get("HDB_WATCHDOG"):  # every thread's stack if a level stalls
                    import faulthandler
                    faulthandler.dump_traceback_later(float(os.environ["HDB_WATCHDOG"]), exit=False)
            if processed >= n:
                levels.append(level)
                break
            # ---- big subsets: samples (D2), keyed nearest sample (D3), bubbles
            brows = torch.cat([alive[s0:s0 + cnt] for _, s0, cnt in big])
            bkey_local = torch.cat([torch.full((cnt,), i, dtype=torch.int32, device=dev)
                                    for i, (_, _, cnt) in enumerate(big)])
            s_gid, s_key, s_off = [], [], [0]
            for i, (kk, s0, cnt) in enumerate(big):
                sp = torch.from_numpy(sample_ids(cnt, self.k, self.samples_per_subset, self.seed, iteration - 1, kk))
                s_gid.append(alive[s0:s0 + cnt][sp.to(dev)])
                s_key.append(torch.full((sp.shape[0],), i, dtype=torch.int32, device=dev))
                s_off.append(s_off[-1] + sp.shape[0])
            s_gid = torch.cat(s_gid)
            s_key = torch.cat(s_key)
            Xb = X.index_select(0, brows).contiguous()
            S = X.index_select(0, s_gid).contiguous()
            lo, hi = P.chunk(brows.shape[0], world, rank)  # this rank's points (all of them at N = 1)
            nearest = torch.empty(hi - lo, dtype=torch.int32, device=dev)
            if hi > lo:
                A.check(A.lib().hdb_nearest_sample(c.h, Xb[lo:hi].data_ptr(), hi - lo, S.data_ptr(), S.shape[0], d,
                                                   self.metric, bkey_local[lo:hi].data_ptr(), s_key.data_ptr(),
                                                   nearest.data_ptr(), None), "FirstStep.nearest")
            if world > 1:
                nearest = P.allgather_var(nearest, self.group)
            if self.profile:
                self._lvl["phase_s"]["nearest_sample"] = self._mark("nearest_sample")
            # nearest is the list position in S (keyed: within the point's own subset)
            nb = S.shape[0]
            ls = torch.empty((nb, d), dtype=torch.float64, device=dev)
            ss, rep = torch.empty_like(ls), torch.empty_like(ls)
            info = torch.empty((nb, 3), dtype=torch.float64, device=dev)
            if self.bubble_slices > 1:
                self._bubbles_sliced(c, Xb, nearest, nb, world, rank, ls, ss, rep, info)
            else:
                A.check(A.lib().hdb_bubble_stats(c.h, Xb.data_ptr(), Xb.shape[0], d, nearest.data_ptr(), nb,
                                                 A.BUBBLE_COMBINESTEP, ls.data_ptr(), ss.data_ptr(), rep.data_ptr(),
                                                 info.data_ptr()), "CombineStep")
            rep_h, info_h = rep.cpu().numpy(), info.cpu().numpy()
            if self.profile:
                self._lvl["phase_s"]["bubbles"] = self._mark("bubbles")
            s_gid_h = s_gid.cpu().numpy()
            new_key_of_bubble = np.full(nb, -2, np.int64)
            # local models: LPT over the ranks on b^2, results gathered, applied in subset order
            nonempty_of = [np.nonzero(info_h[s_off[i]:s_off[i + 1], 2] > 0)[0] for i in range(len(big))]  # D4
            owner = P.lpt([int(ne.shape[0]) ** 2 for ne in nonempty_of], world)
            core_s = {}  # cores-first: seconds of each model's core pass (added to its task time)

            def model(i, core=None):
                import time
                t0 = time.perf_counter()
                try:
                    return model_body(i, core)
                finally:
                    self._task("local_models", float(nonempty_of[i].shape[0]) ** 2,
                               time.perf_counter() - t0 + core_s.get(i, 0.0))

            def model_core(i):
                import time
                t0 = time.perf_counter()
                a, b = s_off[i], s_off[i + 1]
                nonempty = nonempty_of[i]
                core = None
                if nonempty.shape[0] >= 2:
                    core = self._model_cores(rep_h[a:b][nonempty], info_h[a:b][nonempty])
                core_s[i] = time.perf_counter() - t0
                return core

            def model_body(i, core=None):
                a, b = s_off[i], s_off[i + 1]
                nonempty = nonempty_of[i]
                if nonempty.shape[0] < 2:
                    return None, None, None
                try:
                    labels, (iva, ivb, iw) = self._local_model(rep_h[a:b][nonempty], info_h[a:b][nonempty],
                                                               threaded=True, core=core)
                except A.HdbError as e:  # D10: the reference's own exceptions only
                    if e.code > -10:
                        raise
                    return None, e.code, None
                inter = None
                if iw.shape[0]:
                    gid = s_gid_h[a:b][nonempty].astype(np.int32)
                    inter = (gid[iva], gid[ivb], iw) if self.all_inter_edges else (iva[:1], ivb[:1], iw[:1])
                return labels, None, inter

            def run_models(grp, fn):
                """one rank's models as the pool runs them (cores-first when it holds several)"""
                if self.cores_first and len(grp) > 1 and self.model_threads > 1:
                    cores = dict(zip(grp, self._run_group(model_core, grp)))
                    return dict(zip(grp, self._run_group(lambda i: fn(i, cores[i]), grp)))
                return dict(zip(grp, self._run_group(fn, grp)))

            mine = [i for i in range(len(big)) if owner[i] == rank]
            results = run_models(mine, model)
            if self.profile and self.emulate_ranks and world == 1:
                self._lvl["emulated_local_models"] = self._emulate(
                    [int(ne.shape[0]) ** 2 for ne in nonempty_of], lambda grp: run_models(grp, model_body))
            if world > 1:
                for part in P.allgather_object(results, self.group):
                    results.update(part)
            inter_i = 0
            for i, (kk, s0, cnt) in enumerate(big):
                a = s_off[i]
                nonempty = nonempty_of[i]
                labels, code, inter = results[i]
                if code is not None:
                    level.setdefault("model_errors", {})[kk] = code
                if inter is not None:  # D7 block: kept by the rank that computed the model
                    bid = (iteration - 1, 1, inter_i)
                    block_size[bid] = int(inter[2].shape[0])
                    if owner[i] == rank:
                        blocks.append((bid, tuple(torch.from_numpy(np.ascontiguousarray(x, dt)).to(dev) for x, dt in
                                                  zip(inter, (np.int32, np.int32, np.float64)))))
                    inter_i += 1
                if labels is None:
                    labels = np.full(nonempty.shape[0], 2, np.int32)
                labels = np.array(labels, np.int32)
                level["labels"][kk] = labels.copy()
                for cl in sorted(set(labels.tolist())):  # Main.java:272-289 (in-place relabel)
                    labels[labels == cl] = next_id
                    next_id += 1
                nk = sorted(set(labels.tolist()))
                level["new_keys"][kk] = nk
                if len(nk) == 1:
                    forced.add(nk[0])  # D9
                new_key_of_bubble[a + nonempty] = labels
            # LabelClassification.java:21-37 (bubble of the point -> relabelled label)
            if self.profile:
                self._lvl["phase_s"]["local_models"] = self._mark("local_models")
            tbl = torch.from_numpy(new_key_of_bubble).to(dev)
            key_of[brows] = tbl[nearest.long()]
            alive = brows
            levels.append(level)
        self._mark("bookkeeping")
        if pending:
            # every level's leaves in one batch: LPT over the ranks on n^2 across the whole job
            # (a level with one big leaf no longer idles the other ranks)
            if self.profile:
                self._lvl = {"phase_s": {}, "deferred_leaves": True}
                self.level_tasks.append(self._lvl)
            owner = P.lpt([int(r.shape[0]) ** 2 for _, r in pending], world)
            mine = [j for j in range(len(pending)) if owner[j] == rank]
            if mine:
                got = self._leaves(X, [pending[j][1] for j in mine], list(range(len(mine))))
                blocks.extend((pending[j][0], e) for j, e in zip(mine, got))
            if self.profile:
                self._lvl["phase_s"]["leaves"] = self._mark("leaves")
            if self.profile and self.emulate_ranks and world == 1:
                self._lvl["emulated_leaves"] = self._emulate(
                    [int(r.shape[0]) ** 2 for _, r in pending],
                    lambda grp: self._leaves(X, [pending[j][1] for j in grp], list(range(len(grp)))))
        # UnionFindReducer + SortMST: stable descending sort of the iteration-major
        # concatenation (leaf blocks in key order, then the level's inter-cluster blocks)
        order = sorted(block_size)
        off, pos = {}, 0
        for bid in order:
            off[bid] = pos
            pos += block_size[bid]
        blocks.sort(key=lambda t: t[0])
        cat = lambda i, dt: (torch.cat([e[i] for _, e in blocks]) if blocks
                             else torch.zeros(0, dtype=dt, device=dev))
        va, vb, w = cat(0, torch.int32), cat(1, torch.int32), cat(2, torch.float64)
        if world > 1:
            seq = torch.cat([torch.arange(off[bid], off[bid] + block_size[bid], dtype=torch.int64, device=dev)
                             for bid, _ in blocks]) if blocks else torch.zeros(0, dtype=torch.int64, device=dev)
            import torch.distributed as dist
            if self._comm is None and dist.get_backend(self.group) == "nccl":
                self._comm = P.HdbComm(c, self.group)
            va, vb, w = P.merge_local_msts(va.contiguous(), vb.contiguous(), w.contiguous(), self.group, seq=seq,
                                           comm=self._comm)
        elif w.shape[0]:
            A.check(A.lib().hdb_sort_edges_desc(c.h, va.data_ptr(), vb.data_ptr(), w.data_ptr(), w.shape[0]),
                    "SortMST")
        out = dict(edges=(va, vb, w), levels=levels, leaf_of=leaf_of, iterations=iteration)
        self._mark("merge")
        if self.flat_labels and self.all_inter_edges:
            # D6: the global hierarchy + flat partition over the merged MST (replaces the
            # System.exit(1) of Main.java:408); D7 makes the merged edges a spanning tree
            labels = torch.empty(n, dtype=torch.int32, device=dev)
            k = np.zeros(1, np.int64)
            A.check(A.lib().hdb_flat_labels(c.h, va.data_ptr(), vb.data_ptr(), w.data_ptr(), w.shape[0], n,
                                            self.minClSize, labels.data_ptr(), k.ctypes.data), "flat labels")
            out["labels"] = labels
            out["n_clusters"] = int(k[0])
            self._mark("flat_labels")
        return out

    def _run_group(self, fn, grp):
        """run fn over the items of one (emulated) rank as the model pool would"""
        if len(grp) > 1 and self.model_threads > 1:
            if self._pool is None:
                from concurrent.futures import ThreadPoolExecutor
                self._pool = ThreadPoolExecutor(self.model_threads)
            return list(self._pool.map(fn, grp))
        return [fn(i) for i in grp]

    def _emulate(self, costs, run):
        """profile: {N: wall time of the slowest rank} with the items dealt by the driver's LPT
        to N ranks, every rank's share run alone (synchronised), one rank after another"""
        import time
        import torch
        out = {}
        torch.cuda.synchronize(self.device)
        t_in = time.perf_counter()
        self._emulating = True
        try:
            for N in self.emulate_ranks:
                own = P.lpt(costs, N)
                worst = 0.0
                for r in range(N):
                    grp = [i for i in range(len(costs)) if own[i] == r]
                    if not grp:
                        continue
                    torch.cuda.synchronize(self.device)
                    t0 = time.perf_counter()
                    run(grp)
                    torch.cuda.synchronize(self.device)
                    worst = max(worst, time.perf_counter() - t0)
                out[N] = worst
        finally:
            self._emulating = False
        if self._t0 is not None:  # the phase being measured does not include the emulation
            self._t0 += time.perf_counter() - t_in
        return out

    def _bubbles_sliced(self, c, Xb, nearest, nb, world, rank, ls, ss, rep, info):
        """D11 CombineStep: this rank's slices folded into partials (hdb_bubble_partials), the
        partials of every rank gathered in rank (= slice) order, merged in slice order
        (hdb_bubble_combine) -- the same statistics on every rank and at every world size."""
        import torch
        T, d = Xb.shape
        Sl = self.bubble_slices
        g = [T * s // Sl for s in range(Sl + 1)]          # parallel.chunk(T, Sl, s)
        per = [P.chunk(Sl, world, r) for r in range(world)]  # slices of every rank
        s0, s1 = per[rank]
        k = s1 - s0
        dev = Xb.device
        pls = torch.empty(k * nb * d, dtype=torch.float64, device=dev)
        pss = torch.empty_like(pls)
        pn = torch.empty(k * nb, dtype=torch.float64, device=dev)
        if k:
            r0, r1 = g[s0], g[s1]
            cuts = np.array([g[s] - r0 for s in range(s0, s1 + 1)], np.int64)
            A.check(A.lib().hdb_bubble_partials(c.h, Xb[r0:r1].data_ptr(), r1 - r0, d, nearest[r0:r1].data_ptr(), nb,
                                                cuts.ctypes.data, k, pls.data_ptr(), pss.data_ptr(), pn.data_ptr()),
                    "CombineStep partials")
        if world > 1:
            mine = torch.cat([pls, pss, pn])
            allp = P.allgather_var(mine, self.group).to(dev)
            parts, o = [], 0
            for r0_, r1_ in per:
                kr = r1_ - r0_
                sz = kr * nb * d
                parts.append((allp[o:o + sz], allp[o + sz:o + 2 * sz], allp[o + 2 * sz:o + 2 * sz + kr * nb]))
                o += 2 * sz + kr * nb
            pls = torch.cat([p[0] for p in parts]).contiguous()
            pss = torch.cat([p[1] for p in parts]).contiguous()
            pn = torch.cat([p[2] for p in parts]).contiguous()
        if self.profile:
            self._lvl["phase_s"]["bubble_partials"] = self._mark("bubble_partials")
        A.check(A.lib().hdb_bubble_combine(c.h, pls.data_ptr(), pss.data_ptr(), pn.data_ptr(), Sl, nb, d, ls.data_ptr(),
                                           ss.data_ptr(), rep.data_ptr(), info.data_ptr()), "CombineStep merge")

    def _model_cores(self, rep, info):
        """HdbscanDataBubbles.calculateCoreDistancesBubbles for one model (this thread's context):
        the cores hdb_local_model computes first, from the same (rep, nB, eB, nnB)"""
        rep = np.ascontiguousarray(rep, np.float64)
        info = np.ascontiguousarray(info, np.float64)
        b, d = rep.shape
        eB, nnB = np.ascontiguousarray(info[:, 0]), np.ascontiguousarray(info[:, 1])
        nB = np.ascontiguousarray(info[:, 2].astype(np.int32))  # (int) info[i * 3 + 2], as hdb_local_model
        core = np.zeros(b)
        c = A.Context.get(self.device)
        A.check(A.lib().hdb_bubble_core_distances(c.h, A.ptr(rep), A.ptr(nB), A.ptr(eB), A.ptr(nnB), b, d, self.minPts,
                                                  self.metric, A.ptr(core)), "calculateCoreDistancesBubbles")
        return core

    def _local_model(self, rep, info, threaded=False, core=None):
        """LocalModelReduceByKey.java:88-104 body (D4 ids) -> (labels, inter-cluster edges).
        threaded: this thread's own context (private stream) instead of the driver's; core: the
        model's bubble cores computed beforehand (_model_cores)."""
        rep = np.ascontiguousarray(rep, np.float64)
        info = np.ascontiguousarray(info, np.float64)
        b, d = rep.shape
        ne = 2 * b - 1
        labels = np.zeros(b, np.int32)
        mva, mvb, mw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
        iva, ivb, iw = np.zeros(ne, np.int32), np.zeros(ne, np.int32), np.zeros(ne)
        nic = np.zeros(1, np.int64)
        c = A.Context.get(self.device) if threaded else self._c()
        if core is not None:
            core = np.ascontiguousarray(core, np.float64)
            A.check(A.lib().hdb_local_model_cores(c.h, A.ptr(rep), A.ptr(info), b, d, self.minPts, self.minClSize,
                                                  self.metric, A.ptr(core), A.ptr(labels), A.ptr(mva), A.ptr(mvb),
                                                  A.ptr(mw), A.ptr(iva), A.ptr(ivb), A.ptr(iw), A.ptr(nic)),
                    "LocalModelReduceByKey")
        else:
            A.check(A.lib().hdb_local_model(c.h, A.ptr(rep), A.ptr(info), b, d, self.minPts, self.minClSize,
                                            self.metric, A.ptr(labels), A.ptr(mva), A.ptr(mvb), A.ptr(mw), A.ptr(iva),
                                            A.ptr(ivb), A.ptr(iw), A.ptr(nic)), "LocalModelReduceByKey")
        k = int(nic[0])
        return labels, (iva[:k], ivb[:k], iw[:k])
