"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the MR-HDBSCAN* iteration driver
(main/Main.java:103-347) over the C oracle (hdb_oracle.c).  Only tests/ may use it; the
product driver (232-..._amd/driver.py) never imports it.

It follows the Java loop statement by statement, with the deterministic deviations of
SURVEY.md Appendix A.2 applied as named switches (the reference cannot run as shipped on
the target configs: Spark's sampleByKeyExact is unseeded, record orders are Spark's, and the
recursion can spin forever, Q11):

  D1  input rows are given (whitespace-split, first d columns) -- the caller parses;
  D2  sample ids: a seeded, sorted choice of ceil(k * n_key) (or `samples_per_subset`)
      members of each subset -- sample_ids(), shared verbatim with the product driver;
  D3  nearest sample restricted to the point's own subset (ClusterFeaturesByNodesMapper.java:54);
  D4  empty bubbles dropped, bubbles compacted in ascending sample order (vertex id == position);
  D5  canonical orders: rows ascending by global id inside a subset, subsets ascending by key,
      edge lists concatenated iteration-major (leaf edges, then inter-cluster edges);
  D7  every inter-cluster edge, endpoints mapped to the samples' global ids (OFF: only the
      first edge, in bubble-id space, Main.java:256-261);
  D9  progress guard: a subset whose local model yields one label (or that has one bubble)
      becomes a forced leaf; after max_levels every subset is a leaf;
  D10 a local model that raises one of the reference's exceptions (e.g. Clusters.java:45-46,
      "Cluster cannot have less than 0 points") does not end the run: the subset is treated
      as one label, i.e. a forced leaf (recorded in levels[i]["model_errors"]);
  D11 bubble_slices = S > 1: a level's big-subset rows (concatenated in key order, ascending
      id inside a subset) are cut into S fixed contiguous slices (slice s = rows [T s / S,
      T (s + 1) / S)); CombineStep folds each slice and combines the partials in slice order
      (oracle.bubble_stats cuts=...) -- Spark's map-side combine per partition with the
      partitions fixed; the product driver's sliced bubble statistics.  S = 1: one fold.
"""
from __future__ import annotations

import math

import numpy as np

from . import oracle as O


def sample_ids(n_key: int, k: float, samples_per_subset: int | None, seed: int, iteration: int, key: int):
    """D2: positions (into the subset's rows, ascending global id) of the subset's samples,
    ascending.  Size = sampleByKeyExact's exact size ceil(k * n) (Main.java:141) unless an
    explicit per-subset count is given.  Deterministic in (seed, iteration, key)."""
    m = samples_per_subset if samples_per_subset else int(math.ceil(k * n_key))
    m = max(1, min(n_key, m))
    rng = np.random.Generator(np.random.PCG64([seed, iteration, key]))
    return np.sort(rng.choice(n_key, size=m, replace=False)).astype(np.int64)


def _nearest_chunked(P, S, metric, pool, workers):
    """nearest_sample over row chunks on the pool (each point's first minimum is independent
    of the others: identical to one call)"""
    if pool is None or P.shape[0] < 4 * workers:
        return O.nearest_sample(P, S, metric)[0]
    cuts = np.linspace(0, P.shape[0], workers + 1).astype(np.int64)
    parts = pool.map(lambda i: O.nearest_sample(P[cuts[i]:cuts[i + 1]], S, metric)[0], range(workers))
    return np.concatenate(list(parts))


def run(X, min_pts=4, min_cl_size=4, processing_units=50, k=0.2, samples_per_subset=None, seed=20210101,
        metric="euclidean", all_inter_edges=True, max_levels=64, log=None, flat=True, workers=1, bubble_slices=1):
    """Returns dict(edges=(va, vb, w) merged (stable, descending weight), levels=[...],
    leaf_of=np.array subset key of the leaf that processed each point, iterations).

    workers > 1: the CPU-all variant (Spark local[*]'s stand-in, Main.java:89 with one task per
    subset): a level's leaves run concurrently, its big subsets' nearest sample + bubble stats +
    local model run concurrently (the nearest-sample scan of one subset also split into row
    chunks), on a thread pool over the C oracle (ctypes releases the GIL); the bookkeeping that
    numbers the new subsets stays sequential in key order, so the result is identical."""
    pool = None
    if workers > 1:
        import concurrent.futures as cf
        pool = cf.ThreadPoolExecutor(workers)
    try:
        return _run(X, min_pts, min_cl_size, processing_units, k, samples_per_subset, seed, metric,
                    all_inter_edges, max_levels, log, flat, pool, workers, bubble_slices)
    finally:
        if pool is not None:
            pool.shutdown()


def slice_cuts(sizes, S):
    """D11: per subset (sizes in key order), its local cuts of the level's S fixed slices"""
    T = int(np.sum(sizes))
    g = np.array([T * s // S for s in range(S + 1)], np.int64)  # parallel.chunk(T, S, s)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return [np.clip(g - off[i], 0, sizes[i]) for i in range(len(sizes))]


def _run(X, min_pts, min_cl_size, processing_units, k, samples_per_subset, seed, metric, all_inter_edges,
         max_levels, log, flat, pool, workers, bubble_slices=1):
    X = np.ascontiguousarray(X, np.float64)
    n, d = X.shape
    key_of = np.zeros(n, np.int64)            # MapperDataset_github.java:20: key 0
    alive = np.ones(n, bool)                  # records in the current _unprocessed_ file
    forced = set()                            # D9 forced-leaf keys
    leaf_of = np.full(n, -1, np.int64)
    edge_lists = []
    levels = []
    iteration, processed, next_id = 0, 0, 2   # Main.java:103-105
    while processed < n:                      # Main.java:107
        ids = np.nonzero(alive)[0]
        keys = np.unique(key_of[ids])         # D5: subsets ascending by key
        members = {int(c): ids[key_of[ids] == c] for c in keys}  # ascending global id
        leaf_keys, big_keys = [], []
        for c in keys:                        # Main.java:133-138
            c = int(c)
            cnt = members[c].shape[0]
            if cnt <= processing_units or c in forced or iteration >= max_levels:
                leaf_keys.append(c)
                processed += cnt
            else:
                big_keys.append(c)
        level = dict(iteration=iteration, leaves={c: members[c].shape[0] for c in leaf_keys},
                     big={c: members[c].shape[0] for c in big_keys}, labels={}, new_keys={})
        if log:
            log(f"level {iteration}: {len(leaf_keys)} leaves ({sum(level['leaves'].values())} pts, "
                f"max {max(level['leaves'].values(), default=0)}), {len(big_keys)} big subsets "
                f"({sum(level['big'].values())} pts)")
        # FirstStep leaf branch (FirstStep.java:104-120)
        def leaf(c):
            rows = members[c]
            return O.first_step_leaf(X[rows], rows.astype(np.int32), min_pts, metric)[1]
        leaf_edges = list(pool.map(leaf, leaf_keys)) if pool is not None else [leaf(c) for c in leaf_keys]
        for c in leaf_keys:
            leaf_of[members[c]] = c
        edge_lists.extend(leaf_edges)
        iteration += 1
        if processed >= n:
            levels.append(level)
            break
        # sampling (Main.java:140-163, D2) and nearest sample (FirstStep.java:74-102, D3)
        inter_edges = []
        new_alive = np.zeros(n, bool)
        new_key = np.full(n, -2, np.int64)
        cuts_of = dict(zip(big_keys, slice_cuts([members[c].shape[0] for c in big_keys], bubble_slices))) \
            if bubble_slices > 1 else {}
        def model(c):
            rows = members[c]
            sp = sample_ids(rows.shape[0], k, samples_per_subset, seed, iteration - 1, c)
            S = X[rows[sp]]
            nearest = _nearest_chunked(X[rows], S, metric, pool if len(big_keys) == 1 else None, workers)
            # CombineStep per (subset, sample): fold in ascending global id (D5)
            st = O.bubble_stats(X[rows], nearest, S.shape[0], "combine", cuts=cuts_of.get(c))
            nonempty = np.nonzero(st["info"][:, 2] > 0)[0]  # D4 (a 1-member bubble keeps [0, 0, 1])
            lm, err = None, None
            if nonempty.shape[0] >= 2:
                try:
                    lm = O.local_model(st["rep"][nonempty], st["info"][nonempty], min_pts, min_cl_size,
                                       metric)  # LocalModelReduceByKey.java:88-104
                except O.OracleError as e:                 # D10: the reference throws here
                    err = e.code
            return sp, nearest, nonempty, lm, err
        if pool is not None and len(big_keys) > 1:
            results = list(pool.map(model, big_keys))
        else:
            results = [model(c) for c in big_keys]
        for c, (sp, nearest, nonempty, lm, err) in zip(big_keys, results):
            rows = members[c]
            if err is not None:
                level.setdefault("model_errors", {})[c] = err
            pos = np.full(sp.shape[0], -1, np.int64)
            pos[nonempty] = np.arange(nonempty.shape[0])
            if lm is None:                                 # one bubble (reducer never runs) or D10
                labels = np.full(nonempty.shape[0], 2, np.int32)
            else:
                labels = lm["labels"].copy()
                iva, ivb, iw = lm["inter"]
                if iw.shape[0]:
                    gid = rows[sp[nonempty]].astype(np.int32)
                    if all_inter_edges:                    # D7
                        inter_edges.append((gid[iva], gid[ivb], iw.copy()))
                    else:                                  # Main.java:256-261 literal
                        inter_edges.append((iva[:1].copy(), ivb[:1].copy(), iw[:1].copy()))
            level["labels"][c] = labels.copy()
            # partition induction (Main.java:272-289): ascending labels -> next ids, in place
            distinct = sorted(set(int(x) for x in labels))
            for cl in distinct:
                labels[labels == cl] = next_id
                next_id += 1
            level["new_keys"][c] = sorted(set(int(x) for x in labels))
            if len(level["new_keys"][c]) == 1:
                forced.add(level["new_keys"][c][0])        # D9
            # LabelClassification.java:21-37
            nk = labels[pos[nearest]]
            new_key[rows] = nk
            new_alive[rows] = True
        edge_lists.extend(inter_edges)
        key_of = np.where(new_alive, new_key, key_of)
        alive = new_alive
        levels.append(level)
    va, vb, w = O.merge_edges(edge_lists)                  # UnionFindReducer + SortMST
    out = dict(edges=(va, vb, w), levels=levels, leaf_of=leaf_of, iterations=iteration)
    if all_inter_edges and flat:                           # D6: global flat labels (O(levels n))
        from .flat_labels import flat_labels
        out["labels"], out["n_clusters"] = flat_labels(n, va, vb, w, min_cl_size)
    return out
