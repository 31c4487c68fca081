"""TEST INFRASTRUCTURE ONLY -- CPU restatement of the global HDBSCAN* hierarchy and flat
(FOSC / excess-of-mass) labels over a merged MST: SURVEY.md §8(f) #1, the step the reference
never completes (Main.java:351-408 calls System.exit(1) inside its first level).

It follows the canonical top-down procedure of HDBSCANStar.computeHierarchyAndClusterTree
(HDBSCANStar.java:208-474, commented out in the reference), propagateTree (:505-540) and
findProminentClusters (:567-625), without constraints, with these canonical choices where the
Java's result depends on container iteration order (documented in DESIGN.md, "flat labels"):

  * all edges tied at the current level are removed together (:254-271); every affected
    cluster then splits into the connected components of its remaining edges (:274-390);
    a component is a valid child iff it has >= minClusterSize points (minClusterSize >= 2,
    so a component with one point never has edges and is noise, :320-322, :360-368);
    >= 2 valid children: the cluster dies and each valid child is a new cluster born at the
    level; 1 valid child: the cluster keeps that child's points and the rest become noise;
    0 valid children: every point becomes noise;
  * stability(C) = sum over the levels eps at which points leave C, in descending eps, of
    count * (1/eps - 1/birth(C)) -- Cluster.detachPoints, one term per (cluster, level);
  * propagation (Cluster.propagate): a leaf cluster propagates itself; otherwise the cluster
    itself if stability >= propagated stability (ties keep the parent), else its propagated
    descendants; a parent's propagated stability sums its children's contributions in
    ascending order of the child's smallest point id;
  * the root (all points, birth NaN) is never selected: solution = root's propagated
    descendants; flat label of a point = the selected cluster containing it at that cluster's
    birth (the hierarchy line at the cluster's file offset), numbered 1..K by ascending
    smallest point id; 0 = noise.

Straightforward O(levels * n) restatement for small inputs (the product is the bottom-up
union-find in csrc/flat.cpp).
"""
from __future__ import annotations

import numpy as np


class _Cluster:
    __slots__ = ("birth", "parent", "members", "children", "stab", "minid")

    def __init__(self, birth, parent, members):
        self.birth = birth
        self.parent = parent
        self.members = members          # points at birth
        self.children = []
        self.stab = 0.0
        self.minid = min(members)


def flat_labels(n, va, vb, w, min_cl_size):
    """va, vb, w: tree edges (self edges are ignored).  Returns (labels, n_clusters)."""
    if min_cl_size < 2:
        raise ValueError("min_cl_size must be >= 2")
    if n <= 1:
        return np.zeros(max(n, 0), np.int32), 0
    va, vb, w = np.asarray(va), np.asarray(vb), np.asarray(w, np.float64)
    keep = va != vb
    va, vb, w = va[keep], vb[keep], w[keep]
    if va.shape[0] != n - 1:
        raise ValueError("not a spanning tree")
    adj = [dict() for _ in range(n)]  # neighbour -> edge weight
    for a, b, x in zip(va.tolist(), vb.tolist(), w.tolist()):
        adj[a][b] = x
        adj[b][a] = x
    parent = list(range(n))           # cycle check (the edges must be a tree)

    def find(x):
        while parent[x] != x:
            parent[x] = parent[parent[x]]
            x = parent[x]
        return x
    for a, b in zip(va.tolist(), vb.tolist()):
        ra, rb = find(a), find(b)
        if ra == rb:
            raise ValueError("the edges contain a cycle")
        parent[rb] = ra
    label = np.ones(n, np.int64)      # current cluster per point (0 = noise)
    clusters = {1: _Cluster(np.float64("nan"), None, list(range(n)))}
    next_label = 2
    levels = sorted(set(w.tolist()), reverse=True)
    for eps in levels:
        idx = np.nonzero(w == eps)[0]
        affected = set()
        for e in idx:
            a, b = int(va[e]), int(vb[e])
            del adj[a][b]
            del adj[b][a]
            if label[a] != 0:
                affected.add(int(label[a]))
        for L in sorted(affected):
            pts = np.nonzero(label == L)[0].tolist()
            seen = set()
            comps = []
            for p in pts:
                if p in seen:
                    continue
                comp, stack = [p], [p]
                seen.add(p)
                while stack:
                    u = stack.pop()
                    for v in adj[u]:
                        if v not in seen:
                            seen.add(v)
                            comp.append(v)
                            stack.append(v)
                comps.append(comp)
            if len(comps) == 1:
                continue
            C = clusters[L]
            valid = [c for c in comps if len(c) >= min_cl_size]
            leaving = 0
            if len(valid) >= 2:
                leaving = len(pts)
                for c in sorted(valid, key=min):
                    nc = _Cluster(np.float64(eps), C, c)
                    C.children.append(nc)
                    clusters[next_label] = nc
                    label[c] = next_label
                    next_label += 1
                for c in comps:
                    if len(c) < min_cl_size:
                        label[c] = 0
            else:
                for c in comps:
                    if len(c) < min_cl_size:
                        leaving += len(c)
                        label[c] = 0
                if not valid:
                    leaving = len(pts)
            with np.errstate(divide="ignore", invalid="ignore"):  # IEEE, as Java: 1/0 = inf
                C.stab = np.float64(C.stab) + np.float64(leaving) * (np.float64(1.0) / np.float64(eps)
                                                                     - np.float64(1.0) / C.birth)
    # propagateTree (HDBSCANStar.java:505-540): descending label = every child before its parent
    contrib = {}
    solution = []
    for L in sorted(clusters, reverse=True):
        C = clusters[L]
        prop, desc = np.float64(0.0), []
        for k in C.children:                 # created in ascending min point id
            prop = prop + contrib[id(k)][0]
            desc = desc + contrib[id(k)][1]
        if C.parent is None:                 # root: findProminentClusters takes its descendants
            solution = desc
            continue
        if not C.children or C.stab >= prop:  # Cluster.propagate: ties keep the parent
            contrib[id(C)] = (C.stab, [C])
        else:
            contrib[id(C)] = (prop, desc)
    solution = sorted(solution, key=lambda c: c.minid)
    out = np.zeros(n, np.int32)
    for i, c in enumerate(solution):
        out[c.members] = i + 1
    return out, len(solution)
