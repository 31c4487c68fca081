"""Multi-GPU layer: one process per GPU, torch.distributed over RCCL ("nccl" backend on
ROCm) -- or gloo on CPU for tests.

The only real exchange step on the hot path is the reducers' merge of local MSTs
(UnionFindReducer.java:19-69 / Main.java:302-347): every rank holds the edge lists of its
own partitions; an all-gather of the padded (va, vb, w) blocks builds the concatenation in
rank order, and one stable descending sort (SortMST) on the device merges it.  Partitions
themselves are independent, so no collective runs inside the per-partition kernels.
"""
from __future__ import annotations

import numpy as np


def all_gather_edges(va, vb, w, group=None):
    """All-gather variable-length edge blocks in rank order (RCCL has no allgatherv: counts
    first, then fixed-size padded blocks).  Tensors must live on this rank's device for
    nccl, or on the CPU for gloo."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)
    dev = w.device
    n = torch.tensor([w.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    # pack (va, vb) as one int64 lane and w as float64 so two collectives move everything
    ab = torch.zeros(m, dtype=torch.int64, device=dev)
    ab[: w.shape[0]] = (va.to(torch.int64) << 32) | (vb.to(torch.int64) & 0xFFFFFFFF)
    ww = torch.zeros(m, dtype=torch.float64, device=dev)
    ww[: w.shape[0]] = w
    abs_ = [torch.empty_like(ab) for _ in range(ws)]
    wws = [torch.empty_like(ww) for _ in range(ws)]
    dist.all_gather(abs_, ab, group=group)
    dist.all_gather(wws, ww, group=group)
    ab_all = torch.cat([a[:c] for a, c in zip(abs_, counts)])
    w_all = torch.cat([x[:c] for x, c in zip(wws, counts)])
    va_all = (ab_all >> 32).to(torch.int32)
    vb_all = (ab_all & 0xFFFFFFFF).to(torch.int32)
    return va_all, vb_all, w_all


def merge_local_msts(va, vb, w, group=None, sort: bool = True):
    """All-gather + stable descending sort (SortMST.java:9-17) of every rank's local edges."""
    from .databubbles import sort_edges_desc

    va_all, vb_all, w_all = all_gather_edges(va, vb, w, group)
    if sort:
        if w_all.device.type == "cuda":
            sort_edges_desc(va_all, vb_all, w_all)
        else:
            # CPU (gloo) path for multi-process tests: stable sort by descending weight
            order = np.argsort(-w_all.numpy(), kind="stable")
            import torch
            o = torch.from_numpy(order)
            va_all, vb_all, w_all = va_all[o], vb_all[o], w_all[o]
    return va_all, vb_all, w_all
