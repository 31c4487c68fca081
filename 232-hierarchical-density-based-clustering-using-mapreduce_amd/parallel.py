"""Multi-GPU layer: one process per GPU, torch.distributed over RCCL ("nccl" backend on
ROCm) -- or gloo (CPU tensors) for tests -- plus the library's own RCCL communicator for the
reducers' merge (hdb_merge_edges, the C-ABI a JNI-bound Java driver calls).

SURVEY.md §8(e): partitions are independent, so the per-partition kernels run with no
collective; the exchanges are
  * the reducers' merge of local MSTs (UnionFindReducer.java:19-69 / Main.java:302-347):
    all-gather of every rank's edge list, scatter into the canonical (iteration-major, D5)
    concatenation order via per-edge sequence numbers, one stable descending sort (SortMST);
  * the level loop's small exchanges (driver.py): nearest-sample assignments of a rank's
    point chunk, local-model results of the subsets a rank owns.
Work is split deterministically (every rank computes the same plan): LPT on the cost
estimate (leaves: n_i^2, local models: b_i^2), contiguous chunks for point-parallel work.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi as A


# ------------------------------------------------------------------ process group helpers
def world_rank(group=None):
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0
    return dist.get_world_size(group), dist.get_rank(group)


def _coll_device(group=None):
    """Tensors for collectives: the current HIP device under nccl, the CPU under gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def lpt(costs, world: int):
    """Longest-processing-time assignment: items by descending cost (ties: ascending index)
    to the least-loaded rank (ties: lowest rank).  Deterministic on every rank."""
    owner = np.zeros(len(costs), np.int64)
    load = np.zeros(world, np.float64)
    for i in sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i)):
        r = int(np.argmin(load))
        owner[i] = r
        load[r] += float(costs[i])
    return owner


def chunk(n: int, world: int, rank: int):
    """Contiguous split of [0, n): rank r gets [n r / W, n (r+1) / W)."""
    return n * rank // world, n * (rank + 1) // world


def allgather_object(obj, group=None):
    import torch.distributed as dist
    world, _ = world_rank(group)
    out = [None] * world
    dist.all_gather_object(out, obj, group=group)
    return out


def allgather_var(t, group=None):
    """All-gather of variable-length 1-D tensors in rank order (RCCL has no all-gatherv:
    counts first, then fixed-size padded blocks)."""
    import torch
    import torch.distributed as dist
    world, _ = world_rank(group)
    dev = _coll_device(group)
    src = t.to(dev)
    n = torch.tensor([src.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    pad = torch.zeros(m, dtype=src.dtype, device=dev)
    pad[: src.shape[0]] = src
    blocks = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(blocks, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(blocks, counts)]).to(t.device)


# ------------------------------------------------------------------ the library communicator
class HdbComm:
    """hdb_comm (RCCL) for this rank's context: rank 0 makes the unique id, the process group
    carries it to the others (in a Spark driver: a broadcast variable)."""

    def __init__(self, ctx, group=None):
        import torch.distributed as dist
        world, rank = world_rank(group)
        uid = C.create_string_buffer(128)
        if rank == 0:
            n = A.lib().hdb_comm_unique_id(uid, 128)
            if n < 0:
                A.check(n, "hdb_comm_unique_id")
        box = [uid.raw if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(box, src=0, group=group)
        self.ctx = ctx
        self.h = C.c_void_p()
        A.check(A.lib().hdb_comm_init(ctx.h, world, rank, C.create_string_buffer(box[0], 128), C.byref(self.h)),
                "hdb_comm_init")

    def close(self):
        if self.h:
            A.lib().hdb_comm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gather_sorted_msts(va, vb, w, dst: int = 0, group=None):
    """The reducers' merge when every rank already holds its own list sorted (stable,
    descending -- the order SortMST gives it): gather the blocks in rank order to `dst` only
    (UnionFindReducer runs as one reducer, Main.java:302-347) and merge them there as presorted
    runs (hdb_merge_sorted_runs: lower rank first on equal weights).  Equal to
    merge_local_msts on the unsorted blocks -- a stable sort of a concatenation is the stable
    merge of its stably sorted runs -- without the re-sort of the whole list.  Returns the
    merged (va, vb, w) on `dst`, None on the other ranks."""
    import torch
    import torch.distributed as dist
    world, rank = world_rank(group)
    dev = _coll_device(group)
    n = torch.tensor([w.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    out = []
    for t in (va, vb, w):
        src = t.to(dev)
        if src.shape[0] != m:  # equal block sizes (the usual case) go without a pad copy
            pad = torch.zeros(m, dtype=src.dtype, device=dev)
            pad[: src.shape[0]] = src
            src = pad
        big = torch.empty(world * m, dtype=src.dtype, device=dev) if rank == dst else None
        dist.gather(src, list(big.split(m)) if big is not None else None, dst=dst, group=group)
        out.append(big)
    if rank != dst:
        return None
    if m * world != sum(counts):
        keep = torch.cat([torch.arange(r * m, r * m + c) for r, c in enumerate(counts)]).to(dev)
        out = [x[keep] for x in out]
    out = [x.to(w.device) for x in out]
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    if out[2].device.type == "cuda":
        from .databubbles import merge_sorted_runs
        return merge_sorted_runs(out[0], out[1], out[2], off)
    # CPU tensors (gloo tests): the stable descending order of the concatenation (-0.0 == 0.0)
    key = np.where(out[2].numpy() == 0.0, 0.0, out[2].numpy())
    o = torch.from_numpy(np.argsort(-key, kind="stable"))
    return out[0][o], out[1][o], out[2][o]


def _merge_via_comm(comm: HdbComm, va, vb, w, seq):
    import torch
    ctx = comm.ctx
    pa, pb, pw = C.c_void_p(), C.c_void_p(), C.c_void_p()
    e = C.c_int64()
    # an empty tensor's data_ptr() is 0: the library treats a rank with no local edges as
    # consistent with either seq mode, so NULL is fine there
    s = seq.to(torch.int64).contiguous() if seq is not None else None
    A.check(A.lib().hdb_merge_edges(comm.h, va.data_ptr(), vb.data_ptr(), w.data_ptr(),
                                    s.data_ptr() if s is not None else None, w.shape[0], C.byref(pa), C.byref(pb),
                                    C.byref(pw), C.byref(e)), "hdb_merge_edges")
    E = int(e.value)
    dev = w.device
    out = (torch.empty(E, dtype=torch.int32, device=dev), torch.empty(E, dtype=torch.int32, device=dev),
           torch.empty(E, dtype=torch.float64, device=dev))
    try:
        for t, p in zip(out, (pa, pb, pw)):
            A.check(A.lib().hdb_copy(ctx.h, t.data_ptr(), p, t.element_size() * E), "hdb_copy")
    finally:
        for p in (pa, pb, pw):
            A.lib().hdb_free(p)
    return out


def merge_local_msts(va, vb, w, group=None, seq=None, comm: HdbComm | None = None, sort: bool = True):
    """UnionFindReducer + SortMST over every rank's local edges: all-gather, place each edge
    at its canonical position `seq` (a permutation of [0, E) over all ranks; None = rank-major
    concatenation), stable descending sort.  With an HdbComm the library does it over RCCL
    (hdb_merge_edges); otherwise torch.distributed carries the blocks (gloo tests, CPU)."""
    import torch
    if comm is not None:
        return _merge_via_comm(comm, va, vb, w, seq)
    va_all, vb_all = allgather_var(va, group), allgather_var(vb, group)
    w_all = allgather_var(w, group)
    if seq is not None:
        s_all = allgather_var(seq.to(torch.int64), group)
        E = w_all.shape[0]
        if s_all.shape[0] != E or not torch.equal(torch.sort(s_all.cpu())[0], torch.arange(E)):
            raise A.HdbError(-1, "merge: seq is not a permutation of the merged positions")
        inv = torch.empty_like(s_all)
        inv[s_all] = torch.arange(E, dtype=s_all.dtype, device=s_all.device)
        va_all, vb_all, w_all = va_all[inv], vb_all[inv], w_all[inv]
    if sort and w_all.shape[0]:
        if w_all.device.type == "cuda":
            from .databubbles import sort_edges_desc
            va_all, vb_all, w_all = va_all.contiguous(), vb_all.contiguous(), w_all.contiguous()
            sort_edges_desc(va_all, vb_all, w_all)
        else:  # CPU tensors (gloo tests): stable sort by descending weight (-0.0 == 0.0)
            key = np.where(w_all.numpy() == 0.0, 0.0, w_all.numpy())
            o = torch.from_numpy(np.argsort(-key, kind="stable"))
            va_all, vb_all, w_all = va_all[o], vb_all[o], w_all[o]
    return va_all, vb_all, w_all
