// comm.cpp -- the reducers' cross-GPU merge (SURVEY.md §8(b) hdb_merge_edges, §8(e)):
// UnionFindReducer.call + SortMST (UnionFindReducer.java:19-69, SortMST.java:9-17) over the
// local edge lists of every rank: RCCL all-gather (counts, then padded blocks -- RCCL has no
// all-gatherv) over xGMI, then one stable descending radix sort on every rank.
//
// Order: Spark concatenates the reducers' inputs in its own order; the product fixes it
// (D5): with `seq` (the canonical position of each local edge in the iteration-major
// concatenation, a permutation of [0, E) over all ranks) every edge is scattered to that
// position before the stable sort, so the merged list does not depend on which rank
// computed which partition; without it the concatenation is rank-major.
//
// RCCL is resolved at run time (dlopen of librccl.so.1): inside a PyTorch process this is the
// copy torch already loaded, in a JNI process the ROCm one.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <mutex>

#include "internal.hpp"

namespace hdb {
namespace {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    std::string err;
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            r.err = std::string("cannot load librccl.so.1: ") + dlerror();
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy)
            r.err = "librccl.so.1 lacks the NCCL API symbols";
    });
    if (!r.err.empty()) HDB_THROW(HDB_EDEVICE, r.err);
    return r;
}

#define RCCL_CHECK(expr)                                                                             \
    do {                                                                                             \
        ncclResult_t _r = (expr);                                                                    \
        if (_r != ncclSuccess)                                                                       \
            HDB_THROW(HDB_EDEVICE, std::string(#expr) + ": " +                                       \
                                       (rccl().error_string ? rccl().error_string(_r) : "RCCL error")); \
    } while (0)

}  // namespace

// scatter the gathered, padded rank blocks into the merged order
__global__ void merge_place_kernel(const int32_t *__restrict__ ga, const int32_t *__restrict__ gb,
                                   const double *__restrict__ gw, const int64_t *__restrict__ gs,
                                   const int64_t *__restrict__ offs, int nranks, int64_t maxc, int64_t total,
                                   int32_t *__restrict__ va, int32_t *__restrict__ vb, double *__restrict__ w,
                                   int32_t *__restrict__ seen, int *__restrict__ err) {
    HDB_GRID_STRIDE(i, (int64_t)nranks * maxc) {
        const int r = (int)(i / maxc);
        const int64_t k = i - (int64_t)r * maxc;
        if (k >= offs[r + 1] - offs[r]) continue;
        int64_t dst = offs[r] + k;
        if (gs) {
            dst = gs[i];
            if (dst < 0 || dst >= total || atomicExch(&seen[dst], 1) != 0) {
                atomicOr(err, 1);
                continue;
            }
        }
        va[dst] = ga[i];
        vb[dst] = gb[i];
        w[dst] = gw[i];
    }
}

}  // namespace hdb

struct hdb_comm {
    hdb_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
};

using namespace hdb;

extern "C" {

int hdb_comm_unique_id(void *id_out, int32_t cap) {
    try {
        if (!id_out || cap < (int32_t)sizeof(ncclUniqueId)) HDB_THROW(HDB_EINVAL, "id buffer too small");
        ncclUniqueId id;
        RCCL_CHECK(rccl().get_unique_id(&id));
        std::memcpy(id_out, &id, sizeof(id));
        return (int)sizeof(id);
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

int hdb_comm_init(hdb_ctx *ctx, int32_t nranks, int32_t rank, const void *id, hdb_comm **out) {
    try {
        if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) HDB_THROW(HDB_EINVAL, "bad arguments");
        HIP_CHECK(hipSetDevice(ctx->device));
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        hdb_comm *c = new hdb_comm();
        c->ctx = ctx;
        c->nranks = nranks;
        c->rank = rank;
        ncclResult_t r = rccl().comm_init_rank(&c->comm, nranks, uid, rank);
        if (r != ncclSuccess) {
            delete c;
            RCCL_CHECK(r);
        }
        *out = c;
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

void hdb_comm_destroy(hdb_comm *comm) {
    if (!comm) return;
    try {
        if (comm->comm) rccl().comm_destroy(comm->comm);
    } catch (const Error &) {
    }
    delete comm;
}

int hdb_free(void *p) {
    if (!p) return HDB_OK;
    return hipFree(p) == hipSuccess ? HDB_OK : HDB_EDEVICE;
}

int hdb_copy(hdb_ctx *ctx, void *dst, const void *src, int64_t bytes) {
    if (!ctx || bytes < 0 || (bytes && (!dst || !src))) return HDB_EINVAL;
    try {
        HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

int hdb_merge_edges(hdb_comm *comm, const int32_t *va, const int32_t *vb, const double *w, const int64_t *seq,
                    int64_t e_local, int32_t **va_all, int32_t **vb_all, double **w_all, int64_t *e_all) {
    if (!comm || !comm->ctx) {
        set_error("comm is NULL");
        return HDB_EINVAL;
    }
    hdb_ctx *ctx = comm->ctx;
    try {
        if (e_local < 0 || !va_all || !vb_all || !w_all || !e_all || (e_local > 0 && (!va || !vb || !w)))
            HDB_THROW(HDB_EINVAL, "bad arguments");
        HIP_CHECK(hipSetDevice(ctx->device));
        hipStream_t st = ctx->stream;
        Stager sg(ctx);
        const int32_t *da = sg.in(va, (size_t)e_local), *db = sg.in(vb, (size_t)e_local);
        const double *dw = sg.in(w, (size_t)e_local);
        const int64_t *ds = sg.in(seq, (size_t)e_local);
        const int R = comm->nranks;
        KernelTimer t(ctx, "merge_edges");
        // 1. counts (and whether every rank passes seq: all or none; a rank with no local
        //    edges is consistent with either -- its seq pointer may well be NULL)
        int64_t *cnt_dev = nullptr;
        HIP_CHECK(hipMallocAsync((void **)&cnt_dev, sizeof(int64_t) * 2 * (R + 1), st));
        int64_t mine[2] = {e_local, e_local == 0 ? -1 : (seq ? 1 : 0)};
        HIP_CHECK(hipMemcpyAsync(cnt_dev + 2 * R, mine, sizeof(mine), hipMemcpyHostToDevice, st));
        RCCL_CHECK(rccl().all_gather(cnt_dev + 2 * R, cnt_dev, 2, ncclInt64, comm->comm, st));
        std::vector<int64_t> cnt(2 * R);
        HIP_CHECK(hipMemcpyAsync(cnt.data(), cnt_dev, sizeof(int64_t) * 2 * R, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        std::vector<int64_t> offs(R + 1, 0);
        int64_t maxc = 0, with_seq = 0, without_seq = 0;
        for (int r = 0; r < R; r++) {
            offs[r + 1] = offs[r] + cnt[2 * r];
            maxc = std::max(maxc, cnt[2 * r]);
            with_seq += cnt[2 * r + 1] == 1;
            without_seq += cnt[2 * r + 1] == 0;
        }
        if (with_seq && without_seq)
            HDB_THROW(HDB_EINVAL, "merge_edges: seq must be given on every rank with local edges or on none");
        const int64_t nseq = with_seq;
        const int64_t E = offs[R];
        // 2. padded blocks: [va | vb | w | seq] per rank
        const size_t blk = (size_t)maxc * (4 + 4 + 8 + (nseq ? 8 : 0));
        char *send = nullptr, *recv = nullptr;
        HIP_CHECK(hipMallocAsync((void **)&send, std::max<size_t>(blk, 16), st));
        HIP_CHECK(hipMallocAsync((void **)&recv, std::max<size_t>(blk * R, 16), st));
        auto part = [&](char *base, int k) {  // k: 0 va, 1 vb, 2 w, 3 seq
            static const size_t pre[4] = {0, 4, 8, 16};
            return base + (size_t)maxc * pre[k];
        };
        if (e_local) {
            HIP_CHECK(hipMemcpyAsync(part(send, 0), da, 4 * e_local, hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(part(send, 1), db, 4 * e_local, hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(part(send, 2), dw, 8 * e_local, hipMemcpyDeviceToDevice, st));
            if (nseq) HIP_CHECK(hipMemcpyAsync(part(send, 3), ds, 8 * e_local, hipMemcpyDeviceToDevice, st));
        }
        if (blk) RCCL_CHECK(rccl().all_gather(send, recv, blk, ncclInt8, comm->comm, st));
        // 3. rank blocks -> merged order (library-allocated outputs, hdb_free)
        int32_t *oa = nullptr, *ob = nullptr;
        double *ow = nullptr;
        HIP_CHECK(hipMalloc((void **)&oa, sizeof(int32_t) * std::max<int64_t>(E, 1)));
        HIP_CHECK(hipMalloc((void **)&ob, sizeof(int32_t) * std::max<int64_t>(E, 1)));
        HIP_CHECK(hipMalloc((void **)&ow, sizeof(double) * std::max<int64_t>(E, 1)));
        int64_t *offs_dev = cnt_dev;  // reuse: R + 1 words
        HIP_CHECK(hipMemcpyAsync(offs_dev, offs.data(), sizeof(int64_t) * (R + 1), hipMemcpyHostToDevice, st));
        int32_t *seen = nullptr;
        int *err = nullptr;
        HIP_CHECK(hipMallocAsync((void **)&seen, sizeof(int32_t) * std::max<int64_t>(E, 1) + 16, st));
        err = (int *)(seen + std::max<int64_t>(E, 1));
        HIP_CHECK(hipMemsetAsync(seen, 0, sizeof(int32_t) * std::max<int64_t>(E, 1) + 16, st));
        char *lay = nullptr;
        HIP_CHECK(hipMallocAsync((void **)&lay, std::max<size_t>(blk * R, 16), st));
        // recv is R blocks of [va(maxc) vb(maxc) w(maxc) seq(maxc)]; make each field contiguous over ranks
        for (int r = 0; r < R && maxc; r++) {
            char *src = recv + blk * r;
            HIP_CHECK(hipMemcpyAsync(lay + (size_t)maxc * 4 * r, src, 4 * maxc, hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(lay + (size_t)maxc * (4 * R + 4 * r), src + 4 * maxc, 4 * maxc,
                                     hipMemcpyDeviceToDevice, st));
            HIP_CHECK(hipMemcpyAsync(lay + (size_t)maxc * (8 * R + 8 * r), src + 8 * maxc, 8 * maxc,
                                     hipMemcpyDeviceToDevice, st));
            if (nseq)
                HIP_CHECK(hipMemcpyAsync(lay + (size_t)maxc * (16 * R + 8 * r), src + 16 * maxc, 8 * maxc,
                                         hipMemcpyDeviceToDevice, st));
        }
        if (E) {
            const int g = (int)std::min<int64_t>(ceil_div((int64_t)R * maxc, 256), 16384);
            hipLaunchKernelGGL(merge_place_kernel, dim3(g), dim3(256), 0, st, (const int32_t *)lay,
                               (const int32_t *)(lay + (size_t)maxc * 4 * R), (const double *)(lay + (size_t)maxc * 8 * R),
                               nseq ? (const int64_t *)(lay + (size_t)maxc * 16 * R) : nullptr, offs_dev, R, maxc, E,
                               oa, ob, ow, seen, err);
            HIP_CHECK(hipGetLastError());
        }
        int herr = 0;
        HIP_CHECK(hipMemcpyAsync(&herr, err, sizeof(int), hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        (void)hipFreeAsync(send, st);
        (void)hipFreeAsync(recv, st);
        (void)hipFreeAsync(lay, st);
        (void)hipFreeAsync(seen, st);
        (void)hipFreeAsync(cnt_dev, st);
        if (herr) {
            (void)hipFree(oa);
            (void)hipFree(ob);
            (void)hipFree(ow);
            HDB_THROW(HDB_EINVAL, "merge_edges: seq is not a permutation of the merged positions");
        }
        // 4. SortMST: stable, descending weight
        sort_edges_desc_device(ctx, oa, ob, ow, E);
        HIP_CHECK(hipStreamSynchronize(st));
        sg.finish();
        *va_all = oa;
        *vb_all = ob;
        *w_all = ow;
        *e_all = E;
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return HDB_ENOMEM;
    }
}

}  // extern "C"
