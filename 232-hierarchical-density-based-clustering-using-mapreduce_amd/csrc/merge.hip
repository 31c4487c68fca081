// merge.hip -- a20: the reducers' merge of local MSTs (UnionFindReducer.java:19-69 with
// SortMST.java:9-17): stable sort of the concatenated edge lists by DESCENDING weight.
// LSD radix sort is stable, so equal weights keep their concatenation order exactly as
// Java's TimSort does.  -0.0 keys are canonicalised to +0.0 (Java's comparator treats them
// as equal).  The cross-GPU all-gather that builds the concatenation runs over RCCL in
// the host layer; this is the device-side reduce.
#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "sort.hpp"
#include "ssort.hpp"

namespace hdb {

__global__ void edge_keys_kernel(const double *__restrict__ w, int64_t ne, double *__restrict__ keys,
                                 int32_t *__restrict__ iota) {
    HDB_GRID_STRIDE(i, ne) {
        double x = w[i];
        keys[i] = (x == 0.0) ? 0.0 : x;
        iota[i] = (int32_t)i;
    }
}

__global__ void pos_fill_kernel(int32_t *__restrict__ p, int64_t n) {
    HDB_GRID_STRIDE(i, n) p[i] = (int32_t)i;
}

__global__ void edge_gather_kernel(const int32_t *__restrict__ perm, int64_t ne, const int32_t *__restrict__ a_in,
                                   const int32_t *__restrict__ b_in, const double *__restrict__ w_in,
                                   int32_t *__restrict__ a_out, int32_t *__restrict__ b_out,
                                   double *__restrict__ w_out) {
    HDB_GRID_STRIDE(i, ne) {
        int32_t p = perm[i];
        a_out[i] = a_in[p];
        b_out[i] = b_in[p];
        w_out[i] = w_in[p];
    }
}

// --- run-aware merge.  The exact leaf hands over its n-1 tree edges ascending by (w, lo, hi)
// followed by n self edges in id order, and the reducers' concatenations keep such runs: a
// non-decreasing prefix P (length p) and a rest R.  The stable descending order of P ++ R is
// then: R radix-sorted alone (stable, descending), P reversed tie group by tie group (equal
// weights keep their input order), and the two merged with P first on equal weights --
// output position of P[i] = its place in reversed P + #(R > w_i), of R'[j] = j + #(P >= w).
// Both counts are binary searches in sorted arrays.  Identical to the full stable sort.
// first descent f (w[f-1] > w[f]) kept as ne - f by atomicMax on a zeroed word
__global__ void run_scan_kernel(const double *__restrict__ w, int64_t ne, int64_t *__restrict__ first_desc,
                                int *__restrict__ nan) {
    int64_t f = ne;
    int bad = 0;
    HDB_GRID_STRIDE(i, ne) {
        const double a = w[i];
        if (a != a) bad = 1;
        if (i + 1 < ne && a > w[i + 1]) f = min(f, i + 1);
    }
    for (int o = 32; o >= 1; o >>= 1) {
        f = min(f, (int64_t)__shfl_xor((long long)f, o));
        bad |= __shfl_xor(bad, o);
    }
    if ((threadIdx.x & 63) == 0) {
        if (f < ne) atomicMax((unsigned long long *)first_desc, (unsigned long long)(ne - f));
        if (bad) atomicOr(nan, 1);
    }
}

__global__ void run_keys_kernel(const double *__restrict__ w, int64_t p, int64_t r, double *__restrict__ keys,
                                int32_t *__restrict__ iota) {
    HDB_GRID_STRIDE(j, r) {
        const double x = w[p + j];
        keys[j] = (x == 0.0) ? 0.0 : x;
        iota[j] = (int32_t)(p + j);
    }
}

// first index in ascending a[0, n) with a[k] >= x (k = n: none)
__device__ __forceinline__ int64_t lower_bound_asc(const double *a, int64_t n, double x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int64_t upper_bound_asc(const double *a, int64_t n, double x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
// first index in descending a[0, n) with a[k] <= x = #(a > x)
__device__ __forceinline__ int64_t count_greater_desc(const double *a, int64_t n, double x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] > x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void run_place_p_kernel(const int32_t *__restrict__ va, const int32_t *__restrict__ vb,
                                   const double *__restrict__ w, int64_t p, const double *__restrict__ rkeys, int64_t r,
                                   int32_t *__restrict__ oa, int32_t *__restrict__ ob, double *__restrict__ ow) {
    HDB_GRID_STRIDE(i, p) {
        const double x = w[i];
        int64_t gs = i, ge = i + 1;
        if ((i > 0 && w[i - 1] == x) || (i + 1 < p && w[i + 1] == x)) {  // a tie group (rare)
            gs = lower_bound_asc(w, p, x);
            ge = upper_bound_asc(w, p, x);
        }
        const int64_t o = (p - ge) + (i - gs) + count_greater_desc(rkeys, r, x);
        oa[o] = va[i];
        ob[o] = vb[i];
        ow[o] = x;
    }
}

__global__ void run_place_r_kernel(const int32_t *__restrict__ va, const int32_t *__restrict__ vb,
                                   const double *__restrict__ w, int64_t p, const double *__restrict__ rkeys,
                                   const int32_t *__restrict__ rperm, int64_t r, int32_t *__restrict__ oa,
                                   int32_t *__restrict__ ob, double *__restrict__ ow) {
    HDB_GRID_STRIDE(j, r) {
        const int32_t s = rperm[j];
        const int64_t o = j + (p - lower_bound_asc(w, p, rkeys[j]));
        oa[o] = va[s];
        ob[o] = vb[s];
        ow[o] = w[s];
    }
}

// ssort functors of the stable descending sort: the weight (order-preserving map of doubles
// to u64, -0.0 read as +0.0 like edge_keys_kernel's keys), ties by input position
struct DescKeyF {
    const double *w;
    __device__ SKey operator()(int64_t i) const {
        const double x = w[i];
        const uint64_t b = (uint64_t)__double_as_longlong(x == 0.0 ? 0.0 : x);
        return SKey{~((b >> 63) ? ~b : (b | 0x8000000000000000ull)), (uint64_t)i};
    }
};
struct GatherEmitF {
    const int32_t *va, *vb;
    const double *w;
    int32_t *oa, *ob;
    double *ow;
    __device__ void operator()(int64_t r, const SKey &k) const {
        const int64_t p = (int64_t)k.lo;
        oa[r] = va[p];
        ob[r] = vb[p];
        ow[r] = w[p];
    }
};

// in-place stable descending sort of (va, vb, w)
void sort_edges_desc_device(hdb_ctx *ctx, int32_t *va, int32_t *vb, double *w, int64_t ne) {
    if (ne <= 1) return;
    if (ne > INT32_MAX) HDB_THROW(HDB_EINVAL, "too many edges for one sort");
    if (ctx->ssort && !ctx->merge_runs) {
        const SsPlan pl = ss_plan(ne, ctx->ssort_cap);
        if (pl.nb) {
            KernelTimer t(ctx, "merge_sort");
            const size_t eb = ((size_t)ne * 4 + 255) & ~size_t(255);
            char *tmp = (char *)arena(ctx, A_WORK3, 2 * eb + (size_t)ne * 8);
            int32_t *ta = (int32_t *)tmp, *tb_ = (int32_t *)(tmp + eb);
            double *tw = (double *)(tmp + 2 * eb);
            ssort(pl, (char *)arena(ctx, A_SS, pl.bytes), DescKeyF{w}, GatherEmitF{va, vb, w, ta, tb_, tw}, ctx->stream);
            HIP_CHECK(hipMemcpyAsync(va, ta, sizeof(int32_t) * ne, hipMemcpyDeviceToDevice, ctx->stream));
            HIP_CHECK(hipMemcpyAsync(vb, tb_, sizeof(int32_t) * ne, hipMemcpyDeviceToDevice, ctx->stream));
            HIP_CHECK(hipMemcpyAsync(w, tw, sizeof(double) * ne, hipMemcpyDeviceToDevice, ctx->stream));
            return;
        }
    }
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t o_k = carve(sizeof(double) * ne), o_k2 = carve(sizeof(double) * ne), o_i = carve(sizeof(int32_t) * ne),
           o_p = carve(sizeof(int32_t) * ne), o_a = carve(sizeof(int32_t) * ne), o_b = carve(sizeof(int32_t) * ne),
           o_w = carve(sizeof(double) * ne), o_x = carve(sizeof(int64_t) * 2);
    char *base = (char *)arena(ctx, A_WORK3, off);
    double *keys = (double *)(base + o_k), *keys2 = (double *)(base + o_k2);
    int32_t *iota = (int32_t *)(base + o_i), *perm = (int32_t *)(base + o_p);
    int32_t *ta = (int32_t *)(base + o_a), *tb_ = (int32_t *)(base + o_b);
    double *tw = (double *)(base + o_w);
    int64_t *xw = (int64_t *)(base + o_x);
    int g = (int)std::min<int64_t>(ceil_div(ne, 256), 8192);
    hipStream_t st = ctx->stream;
    KernelTimer t(ctx, "merge_sort");
    int64_t p = 0;
    if (ctx->merge_runs && ne >= 4096) {
        int64_t *pin = pinned_words(ctx) + PINNED_WORDS - 16;  // private slice
        HIP_CHECK(hipMemsetAsync(xw, 0, sizeof(int64_t) * 2, st));
        hipLaunchKernelGGL(run_scan_kernel, dim3(g), dim3(256), 0, st, w, ne, xw, (int *)(xw + 1));
        HIP_CHECK(hipMemcpyAsync(pin, xw, sizeof(int64_t) * 2, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        const int64_t pre = ne - pin[0];  // the device keeps ne - (first descent), 0: none
        // a short prefix does not pay for the extra pass; NaN keys keep the radix order
        if (pin[1] == 0 && pre >= ne / 4) p = pre;
    }
    if (p > 0) {
        const int64_t r = ne - p;
        if (r > 0) {
            const int gr = (int)std::min<int64_t>(ceil_div(r, 256), 8192);
            hipLaunchKernelGGL(run_keys_kernel, dim3(gr), dim3(256), 0, st, w, p, r, keys, iota);
            size_t tb = 0;
            HIP_CHECK(sort_pairs_desc(nullptr, tb, keys, keys2, iota, perm, r, 0, 64, st));
            void *tmp = arena(ctx, A_SORT, tb);
            HIP_CHECK(sort_pairs_desc(tmp, tb, keys, keys2, iota, perm, r, 0, 64, st));
            hipLaunchKernelGGL(run_place_r_kernel, dim3(gr), dim3(256), 0, st, va, vb, w, p, keys2, perm, r, ta, tb_,
                               tw);
        }
        hipLaunchKernelGGL(run_place_p_kernel, dim3((int)std::min<int64_t>(ceil_div(p, 256), 8192)), dim3(256), 0, st,
                           va, vb, w, p, keys2, r, ta, tb_, tw);
    } else {
        hipLaunchKernelGGL(edge_keys_kernel, dim3(g), dim3(256), 0, st, w, ne, keys, iota);
        size_t tb = 0;
        HIP_CHECK(sort_pairs_desc(nullptr, tb, keys, keys2, iota, perm, ne, 0, 64, st));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(sort_pairs_desc(tmp, tb, keys, keys2, iota, perm, ne, 0, 64, st));
        hipLaunchKernelGGL(edge_gather_kernel, dim3(g), dim3(256), 0, st, perm, ne, va, vb, w, ta, tb_, tw);
    }
    HIP_CHECK(hipMemcpyAsync(va, ta, sizeof(int32_t) * ne, hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipMemcpyAsync(vb, tb_, sizeof(int32_t) * ne, hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipMemcpyAsync(w, tw, sizeof(double) * ne, hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------ merge of presorted runs
// Stable merge of two descending runs A, B (A first on equal weights) by merge-path tiles:
// a workgroup finds where its MP_T outputs start in A and B (one diagonal binary search per
// end), stages both slices' weights in LDS, and every thread places its outputs with a binary
// search inside the tile.
constexpr int MP_T = 1024, MP_TB = 256;
__device__ __forceinline__ int64_t mp_split(const double *wA, int64_t na, const double *wB, int64_t nb, int64_t k) {
    int64_t lo = k - nb > 0 ? k - nb : 0, hi = k < na ? k : na;
    while (lo < hi) {  // the number of A elements among the first k outputs
        const int64_t mid = (lo + hi) >> 1;
        if (wA[mid] >= wB[k - mid - 1]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(MP_TB) void merge_path_kernel(const int32_t *__restrict__ aA, const int32_t *__restrict__ bA,
                                                         const double *__restrict__ wA, int64_t na,
                                                         const int32_t *__restrict__ aB, const int32_t *__restrict__ bB,
                                                         const double *__restrict__ wB, int64_t nb,
                                                         int32_t *__restrict__ oa, int32_t *__restrict__ ob,
                                                         double *__restrict__ ow) {
    __shared__ double sw[2 * MP_T];
    __shared__ int64_t s_i[2];
    const int64_t k0 = (int64_t)blockIdx.x * MP_T, k1 = min(k0 + MP_T, na + nb);
    if (threadIdx.x < 2) s_i[threadIdx.x] = mp_split(wA, na, wB, nb, threadIdx.x ? k1 : k0);
    __syncthreads();
    const int64_t i0 = s_i[0], j0 = k0 - i0, i1 = s_i[1], j1 = k1 - i1;
    const int nA = (int)(i1 - i0), nB = (int)(j1 - j0);
    for (int t = threadIdx.x; t < nA; t += MP_TB) sw[t] = wA[i0 + t];
    for (int t = threadIdx.x; t < nB; t += MP_TB) sw[nA + t] = wB[j0 + t];
    __syncthreads();
    const int cnt = (int)(k1 - k0);
    for (int t = threadIdx.x; t < cnt; t += MP_TB) {
        int lo = t - nB > 0 ? t - nB : 0, hi = t < nA ? t : nA;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sw[mid] >= sw[nA + t - mid - 1]) lo = mid + 1;
            else hi = mid;
        }
        const int i = lo, j = t - lo;
        const bool takeA = j >= nB || (i < nA && sw[i] >= sw[nA + j]);
        const int64_t k = k0 + t;
        if (takeA) {
            oa[k] = aA[i0 + i];
            ob[k] = bA[i0 + i];
            ow[k] = sw[i];
        } else {
            oa[k] = aB[j0 + j];
            ob[k] = bB[j0 + j];
            ow[k] = sw[nA + j];
        }
    }
}

// two descending runs in separate arrays, A first on equal weights (the exact leaf's merged
// order: its tree edges and its self edges)
void merge_two_runs_device(hdb_ctx *ctx, const int32_t *aA, const int32_t *bA, const double *wA, int64_t na,
                           const int32_t *aB, const int32_t *bB, const double *wB, int64_t nb, int32_t *oa,
                           int32_t *ob, double *ow) {
    if (na + nb <= 0) return;
    hipLaunchKernelGGL(merge_path_kernel, dim3((unsigned)ceil_div(na + nb, (int64_t)MP_T)), dim3(MP_TB), 0, ctx->stream,
                       aA, bA, wA, na, aB, bB, wB, nb, oa, ob, ow);
    HIP_CHECK(hipGetLastError());
}

// precondition check: no NaN, every run non-increasing (bit 0 / bit 1)
__global__ void runs_check_kernel(const double *__restrict__ w, int64_t ne, const int64_t *__restrict__ run_end_flag,
                                  int *__restrict__ err) {
    int e = 0;
    HDB_GRID_STRIDE(i, ne) {
        const double x = w[i];
        if (x != x) e |= 1;
        if (i + 1 < ne && !run_end_flag[i] && x < w[i + 1]) e |= 2;
    }
    if (e) atomicOr(err, e);
}

void merge_sorted_runs_device(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w,
                              const std::vector<int64_t> &off, int32_t *oa, int32_t *ob, double *ow) {
    hipStream_t st = ctx->stream;
    const int nr = (int)off.size() - 1;
    const int64_t ne = off.back();
    if (ne <= 0) return;
    KernelTimer t(ctx, "merge_runs");
    // scratch: the ping-pong buffer, the run-end flags, the error word
    const size_t sb = ((size_t)ne * 16 + 255) & ~size_t(255);
    char *base = (char *)arena(ctx, A_WORK3, sb + (size_t)ne * 8 + 512);
    int32_t *ta = (int32_t *)base, *tb_ = ta + ne;
    double *tw = (double *)(base + (((size_t)ne * 8 + 255) & ~size_t(255)));
    int64_t *flag = (int64_t *)(base + sb);
    int *err = (int *)(flag + ne);
    HIP_CHECK(hipMemsetAsync(flag, 0, (size_t)ne * 8 + 512, st));
    std::vector<int64_t> ends;
    for (int r = 0; r < nr; r++)
        if (off[r + 1] > off[r]) ends.push_back(off[r + 1] - 1);
    for (int64_t e : ends) HIP_CHECK(hipMemsetAsync(flag + e, 0xff, 8, st));
    hipLaunchKernelGGL(runs_check_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(ne, 256), 8192)), dim3(256), 0, st,
                       w, ne, flag, err);
    // pairwise rounds; the last round writes the outputs
    std::vector<int64_t> cur = off;
    const int32_t *sa = va, *sbv = vb;
    const double *sw = w;
    int rounds = 0;
    for (int k = 1; k < nr; k <<= 1) rounds++;
    if (rounds == 0) {
        HIP_CHECK(hipMemcpyAsync(oa, va, 4 * ne, hipMemcpyDeviceToDevice, st));
        HIP_CHECK(hipMemcpyAsync(ob, vb, 4 * ne, hipMemcpyDeviceToDevice, st));
        HIP_CHECK(hipMemcpyAsync(ow, w, 8 * ne, hipMemcpyDeviceToDevice, st));
    }
    for (int r = 0; r < rounds; r++) {
        // the last round lands in the outputs; earlier ones alternate so the input is never overwritten
        const bool last = r == rounds - 1;
        int32_t *da = last ? oa : ((rounds - 1 - r) & 1 ? ta : oa);
        int32_t *db = last ? ob : ((rounds - 1 - r) & 1 ? tb_ : ob);
        double *dw = last ? ow : ((rounds - 1 - r) & 1 ? tw : ow);
        std::vector<int64_t> nxt{0};
        for (size_t p = 0; p + 1 < cur.size(); p += 2) {
            const int64_t a0 = cur[p], a1 = cur[p + 1];
            const int64_t b1 = p + 2 < cur.size() ? cur[p + 2] : a1;  // an odd run passes through
            const int64_t na = a1 - a0, nb = b1 - a1;
            if (na + nb > 0)
                hipLaunchKernelGGL(merge_path_kernel, dim3((unsigned)ceil_div(na + nb, (int64_t)MP_T)), dim3(MP_TB), 0,
                                   st, sa + a0, sbv + a0, sw + a0, na, sa + a1, sbv + a1, sw + a1, nb, da + a0, db + a0,
                                   dw + a0);
            nxt.push_back(b1);
        }
        cur = nxt;
        sa = da;
        sbv = db;
        sw = dw;
    }
    int h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h & 1) HDB_THROW(HDB_EINVAL, "merge_sorted_runs: NaN weight");
    if (h & 2) HDB_THROW(HDB_EINVAL, "merge_sorted_runs: a run is not sorted descending");
}

// ------------------------------------------------ CreateLocalMST record fields
// fake1 / fake2 of CreateLocalMST's records (CreateLocalMST.java:242,266,276-285) are the
// partition-local indices of an edge's two vertices: the position of the global id in the
// partition's `indices` array.  ids sorted once (radix), one binary search per endpoint.
__global__ void local_ids_dup_kernel(const int32_t *__restrict__ keys, int64_t n, int *__restrict__ err) {
    HDB_GRID_STRIDE(i, n - 1) {
        if (keys[i] == keys[i + 1]) atomicOr(err, 1);
    }
}

__device__ __forceinline__ int32_t local_of(const int32_t *keys, const int32_t *pos, int64_t n, int32_t id, int *err) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < id) lo = mid + 1;
        else hi = mid;
    }
    if (lo >= n || keys[lo] != id) {
        atomicOr(err, 2);
        return -1;
    }
    return pos[lo];
}

__global__ void local_ids_kernel(const int32_t *__restrict__ keys, const int32_t *__restrict__ pos, int64_t n,
                                 const int32_t *__restrict__ va, const int32_t *__restrict__ vb,
                                 const double *__restrict__ w, int64_t ne, int32_t node, int32_t *__restrict__ f1,
                                 int32_t *__restrict__ f2, int32_t *__restrict__ nd, int *__restrict__ err) {
    HDB_GRID_STRIDE(e, ne) {
        // a tree edge never relaxed keeps Java's default nearestneighborsID = 0
        // (CreateLocalMST.java:203,242; weight still Double.MAX_VALUE)
        const bool unset = w && e < n - 1 && w[e] == JMAX;
        if (keys) {
            f1[e] = unset ? 0 : local_of(keys, pos, n, va[e], err);
            f2[e] = local_of(keys, pos, n, vb[e], err);
        } else {
            f1[e] = unset ? 0 : va[e];
            f2[e] = vb[e];
        }
        if (nd) nd[e] = node;
    }
}

void local_mst_ids_device(hdb_ctx *ctx, const int32_t *ids, int64_t n, const int32_t *va, const int32_t *vb,
                          const double *w, int64_t ne, int32_t node, int32_t *fake1, int32_t *fake2,
                          int32_t *node_out) {
    if (ne <= 0) return;
    hipStream_t st = ctx->stream;
    const int g = (int)std::min<int64_t>(ceil_div(ne, 256), 8192);
    int32_t *keys = nullptr, *pos = nullptr;
    int *err = nullptr;
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    const size_t o_e = carve(sizeof(int) * 4), o_k = carve(sizeof(int32_t) * std::max<int64_t>(n, 1)),
                 o_k2 = carve(sizeof(int32_t) * std::max<int64_t>(n, 1)), o_p = carve(sizeof(int32_t) * std::max<int64_t>(n, 1)),
                 o_p2 = carve(sizeof(int32_t) * std::max<int64_t>(n, 1));
    char *base = (char *)arena(ctx, A_WORK3, off);
    err = (int *)(base + o_e);
    HIP_CHECK(hipMemsetAsync(err, 0, sizeof(int) * 4, st));
    if (ids) {
        if (n > INT32_MAX) HDB_THROW(HDB_EINVAL, "too many vertices");
        int32_t *k1 = (int32_t *)(base + o_k), *p1 = (int32_t *)(base + o_p);
        keys = (int32_t *)(base + o_k2);
        pos = (int32_t *)(base + o_p2);
        HIP_CHECK(hipMemcpyAsync(k1, ids, sizeof(int32_t) * n, hipMemcpyDefault, st));
        hipLaunchKernelGGL(pos_fill_kernel, dim3((int)std::min<int64_t>(ceil_div(n, 256), 8192)), dim3(256), 0, st, p1, n);
        size_t tb = 0;
        HIP_CHECK(sort_pairs(nullptr, tb, k1, keys, p1, pos, n, 0, 32, st));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(sort_pairs(tmp, tb, k1, keys, p1, pos, n, 0, 32, st));
        hipLaunchKernelGGL(local_ids_dup_kernel, dim3((int)std::min<int64_t>(ceil_div(n, 256), 8192)), dim3(256), 0, st,
                           keys, n, err);
    }
    hipLaunchKernelGGL(local_ids_kernel, dim3(g), dim3(256), 0, st, keys, pos, n, va, vb, w, ne, node, fake1, fake2,
                       node_out, err);
    int h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h & 1) HDB_THROW(HDB_EINVAL, "local MST ids: duplicate vertex ids in the partition");
    if (h & 2) HDB_THROW(HDB_EINVAL, "local MST ids: an edge vertex is not in the partition");
}

// ------------------------------------------------------- pairwise distance
__global__ void distance_rows_kernel(const double *__restrict__ a, const double *__restrict__ b, int64_t n, int d,
                                     int metric, double *__restrict__ out) {
    HDB_GRID_STRIDE(i, n) out[i] = metric_distance(a + i * d, b + i * d, d, metric);
}

void distance_rows_device(hdb_ctx *ctx, const double *a, const double *b, int64_t n, int d, int metric, double *out) {
    if (n <= 0) return;
    int g = (int)std::min<int64_t>(ceil_div(n, 256), 8192);
    hipLaunchKernelGGL(distance_rows_kernel, dim3(g), dim3(256), 0, ctx->stream, a, b, n, d, metric, out);
    HIP_CHECK(hipGetLastError());
}

}  // namespace hdb
