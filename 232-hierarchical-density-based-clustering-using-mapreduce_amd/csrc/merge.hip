// merge.hip -- a20: the reducers' merge of local MSTs (UnionFindReducer.java:19-69 with
// SortMST.java:9-17): stable sort of the concatenated edge lists by DESCENDING weight.
// LSD radix sort is stable, so equal weights keep their concatenation order exactly as
// Java's TimSort does.  -0.0 keys are canonicalised to +0.0 (Java's comparator treats them
// as equal).  The cross-GPU all-gather that builds the concatenation runs over RCCL in
// the host layer; this is the device-side reduce.
#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "sort.hpp"

namespace hdb {

__global__ void edge_keys_kernel(const double *__restrict__ w, int64_t ne, double *__restrict__ keys,
                                 int32_t *__restrict__ iota) {
    HDB_GRID_STRIDE(i, ne) {
        double x = w[i];
        keys[i] = (x == 0.0) ? 0.0 : x;
        iota[i] = (int32_t)i;
    }
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

// in-place stable descending sort of (va, vb, w)
void sort_edges_desc_device(hdb_ctx *ctx, int32_t *va, int32_t *vb, double *w, int64_t ne) {
    if (ne <= 1) return;
    if (ne > INT32_MAX) HDB_THROW(HDB_EINVAL, "too many edges for one sort");
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t o_k = carve(sizeof(double) * ne), o_k2 = carve(sizeof(double) * ne), o_i = carve(sizeof(int32_t) * ne),
           o_p = carve(sizeof(int32_t) * ne), o_a = carve(sizeof(int32_t) * ne), o_b = carve(sizeof(int32_t) * ne),
           o_w = carve(sizeof(double) * ne);
    char *base = (char *)arena(ctx, A_WORK3, off);
    double *keys = (double *)(base + o_k), *keys2 = (double *)(base + o_k2);
    int32_t *iota = (int32_t *)(base + o_i), *perm = (int32_t *)(base + o_p);
    int32_t *ta = (int32_t *)(base + o_a), *tb_ = (int32_t *)(base + o_b);
    double *tw = (double *)(base + o_w);
    int g = (int)std::min<int64_t>(ceil_div(ne, 256), 8192);
    KernelTimer t(ctx, "merge_sort");
    hipLaunchKernelGGL(edge_keys_kernel, dim3(g), dim3(256), 0, ctx->stream, w, ne, keys, iota);
    size_t tb = 0;
    HIP_CHECK(sort_pairs_desc(nullptr, tb, keys, keys2, iota, perm, ne, 0, 64, ctx->stream));
    void *tmp = arena(ctx, A_SORT, tb);
    HIP_CHECK(sort_pairs_desc(tmp, tb, keys, keys2, iota, perm, ne, 0, 64, ctx->stream));
    hipLaunchKernelGGL(edge_gather_kernel, dim3(g), dim3(256), 0, ctx->stream, perm, ne, va, vb, w, ta, tb_, tw);
    HIP_CHECK(hipMemcpyAsync(va, ta, sizeof(int32_t) * ne, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(vb, tb_, sizeof(int32_t) * ne, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(w, tw, sizeof(double) * ne, hipMemcpyDeviceToDevice, ctx->stream));
    HIP_CHECK(hipGetLastError());
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
