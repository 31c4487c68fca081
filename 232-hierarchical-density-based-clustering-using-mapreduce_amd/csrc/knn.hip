// knn.hip -- K1: tiled FP64 k-nearest-neighbour lists and the three core-distance
// semantics of the reference (HDBSCANStar.java:71-106, CoreDistanceMapper.java:71-109,
// CreateLocalMST.java:138-185).
//
// Layout: X is repacked into Xp[n][DP] (DP = d rounded up to even, zero padded) so one
// candidate row is an aligned 16/32/64-byte scalar load.  Every lane owns Q queries in
// registers; the candidate loop index is wave-uniform, so candidate rows arrive through
// the scalar cache into SGPRs and feed v_add_f64/v_mul_f64 directly (no LDS round trip).
// Per pair: d v_add_f64 (sub), d v_mul_f64, d-1 v_add_f64, 1 v_cmp_f64 (the reference's
// exact operation order; no FMA: -ffp-contract=off).  Euclidean selects on the squared
// distance and takes the sqrt once per kept value (sqrt is monotone, so the k smallest
// sqrt values are the sqrt of the k smallest squares).  A rare predicated insertion
// network keeps the per-query top-K sorted in registers.
#include "knn_impl.hpp"

namespace hdb {

// ------------------------------------------------------------------ pack
__global__ void pack_rows_kernel(const double *__restrict__ X, int64_t n, int d, int dp,
                                 double *__restrict__ Xp) {
    HDB_GRID_STRIDE(t, n * dp) {
        int64_t r = t / dp;
        int c = (int)(t - r * dp);
        Xp[t] = c < d ? X[r * d + c] : 0.0;
    }
}

void pack_rows(hdb_ctx *ctx, const double *X, int64_t n, int d, int dp, double *Xp) {
    if (n <= 0) return;
    int64_t tot = n * dp;
    int grid = (int)std::min<int64_t>(ceil_div(tot, 256), 8192);
    hipLaunchKernelGGL(pack_rows_kernel, dim3(grid), dim3(256), 0, ctx->stream, X, n, d, dp, Xp);
    HIP_CHECK(hipGetLastError());
}

thread_local F32Screen g_screen;

// bounding box per dimension (one block per dimension)
__global__ void knn_bbox_kernel(const double *__restrict__ X, int64_t n, int d, double *__restrict__ lo,
                                double *__restrict__ hi) {
    const int c = blockIdx.x;
    __shared__ double sl[256], sh[256];
    double l = INFINITY, h = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        double v = X[i * d + c];
        l = v < l ? v : l;
        h = v > h ? v : h;
        if (v != v) {  // NaN poisons the box -> FP64-only path
            l = NAN;
            h = NAN;
        }
    }
    sl[threadIdx.x] = l;
    sh[threadIdx.x] = h;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            double a = sl[threadIdx.x], b = sl[threadIdx.x + s];
            sl[threadIdx.x] = (a != a || b != b) ? NAN : (a < b ? a : b);
            a = sh[threadIdx.x];
            b = sh[threadIdx.x + s];
            sh[threadIdx.x] = (a != a || b != b) ? NAN : (a > b ? a : b);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        lo[c] = sl[0];
        hi[c] = sh[0];
    }
}

// shift + FP32 pack; params[0] = E, params[1] = 1 if the FP32 screen is usable
__global__ void knn_pack_f32_kernel(const double *__restrict__ X, int64_t n, int d, int df,
                                    const double *__restrict__ lo, const double *__restrict__ hi,
                                    float *__restrict__ Xf, double *__restrict__ params) {
    double Mp = 0;
    bool ok = true;
    for (int c = 0; c < d; c++) {
        double l = lo[c], h = hi[c];
        if (!(l <= h) || !(h - l < 1e300)) ok = false;
        double half = (h - l) * 0.5;
        Mp = half > Mp ? half : Mp;
    }
    ok = ok && Mp <= 1e15;
    HDB_GRID_STRIDE(t, n * df) {
        int64_t r = t / df;
        int c = (int)(t - r * df);
        float v = 0.0f;
        if (c < d && ok) {
            double ctr = lo[c] + (hi[c] - lo[c]) * 0.5;
            v = (float)(X[r * d + c] - ctr);
        }
        Xf[t] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // |x - ctr| <= M' (+ rounding of ctr): pad M' by 1e-12 relative
        params[0] = sqrt((double)d) * 4.0 * 5.9604644775390625e-08 * (Mp * (1.0 + 1e-12)) * 1.01 + 1e-300;
        params[1] = ok ? 1.0 : 0.0;
    }
}

// ------------------------------------------------ generic (any metric, any d)
// One query per lane; values compared directly as in Java (buffer init Double.MAX_VALUE).
template <int K>
__global__ __launch_bounds__(256) void knn_generic_kernel(const double *__restrict__ X, int64_t n, int d,
                                                          int metric, int excl, int64_t cand_chunk,
                                                          double *__restrict__ part_v) {
    const int64_t qi = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t c_lo = (int64_t)blockIdx.y * cand_chunk;
    const int64_t c_hi = min(c_lo + cand_chunk, n);
    const int64_t r = qi < n ? qi : 0;
    double buf[K];
#pragma unroll
    for (int k = 0; k < K; k++) buf[k] = JMAX;
    for (int64_t j = c_lo; j < c_hi; j++) {
        if (excl && j == qi) continue;
        double v = metric_distance(X + r * d, X + j * d, d, metric);
        topk_insert<K>(buf, v);
    }
    if (qi < n)
        for (int k = 0; k < K; k++) part_v[((int64_t)blockIdx.y * n + qi) * K + k] = buf[k];
}

template <int K>
__global__ void knn_merge_generic_kernel(const double *__restrict__ part_v, int64_t n, int S,
                                         double *__restrict__ out_v) {
    HDB_GRID_STRIDE(qi, n) {
        double buf[K];
        for (int k = 0; k < K; k++) buf[k] = part_v[qi * K + k];
        for (int s = 1; s < S; s++)
            for (int k = 0; k < K; k++) topk_insert<K>(buf, part_v[((int64_t)s * n + qi) * K + k]);
        for (int k = 0; k < K; k++) out_v[qi * K + k] = buf[k];
    }
}

// ------------------------------------------------------------- epilogues
// lists: n x KC (ascending, MAX padded); core = element K-1 (K <= KC)
__global__ void core_from_lists_kernel(const double *__restrict__ lists, int64_t n, int KC, int K,
                                       double *__restrict__ core) {
    HDB_GRID_STRIDE(i, n) core[i] = lists[i * KC + (K - 1)];
}

// INCL_SELF_CUMULATIVE (HDBSCANStar.java:79-103): the buffer is never reset, so
// core[i] = K-th smallest of the union of rows 0..i.  Chunked prefix merge.
template <int K>
__device__ __forceinline__ void merge_list(double (&buf)[K], const double *l, int KC) {
    for (int k = 0; k < K; k++) {
        double v = l[k];
        if (!(v < buf[K - 1])) break;
        topk_insert<K>(buf, v);
    }
}
template <int K>
__global__ void cumul_chunk_kernel(const double *__restrict__ lists, int64_t n, int KC, int64_t CH,
                                   double *__restrict__ agg) {
    HDB_GRID_STRIDE(c, ceil_div(n, CH)) {
        double buf[K];
        for (int k = 0; k < K; k++) buf[k] = JMAX;
        int64_t hi = min(n, (c + 1) * CH);
        for (int64_t i = c * CH; i < hi; i++) merge_list<K>(buf, lists + i * KC, KC);
        for (int k = 0; k < K; k++) agg[c * K + k] = buf[k];
    }
}
template <int K>
__global__ void cumul_scan_kernel(double *__restrict__ agg, int64_t nch) {
    // exclusive prefix over chunk aggregates, one lane (nch is small)
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double buf[K];
    for (int k = 0; k < K; k++) buf[k] = JMAX;
    for (int64_t c = 0; c < nch; c++) {
        double cur[K];
        for (int k = 0; k < K; k++) cur[k] = agg[c * K + k];
        for (int k = 0; k < K; k++) agg[c * K + k] = buf[k];
        for (int k = 0; k < K; k++) topk_insert<K>(buf, cur[k]);
    }
}
template <int K>
__global__ void cumul_apply_kernel(const double *__restrict__ lists, int64_t n, int KC, int64_t CH,
                                   const double *__restrict__ agg, double *__restrict__ core) {
    HDB_GRID_STRIDE(c, ceil_div(n, CH)) {
        double buf[K];
        for (int k = 0; k < K; k++) buf[k] = agg[c * K + k];
        int64_t hi = min(n, (c + 1) * CH);
        for (int64_t i = c * CH; i < hi; i++) {
            merge_list<K>(buf, lists + i * KC, KC);
            core[i] = buf[K - 1];
        }
    }
}

// ----------------------------------------------------------------- host
static bool dispatch_d(hdb_ctx *ctx, int d, int KC, bool excl, bool idx, const double *Xp, int64_t n, double *ov,
                       int32_t *oi) {
    switch (d) {
#define HDB_KNN_CASE(DD)                                     \
    case DD: knn_run_d##DD(ctx, KC, excl, idx, Xp, n, ov, oi); return true;
        HDB_KNN_DIMS(HDB_KNN_CASE)
#undef HDB_KNN_CASE
    default: return false;
    }
}

// Computes n x KC lists (KC = bucket >= k) into dev_v (and dev_i) on device.
// X_dev: n x d row-major on device.
void knn_lists_device(hdb_ctx *ctx, const double *X_dev, int64_t n, int d, int k, int metric, bool excl,
                      double *lists_v, int32_t *lists_i, int *KC_out) {
    int KC = pick_kc(k);
    if (KC < 0) HDB_THROW(HDB_EINVAL, "k too large (max 31)");
    *KC_out = KC;
    if (n == 0) return;
    if (metric == HDB_METRIC_EUCLIDEAN && !lists_i && ctx->knn_tree && n >= ctx->knn_tree_min_n &&
        knn_tree_device(ctx, X_dev, n, d, KC, excl, lists_v))
        return;
    // high-dimensional euclidean: K1m (bf16-split MFMA screen + exact FP64 re-check)
    if (metric == HDB_METRIC_EUCLIDEAN && !lists_i && ctx->knn_mfma && d > 16 && n >= ctx->knn_mfma_min_n &&
        knn_mfma_device(ctx, X_dev, n, d, KC, excl, lists_v))
        return;
    if (metric == HDB_METRIC_EUCLIDEAN) {
        int dp = (d + 1) & ~1;
        int df = d <= 4 ? 4 : (d <= 8 ? 8 : 16);
        // carve: Xp (FP64 padded) | Xf (FP32 shifted) | bbox lo/hi | params
        size_t b_xp = ((sizeof(double) * (size_t)(n * dp)) + 255) & ~size_t(255);
        size_t b_xf = ((sizeof(float) * (size_t)(n * df)) + 255) & ~size_t(255);
        char *base = (char *)arena(ctx, A_PAD, b_xp + b_xf + 1024 + 64 * 16);
        double *Xp = (double *)base;
        float *Xf = (float *)(base + b_xp);
        double *blo = (double *)(base + b_xp + b_xf), *bhi = blo + 64, *prm = bhi + 64;
        pack_rows(ctx, X_dev, n, d, dp, Xp);
        g_screen = F32Screen();
        if (d <= 16 && !ctx->force_fp64) {
            hipLaunchKernelGGL(knn_bbox_kernel, dim3(d), dim3(256), 0, ctx->stream, X_dev, n, d, blo, bhi);
            int g = (int)std::min<int64_t>(ceil_div(n * df, 256), 8192);
            hipLaunchKernelGGL(knn_pack_f32_kernel, dim3(g), dim3(256), 0, ctx->stream, X_dev, n, d, df, blo, bhi, Xf,
                               prm);
            HIP_CHECK(hipGetLastError());
            double h_ok = 0;
            HIP_CHECK(hipMemcpyAsync(&h_ok, prm + 1, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
            HIP_CHECK(hipStreamSynchronize(ctx->stream));
            g_screen.on = h_ok == 1.0;
            g_screen.Xf = Xf;
            g_screen.params = prm;
        }
        if (dispatch_d(ctx, d, KC, excl, lists_i != nullptr, Xp, n, lists_v, lists_i)) return;
    }
    if (lists_i) HDB_THROW(HDB_EINVAL, "neighbour indices need the euclidean metric with d in {1..6,8,16}");
    // generic path
    int tiles = (int)ceil_div(n, 256);
    int S = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ctx->num_cus * 8, tiles), 64));
    while (S > 1 && n / S < 256) S--;
    int64_t chunk = ceil_div(n, S);
    double *pv = (double *)arena(ctx, A_WORK2, sizeof(double) * (size_t)(S * n * KC));
    int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
#define GEN_CASE(KK)                                                                                     \
    case KK: {                                                                                           \
        KernelTimer t(ctx, "knn_generic");                                                               \
        hipLaunchKernelGGL(knn_generic_kernel<KK>, dim3(tiles, S), dim3(256), 0, ctx->stream, X_dev, n, d, \
                           metric, (int)excl, chunk, pv);                                                \
    }                                                                                                    \
        hipLaunchKernelGGL(knn_merge_generic_kernel<KK>, dim3(g), dim3(256), 0, ctx->stream, pv, n, S,     \
                           lists_v);                                                                     \
        break;
    switch (KC) {
        GEN_CASE(1)
        GEN_CASE(3)
        GEN_CASE(7)
        GEN_CASE(15)
        GEN_CASE(31)
    }
#undef GEN_CASE
    HIP_CHECK(hipGetLastError());
}

// core distances from per-row lists (n x KC, ascending, MAX padded): element K-1 per row,
// or the cumulative prefix merge of INCL_SELF_CUMULATIVE (HDBSCANStar.java:79-103)
void core_epilogue_device(hdb_ctx *ctx, const double *lists, int64_t n, int KC, int K, int semantics, double *core) {
    int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    if (semantics != HDB_CORE_INCL_SELF_CUMULATIVE) {
        hipLaunchKernelGGL(core_from_lists_kernel, dim3(g), dim3(256), 0, ctx->stream, lists, n, KC, K, core);
        HIP_CHECK(hipGetLastError());
        return;
    }
    const int64_t CH = 256;
    int64_t nch = ceil_div(n, CH);
    double *agg = (double *)arena(ctx, A_WORK2, sizeof(double) * (size_t)(nch * 32));
    int gc = (int)std::min<int64_t>(ceil_div(nch, 64), 4096);
#define CUM_CASE(KK)                                                                                          \
    case KK:                                                                                                  \
        hipLaunchKernelGGL(cumul_chunk_kernel<KK>, dim3(gc), dim3(64), 0, ctx->stream, lists, n, KC, CH, agg);  \
        hipLaunchKernelGGL(cumul_scan_kernel<KK>, dim3(1), dim3(64), 0, ctx->stream, agg, nch);                \
        hipLaunchKernelGGL(cumul_apply_kernel<KK>, dim3(gc), dim3(64), 0, ctx->stream, lists, n, KC, CH, agg,   \
                           core);                                                                             \
        break;
    switch (K) {
        CUM_CASE(1) CUM_CASE(2) CUM_CASE(3) CUM_CASE(4) CUM_CASE(5) CUM_CASE(6) CUM_CASE(7) CUM_CASE(8)
        CUM_CASE(9) CUM_CASE(10) CUM_CASE(11) CUM_CASE(12) CUM_CASE(13) CUM_CASE(14) CUM_CASE(15) CUM_CASE(16)
        CUM_CASE(17) CUM_CASE(18) CUM_CASE(19) CUM_CASE(20) CUM_CASE(21) CUM_CASE(22) CUM_CASE(23)
        CUM_CASE(24) CUM_CASE(25) CUM_CASE(26) CUM_CASE(27) CUM_CASE(28) CUM_CASE(29) CUM_CASE(30)
        CUM_CASE(31)
    default: HDB_THROW(HDB_EINVAL, "minPts too large");
    }
#undef CUM_CASE
    HIP_CHECK(hipGetLastError());
}

// core distances on device buffers
void core_distances_device(hdb_ctx *ctx, const double *X_dev, int64_t n, int d, int min_pts, int metric,
                           int semantics, double *core) {
    if (min_pts < 1) HDB_THROW(HDB_EINVAL, "minPts must be >= 1");
    if (n == 0) return;
    if (min_pts == 1) {  // HDBSCANStar.java:75-77
        HIP_CHECK(hipMemsetAsync(core, 0, sizeof(double) * (size_t)n, ctx->stream));
        return;
    }
    int K = min_pts - 1;
    int KC = pick_kc(K);
    if (KC < 0) HDB_THROW(HDB_EINVAL, "minPts too large (max 32)");
    double *lists = (double *)arena(ctx, A_WORK0, sizeof(double) * (size_t)(n * KC));
    bool excl = semantics == HDB_CORE_EXCL_SELF;
    knn_lists_device(ctx, X_dev, n, d, K, metric, excl, lists, nullptr, &KC);
    core_epilogue_device(ctx, lists, n, KC, K, semantics, core);
}

}  // namespace hdb
