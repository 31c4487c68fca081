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
#include "internal.hpp"

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

// ------------------------------------------------------------ main kernel
// grid.x = query tiles of 256*Q rows, grid.y = candidate splits.
// part_v/part_i: [split][n][K] squared-domain partial lists (split 0 only when S == 1,
// in which case the sqrt epilogue is applied here and written to out).
template <int D, int DP, int K, int Q, int U, bool EXCL, bool IDX>
__global__ __launch_bounds__(256) void knn_sq_kernel(const double *__restrict__ Xp, int64_t n,
                                                     int64_t cand_chunk, double *__restrict__ part_v,
                                                     int32_t *__restrict__ part_i, int finalize) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * Q);
    const int64_t qhi = min(q0 + (int64_t)256 * Q, n);
    const int64_t c_lo = (int64_t)blockIdx.y * cand_chunk;
    const int64_t c_hi = min(c_lo + cand_chunk, n);

    double xq[Q][D];
    double buf[Q][K];
    int bidx[Q][K];
    int64_t qi[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
        qi[q] = q0 + threadIdx.x + (int64_t)q * 256;
        const int64_t r = qi[q] < n ? qi[q] : 0;
#pragma unroll
        for (int c = 0; c < D; c++) xq[q][c] = Xp[r * DP + c];
#pragma unroll
        for (int k = 0; k < K; k++) {
            buf[q][k] = INFINITY;
            bidx[q][k] = -1;
        }
    }

    // candidate segments: [c_lo, a) plain, [a, b) self-check (EXCL only), [b, c_hi) plain
    int64_t a = c_hi, b = c_hi;
    if (EXCL) {
        a = max(c_lo, min(c_hi, q0));
        b = max(a, min(c_hi, qhi));
    }
#pragma unroll 1
    for (int seg = 0; seg < 3; seg++) {
        int64_t s_lo = seg == 0 ? c_lo : (seg == 1 ? a : b);
        int64_t s_hi = seg == 0 ? a : (seg == 1 ? b : c_hi);
        const bool chk = EXCL && seg == 1;
        int64_t j = s_lo;
#pragma unroll 1
        for (; j + U <= s_hi; j += U) {
            double s[U][Q];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const double *cr = Xp + (j + u) * DP;
                double cc[D];
#pragma unroll
                for (int c = 0; c < D; c++) cc[c] = cr[c];
#pragma unroll
                for (int q = 0; q < Q; q++) {
                    double acc = sq_diff(xq[q][0], cc[0]);
#pragma unroll
                    for (int c = 1; c < D; c++) acc = acc + sq_diff(xq[q][c], cc[c]);
                    if (chk && qi[q] == j + u) acc = INFINITY;
                    s[u][q] = acc;
                }
            }
            bool hit = false;
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int q = 0; q < Q; q++) hit |= s[u][q] < buf[q][K - 1];
            if (hit) {
#pragma unroll
                for (int u = 0; u < U; u++)
#pragma unroll
                    for (int q = 0; q < Q; q++) {
                        if (IDX) topk_insert_idx<K>(buf[q], bidx[q], s[u][q], (int)(j + u));
                        else topk_insert<K>(buf[q], s[u][q]);
                    }
            }
        }
#pragma unroll 1
        for (; j < s_hi; j++) {
            const double *cr = Xp + j * DP;
            double cc[D];
#pragma unroll
            for (int c = 0; c < D; c++) cc[c] = cr[c];
#pragma unroll
            for (int q = 0; q < Q; q++) {
                double acc = sq_diff(xq[q][0], cc[0]);
#pragma unroll
                for (int c = 1; c < D; c++) acc = acc + sq_diff(xq[q][c], cc[c]);
                if (chk && qi[q] == j) acc = INFINITY;
                if (IDX) topk_insert_idx<K>(buf[q], bidx[q], acc, (int)j);
                else topk_insert<K>(buf[q], acc);
            }
        }
    }

#pragma unroll
    for (int q = 0; q < Q; q++) {
        if (qi[q] >= n) continue;
        const int64_t o = ((int64_t)blockIdx.y * n + qi[q]) * K;
#pragma unroll
        for (int k = 0; k < K; k++) {
            double v = buf[q][k];
            if (finalize) v = (v < INFINITY) ? sqrt(v) : JMAX;  // Java keeps Double.MAX_VALUE
            part_v[o + k] = v;
            if (IDX) part_i[o + k] = (finalize && !(buf[q][k] < INFINITY)) ? -1 : bidx[q][k];
        }
    }
}

// ----------------------------------------------- FP32-filtered exact kernel
// Same contract as knn_sq_kernel, but each pair is first screened in FP32 (2-cycle VALU
// ops instead of 4-cycle FP64): coordinates are shifted by the data's bounding-box centre
// and rounded to FP32 (Xf), s32 = sum (xf - cf)^2 with fmaf.  A rigorous bound makes the
// screen conservative: with M' = max |x - centre| and E = sqrt(d) * 4 * 2^-24 * M' * 1.01,
//   ||x - c|| >= sqrt(s32 / (1 + d 2^-24)) - E,
// so s32 >= thr(tau) = ((sqrt(tau (1+1e-14)) + E)^2 (1 + 1e-5)) rounded up to FP32 proves
// the exact FP64 s64 >= tau (no insertion).  A group of U x Q pairs goes to the exact FP64
// path (the reference's operation order, identical to knn_sq_kernel) only when some lane
// has a pair below its threshold -- rare once the top-K has warmed up.  Results are the
// FP64 results bit for bit; the filter only skips provably rejected pairs.
__device__ __forceinline__ float knn_thr32(double tau, double E) {
    if (!(tau < INFINITY)) return INFINITY;
    double r = sqrt(tau * (1.0 + 1e-14)) + E;
    double T = (r * r) * (1.0 + 1e-5);
    float f = (float)T;
    if ((double)f < T) f = nextafterf(f, INFINITY);
    return f;
}

template <int D, int DF, int DP, int K, int Q, int U, bool EXCL, bool IDX>
__global__ __launch_bounds__(256) void knn_f32x_kernel(const float *__restrict__ Xf, const double *__restrict__ Xp,
                                                       const double *__restrict__ params, int64_t n,
                                                       int64_t cand_chunk, double *__restrict__ part_v,
                                                       int32_t *__restrict__ part_i, int finalize) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * Q);
    const int64_t qhi = min(q0 + (int64_t)256 * Q, n);
    const int64_t c_lo = (int64_t)blockIdx.y * cand_chunk;
    const int64_t c_hi = min(c_lo + cand_chunk, n);
    const double E = params[0];

    float xf[Q][D];
    double xq[Q][D];
    double buf[Q][K];
    int bidx[Q][K];
    float thr[Q];
    int64_t qi[Q];
#pragma unroll
    for (int q = 0; q < Q; q++) {
        qi[q] = q0 + threadIdx.x + (int64_t)q * 256;
        const int64_t r = qi[q] < n ? qi[q] : 0;
#pragma unroll
        for (int c = 0; c < D; c++) {
            xq[q][c] = Xp[r * DP + c];
            xf[q][c] = Xf[r * DF + c];
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            buf[q][k] = INFINITY;
            bidx[q][k] = -1;
        }
        thr[q] = INFINITY;
    }
    // exact FP64 test of one pair (reference operation order) + insertion
    auto exact = [&](int q, const double (&cc)[D], int64_t jcand, bool self_chk) {
        double acc = sq_diff(xq[q][0], cc[0]);
#pragma unroll
        for (int c = 1; c < D; c++) acc = acc + sq_diff(xq[q][c], cc[c]);
        if (self_chk && qi[q] == jcand) acc = INFINITY;
        if (acc < buf[q][K - 1]) {
            if (IDX) topk_insert_idx<K>(buf[q], bidx[q], acc, (int)jcand);
            else topk_insert<K>(buf[q], acc);
            thr[q] = knn_thr32(buf[q][K - 1], E);
        }
    };
    auto exact_range = [&](int64_t lo, int64_t hi, bool self_chk) {
#pragma unroll 1
        for (int64_t j = lo; j < hi; j++) {
            const double *cr = Xp + j * DP;
            double cc[D];
#pragma unroll
            for (int c = 0; c < D; c++) cc[c] = cr[c];
#pragma unroll
            for (int q = 0; q < Q; q++) exact(q, cc, j, self_chk);
        }
    };
    // screened range, candidates staged through LDS: the block's 4 waves share every chunk
    // of CH candidates (FP32, DF floats each) -- one coalesced global load per thread per
    // chunk, double-buffered, one barrier per chunk; waves read candidates with broadcast
    // ds_reads (in order, so reads run ahead of use).  FP32 test per pair; the exact FP64
    // re-test runs only for (candidate, query) pairs some lane screened in.
    constexpr int CH = 256;
    constexpr int V4 = DF / 4;  // float4 per candidate
    __shared__ float4 sc[2][CH * V4];
    auto screened_range = [&](int64_t lo, int64_t hi) {
        if (lo >= hi) return;
        const int64_t nch = (hi - lo + CH - 1) / CH;
        float4 pre[V4];
        auto prefetch = [&](int64_t k) {
            const int64_t j = lo + k * CH + threadIdx.x;
            const float4 *src = reinterpret_cast<const float4 *>(Xf + (j < hi ? j : lo) * DF);
#pragma unroll
            for (int v = 0; v < V4; v++) pre[v] = src[v];
        };
        auto stage = [&](int buf) {
#pragma unroll
            for (int v = 0; v < V4; v++) sc[buf][threadIdx.x * V4 + v] = pre[v];
        };
        prefetch(0);
        stage(0);
        __syncthreads();
#pragma unroll 1
        for (int64_t k = 0; k < nch; k++) {
            const int buf = (int)(k & 1);
            if (k + 1 < nch) prefetch(k + 1);
            const int64_t jb = lo + k * CH;
            const int cnt = (int)min((int64_t)CH, hi - jb);
            const int ng = cnt / U;
#pragma unroll 1
            for (int g = 0; g < ng; g++) {
                bool pass[U][Q];
                bool any = false;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    const float4 c4 = sc[buf][(g * U + u) * V4];
                    float cf[D];
#pragma unroll
                    for (int c = 0; c < D; c++) {
                        if (c < 4) cf[c] = c == 0 ? c4.x : (c == 1 ? c4.y : (c == 2 ? c4.z : c4.w));
                        else {
                            const float4 e = sc[buf][(g * U + u) * V4 + c / 4];
                            const int r = c & 3;
                            cf[c] = r == 0 ? e.x : (r == 1 ? e.y : (r == 2 ? e.z : e.w));
                        }
                    }
#pragma unroll
                    for (int q = 0; q < Q; q++) {
                        float t0 = xf[q][0] - cf[0];
                        float acc = t0 * t0;
#pragma unroll
                        for (int c = 1; c < D; c++) {
                            float t = xf[q][c] - cf[c];
                            acc = __builtin_fmaf(t, t, acc);
                        }
                        pass[u][q] = !(acc >= thr[q]);
                        any |= pass[u][q];
                    }
                }
                if (!any) continue;
                const int64_t j = jb + g * U;
#pragma unroll
                for (int u = 0; u < U; u++) {
                    bool pu = false;
#pragma unroll
                    for (int q = 0; q < Q; q++) pu |= pass[u][q];
                    if (!pu) continue;
                    const double *cr = Xp + (j + u) * DP;
                    double cc[D];
#pragma unroll
                    for (int c = 0; c < D; c++) cc[c] = cr[c];
#pragma unroll
                    for (int q = 0; q < Q; q++)
                        if (pass[u][q]) exact(q, cc, j + u, false);
                }
            }
            exact_range(jb + (int64_t)ng * U, jb + cnt, false);  // chunk tail
            if (k + 1 < nch) stage(buf ^ 1);
            __syncthreads();
        }
    };
    if (EXCL) {
        const int64_t a = max(c_lo, min(c_hi, q0));
        const int64_t b = max(a, min(c_hi, qhi));
        screened_range(c_lo, a);
        exact_range(a, b, true);  // the query tile itself: self pairs excluded
        screened_range(b, c_hi);
    } else {
        screened_range(c_lo, c_hi);
    }
#pragma unroll
    for (int q = 0; q < Q; q++) {
        if (qi[q] >= n) continue;
        const int64_t o = ((int64_t)blockIdx.y * n + qi[q]) * K;
#pragma unroll
        for (int k = 0; k < K; k++) {
            double v = buf[q][k];
            if (finalize) v = (v < INFINITY) ? sqrt(v) : JMAX;
            part_v[o + k] = v;
            if (IDX) part_i[o + k] = (finalize && !(buf[q][k] < INFINITY)) ? -1 : bidx[q][k];
        }
    }
}

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

// merge S partial squared-domain lists per query and finalize (sqrt, MAX padding)
template <int K, bool IDX>
__global__ void knn_merge_kernel(const double *__restrict__ part_v, const int32_t *__restrict__ part_i,
                                 int64_t n, int S, double *__restrict__ out_v, int32_t *__restrict__ out_i) {
    HDB_GRID_STRIDE(qi, n) {
        double buf[K];
        int bidx[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            buf[k] = part_v[qi * K + k];
            bidx[k] = IDX ? part_i[qi * K + k] : -1;
        }
        for (int s = 1; s < S; s++) {
            const int64_t o = ((int64_t)s * n + qi) * K;
            for (int k = 0; k < K; k++) {
                double v = part_v[o + k];
                if (!(v < buf[K - 1])) break;  // lists are ascending
                if (IDX) topk_insert_idx<K>(buf, bidx, v, part_i[o + k]);
                else topk_insert<K>(buf, v);
            }
        }
#pragma unroll
        for (int k = 0; k < K; k++) {
            bool fin = buf[k] < INFINITY;
            out_v[qi * K + k] = fin ? sqrt(buf[k]) : JMAX;
            if (IDX) out_i[qi * K + k] = fin ? bidx[k] : -1;
        }
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
static int pick_kc(int k) {
    if (k <= 1) return 1;
    if (k <= 3) return 3;
    if (k <= 7) return 7;
    if (k <= 15) return 15;
    if (k <= 31) return 31;
    return -1;
}

struct KnnPlan {
    int Q;
    int S;
    int64_t chunk;
    int tiles;
};

static KnnPlan plan_knn(hdb_ctx *ctx, int64_t n, int Q) {
    KnnPlan p;
    p.Q = Q;
    p.tiles = (int)ceil_div(n, 256 * Q);
    int target = ctx->num_cus * 8;  // >= 8 workgroups per CU in flight
    int S = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(target, p.tiles), 64));
    // each split should still scan a meaningful candidate range
    while (S > 1 && n / S < 1024) S--;
    p.S = S;
    p.chunk = ceil_div(n, S);
    return p;
}

// FP32-screen state for the current call (set by knn_lists_device)
struct F32Screen {
    const float *Xf = nullptr;
    const double *params = nullptr;
    bool on = false;
};
static thread_local F32Screen g_screen;

template <int D, int K, int Q, bool EXCL, bool IDX>
static void launch_knn_sq(hdb_ctx *ctx, const double *Xp, int64_t n, double *out_v, int32_t *out_i) {
    constexpr int DP = (D + 1) & ~1;
    constexpr int DF = D <= 4 ? 4 : (D <= 8 ? 8 : 16);
#ifndef HDB_KNN_U
#define HDB_KNN_U 4
#endif
    constexpr int U = (D <= 4) ? HDB_KNN_U : 2;
#ifndef HDB_KNN_US
#define HDB_KNN_US 8
#endif
    constexpr int US = (D <= 4) ? HDB_KNN_US : (D <= 8 ? 4 : 2);  // screen kernel group
    KnnPlan p = plan_knn(ctx, n, Q);
    dim3 grid(p.tiles, p.S);
    const bool f32 = g_screen.on;
    double *pv = out_v;
    int32_t *pi = out_i;
    if (p.S > 1) {
        pv = (double *)arena(ctx, A_WORK2, sizeof(double) * (size_t)(p.S * n * K));
        pi = IDX ? (int32_t *)arena(ctx, A_WORK3, sizeof(int32_t) * (size_t)(p.S * n * K)) : nullptr;
    }
    {
        KernelTimer t(ctx, "knn_sq");
        if (f32)
            hipLaunchKernelGGL((knn_f32x_kernel<D, DF, DP, K, Q, US, EXCL, IDX>), grid, dim3(256), 0, ctx->stream,
                               g_screen.Xf, Xp, g_screen.params, n, p.chunk, pv, pi, p.S == 1 ? 1 : 0);
        else
            hipLaunchKernelGGL((knn_sq_kernel<D, DP, K, Q, U, EXCL, IDX>), grid, dim3(256), 0, ctx->stream, Xp, n,
                               p.chunk, pv, pi, p.S == 1 ? 1 : 0);
        HIP_CHECK(hipGetLastError());
    }
    if (p.S == 1) return;
    int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    hipLaunchKernelGGL((knn_merge_kernel<K, IDX>), dim3(g), dim3(256), 0, ctx->stream, pv, pi, n, p.S, out_v,
                       out_i);
    HIP_CHECK(hipGetLastError());
}

#ifndef HDB_KNN_Q
#define HDB_KNN_Q 4
#endif
template <int D, int K, bool EXCL, bool IDX>
static void dispatch_q(hdb_ctx *ctx, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    // queries per lane: keep D*Q + K*Q doubles well inside the register budget
    constexpr int Q = (D * 2 + K * (IDX ? 3 : 2) <= 24) ? HDB_KNN_Q : ((D + K) <= 24 ? 2 : 1);
    launch_knn_sq<D, K, Q, EXCL, IDX>(ctx, Xp, n, ov, oi);
}

template <int D, bool EXCL, bool IDX>
static void dispatch_k(hdb_ctx *ctx, int KC, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    switch (KC) {
    case 1: dispatch_q<D, 1, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 3: dispatch_q<D, 3, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 7: dispatch_q<D, 7, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 15: dispatch_q<D, 15, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 31: dispatch_q<D, 31, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    default: HDB_THROW(HDB_EINVAL, "k too large (max 31)");
    }
}

template <bool EXCL, bool IDX>
static bool dispatch_d(hdb_ctx *ctx, int d, int KC, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    switch (d) {
    case 1: dispatch_k<1, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 2: dispatch_k<2, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 3: dispatch_k<3, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 4: dispatch_k<4, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 5: dispatch_k<5, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 6: dispatch_k<6, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 8: dispatch_k<8, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
    case 16: dispatch_k<16, EXCL, IDX>(ctx, KC, Xp, n, ov, oi); return true;
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
        bool ok;
        if (lists_i) ok = excl ? dispatch_d<true, true>(ctx, d, KC, Xp, n, lists_v, lists_i)
                               : dispatch_d<false, true>(ctx, d, KC, Xp, n, lists_v, lists_i);
        else ok = excl ? dispatch_d<true, false>(ctx, d, KC, Xp, n, lists_v, nullptr)
                       : dispatch_d<false, false>(ctx, d, KC, Xp, n, lists_v, nullptr);
        if (ok) return;
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
    int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    if (semantics != HDB_CORE_INCL_SELF_CUMULATIVE) {
        hipLaunchKernelGGL(core_from_lists_kernel, dim3(g), dim3(256), 0, ctx->stream, lists, n, KC, K, core);
        HIP_CHECK(hipGetLastError());
        return;
    }
    const int64_t CH = 256;
    int64_t nch = ceil_div(n, CH);
    double *agg = (double *)arena(ctx, A_WORK1, sizeof(double) * (size_t)(nch * 32));
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

}  // namespace hdb
