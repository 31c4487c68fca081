// knn_impl.hpp -- K1 (all-pairs tiled k-NN) kernel templates and their launch plan, shared
// by knn.hip and the per-dimension instantiation units knn_d*.hip (split so the heavy
// template instantiations compile in parallel).  See knn.hip for the design notes.
#pragma once
#include "internal.hpp"

namespace hdb {

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

// ----------------------------------------------------------------- host

struct KnnPlan {
    int Q;
    int S;
    int64_t chunk;
    int tiles;
};

inline KnnPlan plan_knn(hdb_ctx *ctx, int64_t n, int Q) {
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
extern thread_local F32Screen g_screen;

template <int D, int K, int Q, bool EXCL, bool IDX>
void launch_knn_sq(hdb_ctx *ctx, const double *Xp, int64_t n, double *out_v, int32_t *out_i) {
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
void dispatch_q(hdb_ctx *ctx, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    // queries per lane: keep D*Q + K*Q doubles well inside the register budget
    constexpr int Q = (D * 2 + K * (IDX ? 3 : 2) <= 24) ? HDB_KNN_Q : ((D + K) <= 24 ? 2 : 1);
    launch_knn_sq<D, K, Q, EXCL, IDX>(ctx, Xp, n, ov, oi);
}

template <int D, bool EXCL, bool IDX>
void dispatch_k(hdb_ctx *ctx, int KC, const double *Xp, int64_t n, double *ov, int32_t *oi) {
    switch (KC) {
    case 1: dispatch_q<D, 1, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 3: dispatch_q<D, 3, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 7: dispatch_q<D, 7, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 15: dispatch_q<D, 15, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    case 31: dispatch_q<D, 31, EXCL, IDX>(ctx, Xp, n, ov, oi); break;
    default: HDB_THROW(HDB_EINVAL, "k too large (max 31)");
    }
}

// one instantiation unit per supported d (knn_d<D>.hip)
#define HDB_KNN_DIMS(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(16)
#define HDB_KNN_DECL(DD) \
    void knn_run_d##DD(hdb_ctx *ctx, int KC, bool excl, bool idx, const double *Xp, int64_t n, double *ov, int32_t *oi);
HDB_KNN_DIMS(HDB_KNN_DECL)
#undef HDB_KNN_DECL

}  // namespace hdb
