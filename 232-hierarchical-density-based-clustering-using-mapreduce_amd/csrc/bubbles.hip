// bubbles.hip -- K4 data-bubble statistics and K5 bubble k-NN.
//
// K4 (CombineStep.java:18-64 / ClusterFeatureDataBubbles.java:192-215): members of a
// bubble are folded in ascending point order (D5) -- the fold order fixes the FP sums, so
// the points are stably radix-sorted by bubble id and each bubble is folded sequentially
// by one lane (parallel over bubbles), then the per-bubble epilogue computes rep, extent
// and nnDist from the final (LS, SS, n) exactly as the last CombineStep call does.
//
// K5 (HdbscanDataBubbles.calculateCoreDistancesBubbles, :75-146): per bubble p the lane
// scans q != p in index order with the reference's insertion (strict '<') on the
// transformed distance distanceBubbles(...) and logs, per buffer position, the LAST
// neighbour inserted there during p's scan.  The reference's indexBubbles[] is never
// reset across points (:79-83,118), so its state before point p's formula is the
// last-writer prefix of these logs -- resolved by the host epilogue in point order.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>

#include "common.hpp"

namespace hdb {

__global__ void iota32_kernel(int32_t *a, int64_t n) { HDB_GRID_STRIDE(i, n) a[i] = (int32_t)i; }

__global__ void bubble_count_kernel(const int32_t *__restrict__ bo, int64_t n, int64_t nb, int32_t *__restrict__ cnt,
                                    int *__restrict__ bad) {
    HDB_GRID_STRIDE(i, n) {
        int32_t b = bo[i];
        if (b < 0 || b >= nb) {
            *bad = 1;
            continue;
        }
        atomicAdd(&cnt[b], 1);
    }
}

// K4 fold, one lane per (bubble, dimension): a coordinate's LS and SS are two independent
// sequential chains over the bubble's members (ascending id, D5), kept in registers -- the same
// additions in the same order as the per-bubble fold, bit for bit.  nb x d lanes instead of nb
// (16,384 bubbles: 256 waves -> 2,048 at d = 8), and no read-modify-write of the outputs per
// member.  The epilogue (rep, extent, nnDist: sequential over dimensions) runs per bubble after.
__global__ void bubble_fold_dim_kernel(const double *__restrict__ X, int d, const int32_t *__restrict__ perm,
                                       const int64_t *__restrict__ off, int64_t nb, double *__restrict__ ls,
                                       double *__restrict__ ss) {
    HDB_GRID_STRIDE(t, nb * d) {
        const int64_t b = t / d;
        const int c = (int)(t - b * d);
        const int64_t lo = off[b], hi = off[b + 1];
        double L = 0.0, Q = 0.0;
        if (lo < hi) {
            const double v0 = X[(int64_t)perm[lo] * d + c];
            L = v0;
            Q = v0 * v0;
#pragma unroll 4
            for (int64_t k = lo + 1; k < hi; k++) {
                const double v = X[(int64_t)perm[k] * d + c];
                L = L + v;
                Q = Q + (v * v);
            }
        }
        ls[t] = L;
        ss[t] = Q;
    }
}

// per-bubble epilogue of the folded (LS, SS, n): exactly the tail of bubble_fold_kernel.
// Member counts from the segment offsets, or (cntd != nullptr) from combined slice partials
__global__ void bubble_epilogue_kernel(int d, const int64_t *__restrict__ off, int64_t nb, int variant,
                                       const double *__restrict__ ls, const double *__restrict__ ss,
                                       double *__restrict__ rep, double *__restrict__ info,
                                       const double *__restrict__ cntd = nullptr) {
    HDB_GRID_STRIDE(b, nb) {
        const int64_t cnt = cntd ? (int64_t)cntd[b] : off[b + 1] - off[b];
        const double *L = ls + b * d, *Q = ss + b * d;
        double *R = rep + b * d, *I = info + b * 3;
        if (cnt == 0) {
            for (int c = 0; c < d; c++) R[c] = 0;
            I[0] = I[1] = I[2] = 0;
            continue;
        }
        if (cnt == 1) {
            for (int c = 0; c < d; c++) R[c] = L[c];  // rep = ls (FirstStep.java:100)
            I[0] = 0;
            I[1] = 0;
            I[2] = 1;
            continue;
        }
        if (variant == HDB_BUBBLE_COMBINESTEP) {
            const double n = (double)cnt;  // n += 1 per call == member count (sequential fold)
            for (int c = 0; c < d; c++) R[c] = L[c] / n;  // computeRepBubble (:58-64)
            double extent = 0.0;                          // computeExtentBubble (:46-56)
            for (int c = 0; c < d; c++) {
                double v = ((2 * n * Q[c]) - (2 * (L[c] * L[c])));
                if (v >= 0) extent += sqrt(v / (n * (n - 1)));
            }
            extent = extent / d;
            I[0] = extent;
            // computeNNDistBubble (:42-44): pow(1/n, (int)(1/d)) * extent
            I[1] = pow((1 / n), (double)(1 / d)) * extent;
            I[2] = n;
        } else {
            const int32_t n = (int32_t)cnt;
            for (int c = 0; c < d; c++) R[c] = L[c] / n;
            const int32_t prod = (int32_t)((uint32_t)n * (uint32_t)(n - 1));  // Java int overflow
            double sum = 0.0;
            for (int c = 0; c < d; c++) sum = sum + (((2 * n * Q[c]) - (2 * (L[c] * L[c]))) / prod);
            const double extent = sqrt(sum);
            I[0] = extent;
            I[1] = pow((double)1 / n, (double)1 / d) * extent;
            I[2] = n;
        }
    }
}

// one lane per bubble: sequential fold in member order
__global__ void bubble_fold_kernel(const double *__restrict__ X, int d, const int32_t *__restrict__ perm,
                                   const int64_t *__restrict__ off, int64_t nb, int variant,
                                   double *__restrict__ ls, double *__restrict__ ss, double *__restrict__ rep,
                                   double *__restrict__ info) {
    HDB_GRID_STRIDE(b, nb) {
        const int64_t lo = off[b], hi = off[b + 1];
        double *L = ls + b * d, *Q = ss + b * d, *R = rep + b * d, *I = info + b * 3;
        if (lo == hi) {
            for (int c = 0; c < d; c++) L[c] = Q[c] = R[c] = 0;
            I[0] = I[1] = I[2] = 0;
            continue;
        }
        const double *x0 = X + (int64_t)perm[lo] * d;
        for (int c = 0; c < d; c++) {
            double v = x0[c];
            L[c] = v;
            Q[c] = v * v;
        }
        for (int64_t k = lo + 1; k < hi; k++) {
            const double *x = X + (int64_t)perm[k] * d;
            for (int c = 0; c < d; c++) {
                double v = x[c];
                L[c] = L[c] + v;
                Q[c] = Q[c] + (v * v);
            }
        }
        const int64_t cnt = hi - lo;
        if (cnt == 1) {
            for (int c = 0; c < d; c++) R[c] = L[c];  // rep = ls (FirstStep.java:100)
            I[0] = 0;
            I[1] = 0;
            I[2] = 1;
            continue;
        }
        if (variant == HDB_BUBBLE_COMBINESTEP) {
            const double n = (double)cnt;  // n += 1 per call == member count (sequential fold)
            for (int c = 0; c < d; c++) R[c] = L[c] / n;  // computeRepBubble (:58-64)
            double extent = 0.0;                          // computeExtentBubble (:46-56)
            for (int c = 0; c < d; c++) {
                double v = ((2 * n * Q[c]) - (2 * (L[c] * L[c])));
                if (v >= 0) extent += sqrt(v / (n * (n - 1)));
            }
            extent = extent / d;
            I[0] = extent;
            // computeNNDistBubble (:42-44): pow(1/n, (int)(1/d)) * extent
            I[1] = pow((1 / n), (double)(1 / d)) * extent;
            I[2] = n;
        } else {
            const int32_t n = (int32_t)cnt;
            for (int c = 0; c < d; c++) R[c] = L[c] / n;
            const int32_t prod = (int32_t)((uint32_t)n * (uint32_t)(n - 1));  // Java int overflow
            double sum = 0.0;
            for (int c = 0; c < d; c++) sum = sum + (((2 * n * Q[c]) - (2 * (L[c] * L[c]))) / prod);
            const double extent = sqrt(sum);
            I[0] = extent;
            I[1] = pow((double)1 / n, (double)1 / d) * extent;
            I[2] = n;
        }
    }
}

void bubble_stats_device(hdb_ctx *ctx, const double *X, int64_t n, int d, const int32_t *bo, int64_t nb, int variant,
                         double *ls, double *ss, double *rep, double *info) {
    if (nb <= 0) return;
    if (n > INT32_MAX) HDB_THROW(HDB_EINVAL, "n exceeds int32");
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t o_keys = carve(sizeof(int32_t) * (n + 1)), o_perm = carve(sizeof(int32_t) * (n + 1)),
           o_iota = carve(sizeof(int32_t) * (n + 1)), o_cnt = carve(sizeof(int32_t) * (nb + 1)),
           o_off = carve(sizeof(int64_t) * (nb + 1)), o_bad = carve(sizeof(int));
    char *base = (char *)arena(ctx, A_WORK0, off);
    int32_t *keys = (int32_t *)(base + o_keys), *perm = (int32_t *)(base + o_perm), *iota = (int32_t *)(base + o_iota);
    int32_t *cnt = (int32_t *)(base + o_cnt);
    int64_t *offs = (int64_t *)(base + o_off);
    int *bad = (int *)(base + o_bad);
    int g = 2048;
    HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (nb + 1), ctx->stream));
    HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), ctx->stream));
    KernelTimer t(ctx, "bubble_stats");
    if (n > 0) {
        hipLaunchKernelGGL(iota32_kernel, dim3(g), dim3(256), 0, ctx->stream, iota, n);
        hipLaunchKernelGGL(bubble_count_kernel, dim3(g), dim3(256), 0, ctx->stream, bo, n, nb, cnt, bad);
        size_t tb = 0;
        int end_bit = 1;
        while (end_bit < 32 && (int64_t(1) << end_bit) < nb) end_bit++;
        HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, bo, keys, iota, perm, (int)n, 0, end_bit, ctx->stream));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, bo, keys, iota, perm, (int)n, 0, end_bit, ctx->stream));
    }
    // exclusive scan of counts (int32) into int64 offsets
    {
        size_t tb = 0;
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, offs, (int)(nb + 1), ctx->stream));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, offs, (int)(nb + 1), ctx->stream));
    }
    if (ctx->bubble_fold_dim) {
        hipLaunchKernelGGL(bubble_fold_dim_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nb * d, 256), 16384)),
                           dim3(256), 0, ctx->stream, X, d, perm, offs, nb, ls, ss);
        hipLaunchKernelGGL(bubble_epilogue_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nb, 64), 4096)), dim3(64),
                           0, ctx->stream, d, offs, nb, variant, ls, ss, rep, info);
    } else
        hipLaunchKernelGGL(bubble_fold_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nb, 64), 4096)), dim3(64), 0,
                           ctx->stream, X, d, perm, offs, nb, variant, ls, ss, rep, info);
    HIP_CHECK(hipGetLastError());
    int h_bad = 0;
    HIP_CHECK(hipMemcpyAsync(&h_bad, bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (h_bad) HDB_THROW(HDB_EINVAL, "bubble_of out of range");
}

// ---------------------------------------------- K4 over slices (D11)
// CombineStep as Spark shapes it (reduceByKey: a map-side fold per partition, then the
// partials merged; CombineStep.java:18-40 via Main.java:236-237) with the partitions fixed:
// the rows are cut into S contiguous slices, each slice folds its members (ascending order,
// the same chains as K4), and the partials of a bubble are combined in slice order.  A rank
// folds only its own slices; the partials are gathered and combined in slice order on every
// rank, so the result is the same at every rank count (oracle: orc_bubble_stats_combine_sliced).
struct SliceCuts {
    int64_t c[HDB_MAX_BUBBLE_SLICES + 1];
    int S;
};

__global__ void slice_key_kernel(const int32_t *__restrict__ bo, int64_t n, int64_t nb, SliceCuts sc,
                                 int32_t *__restrict__ key, int32_t *__restrict__ cnt, int *__restrict__ bad) {
    HDB_GRID_STRIDE(i, n) {
        const int32_t b = bo[i];
        if (b < 0 || b >= nb) {
            *bad = 1;
            key[i] = 0;
            continue;
        }
        int s = 0;
        while (s + 1 < sc.S && i >= sc.c[s + 1]) s++;
        const int32_t k = (int32_t)(s * nb + b);
        key[i] = k;
        atomicAdd(&cnt[k], 1);
    }
}

__global__ void counts_to_double_kernel(const int64_t *__restrict__ off, int64_t m, double *__restrict__ out) {
    HDB_GRID_STRIDE(k, m) out[k] = (double)(off[k + 1] - off[k]);
}

// per (bubble, dimension): the slice partials in slice order, empty slices skipped
__global__ void bubble_combine_dim_kernel(const double *__restrict__ pls, const double *__restrict__ pss,
                                          const double *__restrict__ pn, int S, int64_t nb, int d,
                                          double *__restrict__ ls, double *__restrict__ ss) {
    HDB_GRID_STRIDE(t, nb * d) {
        const int64_t b = t / d;
        double L = 0.0, Q = 0.0;
        bool first = true;
        for (int s = 0; s < S; s++) {
            if (pn[(int64_t)s * nb + b] == 0) continue;
            const double l = pls[(int64_t)s * nb * d + t], q = pss[(int64_t)s * nb * d + t];
            L = first ? l : L + l;
            Q = first ? q : Q + q;
            first = false;
        }
        ls[t] = L;
        ss[t] = Q;
    }
}

__global__ void bubble_combine_n_kernel(const double *__restrict__ pn, int S, int64_t nb, double *__restrict__ n_out) {
    HDB_GRID_STRIDE(b, nb) {
        double c = 0;
        for (int s = 0; s < S; s++) c += pn[(int64_t)s * nb + b];
        n_out[b] = c;
    }
}

void bubble_partials_device(hdb_ctx *ctx, const double *X, int64_t n, int d, const int32_t *bo, int64_t nb,
                            const int64_t *h_cuts, int S, double *pls, double *pss, double *pn) {
    if (S < 1 || S > HDB_MAX_BUBBLE_SLICES) HDB_THROW(HDB_EINVAL, "bubble slices: 1..64");
    if (h_cuts[0] != 0 || h_cuts[S] != n) HDB_THROW(HDB_EINVAL, "bubble slices: cuts must span [0, n]");
    for (int s = 0; s < S; s++)
        if (h_cuts[s + 1] < h_cuts[s]) HDB_THROW(HDB_EINVAL, "bubble slices: cuts must be non-decreasing");
    if (n > INT32_MAX || (int64_t)S * nb > INT32_MAX) HDB_THROW(HDB_EINVAL, "bubble slices: too large");
    const int64_t m = (int64_t)S * nb;
    if (m <= 0) return;
    SliceCuts sc{};
    for (int s = 0; s <= S; s++) sc.c[s] = h_cuts[s];
    sc.S = S;
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t o_key = carve(sizeof(int32_t) * (n + 1)), o_skey = carve(sizeof(int32_t) * (n + 1)),
           o_perm = carve(sizeof(int32_t) * (n + 1)), o_iota = carve(sizeof(int32_t) * (n + 1)),
           o_cnt = carve(sizeof(int32_t) * (m + 1)), o_off = carve(sizeof(int64_t) * (m + 1)), o_bad = carve(sizeof(int));
    char *base = (char *)arena(ctx, A_WORK0, off);
    int32_t *key = (int32_t *)(base + o_key), *skey = (int32_t *)(base + o_skey), *perm = (int32_t *)(base + o_perm),
            *iota = (int32_t *)(base + o_iota), *cnt = (int32_t *)(base + o_cnt);
    int64_t *offs = (int64_t *)(base + o_off);
    int *bad = (int *)(base + o_bad);
    const int g = 2048;
    HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (m + 1), ctx->stream));
    HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), ctx->stream));
    KernelTimer t(ctx, "bubble_stats");
    if (n > 0) {
        hipLaunchKernelGGL(iota32_kernel, dim3(g), dim3(256), 0, ctx->stream, iota, n);
        hipLaunchKernelGGL(slice_key_kernel, dim3(g), dim3(256), 0, ctx->stream, bo, n, nb, sc, key, cnt, bad);
        int end_bit = 1;
        while (end_bit < 32 && (int64_t(1) << end_bit) < m) end_bit++;
        size_t tb = 0;
        HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key, skey, iota, perm, (int)n, 0, end_bit, ctx->stream));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, skey, iota, perm, (int)n, 0, end_bit, ctx->stream));
    }
    {
        size_t tb = 0;
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, offs, (int)(m + 1), ctx->stream));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, offs, (int)(m + 1), ctx->stream));
    }
    // a (slice, bubble) segment is a slice's members of the bubble in row order: K4's fold
    hipLaunchKernelGGL(bubble_fold_dim_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(m * d, 256), 16384)), dim3(256),
                       0, ctx->stream, X, d, perm, offs, m, pls, pss);
    hipLaunchKernelGGL(counts_to_double_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(m, 256), 4096)), dim3(256), 0,
                       ctx->stream, offs, m, pn);
    HIP_CHECK(hipGetLastError());
    int *pin = (int *)(pinned_words(ctx) + PINNED_WORDS - 40);
    HIP_CHECK(hipMemcpyAsync(pin, bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (*pin) HDB_THROW(HDB_EINVAL, "bubble_of out of range");
}

void bubble_combine_device(hdb_ctx *ctx, const double *pls, const double *pss, const double *pn, int S, int64_t nb,
                           int d, double *ls, double *ss, double *rep, double *info) {
    if (S < 1) HDB_THROW(HDB_EINVAL, "bubble slices: S >= 1");
    if (nb <= 0) return;
    double *cntd = (double *)arena(ctx, A_WORK1, sizeof(double) * nb);
    KernelTimer t(ctx, "bubble_combine");
    hipLaunchKernelGGL(bubble_combine_dim_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nb * d, 256), 16384)),
                       dim3(256), 0, ctx->stream, pls, pss, pn, S, nb, d, ls, ss);
    hipLaunchKernelGGL(bubble_combine_n_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nb, 256), 4096)), dim3(256), 0,
                       ctx->stream, pn, S, nb, cntd);
    hipLaunchKernelGGL(bubble_epilogue_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(nb, 64), 4096)), dim3(64), 0,
                       ctx->stream, d, nullptr, nb, (int)HDB_BUBBLE_COMBINESTEP, ls, ss, rep, info, cntd);
    HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------ K5 bubble kNN
// knn[b][K] final buffer (transformed distances, MAX padded); log[b][K] last neighbour
// inserted at each position during b's scan (-1 if none).  Buffer init Double.MAX_VALUE,
// strict '<' insertion with shift, exactly HdbscanDataBubbles.java:92-119.
template <int KC>
__global__ __launch_bounds__(256) void bubble_knn_kernel(const double *__restrict__ rep, const double *__restrict__ eB,
                                                         const double *__restrict__ nnB, int64_t b, int d, int metric,
                                                         int K, double *__restrict__ knn_out,
                                                         int32_t *__restrict__ log_out) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t pr = p < b ? p : 0;
    double buf[KC];
    int32_t lg[KC];
#pragma unroll
    for (int k = 0; k < KC; k++) {
        buf[k] = JMAX;
        lg[k] = -1;
    }
    const double ep = eB[pr], np_ = nnB[pr];
    const double *xp = rep + pr * d;
    for (int64_t q = 0; q < b; q++) {  // wave-uniform loop
        if (q == p) continue;
        double dist = metric_distance(xp, rep + q * d, d, metric);
        dist = distance_bubbles(dist, ep, eB[q], np_, nnB[q]);
        // insertion: position = count of buffer entries <= dist (among the first K)
        if (dist < buf[K - 1 < KC ? K - 1 : KC - 1]) {
            int pos = K;
#pragma unroll
            for (int k = KC - 1; k >= 0; k--)
                if (k < K && dist < buf[k]) pos = k;
            // shift right from pos, insert
#pragma unroll
            for (int k = KC - 1; k > 0; k--)
                if (k < K && k > pos) buf[k] = buf[k - 1];
#pragma unroll
            for (int k = 0; k < KC; k++)
                if (k == pos) {
                    buf[k] = dist;
                    lg[k] = (int32_t)q;
                }
        }
    }
    if (p < b) {
#pragma unroll
        for (int k = 0; k < KC; k++)
            if (k < K) {
                knn_out[p * K + k] = buf[k];
                log_out[p * K + k] = lg[k];
            }
    }
}

// The candidate range split in S chunks (grid.y): a 16k-bubble model as one thread per bubble
// is 256 waves -- one per CU, latency bound.  The sequential kernel's log is an insertion log
// per position (lg is not shifted: the stale indexBubbles emulation), so the chunks cannot be
// merged as lists.  Instead each chunk scans its candidates with a chunk-local buffer and
// records every local insertion (q, dist) in q order.  Every insertion of the sequential scan
// is among them: the chunk's buffer holds a subset of the sequential buffer's candidates, so
// its K-th value is never smaller.  Replaying the recorded events of chunks 0..S-1 in q order
// with the sequential rule then reproduces the buffer and the log exactly (a recorded event
// the sequential scan would not insert fails the same test in the replay; an unrecorded one
// would not have changed the state).  A chunk with more insertions than it can record sets a flag and
// the sequential kernel runs instead (BK_EV events per chunk).
constexpr int BK_EV = 64;
template <int KC>
__global__ __launch_bounds__(256) void bubble_knn_part_kernel(const double *__restrict__ rep,
                                                              const double *__restrict__ eB,
                                                              const double *__restrict__ nnB, int64_t b, int d,
                                                              int metric, int K, int S, double *__restrict__ evd,
                                                              int32_t *__restrict__ evq, int32_t *__restrict__ evn,
                                                              int *__restrict__ overflow) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int s = blockIdx.y;
    const int64_t pr = p < b ? p : 0;
    const int64_t q0 = b * s / S, q1 = b * (s + 1) / S;
    const int64_t eo = ((int64_t)s * b + pr) * BK_EV;
    double buf[KC];
#pragma unroll
    for (int k = 0; k < KC; k++) buf[k] = JMAX;
    int ne = 0;
    const double ep = eB[pr], np_ = nnB[pr];
    const double *xp = rep + pr * d;
    for (int64_t q = q0; q < q1; q++) {  // wave-uniform loop
        if (q == p) continue;
        double dist = metric_distance(xp, rep + q * d, d, metric);
        dist = distance_bubbles(dist, ep, eB[q], np_, nnB[q]);
        if (dist < buf[K - 1 < KC ? K - 1 : KC - 1]) {
            int pos = K;
#pragma unroll
            for (int k = KC - 1; k >= 0; k--)
                if (k < K && dist < buf[k]) pos = k;
#pragma unroll
            for (int k = KC - 1; k > 0; k--)
                if (k < K && k > pos) buf[k] = buf[k - 1];
#pragma unroll
            for (int k = 0; k < KC; k++)
                if (k == pos) buf[k] = dist;
            if (p < b && ne < BK_EV) {
                evd[eo + ne] = dist;
                evq[eo + ne] = (int32_t)q;
            }
            ne++;
        }
    }
    if (p < b) {
        evn[(int64_t)s * b + p] = ne < BK_EV ? ne : BK_EV;
        if (ne > BK_EV) atomicOr(overflow, 1);
    }
}

template <int KC>
__global__ __launch_bounds__(256) void bubble_knn_replay_kernel(const double *__restrict__ evd,
                                                                const int32_t *__restrict__ evq,
                                                                const int32_t *__restrict__ evn, int64_t b, int K, int S,
                                                                double *__restrict__ knn_out,
                                                                int32_t *__restrict__ log_out) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= b) return;
    double buf[KC];
    int32_t lg[KC];
#pragma unroll
    for (int k = 0; k < KC; k++) {
        buf[k] = JMAX;
        lg[k] = -1;
    }
    for (int s = 0; s < S; s++) {
        const int64_t eo = ((int64_t)s * b + p) * BK_EV;
        const int ne = evn[(int64_t)s * b + p];
        for (int e = 0; e < ne; e++) {  // the sequential kernel's insertion, event by event
            const double dist = evd[eo + e];
            if (!(dist < buf[K - 1 < KC ? K - 1 : KC - 1])) continue;
            int pos = K;
#pragma unroll
            for (int k = KC - 1; k >= 0; k--)
                if (k < K && dist < buf[k]) pos = k;
#pragma unroll
            for (int k = KC - 1; k > 0; k--)
                if (k < K && k > pos) buf[k] = buf[k - 1];
#pragma unroll
            for (int k = 0; k < KC; k++)
                if (k == pos) {
                    buf[k] = dist;
                    lg[k] = evq[eo + e];
                }
        }
    }
#pragma unroll
    for (int k = 0; k < KC; k++)
        if (k < K) {
            knn_out[p * K + k] = buf[k];
            log_out[p * K + k] = lg[k];
        }
}

template <int KC>
static void bubble_knn_launch(hdb_ctx *ctx, const double *rep, const double *eB, const double *nnB, int64_t b, int d,
                              int metric, int K, double *knn_out, int32_t *log_out) {
    // chunks: >= ~256k threads per model, >= 256 candidates per chunk, and short enough that a
    // chunk's expected insertions in random order, K (1 + ln(L / K)) for L candidates, stay
    // under half the BK_EV it can record (at K >= 7 a 1k-candidate chunk overflows
    // most of the time, and the plain scan then runs after the split anyway) -- L <= K e^(32/K - 1);
    // when that is below 256 the plain scan runs directly
    int64_t S = std::min<int64_t>(ceil_div(262144, std::max<int64_t>(b, 1)), std::max<int64_t>(b / 256, 1));
    const double lmax = K * std::exp(0.5 * BK_EV / K - 1.0);
    if (lmax < 256.0) S = 1;
    else S = std::max<int64_t>(S, (int64_t)std::ceil((double)b / lmax));
    S = std::max<int64_t>(1, std::min<int64_t>({S, (int64_t)64, std::max<int64_t>(b / 256, 1)}));
    if (!ctx->bubble_knn_split) S = 1;
    const dim3 g1((unsigned)ceil_div(b, 256));
    if (S > 1) {
        const size_t ev = (size_t)S * b * BK_EV;
        char *base = (char *)arena(ctx, A_WORK2, ev * (sizeof(double) + sizeof(int32_t)) + (size_t)S * b * 4 + 1024);
        double *evd = (double *)base;
        int32_t *evq = (int32_t *)(base + ev * sizeof(double));
        int32_t *evn = evq + ev;
        int *ovf = (int *)(((uintptr_t)(evn + (size_t)S * b) + 255) & ~uintptr_t(255));
        HIP_CHECK(hipMemsetAsync(ovf, 0, sizeof(int), ctx->stream));
        hipLaunchKernelGGL(bubble_knn_part_kernel<KC>, dim3(g1.x, (unsigned)S), dim3(256), 0, ctx->stream, rep, eB, nnB,
                           b, d, metric, K, (int)S, evd, evq, evn, ovf);
        hipLaunchKernelGGL(bubble_knn_replay_kernel<KC>, g1, dim3(256), 0, ctx->stream, evd, evq, evn, b, K, (int)S,
                           knn_out, log_out);
        int *pin = (int *)(pinned_words(ctx) + PINNED_WORDS - 24);
        HIP_CHECK(hipMemcpyAsync(pin, ovf, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        if (*pin == 0) return;
        ctx->stats["bubble_knn_replay_overflows"] += 1;  // adversarial candidate order: the plain scan
    }
    hipLaunchKernelGGL(bubble_knn_kernel<KC>, g1, dim3(256), 0, ctx->stream, rep, eB, nnB, b, d, metric, K, knn_out,
                       log_out);
}

void bubble_knn_device(hdb_ctx *ctx, const double *rep, const double *eB, const double *nnB, int64_t b, int d,
                       int metric, int K, double *knn_out, int32_t *log_out) {
    if (b <= 0 || K <= 0) return;
    KernelTimer t(ctx, "bubble_knn");
    if (K <= 3)
        bubble_knn_launch<3>(ctx, rep, eB, nnB, b, d, metric, K, knn_out, log_out);
    else if (K <= 7)
        bubble_knn_launch<7>(ctx, rep, eB, nnB, b, d, metric, K, knn_out, log_out);
    else if (K <= 15)
        bubble_knn_launch<15>(ctx, rep, eB, nnB, b, d, metric, K, knn_out, log_out);
    else if (K <= 31)
        bubble_knn_launch<31>(ctx, rep, eB, nnB, b, d, metric, K, knn_out, log_out);
    else
        HDB_THROW(HDB_EINVAL, "minPts too large (max 32)");
    HIP_CHECK(hipGetLastError());
}

}  // namespace hdb
