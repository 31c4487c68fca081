// nearest.hip -- K3: nearest-sample assignment with the reference's FIRST-minimum rule
// (FirstStep.java:74-85: strict '<' over the sample list in order, minDistance starts at
// Double.MAX_VALUE, nearest at 0).
//
// Exactness: Java compares sqrt values.  Distinct squared distances can round to the
// same sqrt, so the lane keeps (s_best, r_best = sqrt(s_best), i_best) and replaces iff
// s < s_best AND sqrt(s) < r_best -- the squared test is only a filter (sqrt is monotone),
// the decision is on sqrt values exactly as in Java.  sqrt runs only when the running
// minimum improves.  Candidate splits merge by (r, index) with ties to the smaller index.
//
// Keyed mode (D3, ClusterFeaturesByNodesMapper.java:53-61): samples and points are
// stably sorted by key; each lane scans only its key's sample range (the wave loops over
// the union of its lanes' ranges with per-lane masks; sorted points make it uniform).
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace hdb {

void pack_rows(hdb_ctx *ctx, const double *X, int64_t n, int d, int dp, double *Xp);

struct NN {
    double s, r;
    int i;
};

__device__ __forceinline__ void nn_consider(NN &b, double s, int j) {
    if (s < b.s) {
        double r = sqrt(s);
        if (r < b.r) {
            b.r = r;
            b.s = s;
            b.i = j;
        }
    }
}

// grid.x = point tiles (256*Q), grid.y = sample splits.  Unkeyed when skeys == nullptr.
template <int D, int DP, int Q, int U>
__global__ __launch_bounds__(256) void nearest_sq_kernel(const double *__restrict__ Xp, int64_t n,
                                                         const double *__restrict__ Sp, int64_t m,
                                                         const int32_t *__restrict__ xkeys,
                                                         const int32_t *__restrict__ skeys, int64_t chunk,
                                                         double *__restrict__ part_r, int32_t *__restrict__ part_i) {
    const int64_t q0 = (int64_t)blockIdx.x * (256 * Q);
    const int64_t c_lo = (int64_t)blockIdx.y * chunk;
    const int64_t c_hi = min(c_lo + chunk, m);
    double xq[Q][D];
    NN best[Q];
    int64_t qi[Q];
    int64_t lo[Q], hi[Q];
    int64_t wlo = c_hi, whi = c_lo;
#pragma unroll
    for (int q = 0; q < Q; q++) {
        qi[q] = q0 + threadIdx.x + (int64_t)q * 256;
        const int64_t r = qi[q] < n ? qi[q] : 0;
#pragma unroll
        for (int c = 0; c < D; c++) xq[q][c] = Xp[r * DP + c];
        best[q].s = INFINITY;
        best[q].r = JMAX;
        best[q].i = -1;
        lo[q] = c_lo;
        hi[q] = c_hi;
        if (skeys) {
            int32_t key = xkeys[r];
            // lower_bound / upper_bound of key in sorted skeys
            int64_t a = 0, b = m;
            while (a < b) {
                int64_t mid = (a + b) >> 1;
                if (skeys[mid] < key) a = mid + 1;
                else b = mid;
            }
            int64_t e = a, f = m;
            while (e < f) {
                int64_t mid = (e + f) >> 1;
                if (skeys[mid] <= key) e = mid + 1;
                else f = mid;
            }
            lo[q] = max(c_lo, a);
            hi[q] = min(c_hi, e);
        }
        if (qi[q] >= n) {
            lo[q] = c_hi;
            hi[q] = c_hi;
        }
        if (lo[q] < hi[q]) {
            wlo = min(wlo, lo[q]);
            whi = max(whi, hi[q]);
        }
    }
    // wave-uniform union range
    for (int off = 32; off >= 1; off >>= 1) {
        wlo = min(wlo, (int64_t)__shfl_xor((long long)wlo, off));
        whi = max(whi, (int64_t)__shfl_xor((long long)whi, off));
    }
    wlo = __builtin_amdgcn_readfirstlane((int)wlo) | ((int64_t)__builtin_amdgcn_readfirstlane((int)(wlo >> 32)) << 32);
    whi = __builtin_amdgcn_readfirstlane((int)whi) | ((int64_t)__builtin_amdgcn_readfirstlane((int)(whi >> 32)) << 32);
    const bool masked = skeys != nullptr;

    int64_t j = wlo;
#pragma unroll 1
    for (; j + U <= whi; j += U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const double *cr = Sp + (j + u) * DP;
            double cc[D];
#pragma unroll
            for (int c = 0; c < D; c++) cc[c] = cr[c];
#pragma unroll
            for (int q = 0; q < Q; q++) {
                double acc = sq_diff(xq[q][0], cc[0]);
#pragma unroll
                for (int c = 1; c < D; c++) acc = acc + sq_diff(xq[q][c], cc[c]);
                if (masked && (j + u < lo[q] || j + u >= hi[q])) acc = INFINITY;
                nn_consider(best[q], acc, (int)(j + u));
            }
        }
    }
#pragma unroll 1
    for (; j < whi; j++) {
        const double *cr = Sp + j * DP;
        double cc[D];
#pragma unroll
        for (int c = 0; c < D; c++) cc[c] = cr[c];
#pragma unroll
        for (int q = 0; q < Q; q++) {
            double acc = sq_diff(xq[q][0], cc[0]);
#pragma unroll
            for (int c = 1; c < D; c++) acc = acc + sq_diff(xq[q][c], cc[c]);
            if (masked && (j < lo[q] || j >= hi[q])) acc = INFINITY;
            nn_consider(best[q], acc, (int)j);
        }
    }
#pragma unroll
    for (int q = 0; q < Q; q++) {
        if (qi[q] >= n) continue;
        int64_t o = (int64_t)blockIdx.y * n + qi[q];
        part_r[o] = best[q].r;
        part_i[o] = best[q].i;
    }
}

// generic metrics: Java semantics on the values themselves
__global__ __launch_bounds__(256) void nearest_generic_kernel(const double *__restrict__ X, int64_t n,
                                                              const double *__restrict__ S, int64_t m, int d,
                                                              int metric, const int32_t *__restrict__ xkeys,
                                                              const int32_t *__restrict__ skeys, int64_t chunk,
                                                              double *__restrict__ part_r,
                                                              int32_t *__restrict__ part_i) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const int64_t c_lo = (int64_t)blockIdx.y * chunk;
    const int64_t c_hi = min(c_lo + chunk, m);
    double bd = JMAX;
    int bi = -1;
    for (int64_t j = c_lo; j < c_hi; j++) {
        if (skeys && skeys[j] != xkeys[p]) continue;
        double v = metric_distance(X + p * d, S + j * d, d, metric);
        if (v < bd) {
            bd = v;
            bi = (int)j;
        }
    }
    part_r[(int64_t)blockIdx.y * n + p] = bd;
    part_i[(int64_t)blockIdx.y * n + p] = bi;
}

// merge splits: smaller value wins, ties -> smaller sample index (first minimum);
// no candidate -> index 0 (Java init), dist MAX.  perm maps sorted positions back.
__global__ void nearest_merge_kernel(const double *__restrict__ part_r, const int32_t *__restrict__ part_i,
                                     int64_t n, int S, const int32_t *__restrict__ sperm,
                                     const int32_t *__restrict__ xperm, int32_t *__restrict__ out_i,
                                     double *__restrict__ out_d) {
    HDB_GRID_STRIDE(p, n) {
        double bd = JMAX;
        int bi = -1;
        for (int s = 0; s < S; s++) {
            double v = part_r[(int64_t)s * n + p];
            int i = part_i[(int64_t)s * n + p];
            if (i < 0) continue;
            if (bi < 0 || v < bd || (v == bd && i < bi)) {
                // a split's candidate only exists if v < MAX (Java strict '<' from MAX)
                bd = v;
                bi = i;
            }
        }
        int res = bi < 0 ? 0 : (sperm ? sperm[bi] : bi);
        int64_t dst = xperm ? xperm[p] : p;
        out_i[dst] = res;
        if (out_d) out_d[dst] = bi < 0 ? JMAX : bd;
    }
}

__global__ void iota_kernel(int32_t *a, int64_t n) { HDB_GRID_STRIDE(i, n) a[i] = (int32_t)i; }
__global__ void gather_rows_kernel(const double *__restrict__ X, const int32_t *__restrict__ perm, int64_t n,
                                   int d, double *__restrict__ out) {
    HDB_GRID_STRIDE(t, n * d) {
        int64_t r = t / d;
        int c = (int)(t - r * d);
        out[t] = X[(int64_t)perm[r] * d + c];
    }
}

template <int D>
static void launch_nearest(hdb_ctx *ctx, const double *Xp, int64_t n, const double *Sp, int64_t m,
                           const int32_t *xk, const int32_t *sk, double *pr, int32_t *pi, int S, int64_t chunk) {
    constexpr int DP = (D + 1) & ~1;
    constexpr int Q = D <= 4 ? 4 : (D <= 8 ? 2 : 1);
    constexpr int U = D <= 4 ? 4 : 2;
    dim3 grid((unsigned)ceil_div(n, 256 * Q), S);
    KernelTimer t(ctx, "nearest_sq");
    hipLaunchKernelGGL((nearest_sq_kernel<D, DP, Q, U>), grid, dim3(256), 0, ctx->stream, Xp, n, Sp, m, xk, sk,
                       chunk, pr, pi);
    HIP_CHECK(hipGetLastError());
}

static void stable_sort_by_key(hdb_ctx *ctx, const int32_t *keys, int64_t n, int32_t *keys_out, int32_t *perm_out,
                               int32_t *perm_tmp) {
    int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    hipLaunchKernelGGL(iota_kernel, dim3(g), dim3(256), 0, ctx->stream, perm_tmp, n);
    size_t tb = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys_out, perm_tmp, perm_out, (int)n, 0, 32,
                                                 ctx->stream));
    void *tmp = arena(ctx, A_SORT, tb);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys_out, perm_tmp, perm_out, (int)n, 0, 32,
                                                 ctx->stream));
}

void nearest_sample_device(hdb_ctx *ctx, const double *X, int64_t n, const double *S, int64_t m, int d,
                           int metric, const int32_t *xkey, const int32_t *skey, int32_t *out_i, double *out_d) {
    if (n == 0) return;
    if (n > INT32_MAX || m > INT32_MAX) HDB_THROW(HDB_EINVAL, "n or m exceeds int32");
    const bool keyed = xkey && skey;
    // scratch carve
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    int dp = (d + 1) & ~1;
    const bool fast = metric == HDB_METRIC_EUCLIDEAN && (d <= 6 || d == 8 || d == 16);
    int tiles = (int)ceil_div(n, fast ? 256 * (d <= 4 ? 4 : (d <= 8 ? 2 : 1)) : 256);
    int SPL = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ctx->num_cus * 8, tiles), 64));
    while (SPL > 1 && m / SPL < 512) SPL--;
    if (keyed) SPL = 1;  // key ranges are small; one split keeps the lane ranges simple
    int64_t chunk = ceil_div(std::max<int64_t>(m, 1), SPL);

    size_t o_xp = carve(sizeof(double) * n * dp), o_sp = carve(sizeof(double) * m * dp);
    size_t o_pr = carve(sizeof(double) * n * SPL), o_pi = carve(sizeof(int32_t) * n * SPL);
    size_t o_xk = carve(sizeof(int32_t) * n), o_sk = carve(sizeof(int32_t) * m);
    size_t o_xperm = carve(sizeof(int32_t) * n), o_sperm = carve(sizeof(int32_t) * m);
    size_t o_tmp = carve(sizeof(int32_t) * std::max(n, m));
    size_t o_xs = carve(sizeof(double) * n * d), o_ss = carve(sizeof(double) * m * d);
    char *base = (char *)arena(ctx, A_WORK0, off);
    double *Xp = (double *)(base + o_xp), *Sp = (double *)(base + o_sp);
    double *pr = (double *)(base + o_pr);
    int32_t *pi = (int32_t *)(base + o_pi);
    int32_t *xks = nullptr, *sks = nullptr, *xperm = nullptr, *sperm = nullptr;
    const double *Xsrc = X, *Ssrc = S;
    int g = 1024;
    if (keyed) {
        xks = (int32_t *)(base + o_xk);
        sks = (int32_t *)(base + o_sk);
        xperm = (int32_t *)(base + o_xperm);
        sperm = (int32_t *)(base + o_sperm);
        int32_t *tmp = (int32_t *)(base + o_tmp);
        stable_sort_by_key(ctx, xkey, n, xks, xperm, tmp);
        stable_sort_by_key(ctx, skey, m, sks, sperm, tmp);
        double *Xs = (double *)(base + o_xs), *Ss = (double *)(base + o_ss);
        hipLaunchKernelGGL(gather_rows_kernel, dim3(g), dim3(256), 0, ctx->stream, X, xperm, n, d, Xs);
        if (m) hipLaunchKernelGGL(gather_rows_kernel, dim3(g), dim3(256), 0, ctx->stream, S, sperm, m, d, Ss);
        Xsrc = Xs;
        Ssrc = Ss;
    }
    if (fast) {
        pack_rows(ctx, Xsrc, n, d, dp, Xp);
        pack_rows(ctx, Ssrc, m, d, dp, Sp);
        switch (d) {
        case 1: launch_nearest<1>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 2: launch_nearest<2>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 3: launch_nearest<3>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 4: launch_nearest<4>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 5: launch_nearest<5>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 6: launch_nearest<6>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 8: launch_nearest<8>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        case 16: launch_nearest<16>(ctx, Xp, n, Sp, m, xks, sks, pr, pi, SPL, chunk); break;
        }
    } else {
        KernelTimer t(ctx, "nearest_generic");
        hipLaunchKernelGGL(nearest_generic_kernel, dim3((unsigned)ceil_div(n, 256), SPL), dim3(256), 0, ctx->stream,
                           Xsrc, n, Ssrc, m, d, metric, xks, sks, chunk, pr, pi);
    }
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(nearest_merge_kernel, dim3(g), dim3(256), 0, ctx->stream, pr, pi, n, SPL, sperm, xperm, out_i,
                       out_d);
    HIP_CHECK(hipGetLastError());
}

}  // namespace hdb
