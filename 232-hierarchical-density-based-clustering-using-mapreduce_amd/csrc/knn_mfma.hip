// knn_mfma.hip -- K1m: exact k-NN lists for high-dimensional euclidean data (BASELINE
// config 4, 2M x 128) on the matrix cores.
//
// The reference computes every distance as sqrt(((0 + (a0-b0)^2) + (a1-b1)^2) + ...) in
// double (EuclideanDistance.java:28-36) and keeps the k smallest per row with a strict '<'
// insertion (HDBSCANStar.java:84-97).  At d = 128 that is 3d FP64 VALU ops per pair.  K1m
// instead screens every (query, candidate) pair with the norm expansion
//     |q - c|^2 = |q|^2 + |c|^2 - 2 q.c
// on bf16 MFMA (v_mfma_f32_32x32x16_bf16, FP32 accumulate), and re-computes only the pairs
// the screen cannot rule out in exact FP64, in the reference's order.  The lists are
// therefore bit-identical to the FP64 scan (K1).
//
// Screen precision: each centred, power-of-two-scaled coordinate x is split x = h + l + e
// with h = bf16(x), l = bf16(x - h), |e| <= 2^-16 (1 + 2^-7) |x|; the dot product takes the
// three products h.h' + h.l' + l.h' (the dropped l.l' and the e terms are <= 3.1 * 2^-16
// sum |x_i y_i|), all exact in FP32, accumulated by the MFMA in FP32 (<= 3 * DP additions:
// gamma <= 3 DP 2^-24).  With Cauchy-Schwarz sum |x_i y_i| <= |x| |y|, the screen error is
//     |approx - |x - y|^2| <= 2 (3.1 * 2^-16 + 3 DP 2^-24) |x| |y| + 4e-13 (|x|^2 + |y|^2) + tiny
// (the second term, 4e-13 (|x|^2 + |y|^2), covers the FP64 centring, norms and final
// combination, and the rounding of the exact value itself, <= 2 d 2^-53 |x - y|^2).  A pair is
// skipped only when approx - bound > T, T = the query's current KC-th smallest exact value:
// its exact value is then > T and could not enter the list.
//
// Work decomposition: a workgroup owns 128 queries (their bf16 fragments stay in VGPRs) and
// streams all candidates in blocks of 64 through LDS; its 8 waves each produce one 32 x 32
// tile of the 128 x 64 block.  Pairs that pass the screen are re-checked by the lane holding
// them and appended to the query's LDS buffer; after the block, 128 owner threads merge the
// buffers into register top-KC lists (the same insertion network as K1) and publish the new
// thresholds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "internal.hpp"

namespace hdb {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MQ = 128;  // queries per workgroup (8 waves: 4 query rows x 2 candidate columns of 32)
constexpr int NT = 512;  // threads per workgroup
constexpr int MC = 64;  // candidates per streamed block
constexpr int KS = 16;  // k per MFMA step

// ---------------------------------------------------------------- prep
// per-column partial sums (centre) and max |x| over row slices; coalesced: consecutive
// threads read consecutive columns of one row
__global__ __launch_bounds__(256) void col_stats_kernel(const double *__restrict__ X, int64_t n, int d, int nb,
                                                        double *__restrict__ part_sum, double *__restrict__ part_max) {
    const int64_t r0 = (int64_t)blockIdx.x * n / nb, r1 = (int64_t)(blockIdx.x + 1) * n / nb;
    for (int c = threadIdx.x; c < d; c += blockDim.x) {
        double s = 0, m = 0;
        for (int64_t r = r0; r < r1; r++) {
            const double v = X[r * d + c];
            s += v;
            m = fmax(m, fabs(v));  // NaN ignored here; checked separately
        }
        part_sum[(int64_t)blockIdx.x * d + c] = s;
        part_max[(int64_t)blockIdx.x * d + c] = m;
    }
}

// centre, finiteness flag and the power-of-two scale that brings max |x - mu| to [0.5, 1)
__global__ void centre_kernel(const double *__restrict__ part_sum, const double *__restrict__ part_max, int nb,
                              int64_t n, int d, double *__restrict__ mu, double *__restrict__ prm) {
    __shared__ double smax[256];
    double m = 0;
    bool finite = true;
    for (int c = threadIdx.x; c < d; c += blockDim.x) {
        double s = 0, mx = 0;
        for (int b = 0; b < nb; b++) {
            s += part_sum[(int64_t)b * d + c];
            mx = fmax(mx, part_max[(int64_t)b * d + c]);
        }
        const double mc = s / (double)n;
        mu[c] = mc;
        if (!isfinite(s) || !isfinite(mx)) finite = false;
        m = fmax(m, mx + fabs(mc));  // bound on |x - mu|
    }
    smax[threadIdx.x] = finite ? m : INFINITY;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double M = smax[0];
        int e = 0;
        if (isfinite(M) && M > 0) frexp(M, &e);
        prm[0] = isfinite(M) ? 1.0 : 0.0;  // usable
        prm[1] = ldexp(1.0, -e);           // scale: exact power of two
    }
}

// bf16 round-to-nearest-even of a finite double via float (|x| <= 1 here)
__device__ __forceinline__ __bf16 to_bf16(double x) { return (__bf16)(float)x; }

// row prep: centred scaled coordinates split into bf16 hi/lo (zero padded to DP), and the
// FP64 norms of the centred scaled row
__global__ __launch_bounds__(256) void split_rows_kernel(const double *__restrict__ X, int64_t n, int64_t n_pad, int d,
                                                         int DP, const double *__restrict__ mu,
                                                         const double *__restrict__ prm, __bf16 *__restrict__ Xh,
                                                         __bf16 *__restrict__ Xl, double *__restrict__ nrm2,
                                                         double *__restrict__ nrm) {
    const double sc = prm[1];
    // one wave per row
    const int lane = threadIdx.x & 63;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n_pad;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        double acc = 0;
        for (int c = lane; c < DP; c += 64) {
            double v = 0;
            if (r < n && c < d) v = (X[r * d + c] - mu[c]) * sc;
            const __bf16 h = to_bf16(v);
            const __bf16 l = to_bf16(v - (double)(float)h);
            Xh[r * DP + c] = h;
            Xl[r * DP + c] = l;
            acc += v * v;
        }
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0) {
            nrm2[r] = acc;
            nrm[r] = sqrt(acc) * (1.0 + 1e-15);
        }
    }
}

// Exact squared distance in the reference's order (EuclideanDistance.java:28-36): the
// additions stay sequential; the loads are issued 8 at a time (independent addresses)
// so a re-check costs d/8 memory round trips instead of d.
template <int DP>
__device__ __forceinline__ double exact_sq(const double *__restrict__ a, const double *__restrict__ b, int d) {
    constexpr int U = 8;
    double sx = 0.0;  // 0 + t0^2 == t0^2 exactly (t^2 >= 0)
    for (int j0 = 0; j0 < d; j0 += U) {
        double av[U], bv[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int j = j0 + u < d ? j0 + u : d - 1;  // clamped: in bounds, unused past d
            av[u] = a[j];
            bv[u] = b[j];
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (j0 + u < d) sx = sx + sq_diff(av[u], bv[u]);
    }
    return sx;
}

// ---------------------------------------------------------------- main
// Two passes over the same MFMA pipeline:
//  PASS_UB (0): per query, the KC smallest UPPER bounds (approx + bound) of the candidates'
//               exact values; thr_out = the KC-th (a rigorous upper bound on the KC-th
//               smallest exact value T*: KC distinct candidates are at or below it).  The
//               screen here is only a heuristic (skipping candidates loosens the bound, it
//               never invalidates it).
//  PASS_EXACT (1): starting from thr_init, a pair is skipped only when approx - bound > thr
//               (its exact value provably exceeds thr >= T*); survivors are re-checked in
//               exact FP64 and merged.  With the pass-0 bound the survivors are ~KC + the
//               few candidates within 2 bound of T*, instead of every running-minimum update
//               of a single pass.
// A cheap FP32 pre-screen (conservative margin) discards most pairs before the FP64 test.
template <int DP, int KC, int PASS>
__global__ __launch_bounds__(NT) void knn_mfma_kernel(const double *__restrict__ X, int64_t n, int64_t n_pad, int d,
                                                       const __bf16 *__restrict__ Xh, const __bf16 *__restrict__ Xl,
                                                       const double *__restrict__ nrm2, const double *__restrict__ nrm,
                                                       const double *__restrict__ prm, int excl,
                                                       const double *__restrict__ thr_init, double *__restrict__ thr_out,
                                                       double *__restrict__ lists, unsigned long long *__restrict__ stats) {
    constexpr int NS = DP / KS;  // MFMA k-steps
    constexpr int LDP = DP + 8;  // LDS row pitch (bf16): 16 B pad breaks the bank aliasing
    constexpr int CH = DP / 8;   // 16-B chunks per row
    constexpr int PF = (MC * CH + NT - 1) / NT;  // prefetched chunks per thread (per array)
    __shared__ __bf16 ch_s[MC * LDP];
    __shared__ __bf16 cl_s[MC * LDP];
    __shared__ double cn2_s[MC], cn_s[MC];
    __shared__ double qn2_s[MQ], qn_s[MQ], thr_s[MQ];
    __shared__ float thrf_s[MQ];
    __shared__ int cnt_s[MQ];
    __shared__ double buf_s[MQ * MC];

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wq = wave & 3, wc = wave >> 2;
    const int64_t qbase = (int64_t)blockIdx.x * MQ;
    const double sc = prm[1], sc2 = sc * sc;
    const double eps_dot = 2.0 * (3.1 * 0x1p-16 + 3.0 * DP * 0x1p-24) * 1.01;
    const int ex = excl & 1;

    // resident query fragments (A operand): row 32wq + (lane & 31), k = 16s + 8 (lane >> 5) + j
    bf16x8 ah[NS], al[NS];
    {
        const int64_t row = qbase + 32 * wq + (lane & 31);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int64_t o = row * DP + KS * s + 8 * (lane >> 5);
            ah[s] = *(const bf16x8 *)(Xh + o);
            al[s] = *(const bf16x8 *)(Xl + o);
        }
    }
    double top[KC];
#pragma unroll
    for (int k = 0; k < KC; k++) top[k] = INFINITY;
    if (tid < MQ) {
        qn2_s[tid] = nrm2[qbase + tid];
        qn_s[tid] = nrm[qbase + tid];
        const double t0 = (PASS == 1 && thr_init) ? thr_init[qbase + tid] : INFINITY;
        thr_s[tid] = t0;
        thrf_s[tid] = (float)(t0 * sc2) * (1.0f + 1e-6f) + 1e-30f;  // rounded up (FP32 pre-screen)
        cnt_s[tid] = 0;
    }
    unsigned long long n_re = 0;
    // prefetch registers for the next candidate block
    bf16x8 ph[PF], pl[PF];
    double pc2 = 0, pcn = 0;
    auto prefetch = [&](int64_t cb) {
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int e = tid + NT * u < MC * CH ? tid + NT * u : MC * CH - 1;  // clamped (DP = 32)
            const int r = e / CH, c8 = (e % CH) * 8;
            const int64_t g = (cb + r) * DP + c8;
            ph[u] = *(const bf16x8 *)(Xh + g);
            pl[u] = *(const bf16x8 *)(Xl + g);
        }
        if (tid < MC) {
            pc2 = nrm2[cb + tid];
            pcn = nrm[cb + tid];
        }
    };
    prefetch(0);

    for (int64_t cbase = 0; cbase < n_pad; cbase += MC) {
        // park the prefetched block in LDS (the previous block's readers are past the barrier)
#pragma unroll
        for (int u = 0; u < PF; u++) {
            const int e = tid + NT * u;
            if (e >= MC * CH) break;
            const int r = e / CH, c8 = (e % CH) * 8;
            *(bf16x8 *)(ch_s + r * LDP + c8) = ph[u];
            *(bf16x8 *)(cl_s + r * LDP + c8) = pl[u];
        }
        if (tid < MC) {
            cn2_s[tid] = pc2;
            cn_s[tid] = pcn;
        }
        __syncthreads();
        if (cbase + MC < n_pad) prefetch(cbase + MC);  // in flight during the MFMAs + epilogue
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; r++) acc[r] = 0.f;
        const int crow = 32 * wc + (lane & 31);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int o = crow * LDP + KS * s + 8 * (lane >> 5);
            const bf16x8 bh = *(const bf16x8 *)(ch_s + o);
            const bf16x8 bl = *(const bf16x8 *)(cl_s + o);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s], bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], bh, acc, 0, 0, 0);
        }
        // screen; C layout: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
        const int cc = 32 * wc + (lane & 31);
        const int64_t cid = cbase + cc;
        const double c2 = cn2_s[cc], cn = cn_s[cc];
        const float c2f = (float)c2, cnf = (float)cn;
        const float epsf = (float)eps_dot * 1.001f;
#pragma unroll
        for (int r = 0; r < 16; r++) {
            const int qr = 32 * wq + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const float q2f = (float)qn2_s[qr];
            // FP32 pre-screen: af is within 8 * 2^-24 (q2 + c2) of the FP64 approx; the
            // 1e-6 (q2 + c2) margin also covers the rounding of the bound itself
            const float af = (q2f + c2f) - 2.0f * acc[r];
            const float bf = epsf * (float)qn_s[qr] * cnf + 1e-6f * (q2f + c2f);
            if (af - bf > thrf_s[qr]) continue;
            const int64_t qid = qbase + qr;
            if (qid >= n || cid >= n || (ex && qid == cid)) continue;
            const double q2 = qn2_s[qr];
            const double approx = (q2 + c2) - 2.0 * (double)acc[r];
            const double bound = eps_dot * qn_s[qr] * cn + 4e-13 * (q2 + c2) + 1e-30;
            double val;
            if (PASS == 0) {
                val = (approx + bound) / sc2;  // rigorous upper bound of the exact value
                if (!(val < thr_s[qr])) continue;
            } else {
                if (approx - bound > thr_s[qr] * sc2) continue;
                val = (excl & 2) ? approx / sc2 : exact_sq<DP>(X + qid * d, X + cid * d, d);
                n_re++;
            }
            const int slot = atomicAdd(&cnt_s[qr], 1);
            buf_s[qr * MC + slot] = val;
        }
        __syncthreads();
        if (tid < MQ) {
            const int m = cnt_s[tid];
            for (int j = 0; j < m; j++) topk_insert<KC>(top, buf_s[tid * MC + j]);
            cnt_s[tid] = 0;
            const double t = top[KC - 1] < thr_s[tid] ? top[KC - 1] : thr_s[tid];
            thr_s[tid] = t;
            thrf_s[tid] = (float)(t * sc2) * (1.0f + 1e-6f) + 1e-30f;
        }
        __syncthreads();
    }
    if (tid < MQ && qbase + tid < n) {
        if (PASS == 0) {
            thr_out[qbase + tid] = top[KC - 1];
        } else {
#pragma unroll
            for (int k = 0; k < KC; k++) {
                const double v = top[k];
                lists[(qbase + tid) * KC + k] = (v < INFINITY) ? sqrt(v) : JMAX;  // Java keeps Double.MAX_VALUE
            }
        }
    }
    if (stats) {
        for (int o = 32; o >= 1; o >>= 1) n_re += __shfl_xor(n_re, o);
        if (lane == 0) atomicAdd(stats, n_re);
    }
}

// ---------------------------------------------------------------- host
template <int DP>
static bool knn_mfma_dp(hdb_ctx *ctx, const double *X, int64_t n, int d, int KC, bool excl, double *lists) {
    const int64_t n_pad = ceil_div(n, (int64_t)MQ) * MQ;
    const int nb = (int)std::min<int64_t>(1024, std::max<int64_t>(1, n / 64));
    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t bytes = 2 * rnd(sizeof(__bf16) * (size_t)(n_pad * DP)) + 3 * rnd(8 * (size_t)n_pad) +
                         2 * rnd(8 * (size_t)nb * d) + rnd(8 * (size_t)d) + 256 + 256;
    char *base = (char *)arena(ctx, A_WORK3, bytes);
    size_t off = 0;
    auto take = [&](size_t b) {
        char *p = base + off;
        off += rnd(b);
        return p;
    };
    __bf16 *Xh = (__bf16 *)take(sizeof(__bf16) * (size_t)(n_pad * DP));
    __bf16 *Xl = (__bf16 *)take(sizeof(__bf16) * (size_t)(n_pad * DP));
    double *nrm2 = (double *)take(8 * (size_t)n_pad), *nrm = (double *)take(8 * (size_t)n_pad);
    double *psum = (double *)take(8 * (size_t)nb * d), *pmax = (double *)take(8 * (size_t)nb * d);
    double *mu = (double *)take(8 * (size_t)d);
    double *thr = (double *)take(8 * (size_t)n_pad);
    const bool two_pass = ctx->knn_mfma_two_pass;
    double *prm = (double *)take(256);
    unsigned long long *stats = (unsigned long long *)take(256);
    hipStream_t st = ctx->stream;
    hipLaunchKernelGGL(col_stats_kernel, dim3(nb), dim3(256), 0, st, X, n, d, nb, psum, pmax);
    hipLaunchKernelGGL(centre_kernel, dim3(1), dim3(256), 0, st, psum, pmax, nb, n, d, mu, prm);
    double h_prm[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(h_prm, prm, 16, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (h_prm[0] != 1.0) return false;  // non-finite input: the FP64 scan handles it
    {
        const int g = (int)std::min<int64_t>(ceil_div(n_pad * 64, 256), 8192);
        hipLaunchKernelGGL(split_rows_kernel, dim3(g), dim3(256), 0, st, X, n, n_pad, d, DP, mu, prm, Xh, Xl, nrm2,
                           nrm);
    }
    if (ctx->count_evals) HIP_CHECK(hipMemsetAsync(stats, 0, 8, st));
    {
        KernelTimer t(ctx, "knn_mfma");
        const dim3 grid((unsigned)(n_pad / MQ));
        const int fl = (excl ? 1 : 0) | (getenv("HDBMI_K1M_DBG") ? 2 : 0);
#define K1M_CASE(KK)                                                                                             \
    case KK:                                                                                                     \
        if (two_pass)                                                                                            \
            hipLaunchKernelGGL((knn_mfma_kernel<DP, KK, 0>), grid, dim3(NT), 0, st, X, n, n_pad, d, Xh, Xl, nrm2, \
                               nrm, prm, fl, nullptr, thr, lists, nullptr);                                     \
        hipLaunchKernelGGL((knn_mfma_kernel<DP, KK, 1>), grid, dim3(NT), 0, st, X, n, n_pad, d, Xh, Xl, nrm2,     \
                           nrm, prm, fl, two_pass ? thr : nullptr, nullptr, lists,                               \
                           ctx->count_evals ? stats : nullptr);                                                  \
        break;
        switch (KC) {
            K1M_CASE(1)
            K1M_CASE(3)
            K1M_CASE(7)
            K1M_CASE(15)
            K1M_CASE(31)
        default: return false;
        }
#undef K1M_CASE
        HIP_CHECK(hipGetLastError());
    }
    if (ctx->count_evals) {
        unsigned long long h = 0;
        HIP_CHECK(hipMemcpyAsync(&h, stats, 8, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        ctx->stats["knn_mfma_rechecks"] = (int64_t)h;
        ctx->stats["last_evals"] = (int64_t)h;
    }
    return true;
}

bool knn_mfma_device(hdb_ctx *ctx, const double *X, int64_t n, int d, int KC, bool excl, double *lists) {
    if (n < 1 || d < 1) return false;
    if (d <= 32) return knn_mfma_dp<32>(ctx, X, n, d, KC, excl, lists);
    if (d <= 64) return knn_mfma_dp<64>(ctx, X, n, d, KC, excl, lists);
    if (d <= 128) return knn_mfma_dp<128>(ctx, X, n, d, KC, excl, lists);
    if (d <= 256) return knn_mfma_dp<256>(ctx, X, n, d, KC, excl, lists);
    return false;
}

}  // namespace hdb
