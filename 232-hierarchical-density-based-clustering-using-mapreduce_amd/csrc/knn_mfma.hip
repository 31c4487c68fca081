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
#include <type_traits>
#include <vector>

#include "internal.hpp"
#include "sort.hpp"

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
                                                         double *__restrict__ nrm, const int *__restrict__ perm,
                                                         double *__restrict__ Xlay = nullptr) {
    const double sc = prm[1];
    // one wave per row
    const int lane = threadIdx.x & 63;
    for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n_pad;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        double acc = 0;
        for (int c = lane; c < DP; c += 64) {
            double v = 0;
            const int64_t src = perm ? (int64_t)perm[r] : (r < n ? r : -1);  // -1: padding row
            const double x = (src >= 0 && c < d) ? X[src * d + c] : 0.0;
            if (Xlay) Xlay[r * DP + c] = x;  // the FP64 row in layout order, zero padded to DP (re-check)
            if (src >= 0 && c < d) v = (x - mu[c]) * sc;
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

// ---------------------------------------------------------------- single pass (default)
// K1m-s: ONE MFMA pass over all pairs (the two-pass kernel above is the fallback).  Per
// query it keeps the KC smallest rigorous UPPER bounds (approx + bound, FP32 rounded up) of
// the candidates seen so far: their largest, thr, is >= the KC-th smallest exact value T*.
// Every candidate whose LOWER bound (approx - bound) is <= the running thr is appended to the
// query's candidate log (id, lower bound rounded down).  thr only decreases, so a candidate
// left out of the log has lb > thr_at_that_time >= thr_final >= T*: its exact value exceeds
// T* and it cannot be among the KC smallest.  A second, tiny kernel re-computes the logged
// candidates with lb <= thr_final in exact FP64 (the reference's order) and keeps the KC
// smallest -- the lists equal the FP64 scan bit for bit.  The deferred re-check takes the
// FP64 work (and its random row loads) out of the MFMA loop; the pass is not repeated.
//
// Tiles: candidates are the MFMA A operand (rows), queries the B operand (columns), so a lane
// holds one query per 32 x 32 tile and its screen constants are per-lane scalars.  A wave
// keeps QT query tiles resident in VGPRs (bf16 hi/lo fragments); the four waves of a
// workgroup share each 32-candidate block, staged global -> LDS by global_load_lds (16 B,
// XOR-swizzled 16-B chunks: conflict-free ds_read_b128), double-buffered, one barrier per
// block.  The screen per pair is one FMA, one subtract and one max: with
//     g = eps |q| / 2,  hc = c2 (1 - 4e-6) / 2,  a = (q2 (1 - 4e-6) - thr) / 2
// a pair can pass the FP64 test  (q2 + c2 - 2 acc) - bound <= thr  only if
//     fma(g, |c|, acc) - hc >= a
// (the 4e-6 (q2 + c2) margin covers every FP32 rounding of this test); a wave branches to
// the rare hit path only when a lane's maximum over its 16 pairs reaches a.
constexpr int S_LOGCAP = 512;  // log entries per query (compacted against thr when full)
struct LogEnt {
    int cid;
    float lb;
};
constexpr int S_CST = 192;  // per 32-candidate block: hc[32], cn[32] (float), c2[32], cn[32] (double)

#ifndef HDB_K1S_WAVES
// waves per workgroup.  The block loop's one barrier per 32-candidate block makes every wave
// wait for the slowest one's hit path; two 4-wave workgroups per CU (128 queries each) wait
// on fewer waves and independently: screen 33.0 -> 31.1 ms at C4 (r05; round 3 measured 8
// against 4 waves x 2 query tiles: 51.9 vs 56.0 ms)
#define HDB_K1S_WAVES 4
#endif
#ifndef HDB_K1S_QT
#define HDB_K1S_QT 1  // query tiles per wave at DP <= 128 (64 fragment VGPRs: 4 waves per SIMD)
#endif
constexpr int NW = HDB_K1S_WAVES;
#ifndef HDB_K1S_XCD
#define HDB_K1S_XCD 1  // contiguous query-group ranges per XCD (A/B at C4: screen 51.8 -> 50.7 ms)
#endif
#ifndef HDB_K1S_REGTOP
// 1: each lane keeps the running top-KC upper bounds of its (query, half-wave) pair in
// registers and logs into its own half of the query's log, so the two half-waves of a wave
// take their hits at the same time and an insertion is a register network instead of a
// dependent LDS shift chain (KC <= 15).  The query's threshold is the KC-th smallest bound of
// the union of its two halves' lists (the halves see disjoint candidate rows, so the union
// holds bounds of distinct candidates: >= the KC-th exact value), refreshed per hit step
#define HDB_K1S_REGTOP 1
#endif
#ifndef HDB_K1S_PROF
#define HDB_K1S_PROF 0  // diagnostic build: per-wave cycle split of the screen loop (stats k1s_prof_*)
#endif
// (round 5 measured two ways of writing the screen's log entries in larger pieces -- an
// 8-entry LDS buffer per (query, half) flushed 64 bytes at a time, and entry pairs held in
// registers and stored as 16 bytes: HBM writes 6.54 -> 3.04 / 5.09 GB per launch at C4, but
// the screen took 36.9 -> 38.2 / 39.0 ms, the longer hit path costing more than the traffic)
#ifndef HDB_K1F_XCD
#define HDB_K1F_XCD 1  // K1m re-check: contiguous 16-query workgroup ranges per XCD (shared candidate rows in one L2)
#endif
#define K1S_XCD HDB_K1S_XCD
// Workgroups are dealt round-robin over the 8 XCDs (block b runs on XCD b mod 8); this maps
// them so XCD x takes one contiguous range of logical blocks (a bijection on [0, G)).
__device__ __forceinline__ int64_t xcd_contig(int64_t b, int64_t G) {
    const int64_t q = G >> 3, r = G & 7, x = b & 7, k = b >> 3;
    return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}
#ifndef HDB_K1S_WPE
#define HDB_K1S_WPE (HDB_K1S_QT == 1 ? (HDB_K1S_REGTOP ? 2 : 4) : 2)  // REGTOP: one 8-wave workgroup per CU
                                                                      // either way; 2 leaves 192 VGPRs (A/B: 37.5 -> 36.9 ms)
#endif
constexpr int K1S_WPE = HDB_K1S_WPE;  // waves per SIMD (A/B at C4: 4 = two workgroups per CU, 51.7 ms, despite
                                      // spilling some fragments; 3 = 168 VGPRs without spills, one workgroup, 57.0 ms)
template <int DP>
struct ScreenCfg {
    static constexpr int QT = DP <= 128 ? HDB_K1S_QT : 1;  // query tiles per wave (VGPR-resident fragments)
    static constexpr int SQ = NW * 32 * QT;       // queries per workgroup
    static constexpr int CH = DP / 8;             // 16-B chunks per bf16 row
    static constexpr int BUF = 2 * 32 * DP;       // bf16 elements per staged block (hi rows, lo rows)
};

// Cross-lane steps without LDS round trips (ds_bpermute: one LDS trip per step, and a chain of
// them per reduction): DPP inside a 16-lane row, v_permlane{16,32}_swap (gfx950) across rows.
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HMIRROR = 0x141, DPP_MIRROR = 0x140;
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    const int b = __float_as_int(v);  // (a lane whose source is off keeps its own value)
    return __int_as_float(__builtin_amdgcn_update_dpp(b, b, CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)b, (int)b, CTRL, 0xf, 0xf, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// the value of lane ^ 32: v_permlane32_swap(v, v) leaves the low half's values in the first
// result's high half and the high half's values in the second result's low half
__device__ __forceinline__ float xor32_f(float v, int lane) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(lane < 32 ? p[1] : p[0]);
}
// maximum over the wave, in every lane (a row's own and partner values both sit in the swap's
// two results, so the symmetric max needs no lane select)
__device__ __forceinline__ float wave_max_f(float v) {
    v = fmaxf(v, dpp_f<DPP_XOR1>(v));
    v = fmaxf(v, dpp_f<DPP_XOR2>(v));
    v = fmaxf(v, dpp_f<DPP_HMIRROR>(v));
    v = fmaxf(v, dpp_f<DPP_MIRROR>(v));
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(v, fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1])));
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(v, fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1])));
}
// minimum over each 16-lane row, in every lane of the row
__device__ __forceinline__ double row_min_d(double v) {
    v = fmin(v, dpp_d<DPP_XOR1>(v));
    v = fmin(v, dpp_d<DPP_XOR2>(v));
    v = fmin(v, dpp_d<DPP_HMIRROR>(v));
    return fmin(v, dpp_d<DPP_MIRROR>(v));
}

// directed conversions (largest float <= x, smallest float >= x), branch-free
__device__ __forceinline__ float f32_down(double x) { return __double2float_rd(x); }
__device__ __forceinline__ float f32_up(double x) { return __double2float_ru(x); }

// per-block screen constants, packed so one global_load_lds stages them
__global__ void screen_consts_kernel(const double *__restrict__ nrm2, const double *__restrict__ nrm, int64_t n_pad,
                                     const int *__restrict__ perm, float *__restrict__ cst) {
    HDB_GRID_STRIDE(r, n_pad) {
        float *b = cst + (r >> 5) * S_CST;
        const int i = (int)(r & 31);
        // a padding row of the layout never passes the screen (hc = +inf)
        b[i] = perm[r] < 0 ? INFINITY : (float)(nrm2[r] * (1.0 - 4e-6) * 0.5);
        b[32 + i] = (float)nrm[r];
        // |c|^2 of a padding row is NaN: its exact-test bound lb = NaN never passes lb <= thr
        ((double *)(b + 64))[i] = perm[r] < 0 ? __builtin_nan("") : nrm2[r];
        ((double *)(b + 128))[i] = nrm[r];
    }
}

// the log of one query (or half-query) is full: keep the entries that can still matter (lb <= thr)
__device__ __noinline__ int log_compact(LogEnt *L, float t, int cap = S_LOGCAP) {
    int w = 0;
    for (int j = 0; j < cap; j++) {
        const LogEnt e = L[j];
        if (e.lb <= t) L[w++] = e;
    }
    return w;
}

// ---------------------------------------------------------------- candidate order (pruned K1m)
// Exact pruning needs spatially compact candidate blocks and query groups.  The rows are
// ordered by a few Lloyd iterations of k-means (KM_K centroids) on a 32-dimensional +-1
// random projection of the bf16 rows, then by the first projected coordinate: clustered data
// (embeddings) lands in runs of one cluster each.  The order only decides how much is
// pruned; every skip below is proven with FP64 balls, whatever the order.  (A random-
// projection tree with median splits was tried first: in 128 dimensions a single projection
// crowds 200 clusters together and every split cuts through dozens of them.)
constexpr int KM_P = 32;   // projected dimensions
constexpr int KM_K = 1024;  // centroids (several per cluster: a cluster without a seed merges)
// Lloyd iterations of the layout's k-means (the layout only steers pruning): A/B at C4 (r05,
// profiles/r05/c4/ab_kmeans_it.log): 2 -> order 2.7 ms, screen 30.0; 3 -> 3.1 / 30.0;
// 4 -> 3.5 / 29.9; 6 -> 4.3 / 30.0 -- the extra passes no longer buy screen time
constexpr int KM_IT = 2;

__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t f32_order(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Y[i] = R x_i, R[p][j] = +-1 (hash of p and j)
__global__ __launch_bounds__(256) void km_project_kernel(const __bf16 *__restrict__ Xh, int DP, int d, int64_t n,
                                                         float *__restrict__ Y) {
    HDB_GRID_STRIDE(i, n) {
        const __bf16 *x = Xh + i * DP;
        float y[KM_P];
#pragma unroll
        for (int p = 0; p < KM_P; p++) y[p] = 0.f;
        for (int j0 = 0; j0 < d; j0 += 8) {
            const bf16x8 v = *(const bf16x8 *)(x + j0);  // zero past d (DP padding)
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const float f = (float)v[u];
                const uint32_t sg = hash_u32((uint32_t)(j0 + u) * 0x9E3779B1u + 0x5bd1e995u);
#pragma unroll
                for (int p = 0; p < KM_P; p++) y[p] += ((sg >> p) & 1u) ? -f : f;
            }
        }
#pragma unroll
        for (int p = 0; p < KM_P; p++) Y[i * KM_P + p] = y[p];
    }
}

// initial centroids: KM_K rows spread over the input
__global__ void km_init_kernel(const float *__restrict__ Y, int64_t n, float *__restrict__ C) {  // grid: k
    const int c = blockIdx.x, p = threadIdx.x;
    const int64_t r = (int64_t)(((unsigned long long)hash_u32(c * 2654435761u + 17u) * (unsigned long long)n) >> 32);
    C[c * KM_P + p] = Y[r * KM_P + p];
}

// The same assignment on the matrix cores: argmin_c |c|^2 - 2 y.c with y and c rounded to
// bf16 (the layout only steers how much the screen prunes -- every skip stays proven with FP64
// balls -- so a rounding-level tie broken differently is harmless).  Centroids (bf16, |c|^2 in
// FP32, padding +inf) sit in LDS; a wave takes 32 rows as the B operand (columns) and runs
// every 32-centroid tile as the A operand: two v_mfma_f32_32x32x16_bf16 per tile (K = 32
// projected dimensions), then each lane folds its 16 centroid rows into (min, argmin) and the
// two half-waves combine by shfl_xor 32 (ties: the lower centroid).
constexpr int KMA_WAVES = 4;
__global__ __launch_bounds__(64 * KMA_WAVES) void km_assign_mfma_kernel(const float *__restrict__ Y, int64_t n,
                                                                       int64_t step, int k,
                                                                       const float *__restrict__ C,
                                                                       int *__restrict__ asg, float *__restrict__ sum,
                                                                       float *__restrict__ cnt, int *__restrict__ hist) {
    static_assert(KM_P == 32, "two 16-deep MFMA steps");
    __shared__ __attribute__((aligned(16))) __bf16 c_s[KM_K * KM_P];
    __shared__ float cn_s[KM_K];
    const int kp = (k + 31) & ~31;  // centroid tiles of 32
    for (int i = threadIdx.x; i < kp * KM_P; i += blockDim.x) c_s[i] = (__bf16)(i < k * KM_P ? C[i] : 0.f);
    __syncthreads();
    for (int c = threadIdx.x; c < kp; c += blockDim.x) {
        float s2 = 0.f;
        if (c < k)
            for (int p = 0; p < KM_P; p++) {
                const float v = (float)c_s[c * KM_P + p];
                s2 = fmaf(v, v, s2);
            }
        cn_s[c] = c < k ? s2 : INFINITY;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, half = lane >> 5, col = lane & 31;
    const int64_t wave = ((int64_t)blockIdx.x * KMA_WAVES + (threadIdx.x >> 6));
    const int64_t nw = (int64_t)gridDim.x * KMA_WAVES;
    for (int64_t r0 = wave * 32; r0 < n; r0 += nw * 32) {
        const int64_t ii = r0 + col;
        const bool real = ii < n;
        const int64_t i = (real ? ii : n - 1) * step;  // the Lloyd iterations run on a strided sample
        // B operand: row i's projected coordinates k = 16 s + 8 half + j
        bf16x8 yb[2];
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
            for (int j = 0; j < 8; j++) yb[s2][j] = (__bf16)Y[i * KM_P + 16 * s2 + 8 * half + j];
        float best = INFINITY;
        int bc = 0;
        for (int t = 0; t < kp; t += 32) {
            f32x16 acc;
#pragma unroll
            for (int r = 0; r < 16; r++) acc[r] = 0.f;
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const bf16x8 a = *(const bf16x8 *)(c_s + (t + col) * KM_P + 16 * s2 + 8 * half);
                acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, yb[s2], acc, 0, 0, 0);
            }
            // C row (centroid t + 8 gi + 4 half + u), column (row r0 + col)
#pragma unroll
            for (int gi = 0; gi < 4; gi++)
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int c = t + 8 * gi + 4 * half + u;
                    const float v = cn_s[c] - 2.f * acc[4 * gi + u];
                    if (v < best) {
                        best = v;
                        bc = c;
                    }
                }
        }
        const float ob = __shfl_xor(best, 32);
        const int oc = __shfl_xor(bc, 32);
        if (ob < best || (ob == best && oc < bc)) {
            best = ob;
            bc = oc;
        }
        if (real && half == 0) {
            asg[i] = bc;
            if (hist) atomicAdd(&hist[bc], 1);
            if (sum) {
#pragma unroll
                for (int p = 0; p < KM_P; p++) atomicAdd(&sum[bc * KM_P + p], Y[i * KM_P + p]);
                atomicAdd(&cnt[bc], 1.f);
            }
        }
    }
}

__global__ void km_update_kernel(float *__restrict__ C, float *__restrict__ sum, float *__restrict__ cnt) {
    const int c = blockIdx.x, p = threadIdx.x;
    const float k = cnt[c];
    if (k > 0.f) C[c * KM_P + p] = sum[c * KM_P + p] / k;
    __syncthreads();
    sum[c * KM_P + p] = 0.f;
    if (p == 0) cnt[c] = 0.f;
}

__global__ void km_keys_kernel(const float *__restrict__ Y, const int *__restrict__ asg, int64_t n,
                               unsigned long long *__restrict__ keys, int *__restrict__ vals) {
    HDB_GRID_STRIDE(i, n) {
        keys[i] = ((unsigned long long)asg[i] << 32) | f32_order(Y[i * KM_P]);
        vals[i] = (int)i;
    }
}

// Ball of G consecutive rows of the order (FP64, scaled domain v = (x - mu) sc, exactly as
// split_rows_kernel computes v): centre, radius and max norm, both rounded up.  One
// workgroup per group; each wave walks every fourth row, a row's d values spread over the
// lanes (coalesced 512-byte loads): column sums for the centre, then per row the squared
// distance to the centre and the squared norm summed over the wave.  Any centre gives a valid
// ball (the radius is measured from it); the 1e-12 padding covers the summation-order error.
__device__ __forceinline__ double wave_sum_d(double v) {
    v = v + dpp_d<DPP_XOR1>(v);
    v = v + dpp_d<DPP_XOR2>(v);
    v = v + dpp_d<DPP_HMIRROR>(v);
    v = v + dpp_d<DPP_MIRROR>(v);  // every lane: its 16-lane row's sum
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)b, (uint32_t)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
    v = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | lo[0]) +
        __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | lo[1]);  // own row + its pair
    const uint64_t b2 = __builtin_bit_cast(uint64_t, v);
    const auto lo2 = __builtin_amdgcn_permlane32_swap((uint32_t)b2, (uint32_t)b2, false, false);
    const auto hi2 = __builtin_amdgcn_permlane32_swap((uint32_t)(b2 >> 32), (uint32_t)(b2 >> 32), false, false);
    return __builtin_bit_cast(double, ((uint64_t)hi2[0] << 32) | lo2[0]) +
           __builtin_bit_cast(double, ((uint64_t)hi2[1] << 32) | lo2[1]);
}

__global__ __launch_bounds__(256) void ball_kernel(const double *__restrict__ X, int d, const double *__restrict__ mu,
                                                   const double *__restrict__ prm, const int *__restrict__ perm,
                                                   const int *__restrict__ g_blk, const int *__restrict__ g_nblk,
                                                   int64_t G, int DPc, double *__restrict__ ctr,
                                                   double *__restrict__ rn) {
    __shared__ double m_s[256], part_s[4][256];
    __shared__ double r_s[4], q_s[4];
    __shared__ int cnt_s[4];
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const double sc = prm[1];
    // rows [r0, r1) of the layout (padding rows, perm < 0, are not part of the ball)
    const int64_t r0 = g_blk ? (int64_t)g_blk[blockIdx.x] * 32 : (int64_t)blockIdx.x * G;
    const int64_t r1 = g_blk ? r0 + (int64_t)g_nblk[blockIdx.x] * 32 : r0 + G;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // columns lane + 64 j (d <= 256)
    int cnt = 0;
    for (int64_t r = r0 + wv; r < r1; r += 4) {
        const int p = perm[r];  // wave-uniform
        if (p < 0) continue;
        cnt++;
        const double *x = X + (int64_t)p * d;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int c = lane + 64 * j;
            if (c < d) acc[j] += (x[c] - mu[c]) * sc;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (lane + 64 * j < d) part_s[wv][lane + 64 * j] = acc[j];
    if (lane == 0) cnt_s[wv] = cnt;
    __syncthreads();
    const int tot = cnt_s[0] + cnt_s[1] + cnt_s[2] + cnt_s[3];
    if (tot == 0) {
        for (int c = tid; c < DPc; c += 256) ctr[(int64_t)blockIdx.x * DPc + c] = 0.0;
        if (tid == 0) rn[2 * blockIdx.x] = rn[2 * blockIdx.x + 1] = 0.0;
        return;
    }
    for (int c = tid; c < d; c += 256) m_s[c] = (((part_s[0][c] + part_s[1][c]) + part_s[2][c]) + part_s[3][c]) / (double)tot;
    __syncthreads();
    for (int c = tid; c < DPc; c += 256) ctr[(int64_t)blockIdx.x * DPc + c] = c < d ? m_s[c] : 0.0;
    double md = 0.0, mn = 0.0;
    for (int64_t r = r0 + wv; r < r1; r += 4) {
        const int p = perm[r];
        if (p < 0) continue;
        const double *x = X + (int64_t)p * d;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int c = lane + 64 * j;
            if (c < d) {
                const double v = (x[c] - mu[c]) * sc, e = v - m_s[c];
                a += e * e;
                b += v * v;
            }
        }
        md = fmax(md, wave_sum_d(a));
        mn = fmax(mn, wave_sum_d(b));
    }
    if (lane == 0) {
        r_s[wv] = md;
        q_s[wv] = mn;
    }
    __syncthreads();
    if (tid == 0) {
        const double R = fmax(fmax(r_s[0], r_s[1]), fmax(r_s[2], r_s[3]));
        const double Q = fmax(fmax(q_s[0], q_s[1]), fmax(q_s[2], q_s[3]));
        rn[2 * blockIdx.x] = sqrt(R) * (1.0 + 1e-12) + 1e-300;
        rn[2 * blockIdx.x + 1] = sqrt(Q) * (1.0 + 1e-12) + 1e-300;
    }
}

typedef __attribute__((address_space(3))) void *lds_ptr_t;

// candidate superblocks (runs of consecutive 32-row blocks of the layout) and their balls
constexpr int NSB_MAX = 2048;
struct SbArgs {
    const double *qctr, *qrn;  // query-group balls (one per workgroup)
    const double *sctr, *srn;  // superblock balls
    const int *sb_blk;         // first block of each superblock
    const int *sb_nblk;        // blocks of each superblock
    const int *perm;           // layout position -> row of X (-1: padding row)
    int nsb;                   // superblocks (<= NSB_MAX)
    int prune;                 // 0: every superblock in index order
    unsigned long long *blocks_done;
    const float *keys;         // [groups][nsbp] visiting keys from sb_keys_kernel
};

// The superblock visiting keys of every (query group, superblock) pair, computed up front in
// one grid: a workgroup takes 16 groups x 64 superblocks, their ball centres staged in LDS
// 32 dimensions at a time, each thread 4 groups of one superblock; the squared centre
// distance sums the dimensions in index order (the order the screen's own setup used).
// The screen kernel then only reads its group's row (coalesced) before sorting it.
template <int DP>
__global__ __launch_bounds__(256) void sb_keys_kernel(const double *__restrict__ qctr, const double *__restrict__ qrn,
                                                      const double *__restrict__ sctr, const double *__restrict__ srn,
                                                      int64_t ngroups, int nsb, int nsbp, double eps_dot,
                                                      float *__restrict__ keys) {
    constexpr int TG = 16, TS = 64, DC = 32;
    __shared__ double q_s[TG][DC + 1], s_s[TS][DC + 1];
    const int tid = threadIdx.x, si = tid & (TS - 1), gq = (tid >> 6) * 4;
    const int64_t g0 = (int64_t)blockIdx.y * TG;
    const int s0 = blockIdx.x * TS;
    double d2[4] = {0.0, 0.0, 0.0, 0.0};
    for (int c0 = 0; c0 < DP; c0 += DC) {
        for (int i = tid; i < TG * DC; i += 256) {
            const int r = i / DC, c = i % DC;
            q_s[r][c] = g0 + r < ngroups ? qctr[(g0 + r) * DP + c0 + c] : 0.0;
        }
        for (int i = tid; i < TS * DC; i += 256) {
            const int r = i / DC, c = i % DC;
            s_s[r][c] = s0 + r < nsb ? sctr[(int64_t)(s0 + r) * DP + c0 + c] : 0.0;
        }
        __syncthreads();
#pragma unroll 8
        for (int c = 0; c < DC; c++) {
            const double sv = s_s[si][c];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const double e = q_s[gq + u][c] - sv;
                d2[u] += e * e;
            }
        }
        __syncthreads();
    }
    const int i = s0 + si;
    if (i >= nsbp) return;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int64_t g = g0 + gq + u;
        if (g >= ngroups) continue;
        float key = INFINITY;
        if (i < nsb) {
            const double RQ = qrn[2 * g], NQ = qrn[2 * g + 1], RS = srn[2 * i], NS = srn[2 * i + 1];
            const double gap = sqrt(d2[u]) * (1.0 - 1e-12) - (RQ + RS) * (1.0 + 1e-12);
            const double lb2 = gap > 0.0 ? gap * gap * (1.0 - 1e-12) : 0.0;
            const double bm = eps_dot * NQ * NS + 4e-13 * (NQ * NQ + NS * NS) + 1e-30;
            key = f32_down(lb2 - 2.0 * bm * (1.0 + 1e-12));
        }
        keys[g * nsbp + i] = key;
    }
}

template <int DP, int KC>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(K1S_WPE, K1S_WPE))) void knn_mfma_screen_kernel(
    const __bf16 *__restrict__ Xh, const __bf16 *__restrict__ Xl, const double *__restrict__ nrm2,
    const double *__restrict__ nrm, const float *__restrict__ cst, int64_t n, int64_t n_pad, int excl,
    LogEnt *__restrict__ logs, int *__restrict__ log_cnt, float *__restrict__ thr_out, int *__restrict__ overflow,
    SbArgs sb) {
    using C = ScreenCfg<DP>;
    constexpr int QT = C::QT, SQ = C::SQ, CH = C::CH, BUF = C::BUF, NS = DP / KS;
    // two distinct LDS objects per double buffer: the compiler's waitcnt pass then knows the
    // LDS-DMA into one buffer does not alias reads of the other (no vmcnt(0) before them)
    __shared__ __attribute__((aligned(16))) __bf16 cb0_s[BUF];
    __shared__ __attribute__((aligned(16))) __bf16 cb1_s[BUF];
    __shared__ __attribute__((aligned(16))) float cst0_s[S_CST];
    __shared__ __attribute__((aligned(16))) float cst1_s[S_CST];
    auto cbuf = [&](auto B) -> __bf16 * {
        if constexpr (decltype(B)::value == 0) return cb0_s;
        else return cb1_s;
    };
    auto cstb = [&](auto B) -> float * {
        if constexpr (decltype(B)::value == 0) return cst0_s;
        else return cst1_s;
    };
    constexpr bool REG = HDB_K1S_REGTOP && KC <= 15;  // register lists (see HDB_K1S_REGTOP)
    static_assert(!REG || QT == 1, "register top lists hold one query per lane");
    constexpr int LH = S_LOGCAP / 2;  // REG: entries per half-query log
    constexpr int KR = REG ? KC : 1, KT = KR - 1;  // register list length, its last slot
    __shared__ float top_s[REG ? 1 : SQ * KC];
    __shared__ int cnt_s[REG ? 1 : SQ];
    __shared__ double qn2_s[SQ], qn_s[SQ];

    __shared__ float sk_s[NSB_MAX];           // superblock keys (lower bound - 2 max bound), ascending
    __shared__ unsigned short si_s[NSB_MAX];  // superblock ids in key order, then their block counts
    __shared__ int sbs_s[NSB_MAX];            // first block of the i-th superblock in key order
    __shared__ float tmax_s[2][NW];           // per-wave max thr, written in alternate iterations
    // REG hit path: a hitting lane's 16 screen values, read back by (dynamic) row index -- an
    // LDS load in place of a 16-way register select chain per hit
    __shared__ __attribute__((aligned(16))) float hacc_s[REG ? NW * 64 * 16 : 1];

    // the wave index as a scalar: the LDS-DMA destinations (M0) and buffer resources derived
    // from it stay in SGPRs (no waterfall loop, no VGPRs spent on uniform addresses)
    const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63,
              half = lane >> 5, col = lane & 31;
#if HDB_K1S_PROF
    const uint64_t p_t0 = __builtin_readcyclecounter();
    uint64_t p_wait = 0, p_mfma = 0, p_hit = 0, p_hitsteps = 0, p_hits = 0, p_setup = 0;
#endif
#if K1S_XCD
    // query groups of one k-means cluster are consecutive and visit the same candidate
    // superblocks: give each XCD (workgroups are dealt round-robin over the 8) a contiguous
    // range of groups, so those candidates are fetched into one L2 instead of eight
    const int64_t gid = xcd_contig(blockIdx.x, gridDim.x);
#else
    const int64_t gid = blockIdx.x;
#endif
    const int64_t qbase = gid * SQ;
    {
        // a group of padding rows only (uniform: every thread reads the same rows)
        bool any = false;
        for (int i = 0; i < SQ && !any; i += 32) any = sb.perm[qbase + i] >= 0;
        if (!any) {
            for (int i = tid; i < (REG ? 2 : 1) * SQ; i += 64 * NW) log_cnt[(REG ? 2 : 1) * qbase + i] = 0;
            return;
        }
    }
    const double eps_dot = 2.0 * (3.1 * 0x1p-16 + 3.0 * DP * 0x1p-24) * 1.01;
    const float epsf = (float)eps_dot * 1.001f;
    const bool ex = excl != 0;

    if constexpr (!REG)
        for (int i = tid; i < SQ * KC; i += 64 * NW) top_s[i] = INFINITY;
    for (int i = tid; i < SQ; i += 64 * NW) {
        if constexpr (!REG) cnt_s[i] = 0;
        qn2_s[i] = nrm2[qbase + i];
        qn_s[i] = nrm[qbase + i];
    }
    // superblock visiting order: ascending lower bound of (FP64 ball gap)^2 minus twice the
    // largest screen bound; a superblock whose key exceeds every query's thr holds no
    // candidate any query could log (lb >= exact - 2 bound >= gap^2 - 2 bound > thr)
    int nsbp = 1;
    while (nsbp < sb.nsb) nsbp <<= 1;
    if (sb.prune) {
        // keys precomputed by sb_keys_kernel: one coalesced row
        for (int i = tid; i < nsbp; i += 64 * NW) {
            sk_s[i] = sb.keys[gid * nsbp + i];
            si_s[i] = (unsigned short)i;
        }
        __syncthreads();
        for (int k = 2; k <= nsbp; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = tid; i < nsbp; i += 64 * NW) {
                    const int ij = i ^ j;
                    if (ij > i) {
                        const bool up = (i & k) == 0;
                        const float x = sk_s[i], y = sk_s[ij];
                        if ((x > y) == up) {
                            sk_s[i] = y;
                            sk_s[ij] = x;
                            const unsigned short t = si_s[i];
                            si_s[i] = si_s[ij];
                            si_s[ij] = t;
                        }
                    }
                }
                __syncthreads();
            }
    } else {
        for (int i = tid; i < nsbp; i += 64 * NW) {
            sk_s[i] = -INFINITY;
            si_s[i] = (unsigned short)i;
        }
    }
    if (tid < 2 * NW) tmax_s[tid / NW][tid % NW] = INFINITY;

    bf16x8 bh[QT][NS], bl[QT][NS];
    float g[QT], qh[QT], a[QT];
    // query t of this lane: row qbase + qloc(t) (recomputed: fewer live registers)
    auto qloc_of = [&](int t) { return wave * 32 * QT + 32 * t + col; };
    unsigned qvm = 0;  // bit t: a real row (not padding)
    // REG: this lane's (query, half) running list of upper bounds (ascending), its half-log
    // length (LH + 1: overflowed) and the query's threshold (KC-th bound of both halves' lists)
    float tl[KR];
#pragma unroll
    for (int k = 0; k < KR; k++) tl[k] = INFINITY;
    int lcnt = 0;
    float thq = INFINITY;
    // KC-th smallest of the union of this lane's list and its partner half's (lane ^ 32):
    // min over i of max(A_(i), B_(KC-i)) with A_(0) = B_(0) = -inf
    auto union_kth = [&]() __attribute__((always_inline)) {
        float pv[KR];
#pragma unroll
        for (int k = 0; k < KR; k++) pv[k] = xor32_f(tl[k], lane);
        float th = fminf(pv[KT], tl[KT]);
#pragma unroll
        for (int i = 1; i < KR; i++) th = fminf(th, fmaxf(tl[i - 1], pv[KT - i]));
        return th;
    };
#pragma unroll
    for (int t = 0; t < QT; t++) {
        const int64_t row = qbase + qloc_of(t);
        if (sb.perm[row] >= 0) qvm |= 1u << t;
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int64_t o = row * DP + KS * s + 8 * half;
            bh[t][s] = *(const bf16x8 *)(Xh + o);
            bl[t][s] = *(const bf16x8 *)(Xl + o);
        }
        g[t] = epsf * (float)nrm[row] * 0.5f;
        qh[t] = (float)(nrm2[row] * (1.0 - 4e-6) * 0.5);
        a[t] = -INFINITY;
    }

    // global -> LDS staging of one 32-candidate block (all of it is LDS-DMA: nothing else is
    // in flight on the vector-memory counter when the barrier drains it).  CH wave-
    // instructions per block (CH/2 per array), CH/NW per wave; each lane's source offset inside
    // the block is fixed (swizzle on the source address, the LDS image stays lane-linear).
    constexpr int GW = (CH + NW - 1) / NW;  // wave-instructions per wave per block
    // buffer loads with a per-block SGPR resource and a 32-bit lane offset (no 64-bit
    // per-lane address registers)
    auto stage = [&](__bf16 *base, float *cdst, int64_t cb) __attribute__((always_inline)) {
        int lr = lane;
        asm volatile("" : "+v"(lr));  // recomputed, not held live across the loop
        const __amdgpu_buffer_rsrc_t rh =
            __builtin_amdgcn_make_buffer_rsrc((void *)(Xh + cb * DP), (short)0, 32 * DP * 2, 0x00020000);
        const __amdgpu_buffer_rsrc_t rl =
            __builtin_amdgcn_make_buffer_rsrc((void *)(Xl + cb * DP), (short)0, 32 * DP * 2, 0x00020000);
#pragma unroll
        for (int k = 0; k < GW; k++) {
            const int i = wave + NW * k;
            if (CH % NW != 0 && i >= CH) break;  // wave-uniform
            const int arr = i >= CH / 2, ii = arr ? i - CH / 2 : i;
            const int p = ii * 64 + lr, row = p / CH, pc = p % CH, lc = pc ^ (row & (CH - 1));
            const int boff = (row * DP + lc * 8) * 2;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(arr ? rl : rh, (lds_ptr_t)(base + arr * 32 * DP + ii * 512), 16,
                                                     boff, 0, 0, 0);
        }
        if (wave == 0 && lane < S_CST / 4) {
            const __amdgpu_buffer_rsrc_t rc =
                __builtin_amdgcn_make_buffer_rsrc((void *)(cst + (cb >> 5) * S_CST), (short)0, S_CST * 4, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rc, (lds_ptr_t)cdst, 16, lr * 16, 0, 0, 0);
        }
    };

    // the block sequence: superblocks in key order while key <= max thr of the group (read
    // one iteration late from alternating slots, so every wave takes the same decision)
    auto sb_blocks = [&](int i) -> int {
        return si_s[i];
    };
    float wmax = INFINITY;  // this wave's max thr over its real queries (uniform)
    int par = 0;
    int ci_sb = 0, ci_b = 0;  // current superblock (key order) and block within it; -1: done
    int64_t nproc = 0;
    // One block step.  The current and the next buffers come in as __restrict__ parameters:
    // inlining them gives the LDS-DMA stores into `nxt` and the ds_reads of `cur` disjoint
    // alias scopes, which is what lets the compiler's waitcnt pass issue the MFMA operand reads
    // without first draining the next block's DMA (two distinct LDS objects alone do not).
    auto body = [&](const __bf16 *__restrict__ cur, __bf16 *__restrict__ nxt, const float *__restrict__ cstc,
                    float *__restrict__ cstn) __attribute__((always_inline)) {
        const int64_t cb = ((int64_t)sbs_s[ci_sb] + ci_b) * 32;
#if HDB_K1S_PROF
        const uint64_t p_a = __builtin_readcyclecounter();
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // block landed everywhere; the other buffer is free
#if HDB_K1S_PROF
        const uint64_t p_b = __builtin_readcyclecounter();
        p_wait += p_b - p_a;
#endif
        float thrmax = tmax_s[par ^ 1][0];
#pragma unroll
        for (int w = 1; w < NW; w++) thrmax = fmaxf(thrmax, tmax_s[par ^ 1][w]);
        int nx_sb = ci_sb, nx_b = ci_b + 1;
        if (nx_b >= sb_blocks(ci_sb)) {
            nx_sb = ci_sb + 1;
            nx_b = 0;
            if (!(nx_sb < sb.nsb && sk_s[nx_sb] <= thrmax)) nx_sb = -1;
        }
        if (nx_sb >= 0) stage(nxt, cstn, ((int64_t)sbs_s[nx_sb] + nx_b) * 32);
        const float *const cst_s = cstc;
        nproc++;

        const __bf16 *hb = cur, *lb = hb + 32 * DP;
        // per-step LDS offsets recomputed each block (an opaque copy of the lane id keeps the
        // compiler from hoisting eight live address registers out of the loop: VGPR pressure)
        int colr = col;
        asm volatile("" : "+v"(colr));
        f32x16 acc[QT];
#pragma unroll
        for (int t = 0; t < QT; t++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[t][r] = 0.f;
#pragma unroll
        for (int s = 0; s < NS; s++) {
            const int pc = (2 * s + half) ^ (colr & (CH - 1));
            const bf16x8 ah = *(const bf16x8 *)(hb + colr * DP + pc * 8);
            const bf16x8 al = *(const bf16x8 *)(lb + colr * DP + pc * 8);
#pragma unroll
            for (int t = 0; t < QT; t++) {
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[t][s], acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[t][s], acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[t][s], acc[t], 0, 0, 0);
            }
        }
        // screen: C row (candidate) = 8 gi + 4 half + u, column (query) = col
        const float4 *hc4 = (const float4 *)cst_s, *cn4 = (const float4 *)(cst_s + 32);
        float m[QT];
#pragma unroll
        for (int t = 0; t < QT; t++) m[t] = -INFINITY;
#pragma unroll
        for (int gi = 0; gi < 4; gi++) {
            const float4 h4 = hc4[2 * gi + half], c4 = cn4[2 * gi + half];
#pragma unroll
            for (int t = 0; t < QT; t++) {
                m[t] = fmaxf(m[t], fmaf(g[t], c4.x, acc[t][4 * gi + 0]) - h4.x);
                m[t] = fmaxf(m[t], fmaf(g[t], c4.y, acc[t][4 * gi + 1]) - h4.y);
                m[t] = fmaxf(m[t], fmaf(g[t], c4.z, acc[t][4 * gi + 2]) - h4.z);
                m[t] = fmaxf(m[t], fmaf(g[t], c4.w, acc[t][4 * gi + 3]) - h4.w);
            }
        }
        bool hit = false;
#pragma unroll
        for (int t = 0; t < QT; t++) hit |= m[t] >= a[t];
#if HDB_K1S_PROF
        const uint64_t p_c = __builtin_readcyclecounter();
        p_mfma += p_c - p_b;
#endif
        if (REG && __ballot(hit)) {
#if HDB_K1S_PROF
            p_hitsteps++;
#endif
            // both half-waves at once: each lane owns its (query, half) list and half-log
            const double *c2d = (const double *)(cst_s + 64), *cnd = (const double *)(cst_s + 128);
            unsigned mk = 0u;
            if (m[0] >= a[0] && (qvm & 1u)) {
#pragma unroll
                for (int gi = 0; gi < 4; gi++) {
                    const float4 h4 = hc4[2 * gi + half], c4 = cn4[2 * gi + half];
                    mk |= (fmaf(g[0], c4.x, acc[0][4 * gi + 0]) - h4.x >= a[0]) ? 1u << (4 * gi + 0) : 0u;
                    mk |= (fmaf(g[0], c4.y, acc[0][4 * gi + 1]) - h4.y >= a[0]) ? 1u << (4 * gi + 1) : 0u;
                    mk |= (fmaf(g[0], c4.z, acc[0][4 * gi + 2]) - h4.z >= a[0]) ? 1u << (4 * gi + 2) : 0u;
                    mk |= (fmaf(g[0], c4.w, acc[0][4 * gi + 3]) - h4.w >= a[0]) ? 1u << (4 * gi + 3) : 0u;
                }
            }
            if (mk) {
                int cq = col;
                asm volatile("" : "+v"(cq));  // recomputed here: no loop-long address registers
                const int ql = wave * 32 + cq;  // qloc_of(0) (QT = 1)
                const int64_t qid = qbase + ql;
                const double q2 = qn2_s[ql], qn = qn_s[ql];
                int hh = half;
                asm volatile("" : "+v"(hh));  // as cq: the half-log base is not hoisted (a 64-bit spill)
                LogEnt *const L = logs + (qid * S_LOGCAP + hh * LH);
                float *const hv = hacc_s + (wave * 64 + lane) * 16;
#pragma unroll
                for (int u = 0; u < 16; u += 4)
                    *(float4 *)(hv + u) = make_float4(acc[0][u], acc[0][u + 1], acc[0][u + 2], acc[0][u + 3]);
                for (; mk; mk &= mk - 1) {
                    const int r = __builtin_ctz(mk);
                    const int ci = 8 * (r >> 2) + 4 * half + (r & 3);
#if HDB_K1S_PROF
                    p_hits++;
#endif
                    const float av = hv[r];  // dynamic element (LDS: no 16-way register select chain)
                    const int64_t cid = cb + ci;
                    if (ex && cid == qid) continue;  // self (a padding row fails the lb test: c2 = NaN)
                    const double c2 = c2d[ci], cn = cnd[ci];
                    const double approx = (q2 + c2) - 2.0 * (double)av;
                    const double bound = eps_dot * qn * cn + 4e-13 * (q2 + c2) + 1e-30;
                    const double lbv = approx - bound;
                    const float thr = fminf(tl[KT], thq);
                    if (!(lbv <= (double)thr)) continue;
                    if (lcnt == LH) {
                        lcnt = log_compact(L, thr, LH);
                        if (lcnt == LH) {
                            atomicAdd(overflow, 1);
                            lcnt = LH + 1;  // this query's lists are not trusted
                        }
                    }
                    if (lcnt < LH) {
                        LogEnt e;
                        e.cid = (int)cid;
                        e.lb = f32_down(lbv);
                        L[lcnt++] = e;
                    }
                    const float ub = f32_up(approx + bound);
                    if (ub < tl[KT]) {  // insertion network (ascending): shift above the slot, ub into it
                        bool lt[KR];
#pragma unroll
                        for (int k = 0; k < KR; k++) lt[k] = ub < tl[k];
#pragma unroll
                        for (int k = KT; k > 0; k--) tl[k] = lt[k - 1] ? tl[k - 1] : (lt[k] ? ub : tl[k]);
                        tl[0] = lt[0] ? ub : tl[0];
                    }
                }
            }
            thq = union_kth();
            const float th = thq;
            a[0] = qh[0] - 0.5f * th;
            const float wm = wave_max_f((qvm & 1u) ? th : -INFINITY);
            wmax = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wm)));  // uniform
#if HDB_K1S_PROF
            p_hit += __builtin_readcyclecounter() - p_c;
#endif
        } else if (!REG && __ballot(hit)) {
#if HDB_K1S_PROF
            p_hitsteps++;
#endif
            // rare: the two half-waves hold the same queries, so they take turns; each lane
            // walks only the set bits of its pass mask
            const double *c2d = (const double *)(cst_s + 64), *cnd = (const double *)(cst_s + 128);
            unsigned hm[QT];
#pragma unroll
            for (int t = 0; t < QT; t++) {
                hm[t] = 0u;
                if (m[t] >= a[t] && ((qvm >> t) & 1u)) {
#pragma unroll
                    for (int gi = 0; gi < 4; gi++) {
                        const float4 h4 = hc4[2 * gi + half], c4 = cn4[2 * gi + half];
                        hm[t] |= (fmaf(g[t], c4.x, acc[t][4 * gi + 0]) - h4.x >= a[t]) ? 1u << (4 * gi + 0) : 0u;
                        hm[t] |= (fmaf(g[t], c4.y, acc[t][4 * gi + 1]) - h4.y >= a[t]) ? 1u << (4 * gi + 1) : 0u;
                        hm[t] |= (fmaf(g[t], c4.z, acc[t][4 * gi + 2]) - h4.z >= a[t]) ? 1u << (4 * gi + 2) : 0u;
                        hm[t] |= (fmaf(g[t], c4.w, acc[t][4 * gi + 3]) - h4.w >= a[t]) ? 1u << (4 * gi + 3) : 0u;
                    }
                }
            }
            for (int h = 0; h < 2; h++) {
                if (half == h) {
#pragma unroll
                    for (int t = 0; t < QT; t++) {
                        const int ql = qloc_of(t);
                        const int64_t qid = qbase + ql;
                        const double q2 = qn2_s[ql], qn = qn_s[ql];
                        float *tp = top_s + ql * KC;
                        for (unsigned mk = hm[t]; mk; mk &= mk - 1) {
                            const int r = __builtin_ctz(mk);
                            const int ci = 8 * (r >> 2) + 4 * half + (r & 3);
#if HDB_K1S_PROF
                            p_hits++;
#endif
                            const float av = acc[t][r];  // dynamic element (rare path)
                            const int64_t cid = cb + ci;
                            if (ex && cid == qid) continue;  // self (a padding row fails the lb test: c2 = NaN)
                            const double c2 = c2d[ci], cn = cnd[ci];
                            const double approx = (q2 + c2) - 2.0 * (double)av;
                            const double bound = eps_dot * qn * cn + 4e-13 * (q2 + c2) + 1e-30;
                            const double lbv = approx - bound;
                            const float thr = tp[KC - 1];
                            if (!(lbv <= (double)thr)) continue;
                            int k = cnt_s[ql];
                            if (k == S_LOGCAP) {
                                k = log_compact(logs + qid * S_LOGCAP, thr);
                                if (k == S_LOGCAP) {
                                    atomicAdd(overflow, 1);
                                    k = S_LOGCAP + 1;  // this query's lists are not trusted
                                }
                                cnt_s[ql] = k;
                            }
                            if (k < S_LOGCAP) {
                                LogEnt e;
                                e.cid = (int)cid;
                                e.lb = f32_down(lbv);
                                logs[qid * S_LOGCAP + k] = e;
                                cnt_s[ql] = k + 1;
                            }
                            const float ub = f32_up(approx + bound);
                            if (ub < thr) {
                                int i = KC - 1;
                                for (; i > 0 && tp[i - 1] > ub; i--) tp[i] = tp[i - 1];
                                tp[i] = ub;
                            }
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            float wm = -INFINITY;
#pragma unroll
            for (int t = 0; t < QT; t++) {
                const float th = top_s[qloc_of(t) * KC + KC - 1];
                a[t] = qh[t] - 0.5f * th;
                if ((qvm >> t) & 1u) wm = fmaxf(wm, th);
            }
            for (int o = 32; o >= 1; o >>= 1) wm = fmaxf(wm, __shfl_xor(wm, o));
            wmax = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wm)));  // uniform
#if HDB_K1S_PROF
            p_hit += __builtin_readcyclecounter() - p_c;
#endif
        }
        if (lane == 0) tmax_s[par][wave] = wmax;
        par ^= 1;
        ci_sb = nx_sb;
        ci_b = nx_b;
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    __syncthreads();
    // the key order's block ranges in LDS (no dependent global loads in the block loop)
    for (int i = tid; i < sb.nsb; i += 64 * NW) {
        const int id = si_s[i];
        sbs_s[i] = sb.sb_blk[id];
        si_s[i] = (unsigned short)sb.sb_nblk[id];
    }
    __syncthreads();
#if HDB_K1S_PROF
    p_setup = __builtin_readcyclecounter() - p_t0;
#endif
    auto step = [&](auto B, auto Bn) { body(cbuf(B), cbuf(Bn), cstb(B), cstb(Bn)); };
    stage(cbuf(B0{}), cstb(B0{}), (int64_t)sbs_s[0] * 32);
    while (true) {
        step(B0{}, B1{});
        if (ci_sb < 0) break;
        step(B1{}, B0{});
        if (ci_sb < 0) break;
    }
    if (sb.blocks_done && tid == 0) atomicAdd(sb.blocks_done, (unsigned long long)nproc);
#if HDB_K1S_PROF
    if (sb.blocks_done) {
        if (lane == 0) {
            atomicAdd(sb.blocks_done + 1, (unsigned long long)p_wait);
            atomicAdd(sb.blocks_done + 2, (unsigned long long)p_mfma);
            atomicAdd(sb.blocks_done + 3, (unsigned long long)p_hit);
            atomicAdd(sb.blocks_done + 4, (unsigned long long)p_hitsteps);
            atomicAdd(sb.blocks_done + 5, (unsigned long long)p_setup);
            atomicAdd(sb.blocks_done + 6, (unsigned long long)nproc);
        }
        atomicAdd(sb.blocks_done + 7, (unsigned long long)p_hits);
    }
#endif
    __syncthreads();
    if constexpr (REG) {
        const int64_t qid = qbase + qloc_of(0);
        const float th = union_kth();
        if (qvm & 1u) {
            log_cnt[2 * qid + half] = lcnt > LH ? -1 : lcnt;
            if (half == 0) thr_out[qid] = th;
        } else {
            log_cnt[2 * qid + half] = 0;
        }
    } else {
        for (int i = tid; i < SQ; i += 64 * NW) {
            const int64_t qid = qbase + i;
            if (sb.perm[qid] < 0) {
                log_cnt[qid] = 0;
            } else {
                log_cnt[qid] = cnt_s[i] > S_LOGCAP ? -1 : cnt_s[i];
                thr_out[qid] = top_s[i * KC + KC - 1];
            }
        }
    }
}

#ifndef HDB_K1F_LAYOUT
#define HDB_K1F_LAYOUT 1  // K1m re-check reads an FP64 copy of the rows in layout order (written by split_rows_kernel)
#endif
#ifndef HDB_K1F_WPE
#define HDB_K1F_WPE 1  // K1m re-check: waves per SIMD the kernel is compiled for (1: no cap)
#endif
#ifndef HDB_K1F_DIST
#define HDB_K1F_DIST 1  // K1m re-check: the group's running top-KC distributed over its 16 lanes
#endif
#ifndef HDB_K1F_LAY_UNROLL
#define HDB_K1F_LAY_UNROLL 1
#endif
#ifndef HDB_K1F_U
#define HDB_K1F_U 16  // doubles per prefetched chunk (r04 C4 A/B, layout rows: 8.87 ms at 8, 8.15 at 16; caller-order rows: 15.2 at 8, 15.6 at 16, 17.1 at 32)
#endif
// exact squared distance in the reference's order with the query row in LDS and the candidate
// row (caller order, runtime length d) streamed in U-double chunks, the next chunk in flight
// while the current one is summed
__device__ __forceinline__ double exact_sq_pf(const double *a_lds, const double *__restrict__ b, int d) {
    constexpr int U = HDB_K1F_U;  // doubles per prefetched chunk
    double nb[U];
#pragma unroll
    for (int u = 0; u < U; u++) nb[u] = b[u < d ? u : d - 1];
    double sx = 0.0;
    for (int j0 = 0; j0 < d; j0 += U) {
        double cb[U];
#pragma unroll
        for (int u = 0; u < U; u++) cb[u] = nb[u];
        if (j0 + U < d) {
#pragma unroll
            for (int u = 0; u < U; u++) nb[u] = b[j0 + U + u < d ? j0 + U + u : d - 1];
        }
#pragma unroll
        for (int u = 0; u < U; u++)
            if (j0 + u < d) sx = sx + sq_diff(a_lds[j0 + u], cb[u]);
    }
    return sx;
}

// the same sum over a layout row zero padded to DP (compile time: no guards, no clamped
// addresses): the padded terms are (0 - 0)^2 = +0, and s + 0 == s, so the value is bit-equal
template <int DP>
__device__ __forceinline__ double exact_sq_lay(const double *a_lds, const double *__restrict__ b) {
    constexpr int U = HDB_K1F_U;
    static_assert(DP % U == 0, "chunk must divide the padded row");
    double nb[U];
#pragma unroll
    for (int u = 0; u < U; u++) nb[u] = b[u];
    double sx = 0.0;
#pragma unroll HDB_K1F_LAY_UNROLL
    for (int j0 = 0; j0 < DP; j0 += U) {
        double cb[U];
#pragma unroll
        for (int u = 0; u < U; u++) cb[u] = nb[u];
        if (j0 + U < DP) {
#pragma unroll
            for (int u = 0; u < U; u++) nb[u] = b[j0 + U + u];
        }
#pragma unroll
        for (int u = 0; u < U; u++) sx = sx + sq_diff(a_lds[j0 + u], cb[u]);
    }
    return sx;
}

// The exact FP64 re-check, 16 lanes per query, four queries per wave: a query keeps ~KC
// survivors, so a wave per query (round 3's kernel, 17.4 ms at C4) left most lanes idle while its
// few lanes streamed 1 KB rows.  Per 16-lane group: the surviving log entries (lb <= thr) are
// compacted into LDS 256 at a time, every lane computes the exact FP64 distances of its
// survivors in the reference's order (one lane per candidate: the sequential sum is the
// bit-exact one), and the KC smallest come out of 16-lane min/ballot selections.  LAY: the rows
// are read from the zero-padded layout copy with the compile-time length DP (16-byte loads, no
// clamps: half the L1 accesses of the caller-order path; 15.6 -> 7.3 ms at C4 with DIST).
// Query rows in dynamic LDS (16 x DP, or 16 x d).
constexpr int K1F_CH = 256;  // compacted survivors per group and pass
template <int KC, int DP, bool LAY>
__global__ __launch_bounds__(256, HDB_K1F_WPE) void knn_mfma_final16_kernel(const double *__restrict__ X, int64_t n, int d,
                                                               const LogEnt *__restrict__ logs,
                                                               const int *__restrict__ log_cnt,
                                                               const float *__restrict__ thr,
                                                               const int *__restrict__ perm,
                                                               double *__restrict__ lists,
                                                               const double *__restrict__ Xlay) {
    constexpr bool REG = HDB_K1S_REGTOP && KC <= 15;
    constexpr int NH = REG ? 2 : 1, LH = S_LOGCAP / NH;
    extern __shared__ __attribute__((aligned(16))) double k1f_dyn[];
    __shared__ int cl_s[16][K1F_CH];
    const int lane = threadIdx.x & 63, sub = lane >> 4, sl = lane & 15;
    const int g = (threadIdx.x >> 6) * 4 + sub;  // query slot in the workgroup
    // consecutive workgroups (one k-means cluster) share candidate rows: with XCD-contiguous
    // ranges those rows are fetched into one L2 instead of eight
    const int64_t q = (HDB_K1F_XCD ? xcd_contig(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x) * 16 + g;
    const bool act = q < n && perm[q] >= 0;  // n: layout rows here (uniform per 16 lanes)
    const int rs = LAY ? DP : d;  // query row length in LDS
    double *qr = k1f_dyn + (size_t)g * rs;
    const int64_t qo = act ? perm[q] : 0;  // the query's row in X (the lists follow X's order)
    // Xlay: the rows in layout order, so a workgroup's 16 consecutive queries (one k-means
    // cluster) and their candidates (the same cluster, mostly) share lines in L2 and pages in
    // the TLB; X: the caller's order, rows gathered through perm
    const double *qsrc = LAY ? Xlay + q * DP : X + qo * d;
    if (act)
        for (int c = sl; c < rs; c += 16) qr[c] = qsrc[c];
    const float t = act ? thr[q] : 0.f;
    // DIST: the group's running KC smallest live one per lane (lane sl: the sl-th), merged with
    // each batch of <= 64 exact values by KC rounds of a 16-lane minimum; otherwise every lane
    // keeps its own sorted top-KC (30 VGPRs at KC = 15) and the lanes are merged at the end
    constexpr bool DIST = HDB_K1F_DIST && KC <= 16;
    double lv = INFINITY;
    double top[KC];
#pragma unroll
    for (int k = 0; k < KC; k++) top[k] = INFINITY;
    const unsigned long long below = (1ull << lane) - 1;
    int *cl = cl_s[g];
    for (int h = 0; h < NH; h++) {
        const int cnt = act ? log_cnt[NH * q + h] : 0;
        const LogEnt *L = logs + q * S_LOGCAP + h * LH;
        for (int j0 = 0; j0 < LH; j0 += K1F_CH) {
            // compaction of entries [j0, j0 + K1F_CH) of this half-log
            int np = 0;
            for (int j1 = j0; j1 < j0 + K1F_CH; j1 += 64) {
                LogEnt e[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {  // four loads in flight per lane
                    const int j = j1 + 16 * u + sl;
                    ok[u] = j < cnt;
                    if (ok[u]) e[u] = L[j];
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const bool sv = ok[u] && e[u].lb <= t;
                    const unsigned long long m = __ballot(sv);
                    const unsigned long long mg = (m >> (16 * sub)) & 0xFFFFull;
                    if (sv) cl[np + __popcll(m & below & (0xFFFFull << (16 * sub)))] = e[u].cid;
                    np += __popcll(mg);
                }
                if (!__ballot(j1 + 64 < cnt)) break;  // wave-uniform: the rest of the pass is empty
            }
            __builtin_amdgcn_wave_barrier();
            if constexpr (DIST) {
                int npm = max(np, __shfl_xor(np, 16));
                npm = max(npm, __shfl_xor(npm, 32));  // wave-uniform batch count
                for (int jb = 0; jb < npm; jb += 64) {
                    double v[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int j = jb + 16 * i + sl;
                        v[i] = INFINITY;
                        if (j < np)
                            v[i] = LAY ? exact_sq_lay<DP>(qr, Xlay + (int64_t)cl[j] * DP)
                                        : exact_sq_pf(qr, X + (int64_t)perm[cl[j]] * d, d);
                    }
                    double nl = INFINITY;
#pragma unroll 1
                    for (int k = 0; k < KC; k++) {
                        const double m = fmin(fmin(lv, fmin(v[0], v[1])), fmin(v[2], v[3]));
                        const double mn = row_min_d(m);
                        const unsigned long long b = (__ballot(m == mn) >> (16 * sub)) & 0xFFFFull;
                        if (sl == __ffsll((long long)b) - 1) {  // the first lane holding it gives it up
                            if (lv == mn) lv = INFINITY;
                            else if (v[0] == mn) v[0] = INFINITY;
                            else if (v[1] == mn) v[1] = INFINITY;
                            else if (v[2] == mn) v[2] = INFINITY;
                            else v[3] = INFINITY;
                        }
                        if (sl == k) nl = mn;
                    }
                    lv = nl;
                }
            } else if constexpr (LAY) {
                for (int j = sl; j < np; j += 16) topk_insert<KC>(top, exact_sq_lay<DP>(qr, Xlay + (int64_t)cl[j] * DP));
            } else {
                for (int j = sl; j < np; j += 16) topk_insert<KC>(top, exact_sq_pf(qr, X + (int64_t)perm[cl[j]] * d, d));
            }
            __builtin_amdgcn_wave_barrier();
            if (!__ballot(j0 + K1F_CH < cnt)) break;  // wave-uniform: no group has more entries
        }
    }
    if constexpr (DIST) {
        if (act && sl < KC) lists[qo * KC + sl] = (lv < INFINITY) ? sqrt(lv) : JMAX;
        return;
    }
    // the KC smallest over the 16 lanes of the group
    for (int k = 0; k < KC; k++) {
        double mn = top[0];
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o));
        const unsigned long long b = (__ballot(top[0] == mn) >> (16 * sub)) & 0xFFFFull;
        if (sl == __ffsll((long long)b) - 1) {
#pragma unroll
            for (int i = 0; i + 1 < KC; i++) top[i] = top[i + 1];
            top[KC - 1] = INFINITY;
        }
        if (act && sl == 0) lists[qo * KC + k] = (mn < INFINITY) ? sqrt(mn) : JMAX;
    }
}

template <int KC, int DP>
static void launch_recheck(hipStream_t st, const double *X, int64_t n, int d, const LogEnt *logs, const int *log_cnt,
                           const float *thr, const int *perm, double *lists, const double *Xlay) {
    // (a 16-lane systolic variant -- lane j adds dimension block j to lane j-1's partial sum of
    // the previous step, the reference's order -- was built and measured in round 4: 27.5 ms at
    // C4 against this kernel's 15.5 ms; its staggered 64-byte segment reads touch 64 cache lines
    // per instruction with little reuse, where a lane streaming its own row reuses each line
    // over eight loads)
    if (Xlay)
        hipLaunchKernelGGL((knn_mfma_final16_kernel<KC, DP, true>), dim3((unsigned)ceil_div(n, 16)), dim3(256),
                           (unsigned)(16 * 8 * DP), st, X, n, d, logs, log_cnt, thr, perm, lists, Xlay);
    else
        hipLaunchKernelGGL((knn_mfma_final16_kernel<KC, DP, false>), dim3((unsigned)ceil_div(n, 16)), dim3(256),
                           (unsigned)(16 * 8 * d), st, X, n, d, logs, log_cnt, thr, perm, lists, Xlay);
}

// ---------------------------------------------------------------- host
template <int DP, int KC>
static void launch_single(hdb_ctx *ctx, const double *X, int64_t n, int64_t n_pad, int d, const __bf16 *Xh,
                          const __bf16 *Xl, const double *nrm2, const double *nrm, const float *cst, int excl,
                          LogEnt *logs, int *log_cnt, float *thr, int *overflow, const int *perm, const SbArgs &sb,
                          double *lists, const double *Xlay) {
    hipStream_t st = ctx->stream;
    using C = ScreenCfg<DP>;
    {
        KernelTimer t(ctx, "knn_mfma");
        hipLaunchKernelGGL((knn_mfma_screen_kernel<DP, KC>), dim3((unsigned)(n_pad / C::SQ)), dim3(64 * NW), 0, st, Xh,
                           Xl, nrm2, nrm, cst, n, n_pad, excl, logs, log_cnt, thr, overflow, sb);
        HIP_CHECK(hipGetLastError());
    }
    {
        KernelTimer t(ctx, "knn_mfma_final");
        launch_recheck<KC, DP>(st, X, n, d, logs, log_cnt, thr, perm, lists, Xlay);
        HIP_CHECK(hipGetLastError());
    }
}

__global__ void order_iota_kernel(int *p, int64_t n, int64_t n_pad) {
    HDB_GRID_STRIDE(i, n_pad) p[i] = i < n ? (int)i : -1;
}

// sorted position p (cluster c = key >> 32, rank p - start[c]) -> layout position off[c] + rank
__global__ void km_scatter_kernel(const unsigned long long *__restrict__ keys, const int *__restrict__ rows, int64_t n,
                                  const int *__restrict__ start, const int *__restrict__ off, int *__restrict__ perm) {
    HDB_GRID_STRIDE(p, n) {
        const int c = (int)(keys[p] >> 32);
        perm[(int64_t)off[c] + (p - start[c])] = rows[p];
    }
}

// number of k-means centroids for n rows (every cluster is padded to a multiple of 256 rows)
static int km_k(int64_t n) { return (int)std::min<int64_t>(KM_K, std::max<int64_t>(1, n / 2048)); }

struct KmBufs {
    unsigned long long *k1, *k2;
    int *vals, *rows, *asg, *hist, *start, *off;
    float *Y, *C, *sum, *cnt;
    void *tmp;
    size_t tmp_bytes;
};

// The candidate layout: rows of each k-means cluster in consecutive positions (ordered by the
// first projected coordinate), every cluster padded to a multiple of 256 rows (perm = -1), so
// no query group and no block mixes clusters.  Superblocks: each cluster's blocks in runs of
// at most sbmax.  Returns the layout's row count (a multiple of 256).
static int64_t km_layout(hdb_ctx *ctx, const __bf16 *Xh, int DP, int d, int64_t n, const KmBufs &b, int *perm,
                         std::vector<int> &sb_blk, std::vector<int> &sb_nblk) {
    hipStream_t st = ctx->stream;
    KernelTimer t(ctx, "knn_mfma_order");
    const int k = km_k(n);
    const int g = (int)std::min<int64_t>(ceil_div(n, 256), 8192);
    hipLaunchKernelGGL(km_project_kernel, dim3(g), dim3(256), 0, st, Xh, DP, d, n, b.Y);
    hipLaunchKernelGGL(km_init_kernel, dim3(k), dim3(KM_P), 0, st, b.Y, n, b.C);
    HIP_CHECK(hipMemsetAsync(b.sum, 0, 4 * (size_t)KM_K * KM_P, st));
    HIP_CHECK(hipMemsetAsync(b.cnt, 0, 4 * (size_t)KM_K, st));
    HIP_CHECK(hipMemsetAsync(b.hist, 0, 4 * (size_t)KM_K, st));
    // Lloyd iterations on a strided sample of <= 128k rows, then every row once
    const int64_t step = std::max<int64_t>(1, n / 131072), m = n / step;
    for (int it = 0; it < KM_IT; it++) {
        hipLaunchKernelGGL(km_assign_mfma_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(m, 32 * KMA_WAVES), 2048)),
                           dim3(64 * KMA_WAVES), 0, st, b.Y, m, step, k, b.C, b.asg, b.sum, b.cnt, (int *)nullptr);
        hipLaunchKernelGGL(km_update_kernel, dim3(k), dim3(KM_P), 0, st, b.C, b.sum, b.cnt);
    }
    hipLaunchKernelGGL(km_assign_mfma_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n, 32 * KMA_WAVES), 2048)),
                       dim3(64 * KMA_WAVES), 0, st, b.Y, n, (int64_t)1, k, b.C, b.asg, (float *)nullptr,
                       (float *)nullptr, b.hist);
    HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(km_keys_kernel, dim3(g), dim3(256), 0, st, b.Y, b.asg, n, b.k1, b.vals);
    size_t tb = b.tmp_bytes;
    HIP_CHECK(sort_pairs(b.tmp, tb, b.k1, b.k2, b.vals, b.rows, n, 0, 48, st));  // KM_K <= 2^16
    std::vector<int> hist(k), start(k), off(k);
    HIP_CHECK(hipMemcpyAsync(hist.data(), b.hist, 4 * (size_t)k, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int64_t s0 = 0, o0 = 0, nbr = 0, nz = 0;
    for (int c = 0; c < k; c++) {
        start[c] = (int)s0;
        off[c] = (int)o0;
        s0 += hist[c];
        o0 += ceil_div((int64_t)hist[c], (int64_t)256) * 256;
        nbr += ceil_div((int64_t)hist[c], (int64_t)32);
        nz += hist[c] > 0;
    }
    const int64_t n_lay = o0;
    const int sbmax = (int)std::max<int64_t>(1, ceil_div(nbr, std::max<int64_t>(1, NSB_MAX - nz)));
    sb_blk.clear();
    sb_nblk.clear();
    for (int c = 0; c < k; c++) {
        const int nb = (int)ceil_div((int64_t)hist[c], (int64_t)32);
        for (int j = 0; j < nb; j += sbmax) {
            sb_blk.push_back(off[c] / 32 + j);
            sb_nblk.push_back(std::min(sbmax, nb - j));
        }
    }
    HIP_CHECK(hipMemcpyAsync(b.start, start.data(), 4 * (size_t)k, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(b.off, off.data(), 4 * (size_t)k, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(perm, 0xff, 4 * (size_t)ceil_div(n_lay, (int64_t)512) * 512, st));
    hipLaunchKernelGGL(km_scatter_kernel, dim3(g), dim3(256), 0, st, b.k2, b.rows, n, b.start, b.off, perm);
    HIP_CHECK(hipStreamSynchronize(st));  // start/off staged from host vectors
    return n_lay;
}

template <int DP>
static bool knn_mfma_dp(hdb_ctx *ctx, const double *X, int64_t n, int d, int KC, bool excl, double *lists) {
    const int64_t n_pad = ceil_div(n, (int64_t)512) * 512;  // multiple of MQ and of every SQ
    const bool single = ctx->knn_mfma_single, prune = single && ctx->knn_mfma_prune;
    // row capacity: the pruned layout pads every k-means cluster to a multiple of 256 rows
    const int64_t n_cap = prune ? ceil_div(n + 256 * (int64_t)km_k(n), (int64_t)512) * 512 : n_pad;
    const int nb = (int)std::min<int64_t>(1024, std::max<int64_t>(1, n / 64));
    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t bytes = 2 * rnd(sizeof(__bf16) * (size_t)(n_cap * DP)) + 3 * rnd(8 * (size_t)n_cap) +
                         2 * rnd(8 * (size_t)nb * d) + rnd(8 * (size_t)d) + 256 + 256 +
                         rnd(4 * (size_t)(n_cap / 32) * S_CST) + 2 * rnd(4 * (size_t)n_cap);
    char *base = (char *)arena(ctx, A_WORK3, bytes);
    size_t off = 0;
    auto take = [&](size_t b) {
        char *p = base + off;
        off += rnd(b);
        return p;
    };
    __bf16 *Xh = (__bf16 *)take(sizeof(__bf16) * (size_t)(n_cap * DP));
    __bf16 *Xl = (__bf16 *)take(sizeof(__bf16) * (size_t)(n_cap * DP));
    double *nrm2 = (double *)take(8 * (size_t)n_cap), *nrm = (double *)take(8 * (size_t)n_cap);
    double *psum = (double *)take(8 * (size_t)nb * d), *pmax = (double *)take(8 * (size_t)nb * d);
    double *mu = (double *)take(8 * (size_t)d);
    double *thr = (double *)take(8 * (size_t)n_cap);
    double *prm = (double *)take(256);
    unsigned long long *stats = (unsigned long long *)take(256);
    float *cst = (float *)take(4 * (size_t)(n_cap / 32) * S_CST);
    int *log_cnt = (int *)take(8 * (size_t)n_cap);  // per query, or per half-query (HDB_K1S_REGTOP)
    float *thr_f = (float *)take(4 * (size_t)n_cap);
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
                           nrm, nullptr);
    }
    if (single) {
        using Cf = ScreenCfg<DP>;
        // layout (A_ORDER): perm, k-means scratch, query-group and superblock balls
        const int64_t n_sortcap = std::max<int64_t>(n, 1);
        size_t sort_tb = 0;
        HIP_CHECK(sort_pairs(nullptr, sort_tb, (const unsigned long long *)nullptr, (unsigned long long *)nullptr,
                             (const int *)nullptr, (int *)nullptr, n_sortcap, 0, 64, st));
        const size_t obytes = rnd(4 * (size_t)n_cap) + 3 * rnd(4 * (size_t)n) + 2 * rnd(8 * (size_t)n) +
                              rnd(sort_tb) + rnd(4 * (size_t)n * KM_P) + 2 * rnd(4 * KM_K * KM_P) +
                              rnd(4 * KM_K) + 3 * rnd(4 * KM_K) + rnd(8 * (size_t)(n_cap / 128) * DP) +
                              rnd(16 * (size_t)(n_cap / 128)) + rnd(8 * (size_t)NSB_MAX * DP) + rnd(16 * NSB_MAX) +
                              2 * rnd(4 * NSB_MAX);
        char *ob = (char *)arena(ctx, A_ORDER, obytes);
        size_t oo = 0;
        auto otake = [&](size_t b) {
            char *p = ob + oo;
            oo += rnd(b);
            return p;
        };
        int *perm = (int *)otake(4 * (size_t)n_cap);
        KmBufs kb;
        kb.vals = (int *)otake(4 * (size_t)n);
        kb.rows = (int *)otake(4 * (size_t)n);
        kb.asg = (int *)otake(4 * (size_t)n);
        kb.k1 = (unsigned long long *)otake(8 * (size_t)n);
        kb.k2 = (unsigned long long *)otake(8 * (size_t)n);
        kb.tmp = otake(sort_tb);
        kb.tmp_bytes = sort_tb;
        kb.Y = (float *)otake(4 * (size_t)n * KM_P);
        kb.C = (float *)otake(4 * KM_K * KM_P);
        kb.sum = (float *)otake(4 * KM_K * KM_P);
        kb.cnt = (float *)otake(4 * KM_K);
        kb.hist = (int *)otake(4 * KM_K);
        kb.start = (int *)otake(4 * KM_K);
        kb.off = (int *)otake(4 * KM_K);
        double *qctr = (double *)otake(8 * (size_t)(n_cap / 128) * DP);
        double *qrn = (double *)otake(16 * (size_t)(n_cap / 128));
        double *sctr = (double *)otake(8 * (size_t)NSB_MAX * DP), *srn = (double *)otake(16 * NSB_MAX);
        int *sb_blk_d = (int *)otake(4 * NSB_MAX), *sb_nblk_d = (int *)otake(4 * NSB_MAX);
        std::vector<int> sb_blk, sb_nblk;
        int64_t n_lay = n;
        if (prune) {
            n_lay = km_layout(ctx, Xh, DP, d, n, kb, perm, sb_blk, sb_nblk);
        } else {
            const int g = (int)std::min<int64_t>(ceil_div(n_pad, 256), 8192);
            hipLaunchKernelGGL(order_iota_kernel, dim3(g), dim3(256), 0, st, perm, n, n_pad);
            const int64_t nbr = ceil_div(n, (int64_t)32);
            const int sbb = (int)ceil_div(nbr, (int64_t)NSB_MAX);
            for (int64_t b0 = 0; b0 < nbr; b0 += sbb) {
                sb_blk.push_back((int)b0);
                sb_nblk.push_back((int)std::min<int64_t>(sbb, nbr - b0));
            }
        }
        const int64_t n_lp = ceil_div(n_lay, (int64_t)512) * 512;  // layout rows incl. padding
        const int nsb = (int)sb_blk.size();
        HIP_CHECK(hipMemcpyAsync(sb_blk_d, sb_blk.data(), 4 * (size_t)nsb, hipMemcpyHostToDevice, st));
        HIP_CHECK(hipMemcpyAsync(sb_nblk_d, sb_nblk.data(), 4 * (size_t)nsb, hipMemcpyHostToDevice, st));
        double *Xlay = nullptr;
        if (prune) {
            // the layout-order FP64 copy (8 n DP bytes, ~2 GB at C4) only speeds the re-check:
            // when the device cannot hold it, the re-check reads the caller-order rows instead
            if (HDB_K1F_LAYOUT) {
                try {
                    Xlay = (double *)arena(ctx, A_XLAY, 8 * (size_t)n_lp * DP);
                } catch (const Error &) {
                    (void)hipGetLastError();  // clear the failed allocation's sticky error
                    Xlay = nullptr;
                }
            }
            const int g = (int)std::min<int64_t>(ceil_div(n_lp * 64, 256), 8192);
            hipLaunchKernelGGL(split_rows_kernel, dim3(g), dim3(256), 0, st, X, n, n_lp, d, DP, mu, prm, Xh, Xl, nrm2,
                               nrm, perm, Xlay);
            hipLaunchKernelGGL(ball_kernel, dim3((unsigned)(n_lp / Cf::SQ)), dim3(256), 0, st, X, d, mu, prm, perm,
                               (const int *)nullptr, (const int *)nullptr, (int64_t)Cf::SQ, DP, qctr, qrn);
            hipLaunchKernelGGL(ball_kernel, dim3((unsigned)nsb), dim3(256), 0, st, X, d, mu, prm, perm, sb_blk_d,
                               sb_nblk_d, (int64_t)0, DP, sctr, srn);
        }
        if (prune && ctx->count_evals) {
            // diagnostic: ball radii (x 1e6, scaled domain) of query groups and superblocks
            const int64_t nqg = n_lp / Cf::SQ;
            std::vector<double> hq(2 * (size_t)nqg), hs(2 * (size_t)nsb);
            HIP_CHECK(hipMemcpyAsync(hq.data(), qrn, 16 * (size_t)nqg, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipMemcpyAsync(hs.data(), srn, 16 * (size_t)nsb, hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            auto med = [](const std::vector<double> &v) {
                std::vector<double> r;
                for (size_t i = 0; i < v.size(); i += 2)
                    if (v[i] > 0) r.push_back(v[i]);
                std::sort(r.begin(), r.end());
                return r.empty() ? 0.0 : r[r.size() / 2];
            };
            ctx->stats["knn_mfma_qrad_med_e6"] = (int64_t)(med(hq) * 1e6);
            ctx->stats["knn_mfma_sbrad_med_e6"] = (int64_t)(med(hs) * 1e6);
            ctx->stats["knn_mfma_nsb"] = nsb;
            ctx->stats["knn_mfma_layout_rows"] = n_lay;
        }
        unsigned long long *blocks_done = stats + 1;
        HIP_CHECK(hipMemsetAsync(blocks_done, 0, HDB_K1S_PROF ? 64 : 8, st));
        float *sb_keys = nullptr;
        if (prune) {
            int nsbp = 1;
            while (nsbp < nsb) nsbp <<= 1;
            const int64_t ngr = n_lp / Cf::SQ;
            sb_keys = (float *)arena(ctx, A_SBKEY, 4 * (size_t)ngr * nsbp);
            const double eps_dot = 2.0 * (3.1 * 0x1p-16 + 3.0 * DP * 0x1p-24) * 1.01;  // the screen's
            hipLaunchKernelGGL(sb_keys_kernel<DP>, dim3((unsigned)ceil_div(nsbp, 64), (unsigned)ceil_div(ngr, (int64_t)16)),
                               dim3(256), 0, st, qctr, qrn, sctr, srn, ngr, nsb, nsbp, eps_dot, sb_keys);
        }
        const SbArgs sbargs{qctr, qrn, sctr, srn, sb_blk_d, sb_nblk_d, perm, nsb, prune ? 1 : 0, blocks_done, sb_keys};
        {
            const int g = (int)std::min<int64_t>(ceil_div(n_lp, 256), 4096);
            hipLaunchKernelGGL(screen_consts_kernel, dim3(g), dim3(256), 0, st, nrm2, nrm, n_lp, perm, cst);
        }
        LogEnt *logs = (LogEnt *)arena(ctx, A_LOG, sizeof(LogEnt) * (size_t)n_lp * S_LOGCAP);
        int *overflow = (int *)stats;
        HIP_CHECK(hipMemsetAsync(overflow, 0, 4, st));
        const int fl = excl ? 1 : 0;
#define K1S_CASE(KK)                                                                                              \
    case KK:                                                                                                      \
        launch_single<DP, KK>(ctx, X, n_lp, n_lp, d, Xh, Xl, nrm2, nrm, cst, fl, logs, log_cnt, thr_f, overflow, \
                              perm, sbargs, lists, Xlay);                                                         \
        break;
        switch (KC) {
            K1S_CASE(1)
            K1S_CASE(3)
            K1S_CASE(7)
            K1S_CASE(15)
            K1S_CASE(31)
        default: return false;
        }
#undef K1S_CASE
        unsigned long long h_st[9] = {};
        HIP_CHECK(hipMemcpyAsync(h_st, stats, HDB_K1S_PROF ? 72 : 16, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        if (HDB_K1S_PROF) {  // summed over waves: cycles waiting, MFMA + screen, hit path; wave-steps
            const char *nm[7] = {"wait", "mfma", "hit", "hitsteps", "setup", "wavesteps", "hits"};
            for (int i = 0; i < 7; i++) ctx->stats[std::string("k1s_prof_") + nm[i]] = (int64_t)h_st[2 + i];
        }
        const int h_ovf = (int)(h_st[0] & 0xffffffffull);
        ctx->stats["knn_mfma_blocks"] = (int64_t)h_st[1];  // (query group, 32-candidate block) pairs computed
        ctx->stats["knn_mfma_group_rows"] = Cf::SQ;
        if (ctx->count_evals) {
            // diagnostic: logged candidates (the FP64 re-checks are those with lb <= thr)
            const int nh = (HDB_K1S_REGTOP && KC <= 15) ? 2 : 1;
            std::vector<int> hc((size_t)n_lp * nh);
            HIP_CHECK(hipMemcpy(hc.data(), log_cnt, 4 * (size_t)n_lp * nh, hipMemcpyDeviceToHost));
            int64_t tot = 0;
            for (int v : hc) tot += v < 0 ? S_LOGCAP / nh : v;
            ctx->stats["knn_mfma_rechecks"] = tot;
            ctx->stats["last_evals"] = tot;
        }
        ctx->stats["knn_mfma_log_overflow"] = h_ovf;
        if (h_ovf == 0) return true;
        // a query's log overflowed (e.g. hundreds of exact duplicates): two-pass kernel for all,
        // on the rows in their own order
        const int g2 = (int)std::min<int64_t>(ceil_div(n_pad * 64, 256), 8192);
        hipLaunchKernelGGL(split_rows_kernel, dim3(g2), dim3(256), 0, st, X, n, n_pad, d, DP, mu, prm, Xh, Xl, nrm2,
                           nrm, nullptr);
    }
    if (ctx->count_evals) HIP_CHECK(hipMemsetAsync(stats, 0, 8, st));
    {
        KernelTimer t(ctx, "knn_mfma");
        const dim3 grid((unsigned)(n_pad / MQ));
        const int fl = (excl ? 1 : 0) | (getenv("HDBMI_K1M_DBG") ? 2 : 0);
#define K1M_CASE(KK)                                                                                             \
    case KK:                                                                                                     \
        hipLaunchKernelGGL((knn_mfma_kernel<DP, KK, 0>), grid, dim3(NT), 0, st, X, n, n_pad, d, Xh, Xl, nrm2,     \
                           nrm, prm, fl, nullptr, thr, lists, nullptr);                                         \
        hipLaunchKernelGGL((knn_mfma_kernel<DP, KK, 1>), grid, dim3(NT), 0, st, X, n, n_pad, d, Xh, Xl, nrm2,     \
                           nrm, prm, fl, thr, nullptr, lists, ctx->count_evals ? stats : nullptr);              \
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
