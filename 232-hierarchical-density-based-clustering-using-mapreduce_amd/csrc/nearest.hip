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

#include <cmath>
#include <numeric>
#include <vector>

#include "common.hpp"
#include "sort.hpp"

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

// ------------------------------------------------------------------ K3g: grouped samples
// Large unkeyed euclidean scans (the recursive-sampling levels of C3/C5: millions of points
// against 4k-16k samples).  The samples are cut on the host into groups of G by recursive
// median splits (widest dimension), each group with its FP64 bounding box; every point
// descends the split tree to a "home" group, and the points are processed in home order so a
// wave's lanes share their candidate groups.  A lane first scans its home group, then the wave
// walks every group's box: a group is scanned (for all lanes) when some lane's box lower bound
// could still reach its best value.  Exact: the box bound uses the reference's own summation
// order on monotonically rounded gaps (every computed sample distance in the box is >= it), a
// group is skipped only when that bound exceeds r^2 (1 + 2^-48) (no sample in it can reach the
// best sqrt value r, ties included), and candidates are kept by (sqrt value, sample index)
// lexicographically -- the reference's first minimum in sample order (FirstStep.java:74-85),
// whatever order the groups are scanned in.
#ifndef HDB_NNG_SB
#define HDB_NNG_SB 16  // K3g: consecutive sample groups tested behind one union box first (0: off; r04 C5 A/B nearest-sample phase: 2.69-2.73 s off, 2.18 at 4, 2.09-2.33 at 8, 2.07-2.09 at 16)
#endif
struct NNg {
    double r, g2;  // best sqrt value, pruning guard r^2 (1 + 2^-48)
    int i;
};

__device__ __forceinline__ void nng_consider(NNg &b, double s, int j) {
    if (s <= b.g2) {  // NaN never passes
        const double r = sqrt(s);
        if (r < b.r || (r == b.r && j < b.i)) {
            b.r = r;
            b.i = j;
            b.g2 = r * r * (1.0 + 0x1p-48);
        }
    }
}

struct KdNode {
    int dim;      // -1: leaf
    double split;
    int left, right;  // children (node ids); leaf: left = group id
};

// home group of every point: descend its key's split tree (keys: sorted distinct sample keys,
// root/glo/ghi per key); a point whose key has no sample gets key slot -1 (Java's init)
__global__ void nng_home_kernel(const double *__restrict__ X, int64_t n, int d, const KdNode *__restrict__ tree,
                                const int32_t *__restrict__ xkey, const int32_t *__restrict__ keys, int nk,
                                const int32_t *__restrict__ root, uint32_t *__restrict__ hkey,
                                int32_t *__restrict__ val, int32_t *__restrict__ kslot) {
    HDB_GRID_STRIDE(p, n) {
        int ks = 0;
        if (xkey) {
            const int32_t k = xkey[p];
            int a = 0, b = nk;
            while (a < b) {
                const int mid = (a + b) >> 1;
                if (keys[mid] < k) a = mid + 1;
                else b = mid;
            }
            ks = (a < nk && keys[a] == k) ? a : -1;
        }
        uint32_t g = 0xffffffffu;  // no sample: sorts last
        if (ks >= 0) {
            int v = root[ks];
            while (tree[v].dim >= 0) v = X[p * d + tree[v].dim] < tree[v].split ? tree[v].left : tree[v].right;
            g = (uint32_t)tree[v].left;
        }
        hkey[p] = g;
        val[p] = (int32_t)p;
        kslot[p] = ks;
    }
}

template <int D, int G>
__global__ __launch_bounds__(256) void nng_search_kernel(const double *__restrict__ X, int64_t n,
                                                         const int32_t *__restrict__ order,
                                                         const uint32_t *__restrict__ home,
                                                         const double *__restrict__ Sg, const int32_t *__restrict__ sidx,
                                                         const double *__restrict__ boxes, int ng,
                                                         const int32_t *__restrict__ kslot,
                                                         const int32_t *__restrict__ glo,
                                                         const int32_t *__restrict__ ghi,
                                                         int32_t *__restrict__ out_i, double *__restrict__ out_d,
                                                         const double *__restrict__ sboxes, int sb) {
    extern __shared__ double box_s[];  // ng x 2D (lo then hi), when it fits
    const bool lds_boxes = ng * 2 * D * 8 <= 65536;
    if (lds_boxes)
        for (int k = threadIdx.x; k < ng * 2 * D; k += blockDim.x) box_s[k] = boxes[k];
    __syncthreads();
    const double *bx = lds_boxes ? box_s : boxes;
    const int64_t pos = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t p = pos < n ? order[pos] : 0;
    const int ks = pos < n ? kslot[p] : -1;
    const bool live = ks >= 0;  // a point whose key has samples
    double x[D];
#pragma unroll
    for (int c = 0; c < D; c++) x[c] = X[p * D + c];
    NNg b{JMAX, INFINITY, -1};
    const int hg = live ? (int)home[pos] : 0;
    const int g_lo = live ? glo[ks] : ng, g_hi = live ? ghi[ks] : 0;  // the key's groups
    int w_lo = g_lo, w_hi = g_hi;
    for (int o = 32; o >= 1; o >>= 1) {
        w_lo = min(w_lo, __shfl_xor(w_lo, o));
        w_hi = max(w_hi, __shfl_xor(w_hi, o));
    }
    // home group first (per-lane addresses)
    for (int k = 0; k < G && live; k++) {
        const double *sr = Sg + ((int64_t)hg * G + k) * D;
        double acc = sq_diff(x[0], sr[0]);
#pragma unroll
        for (int c = 1; c < D; c++) acc = acc + sq_diff(x[c], sr[c]);
        nng_consider(b, acc, sidx[(int64_t)hg * G + k]);
    }
    // box lower bound in the reference's summation order on monotonically rounded gaps
    auto box_lb = [&](const double *lo) -> double {
        const double *hi = lo + D;
        double gap0 = fmax(fmax(lo[0] - x[0], x[0] - hi[0]), 0.0);
        double lb = gap0 * gap0;
#pragma unroll
        for (int c = 1; c < D; c++) {
            const double gc = fmax(fmax(lo[c] - x[c], x[c] - hi[c]), 0.0);
            lb = lb + gc * gc;
        }
        return lb;
    };
    auto scan_group = [&](int g) {
        const bool need = live && g >= g_lo && g < g_hi && g != hg && box_lb(bx + (int64_t)g * 2 * D) <= b.g2;
        if (!__ballot(need)) return;
        for (int k = 0; k < G; k++) {
            const double *sr = Sg + ((int64_t)g * G + k) * D;  // uniform
            double acc = sq_diff(x[0], sr[0]);
#pragma unroll
            for (int c = 1; c < D; c++) acc = acc + sq_diff(x[c], sr[c]);
            if (need) nng_consider(b, acc, sidx[(int64_t)g * G + k]);
        }
    };
    // every group whose box can still reach the lane's best (wave-uniform loop).  sb > 0: runs of
    // sb consecutive groups (neighbours in the split tree) behind the union of their boxes, whose
    // bound is <= each member's (a larger box, the same monotone operations), so a run no lane
    // can reach holds no group any lane would scan
    if (sb > 0) {
        for (int s0 = (w_lo / sb) * sb; s0 < w_hi; s0 += sb) {
            const bool need_s = live && s0 + sb > g_lo && s0 < g_hi && box_lb(sboxes + (int64_t)(s0 / sb) * 2 * D) <= b.g2;
            if (!__ballot(need_s)) continue;
            const int e = min(s0 + sb, w_hi);
            for (int g = max(s0, w_lo); g < e; g++) scan_group(g);
        }
    } else {
        for (int g = w_lo; g < w_hi; g++) scan_group(g);
    }
    if (pos < n) {
        out_i[p] = b.i < 0 ? 0 : b.i;  // no candidate below MAX: Java's initial nearest = 0
        if (out_d) out_d[p] = b.i < 0 ? JMAX : b.r;
    }
}

// host: median-split groups of the samples (per key when keyed); returns false when the path
// does not apply
static bool nearest_grouped(hdb_ctx *ctx, const double *X, int64_t n, const double *S, int64_t m, int d,
                            const int32_t *xkey, const int32_t *skey, int32_t *out_i, double *out_d) {
    if (!ctx->nearest_grouped || !(d == 2 || d == 3 || d == 4 || d == 8 || d == 16)) return false;
    if (m < 1024 || n < 8192 || n > INT32_MAX) return false;
    const int G = d <= 8 ? 32 : 64;
    hipStream_t st = ctx->stream;
    std::vector<double> hs((size_t)m * d);
    std::vector<int32_t> hk(skey ? (size_t)m : 0);
    HIP_CHECK(hipMemcpyAsync(hs.data(), S, sizeof(double) * hs.size(), hipMemcpyDeviceToHost, st));
    if (skey) HIP_CHECK(hipMemcpyAsync(hk.data(), skey, 4 * (size_t)m, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    for (double v : hs)
        if (!std::isfinite(v)) return false;  // the plain scan keeps the reference's NaN/inf behaviour
    // samples of each key, in list order
    std::vector<int32_t> idx((size_t)m);
    std::iota(idx.begin(), idx.end(), 0);
    if (skey) std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return hk[a] < hk[b]; });
    std::vector<int32_t> keys, roots, glo, ghi;
    std::vector<KdNode> tree;
    std::vector<std::pair<int64_t, int64_t>> grp;  // [lo, hi) of idx per group
    struct Task {
        int64_t lo, hi;
        int node;
    };
    std::vector<Task> stack;
    for (int64_t k0 = 0; k0 < m;) {
        int64_t k1 = k0 + 1;
        while (skey && k1 < m && hk[idx[k1]] == hk[idx[k0]]) k1++;
        if (!skey) k1 = m;
        keys.push_back(skey ? hk[idx[k0]] : 0);
        roots.push_back((int)tree.size());
        glo.push_back((int)grp.size());
        tree.push_back(KdNode{-1, 0.0, 0, 0});
        stack.push_back({k0, k1, roots.back()});
        while (!stack.empty()) {
            const Task t = stack.back();
            stack.pop_back();
            if (t.hi - t.lo <= G) {
                tree[t.node] = KdNode{-1, 0.0, (int)grp.size(), 0};
                grp.push_back({t.lo, t.hi});
                continue;
            }
            int dim = 0;
            double best = -1;
            for (int c = 0; c < d; c++) {
                double lo = INFINITY, hi = -INFINITY;
                for (int64_t k = t.lo; k < t.hi; k++) {
                    const double v = hs[(size_t)idx[k] * d + c];
                    lo = std::min(lo, v);
                    hi = std::max(hi, v);
                }
                if (hi - lo > best) {
                    best = hi - lo;
                    dim = c;
                }
            }
            // split at a multiple of G so every group of the node but the last is full
            const int64_t cnt = t.hi - t.lo, halfg = (cnt / G + 1) / 2;
            const int64_t mid = t.lo + std::max<int64_t>(1, halfg) * G;
            std::nth_element(idx.begin() + t.lo, idx.begin() + mid, idx.begin() + t.hi, [&](int32_t a, int32_t b2) {
                const double va = hs[(size_t)a * d + dim], vb = hs[(size_t)b2 * d + dim];
                return va < vb || (va == vb && a < b2);
            });
            const int l = (int)tree.size(), r = l + 1;
            tree.push_back(KdNode{-1, 0.0, 0, 0});
            tree.push_back(KdNode{-1, 0.0, 0, 0});
            tree[t.node] = KdNode{dim, hs[(size_t)idx[mid] * d + dim], l, r};
            stack.push_back({mid, t.hi, r});
            stack.push_back({t.lo, mid, l});
        }
        ghi.push_back((int)grp.size());
        k0 = k1;
    }
    const int ng = (int)grp.size(), nk = (int)keys.size();
    std::vector<double> hg((size_t)ng * G * d, NAN), hb((size_t)ng * 2 * d);
    std::vector<int32_t> hi_((size_t)ng * G, -1);
    for (int g = 0; g < ng; g++) {
        for (int c = 0; c < d; c++) {
            hb[(size_t)g * 2 * d + c] = INFINITY;
            hb[(size_t)g * 2 * d + d + c] = -INFINITY;
        }
        for (int64_t k = grp[g].first; k < grp[g].second; k++) {
            const int64_t slot = (int64_t)g * G + (k - grp[g].first);
            hi_[slot] = idx[k];
            for (int c = 0; c < d; c++) {
                const double v = hs[(size_t)idx[k] * d + c];
                hg[(size_t)slot * d + c] = v;
                hb[(size_t)g * 2 * d + c] = std::min(hb[(size_t)g * 2 * d + c], v);
                hb[(size_t)g * 2 * d + d + c] = std::max(hb[(size_t)g * 2 * d + d + c], v);
            }
        }
    }
    // device scratch (A_WORK1): groups, ids, boxes, tree, key tables, keys/order + sort
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t tb = 0;
    HIP_CHECK(sort_pairs(nullptr, tb, (const uint32_t *)nullptr, (uint32_t *)nullptr, (const int32_t *)nullptr,
                         (int32_t *)nullptr, n, 0, 32, st));
    // runs of SB groups behind one union box (HDB_NNG_SB; 0: group boxes only)
    const int SB = HDB_NNG_SB;
    const int ns = SB > 0 ? (ng + SB - 1) / SB : 0;
    std::vector<double> hsb((size_t)std::max(ns, 1) * 2 * d);
    for (int s2 = 0; s2 < ns; s2++)
        for (int c = 0; c < d; c++) {
            double lo = INFINITY, hi = -INFINITY;
            for (int g = s2 * SB; g < std::min(ng, (s2 + 1) * SB); g++) {
                lo = std::min(lo, hb[(size_t)g * 2 * d + c]);
                hi = std::max(hi, hb[(size_t)g * 2 * d + d + c]);
            }
            hsb[(size_t)s2 * 2 * d + c] = lo;
            hsb[(size_t)s2 * 2 * d + d + c] = hi;
        }
    const size_t o_sb = carve(8 * hsb.size());
    const size_t o_g = carve(sizeof(double) * hg.size()), o_i = carve(4 * hi_.size()), o_b = carve(8 * hb.size()),
                 o_t = carve(sizeof(KdNode) * tree.size()), o_kt = carve(16 * (size_t)nk), o_k1 = carve(4 * (size_t)n),
                 o_k2 = carve(4 * (size_t)n), o_v1 = carve(4 * (size_t)n), o_v2 = carve(4 * (size_t)n),
                 o_ks = carve(4 * (size_t)n), o_tmp = carve(tb);
    char *base = (char *)arena(ctx, A_WORK1, off);
    double *dg = (double *)(base + o_g), *db = (double *)(base + o_b);
    int32_t *di = (int32_t *)(base + o_i);
    KdNode *dt = (KdNode *)(base + o_t);
    int32_t *dkeys = (int32_t *)(base + o_kt), *droot = dkeys + nk, *dglo = droot + nk, *dghi = dglo + nk;
    uint32_t *k1 = (uint32_t *)(base + o_k1), *k2 = (uint32_t *)(base + o_k2);
    int32_t *v1 = (int32_t *)(base + o_v1), *v2 = (int32_t *)(base + o_v2), *kslot = (int32_t *)(base + o_ks);
    std::vector<int32_t> ktab((size_t)4 * nk);
    std::copy(keys.begin(), keys.end(), ktab.begin());
    std::copy(roots.begin(), roots.end(), ktab.begin() + nk);
    std::copy(glo.begin(), glo.end(), ktab.begin() + 2 * nk);
    std::copy(ghi.begin(), ghi.end(), ktab.begin() + 3 * nk);
    HIP_CHECK(hipMemcpyAsync(dg, hg.data(), sizeof(double) * hg.size(), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(di, hi_.data(), 4 * hi_.size(), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(db, hb.data(), 8 * hb.size(), hipMemcpyHostToDevice, st));
    double *dsb = (double *)(base + o_sb);
    HIP_CHECK(hipMemcpyAsync(dsb, hsb.data(), 8 * hsb.size(), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(dt, tree.data(), sizeof(KdNode) * tree.size(), hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(dkeys, ktab.data(), 4 * ktab.size(), hipMemcpyHostToDevice, st));
    KernelTimer t(ctx, "nearest_grouped");
    const int g = (int)std::min<int64_t>(ceil_div(n, 256), 8192);
    hipLaunchKernelGGL(nng_home_kernel, dim3(g), dim3(256), 0, st, X, n, d, dt, skey ? xkey : nullptr, dkeys, nk,
                       droot, k1, v1, kslot);
    HIP_CHECK(sort_pairs((void *)(base + o_tmp), tb, k1, k2, v1, v2, n, 0, 32, st));
    const unsigned blocks = (unsigned)ceil_div(n, 256);
    const size_t lds_arg = (size_t)ng * 2 * d * 8 <= 65536 ? (size_t)ng * 2 * d * 8 : 0;
#define NNG_CASE(DD, GG)                                                                                         \
    case DD:                                                                                                     \
        hipLaunchKernelGGL((nng_search_kernel<DD, GG>), dim3(blocks), dim3(256), lds_arg, st, X, n, v2, k2, dg, \
                           di, db, ng, kslot, dglo, dghi, out_i, out_d, dsb, SB);                                \
        break;
    switch (d) {
        NNG_CASE(2, 32)
        NNG_CASE(3, 32)
        NNG_CASE(4, 32)
        NNG_CASE(8, 32)
        NNG_CASE(16, 64)
    }
#undef NNG_CASE
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipStreamSynchronize(st));  // the host vectors above are read by the copies
    return true;
}

void nearest_sample_device(hdb_ctx *ctx, const double *X, int64_t n, const double *S, int64_t m, int d,
                           int metric, const int32_t *xkey, const int32_t *skey, int32_t *out_i, double *out_d) {
    if (n == 0) return;
    if (n > INT32_MAX || m > INT32_MAX) HDB_THROW(HDB_EINVAL, "n or m exceeds int32");
    const bool keyed = xkey && skey;
    if (metric == HDB_METRIC_EUCLIDEAN &&
        nearest_grouped(ctx, X, n, S, m, d, keyed ? xkey : nullptr, keyed ? skey : nullptr, out_i, out_d))
        return;
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
