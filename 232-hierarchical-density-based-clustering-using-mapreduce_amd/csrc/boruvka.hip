// boruvka.hip -- K2b: exact minimum spanning tree of the mutual-reachability graph for
// graphs too large for the step-serial Prim (config 2: one 1M-point graph).
//
// Result contract: an MST under the strict total order (w, min id, max id) on edges, with
// w = max(sqrt(s), core_p, core_q) computed with exactly the reference Prim's expression
// (HDBSCANStar.java:162-168).  Every MST has the same sorted weight sequence, so the
// weights equal the reference Prim's bit-for-bit; the topology may differ from Prim's only
// among equal-weight edges (Prim breaks ties by scan order).  Edges are returned sorted by
// (w, min id, max id).
//
// Layout: points are sorted by a Morton key over (up to) the first 8 dimensions, cut into
// 64-point tiles with a per-tile bounding box and a per-round "uniform component" tag.
// A wave owns one query tile (lane = point).  It walks candidate tiles outward from its own
// (t, t+1, t-1, t+2, ...), skipping a tile when no lane needs it: either every candidate is
// in the lane's component, or the tile's box is provably farther than the lane's bound.  The
// bound is min(own best, the component's best so far), the latter read from the per-round
// component minimum that other waves publish with atomicMin (a stale read only weakens the
// bound, never prunes a winner: pruning needs LB > bound strictly).
#include <hipcub/hipcub.hpp>

#include "internal.hpp"

namespace hdb {

constexpr int BT = 64;  // tile size (one wave)

template <int D>
struct Rec {
    double x[D];
    double core;
    int32_t comp;
    int32_t id;
};

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }

// ---------------------------------------------------------------- morton
__global__ void bbox_reduce_kernel(const double *__restrict__ X, int64_t n, int d, double *__restrict__ lo,
                                   double *__restrict__ hi) {
    // one block per dimension (d <= 64)
    const int c = blockIdx.x;
    __shared__ double sl[256], sh[256];
    double l = INFINITY, h = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        double v = X[i * d + c];
        l = fmin(l, v);
        h = fmax(h, v);
    }
    sl[threadIdx.x] = l;
    sh[threadIdx.x] = h;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            sl[threadIdx.x] = fmin(sl[threadIdx.x], sl[threadIdx.x + s]);
            sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + s]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        lo[c] = sl[0];
        hi[c] = sh[0];
    }
}

__global__ void morton_kernel(const double *__restrict__ X, int64_t n, int d, const double *__restrict__ lo,
                              const double *__restrict__ hi, uint64_t *__restrict__ keys, int32_t *__restrict__ iota) {
    const int dk = d < 8 ? d : 8;
    const int bits = 63 / dk > 21 ? 21 : 63 / dk;
    HDB_GRID_STRIDE(i, n) {
        uint64_t key = 0;
        uint32_t q[8];
        for (int c = 0; c < dk; c++) {
            double span = hi[c] - lo[c];
            double t = span > 0 ? (X[i * d + c] - lo[c]) / span : 0.0;
            t = t < 0 ? 0 : (t > 1 ? 1 : t);
            if (t != t) t = 0;
            q[c] = (uint32_t)(t * (double)((1u << bits) - 1));
        }
        for (int b = bits - 1; b >= 0; b--)
            for (int c = 0; c < dk; c++) key = (key << 1) | ((q[c] >> b) & 1u);
        keys[i] = key;
        iota[i] = (int32_t)i;
    }
}

template <int D>
__global__ void build_recs_kernel(const double *__restrict__ X, const double *__restrict__ core,
                                  const int32_t *__restrict__ perm, int64_t n, Rec<D> *__restrict__ recs,
                                  int32_t *__restrict__ inv) {
    HDB_GRID_STRIDE(i, n) {
        int32_t o = perm[i];
        Rec<D> r;
        for (int c = 0; c < D; c++) r.x[c] = X[(int64_t)o * D + c];
        r.core = core[o];
        r.comp = (int32_t)i;
        r.id = o;
        recs[i] = r;
        inv[o] = (int32_t)i;
    }
}

// tile boxes (coordinates fixed) and uniform-component tags (per round)
template <int D>
__global__ void tile_box_kernel(const Rec<D> *__restrict__ recs, int64_t n, double *__restrict__ tlo,
                                double *__restrict__ thi) {
    const int64_t t = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t i = t * BT + lane;
    for (int c = 0; c < D; c++) {
        double v = i < n ? recs[i].x[c] : NAN;
        double l = i < n ? v : INFINITY, h = i < n ? v : -INFINITY;
        for (int off = 32; off >= 1; off >>= 1) {
            l = fmin(l, __shfl_xor(l, off));
            h = fmax(h, __shfl_xor(h, off));
        }
        if (lane == 0) {
            tlo[t * D + c] = l;
            thi[t * D + c] = h;
        }
    }
}

template <int D>
__global__ void tile_comp_kernel(const Rec<D> *__restrict__ recs, int64_t n, int32_t *__restrict__ tcomp) {
    const int64_t t = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t i = t * BT + lane;
    int32_t c = i < n ? recs[i].comp : -2;
    int32_t c0 = __shfl(c, 0);
    bool same = (c == c0) || (c == -2);
    bool all = __all(same);
    if (lane == 0) tcomp[t] = all ? c0 : -1;
}

// --------------------------------------------------------------- scan
struct Best {
    double w;
    int32_t lo, hi;  // original ids
};
__device__ __forceinline__ bool key_less(double w, int32_t lo, int32_t hi, const Best &b) {
    if (w < b.w) return true;
    if (w > b.w) return false;
    if (lo != b.lo) return lo < b.lo;
    return hi < b.hi;
}

// BVH over the Morton-ordered tiles: level 0 = tiles (64 points), level L node i covers
// level L-1 nodes 8i .. 8i+7.  Node boxes are fixed; node component tags (uniform
// component id or -1) are rebuilt every round.
constexpr int FAN = 8;
constexpr int MAXLEV = 12;
struct Bvh {
    double *lo, *hi;      // [total_nodes][D]
    int32_t *tag;         // [total_nodes]
    int64_t off[MAXLEV + 1];
    int64_t cnt[MAXLEV];
    int levels;
};

template <int D>
__global__ void bvh_box_kernel(double *__restrict__ lo, double *__restrict__ hi, int64_t child_off, int64_t child_cnt,
                               int64_t off, int64_t cnt) {
    HDB_GRID_STRIDE(i, cnt) {
        int64_t c0 = i * FAN, c1 = min(c0 + FAN, child_cnt);
        for (int c = 0; c < D; c++) {
            double l = INFINITY, h = -INFINITY;
            for (int64_t k = c0; k < c1; k++) {
                double a = lo[(child_off + k) * D + c], b = hi[(child_off + k) * D + c];
                l = a < l ? a : l;
                h = b > h ? b : h;
            }
            lo[(off + i) * D + c] = l;
            hi[(off + i) * D + c] = h;
        }
    }
}

__global__ void bvh_tag_kernel(int32_t *__restrict__ tag, int64_t child_off, int64_t child_cnt, int64_t off,
                               int64_t cnt) {
    HDB_GRID_STRIDE(i, cnt) {
        int64_t c0 = i * FAN, c1 = min(c0 + FAN, child_cnt);
        int32_t t = tag[child_off + c0];
        for (int64_t k = c0 + 1; k < c1 && t >= 0; k++)
            if (tag[child_off + k] != t) t = -1;
        tag[off + i] = t;
    }
}

// lane lower bound (squared) from point x to a box
template <int D>
__device__ __forceinline__ double box_lb2(const double (&x)[D], const double *__restrict__ l,
                                          const double *__restrict__ h) {
    double lb = 0;
#pragma unroll
    for (int c = 0; c < D; c++) {
        double a = l[c], b = h[c];
        double g = x[c] < a ? a - x[c] : (x[c] > b ? x[c] - b : 0.0);
        lb = lb + g * g;
    }
    return lb;
}

template <int D>
__global__ __launch_bounds__(256) void boruvka_bvh_kernel(const Rec<D> *__restrict__ recs, int64_t n, int64_t ntiles,
                                                          Bvh bvh, unsigned long long *__restrict__ comp_w,
                                                          double *__restrict__ best_w, int32_t *__restrict__ best_lo,
                                                          int32_t *__restrict__ best_hi) {
    __shared__ int32_t stack_s[4][MAXLEV * FAN + 8];
    const int w = threadIdx.x >> 6;
    const int64_t t = (int64_t)blockIdx.x * 4 + w;
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    int32_t *stk = stack_s[w];
    const int64_t i = t * BT + lane;
    const bool valid = i < n;
    double mx[D];
    double mcore = 0;
    int32_t mcomp = -3, mid = 0;
    if (valid) {
        const Rec<D> r = recs[i];
#pragma unroll
        for (int c = 0; c < D; c++) mx[c] = r.x[c];
        mcore = r.core;
        mcomp = r.comp;
        mid = r.id;
    } else {
#pragma unroll
        for (int c = 0; c < D; c++) mx[c] = 0;
    }
    Best b{INFINITY, INT32_MAX, INT32_MAX};
    double cbound = INFINITY;
    // query tile box (uniform) for the visit order
    const double *qlo = bvh.lo + t * D, *qhi = bvh.hi + t * D;
    auto refresh = [&]() {
        if (valid) {
            unsigned long long cw = __hip_atomic_load(&comp_w[mcomp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            double cwd = __longlong_as_double((long long)cw);
            if (cwd < cbound) cbound = cwd;
        }
    };
    auto lane_needs = [&](int64_t node) -> bool {
        if (!valid) return false;
        const int32_t tg = bvh.tag[node];
        if (tg >= 0 && tg == mcomp) return false;
        double bound = b.w < cbound ? b.w : cbound;
        if (!(bound < INFINITY)) return true;
        double lb = box_lb2<D>(mx, bvh.lo + node * D, bvh.hi + node * D);
        return !(lb * (1.0 - 1e-12) > bound * bound);
    };
    int sp = 0;
    if (lane == 0) stk[0] = ((bvh.levels - 1) << 26) | 0;
    sp = 1;
    int visits = 0;
    while (sp > 0) {
        __builtin_amdgcn_wave_barrier();
        const int32_t code = __builtin_amdgcn_readfirstlane(stk[sp - 1]);
        sp--;
        const int lev = code >> 26;
        const int64_t idx = code & ((1 << 26) - 1);
        const int64_t node = bvh.off[lev] + idx;
        if ((visits++ & 7) == 0) refresh();
        if (!__any(lane_needs(node))) continue;
        if (lev == 0) {
            // leaf: 64 candidates of tile idx
            const bool need = lane_needs(node);
            const int64_t j0 = idx * BT, j1 = min(j0 + BT, n);
            for (int64_t q = j0; q < j1; q++) {
                const Rec<D> &r = recs[q];  // uniform -> scalar loads
                if (!need) continue;
                if (r.comp == mcomp) continue;
                double s = sq_diff(mx[0], r.x[0]);
#pragma unroll
                for (int c = 1; c < D; c++) s = s + sq_diff(mx[c], r.x[c]);
                // s > fl(b*b)*(1+2^-48) proves fl(sqrt(s)) > b strictly (ties could still win on ids)
                double thr = (b.w * b.w) * 1.0000000000000036;
                if (s > thr) continue;
                double mrd = sqrt(s);  // HDBSCANStar.java:162-168 order
                if (mcore > mrd) mrd = mcore;
                if (r.core > mrd) mrd = r.core;
                int32_t lo = mid < r.id ? mid : r.id;
                int32_t hi = mid < r.id ? r.id : mid;
                if (key_less(mrd, lo, hi, b)) {
                    b.w = mrd;
                    b.lo = lo;
                    b.hi = hi;
                }
            }
            if (need && b.w < cbound) {
                atomicMin(&comp_w[mcomp], (unsigned long long)dbits(b.w));
                cbound = b.w;
            }
            continue;
        }
        // internal: push needed children, farthest first (nearest popped first)
        const int64_t c0 = idx * FAN;
        const int64_t c1 = min(c0 + FAN, bvh.cnt[lev - 1]);
        double key[FAN];
        bool ok[FAN];
#pragma unroll
        for (int k = 0; k < FAN; k++) {
            ok[k] = false;
            key[k] = INFINITY;
            const int64_t c = c0 + k;
            if (c < c1) {
                const int64_t cn = bvh.off[lev - 1] + c;
                ok[k] = __any(lane_needs(cn));
                // box-to-box distance between the query tile and the child (uniform)
                double kk = 0;
                const double *cl = bvh.lo + cn * D, *ch = bvh.hi + cn * D;
#pragma unroll
                for (int d = 0; d < D; d++) {
                    double g = qhi[d] < cl[d] ? cl[d] - qhi[d] : (ch[d] < qlo[d] ? qlo[d] - ch[d] : 0.0);
                    kk = kk + g * g;
                }
                key[k] = kk;
            }
        }
        // selection: push in decreasing key order
#pragma unroll 1
        for (int r = 0; r < FAN; r++) {
            int sel = -1;
            double sk = -1.0;
#pragma unroll
            for (int k = 0; k < FAN; k++)
                if (ok[k] && key[k] > sk) {
                    sk = key[k];
                    sel = k;
                }
            sel = __builtin_amdgcn_readfirstlane(sel);
            if (sel < 0) break;
#pragma unroll
            for (int k = 0; k < FAN; k++)
                if (k == sel) ok[k] = false;
            if (lane == 0) stk[sp] = ((lev - 1) << 26) | (int32_t)(c0 + sel);
            sp++;
        }
    }
    if (valid) {
        best_w[i] = b.w;
        best_lo[i] = b.lo;
        best_hi[i] = b.hi;
        if (b.w < INFINITY) atomicMin(&comp_w[mcomp], (unsigned long long)dbits(b.w));
    }
}

template <int D>
__global__ void comp_key_kernel(const Rec<D> *__restrict__ recs, int64_t n, const unsigned long long *__restrict__ comp_w,
                                const double *__restrict__ best_w, const int32_t *__restrict__ best_lo,
                                const int32_t *__restrict__ best_hi, unsigned long long *__restrict__ comp_key) {
    HDB_GRID_STRIDE(i, n) {
        int32_t c = recs[i].comp;
        double w = best_w[i];
        if (w < INFINITY && dbits(w) == comp_w[c])
            atomicMin(&comp_key[c], ((unsigned long long)(uint32_t)best_lo[i] << 32) | (uint32_t)best_hi[i]);
    }
}

// per component root c: chosen edge -> parent pointer; record edge unless mutual-larger
template <int D>
__global__ void hook_kernel(const Rec<D> *__restrict__ recs, int64_t n, const int32_t *__restrict__ inv,
                            const unsigned long long *__restrict__ comp_w,
                            const unsigned long long *__restrict__ comp_key, int32_t *__restrict__ parent,
                            int32_t *__restrict__ out_a, int32_t *__restrict__ out_b, double *__restrict__ out_w,
                            unsigned long long *__restrict__ n_edges) {
    HDB_GRID_STRIDE(c, n) {
        if (recs[c].comp != (int32_t)c) continue;  // not a root
        unsigned long long k = comp_key[c];
        if (k == ~0ull) {
            parent[c] = (int32_t)c;
            continue;
        }
        int32_t lo = (int32_t)(k >> 32), hi = (int32_t)(k & 0xffffffffu);
        int32_t cl = recs[inv[lo]].comp, ch = recs[inv[hi]].comp;
        int32_t other = cl == (int32_t)c ? ch : cl;
        parent[c] = other;
    }
}

template <int D>
__global__ void hook_fix_kernel(const Rec<D> *__restrict__ recs, int64_t n, const unsigned long long *__restrict__ comp_w,
                                const unsigned long long *__restrict__ comp_key, int32_t *__restrict__ parent,
                                int32_t *__restrict__ parent2, int32_t *__restrict__ out_a, int32_t *__restrict__ out_b,
                                double *__restrict__ out_w, unsigned long long *__restrict__ n_edges) {
    HDB_GRID_STRIDE(c, n) {
        if (recs[c].comp != (int32_t)c) continue;
        int32_t p = parent[c];
        if (p == (int32_t)c) {
            parent2[c] = p;
            continue;
        }
        bool mutual = parent[p] == (int32_t)c;
        if (mutual && (int32_t)c < p) {
            parent2[c] = (int32_t)c;  // smaller id of a mutual pair becomes the root
        } else {
            parent2[c] = p;
        }
        if (!(mutual && (int32_t)c > p)) {
            unsigned long long slot = atomicAdd(n_edges, 1ull);
            unsigned long long k = comp_key[c];
            out_a[slot] = (int32_t)(k >> 32);
            out_b[slot] = (int32_t)(k & 0xffffffffu);
            out_w[slot] = __longlong_as_double((long long)comp_w[c]);
        }
    }
}

__global__ void jump_kernel(int32_t *__restrict__ parent, int64_t n, int *__restrict__ changed) {
    HDB_GRID_STRIDE(c, n) {
        int32_t p = parent[c];
        if (p < 0) continue;
        int32_t pp = parent[p];
        if (pp != p) {
            parent[c] = pp;
            *changed = 1;
        }
    }
}

template <int D>
__global__ void relabel_kernel(Rec<D> *__restrict__ recs, int64_t n, const int32_t *__restrict__ parent) {
    HDB_GRID_STRIDE(i, n) recs[i].comp = parent[recs[i].comp];
}

__global__ void mark_nonroot_kernel(int32_t *__restrict__ parent, int64_t n, const int32_t *__restrict__ is_root) {
    HDB_GRID_STRIDE(c, n) if (!is_root[c]) parent[c] = -1;
}

template <int D>
__global__ void roots_kernel(const Rec<D> *__restrict__ recs, int64_t n, int32_t *__restrict__ is_root) {
    HDB_GRID_STRIDE(c, n) is_root[c] = recs[c].comp == (int32_t)c;
}

__global__ void edge_idkey_kernel(const int32_t *a, const int32_t *b, int64_t m, uint64_t *k, int32_t *io) {
    HDB_GRID_STRIDE(i, m) {
        k[i] = ((uint64_t)(uint32_t)a[i] << 32) | (uint32_t)b[i];
        io[i] = (int32_t)i;
    }
}
__global__ void edge_wkey_kernel(const int32_t *perm_, const double *ww, int64_t m, uint64_t *k) {
    HDB_GRID_STRIDE(i, m) k[i] = (uint64_t)__double_as_longlong(ww[perm_[i]]);
}
__global__ void edge_out_kernel(const int32_t *perm_, const int32_t *a, const int32_t *b, const double *ww, int64_t m,
                                int32_t *oa, int32_t *ob, double *ow) {
    HDB_GRID_STRIDE(i, m) {
        int32_t p = perm_[i];
        oa[i] = a[p];
        ob[i] = b[p];
        ow[i] = ww[p];
    }
}

// ---------------------------------------------------------------- host
template <int D>
static void boruvka_impl(hdb_ctx *ctx, const double *X, int64_t n, const double *core, int32_t *va, int32_t *vb,
                         double *w) {
    if (n > INT32_MAX / 2) HDB_THROW(HDB_EINVAL, "n too large");
    const int64_t ntiles = ceil_div(n, BT);
    Bvh bvh;
    {
        int64_t c = ntiles, tot = 0;
        bvh.levels = 0;
        while (true) {
            if (bvh.levels >= MAXLEV) HDB_THROW(HDB_EINVAL, "boruvka: too many BVH levels");
            bvh.off[bvh.levels] = tot;
            bvh.cnt[bvh.levels] = c;
            tot += c;
            bvh.levels++;
            if (c == 1) break;
            c = ceil_div(c, FAN);
        }
        bvh.off[bvh.levels] = tot;
    }
    const int64_t nnodes = bvh.off[bvh.levels];
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t o_blo = carve(sizeof(double) * D * nnodes), o_bhi = carve(sizeof(double) * D * nnodes),
           o_btag = carve(4 * nnodes);
    size_t o_lo = carve(sizeof(double) * 64), o_hi = carve(sizeof(double) * 64), o_keys = carve(8 * n),
           o_keys2 = carve(8 * n), o_iota = carve(4 * n), o_perm = carve(4 * n), o_recs = carve(sizeof(Rec<D>) * n),
           o_inv = carve(4 * n), o_cw = carve(8 * n), o_ck = carve(8 * n), o_bw = carve(8 * n), o_bl = carve(4 * n),
           o_bh = carve(4 * n), o_par = carve(4 * n), o_par2 = carve(4 * n), o_root = carve(4 * n), o_ne = carve(8),
           o_chg = carve(8), o_ea = carve(4 * n), o_eb = carve(4 * n), o_ew = carve(8 * n);
    char *base = (char *)arena(ctx, A_WORK0, off);
    auto P = [&](size_t o) { return (void *)(base + o); };
    double *blo = (double *)P(o_lo), *bhi = (double *)P(o_hi);
    uint64_t *keys = (uint64_t *)P(o_keys), *keys2 = (uint64_t *)P(o_keys2);
    int32_t *iota = (int32_t *)P(o_iota), *perm = (int32_t *)P(o_perm), *inv = (int32_t *)P(o_inv);
    Rec<D> *recs = (Rec<D> *)P(o_recs);
    bvh.lo = (double *)P(o_blo);
    bvh.hi = (double *)P(o_bhi);
    bvh.tag = (int32_t *)P(o_btag);
    double *tlo = bvh.lo, *thi = bvh.hi;  // level 0 = tiles
    int32_t *tcomp = bvh.tag;
    unsigned long long *comp_w = (unsigned long long *)P(o_cw), *comp_key = (unsigned long long *)P(o_ck);
    double *best_w = (double *)P(o_bw);
    int32_t *best_lo = (int32_t *)P(o_bl), *best_hi = (int32_t *)P(o_bh);
    int32_t *parent = (int32_t *)P(o_par), *parent2 = (int32_t *)P(o_par2), *is_root = (int32_t *)P(o_root);
    unsigned long long *n_edges = (unsigned long long *)P(o_ne);
    int *changed = (int *)P(o_chg);
    int32_t *ea = (int32_t *)P(o_ea), *eb = (int32_t *)P(o_eb);
    double *ew = (double *)P(o_ew);
    const int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    hipStream_t st = ctx->stream;

    KernelTimer tt(ctx, "boruvka_total");
    hipLaunchKernelGGL(bbox_reduce_kernel, dim3(D), dim3(256), 0, st, X, n, D, blo, bhi);
    hipLaunchKernelGGL(morton_kernel, dim3(g), dim3(256), 0, st, X, n, D, blo, bhi, keys, iota);
    {
        size_t tb = 0;
        HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys2, iota, perm, (int)n, 0, 64, st));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys2, iota, perm, (int)n, 0, 64, st));
    }
    hipLaunchKernelGGL(build_recs_kernel<D>, dim3(g), dim3(256), 0, st, X, core, perm, n, recs, inv);
    hipLaunchKernelGGL(tile_box_kernel<D>, dim3((unsigned)ntiles), dim3(64), 0, st, recs, n, tlo, thi);
    for (int L = 1; L < bvh.levels; L++)
        hipLaunchKernelGGL(bvh_box_kernel<D>, dim3((unsigned)std::min<int64_t>(ceil_div(bvh.cnt[L], 256), 4096)), dim3(256),
                           0, st, bvh.lo, bvh.hi, bvh.off[L - 1], bvh.cnt[L - 1], bvh.off[L], bvh.cnt[L]);
    HIP_CHECK(hipMemsetAsync(n_edges, 0, 8, st));
    HIP_CHECK(hipGetLastError());

    int64_t have = 0;
    for (int round = 0; have < n - 1; round++) {
        if (round > 64) HDB_THROW(HDB_EINVAL, "boruvka did not converge (non-finite distances?)");
        hipLaunchKernelGGL(tile_comp_kernel<D>, dim3((unsigned)ntiles), dim3(64), 0, st, recs, n, tcomp);
        for (int L = 1; L < bvh.levels; L++)
            hipLaunchKernelGGL(bvh_tag_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(bvh.cnt[L], 256), 4096)),
                               dim3(256), 0, st, bvh.tag, bvh.off[L - 1], bvh.cnt[L - 1], bvh.off[L], bvh.cnt[L]);
        HIP_CHECK(hipMemsetAsync(comp_w, 0xff, 8 * n, st));
        HIP_CHECK(hipMemsetAsync(comp_key, 0xff, 8 * n, st));
        {
            KernelTimer ts(ctx, "boruvka_scan");
            hipLaunchKernelGGL(boruvka_bvh_kernel<D>, dim3((unsigned)ceil_div(ntiles, 4)), dim3(256), 0, st, recs, n,
                               ntiles, bvh, comp_w, best_w, best_lo, best_hi);
        }
        hipLaunchKernelGGL(comp_key_kernel<D>, dim3(g), dim3(256), 0, st, recs, n, comp_w, best_w, best_lo, best_hi,
                           comp_key);
        hipLaunchKernelGGL(roots_kernel<D>, dim3(g), dim3(256), 0, st, recs, n, is_root);
        hipLaunchKernelGGL(hook_kernel<D>, dim3(g), dim3(256), 0, st, recs, n, inv, comp_w, comp_key, parent, ea, eb,
                           ew, n_edges);
        hipLaunchKernelGGL(hook_fix_kernel<D>, dim3(g), dim3(256), 0, st, recs, n, comp_w, comp_key, parent, parent2,
                           ea, eb, ew, n_edges);
        hipLaunchKernelGGL(mark_nonroot_kernel, dim3(g), dim3(256), 0, st, parent2, n, is_root);
        // pointer jumping to the roots
        for (int it = 0; it < 64; it++) {
            int h_changed = 0;
            HIP_CHECK(hipMemsetAsync(changed, 0, sizeof(int), st));
            for (int r = 0; r < 4; r++) hipLaunchKernelGGL(jump_kernel, dim3(g), dim3(256), 0, st, parent2, n, changed);
            HIP_CHECK(hipMemcpyAsync(&h_changed, changed, sizeof(int), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            if (!h_changed) break;
        }
        hipLaunchKernelGGL(relabel_kernel<D>, dim3(g), dim3(256), 0, st, recs, n, parent2);
        unsigned long long h_ne = 0;
        HIP_CHECK(hipMemcpyAsync(&h_ne, n_edges, 8, hipMemcpyDeviceToHost, st));
        HIP_CHECK(hipStreamSynchronize(st));
        HIP_CHECK(hipGetLastError());
        if ((int64_t)h_ne == have) HDB_THROW(HDB_EINVAL, "boruvka made no progress (non-finite distances?)");
        have = (int64_t)h_ne;
    }
    // sort edges by (w, lo, hi): stable sort by (lo,hi) then stable by w
    {
        int64_t ne = n - 1;
        if (ne > 0) {
            uint64_t *k1 = keys, *k2 = keys2;
            int32_t *p1 = iota, *p2 = perm;
            hipLaunchKernelGGL(edge_idkey_kernel, dim3(g), dim3(256), 0, st, ea, eb, ne, k1, p1);
            size_t tb = 0;
            HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1, k2, p1, p2, (int)ne, 0, 64, st));
            void *tmp = arena(ctx, A_SORT, tb);
            HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k1, k2, p1, p2, (int)ne, 0, 64, st));
            hipLaunchKernelGGL(edge_wkey_kernel, dim3(g), dim3(256), 0, st, p2, ew, ne, k1);
            // stable sort by w (non-negative doubles: bit order == numeric order)
            HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k1, k2, p2, p1, (int)ne, 0, 64, st));
            tmp = arena(ctx, A_SORT, tb);
            HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, k1, k2, p2, p1, (int)ne, 0, 64, st));
            hipLaunchKernelGGL(edge_out_kernel, dim3(g), dim3(256), 0, st, p1, ea, eb, ew, ne, va, vb, w);
            HIP_CHECK(hipGetLastError());
        }
    }
}

void boruvka_device(hdb_ctx *ctx, const double *X, int64_t n, int d, const double *core, int metric, int32_t *va,
                    int32_t *vb, double *w) {
    if (metric != HDB_METRIC_EUCLIDEAN) HDB_THROW(HDB_EINVAL, "boruvka: euclidean metric only");
    if (n <= 1) return;
    switch (d) {
    case 1: boruvka_impl<1>(ctx, X, n, core, va, vb, w); break;
    case 2: boruvka_impl<2>(ctx, X, n, core, va, vb, w); break;
    case 3: boruvka_impl<3>(ctx, X, n, core, va, vb, w); break;
    case 4: boruvka_impl<4>(ctx, X, n, core, va, vb, w); break;
    case 8: boruvka_impl<8>(ctx, X, n, core, va, vb, w); break;
    case 16: boruvka_impl<16>(ctx, X, n, core, va, vb, w); break;
    default: HDB_THROW(HDB_EINVAL, "boruvka: d must be one of 1,2,3,4,8,16");
    }
}

}  // namespace hdb
