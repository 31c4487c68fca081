// flat.hip -- K6: the global HDBSCAN* hierarchy and its flat (FOSC / excess-of-mass) labels
// over a merged MST, on the device.  SURVEY.md §8(f) #1: the step the reference never
// completes (Main.java:351-408); semantics = HDBSCANStar.java:208-625 (computeHierarchy-
// AndClusterTree / propagateTree / findProminentClusters, commented out in the reference)
// with the canonical rules of oracle/flat_labels.py and csrc/flat.cpp (the host algorithm this
// must equal bit for bit): a tie group is removed at once (multi-way dendrogram nodes), one
// stability term per (cluster, node) added in descending level order, FOSC children summed in
// ascending smallest point id, labels 1..K by smallest point id, 0 = noise.
//
// Algorithm (all O(m) or O(m log m) data-parallel passes, m = n - 1 tree edges):
//  1. compact the non-self edges, validate, rank them by ascending weight (the merged list
//     arrives sorted descending: no sort; otherwise one radix sort);
//  2. binary Kruskal (single-linkage) tree by rank divide and conquer: at depth j every rank
//     block [lo, hi) splits into L = [lo, mid) and U = [mid, hi).  Endpoint labels name the
//     component of F_{<lo} (the forest of ranks < lo) by its root edge, or the vertex itself
//     -- such labels are unique across all blocks of a depth, so one union-find array serves
//     them all.  The L edges are united; the lightest U edge touching an L component is the
//     parent of that component's root (its largest L edge); U labels move to the new roots.
//     The parent of edge e = the lightest edge on the boundary of C(e) (e plus the lighter
//     edges connected to it), assigned at exactly one depth.  Component sizes and smallest
//     ids ride along (|C(e)| and min id of C(e) per edge);
//  3. equal-weight parent links merge edges into multi-way nodes (one node per component a
//     tie group leaves); condensation is local: a node is reached iff it is the root or has
//     >= minClSize points, a cluster starts at a valid child of a node with >= 2 valid
//     children; pointer jumping (path halving) finds each node's cluster;
//  4. per-cluster stability = sequential sum of its chain's terms in descending level (one
//     radix sort groups the chains); FOSC over the (few) clusters on the host; labels by
//     pointer jumping to the nearest selected ancestor.
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <numeric>

#include "common.hpp"
#include "internal.hpp"
#include "sort.hpp"
#include "ssort.hpp"

namespace hdb {

namespace {

constexpr int32_t NONE = INT32_MAX;
enum : int { FE_RANGE = 1, FE_NAN = 2, FE_CYCLE = 4, FE_ISOLATED = 8, FE_ROOTS = 16, FE_JUMP = 32 };

// ------------------------------------------------------------------------- union-find
// Randomised linking: the root with the lower (priority, id) hooks under the higher one, so
// trees stay O(log) deep whatever order the unions arrive in (linking by id alone builds
// long chains on the ascending-id paths of an MST).  Contracted labels (>= n: a component of
// the lower ranks, often shared by thousands of edges) outrank every vertex label, so the
// many unions of singletons with a shared label CAS their own entries, never the shared one.
__device__ __forceinline__ uint32_t uf_prio(int32_t x, int64_t n) {
    uint32_t h = (uint32_t)x * 0x9E3779B1u;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return (x >= n ? 0x80000000u : 0u) | (h >> 1);
}

// label records: {uf parent, root edge, size, min id} in 16 bytes (one transaction per label)
struct __align__(16) LRec {
    int32_t uf, rootedge, csize, cmin;
};

// Union-find words are read and written with relaxed agent-scope atomics (global_load / store
// sc1: coherent in the L2, skip the CU's L1).  They were `volatile` until round 6, which on
// gfx950 compiles to system-scope flat accesses (sc0 sc1) with a full vmcnt/lgkmcnt drain after
// each -- every step of a find paid the system-scope round trip.
__device__ __forceinline__ int32_t uf_ld(const int32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void uf_st(int32_t *p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t uf_find(LRec *lr, int32_t x) {
    int32_t *u = &lr->uf;  // stride 4 ints
    while (true) {
        int32_t p = uf_ld(u + 4 * (int64_t)x);
        if (p == x) return x;
        int32_t g = uf_ld(u + 4 * (int64_t)p);
        if (g == p) return p;
        uf_st(u + 4 * (int64_t)x, g);  // path halving: g is an ancestor of x
        x = g;
    }
}

// returns the root this union hooked (every label but its component's final root is hooked
// exactly once), or -1 when a and b were already connected
__device__ __forceinline__ int32_t uf_unite(LRec *uf, int32_t a, int32_t b, int64_t n) {
    while (true) {
        a = uf_find(uf, a);
        b = uf_find(uf, b);
        if (a == b) return -1;
        const uint32_t pa = uf_prio(a, n), pb = uf_prio(b, n);
        if (pa < pb || (pa == pb && a < b)) {
            int32_t t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(&uf[b].uf, b, a) == b) return b;  // b hooks under the higher-priority a
    }
}

// set bit(s) of a flag word once per workgroup (same-address atomics and even GLC reads
// from thousands of waves serialise at one L2 channel); every thread must call it
__device__ __forceinline__ void flag_or(int *flag, int bits) {
    __shared__ int sbits;
    if (threadIdx.x == 0) sbits = 0;
    __syncthreads();
    if (bits) atomicOr(&sbits, bits);
    __syncthreads();
    if (threadIdx.x == 0 && sbits) atomicOr(flag, sbits);
}

// root of x in an "upward" forest (every pointer goes to a larger id, roots point to self),
// compressing as it climbs
__device__ __forceinline__ int32_t up_find(int32_t *up, int32_t x) {
    while (true) {
        int32_t p = uf_ld(up + x);
        if (p == x) return x;
        int32_t g = uf_ld(up + p);
        if (g == p) return p;
        uf_st(up + x, g);
        x = g;
    }
}

// ------------------------------------------------------------------ 1. compact + rank
__global__ void fl_mark(const int32_t *__restrict__ va, const int32_t *__restrict__ vb, const double *__restrict__ w,
                        int64_t ne, int64_t n, int32_t *__restrict__ keep, int *__restrict__ err) {
    int e = 0;
    HDB_GRID_STRIDE(i, ne) {
        int32_t a = va[i], b = vb[i];
        int k = a != b;
        keep[i] = k;
        if (k) {
            if (a < 0 || b < 0 || a >= n || b >= n) e |= FE_RANGE;
            if (w[i] != w[i]) e |= FE_NAN;
        }
    }
    if (e) atomicOr(err, e);
}

__global__ void fl_compact(const int32_t *__restrict__ va, const int32_t *__restrict__ vb, const double *__restrict__ w,
                           int64_t ne, const int32_t *__restrict__ keep, const int32_t *__restrict__ pos,
                           int64_t cap, int32_t *__restrict__ ca, int32_t *__restrict__ cb, double *__restrict__ cw,
                           int64_t *__restrict__ m_out) {
    HDB_GRID_STRIDE(i, ne) {
        if (keep[i]) {
            int32_t p = pos[i];
            if (p < cap) {
                ca[p] = va[i];
                cb[p] = vb[i];
                double x = w[i];
                cw[p] = (x == 0.0) ? 0.0 : x;  // -0.0 ties +0.0 (== in the host algorithm)
            }
        }
        if (i == ne - 1) *m_out = (int64_t)pos[i] + keep[i];
    }
}

// bit 0: not descending, bit 1: not ascending
__global__ void fl_order(const double *__restrict__ cw, const int64_t *__restrict__ m_p, int *__restrict__ flags) {
    const int64_t m = *m_p;
    int f = 0;
    HDB_GRID_STRIDE(i, m - 1) {
        double a = cw[i], b = cw[i + 1];
        if (a < b) f |= 1;
        if (a > b) f |= 2;
    }
    flag_or(flags, f);  // a descending list sets bit 1 in every lane
}

// rank order by ascending weight: src position of rank r = desc ? m-1-r : (perm ? perm[r] : r)
__global__ void fl_rank(const int32_t *__restrict__ ca, const int32_t *__restrict__ cb, const double *__restrict__ cw,
                        int64_t m, int desc, const int32_t *__restrict__ perm, int32_t *__restrict__ ea,
                        int32_t *__restrict__ eb, double *__restrict__ ew, int32_t *__restrict__ lab,
                        int32_t *__restrict__ parent) {
    HDB_GRID_STRIDE(r, m) {
        int64_t s = desc ? m - 1 - r : (perm ? perm[r] : r);
        int32_t a = ca[s], b = cb[s];
        ea[r] = a;
        eb[r] = b;
        ew[r] = cw[s];
        lab[2 * r] = a;  // singleton labels: the vertex id
        lab[2 * r + 1] = b;
        parent[r] = NONE;
    }
}

__global__ void fl_sort_keys(const double *__restrict__ cw, int64_t m, double *__restrict__ keys,
                             int32_t *__restrict__ iota) {
    HDB_GRID_STRIDE(i, m) {
        keys[i] = cw[i];
        iota[i] = (int32_t)i;
    }
}

__global__ void fill_i32(int32_t *__restrict__ p, int64_t count, int32_t v) {
    HDB_GRID_STRIDE(i, count) p[i] = v;
}

// point parents: the lightest edge at each vertex (the dendrogram node a point first joins)
__global__ void fl_point_parent(const int32_t *__restrict__ ea, const int32_t *__restrict__ eb, int64_t m,
                                int32_t *__restrict__ pparent) {
    HDB_GRID_STRIDE(r, m) {
        atomicMin(&pparent[ea[r]], (int32_t)r);
        atomicMin(&pparent[eb[r]], (int32_t)r);
    }
}

// Vertex labels for the divide and conquer ordered by rank (locality): point v becomes
// 2 pp(v) + side, pp(v) = its lightest edge (rank) and side = 1 when v is that edge's second
// endpoint -- unique, < 2m.  A block of ranks [lo, hi) then touches the records of labels near
// [2lo, 2hi) for most of its vertices instead of points scattered over all n ids.
__global__ void fl_relabel_orig(const int32_t *__restrict__ pparent, const int32_t *__restrict__ eb, int64_t n,
                                int32_t *__restrict__ orig) {
    HDB_GRID_STRIDE(v, n) {
        const int32_t p = pparent[v];
        if (p == NONE) continue;  // a point no edge touches (malformed input: the union-find reports it)
        orig[2 * (int64_t)p + (eb[p] == (int32_t)v ? 1 : 0)] = (int32_t)v;
    }
}
__global__ void fl_relabel(const int32_t *__restrict__ ea, const int32_t *__restrict__ eb,
                           const int32_t *__restrict__ pparent, int64_t m, int32_t *__restrict__ lab) {
    HDB_GRID_STRIDE(r, m) {
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const int32_t v = s ? eb[r] : ea[r];
            const int32_t p = pparent[v];
            lab[2 * r + s] = 2 * p + (eb[p] == v ? 1 : 0);
        }
    }
}

// ------------------------------------------------------- 2. Kruskal tree, depth kernels
// L edge #i of depth bit b: rank with bit b clear
__device__ __forceinline__ int64_t l_rank(int64_t i, int b) {
    return ((i >> b) << (b + 1)) | (i & ((int64_t(1) << b) - 1));
}

struct DC {
    int32_t *lab;       // 2m endpoint labels (vertex id < n, or n + root edge rank)
    LRec *lr;           // n + m label records
    int32_t *stamp;     // n + m: 2j = a label of an L edge at depth j
    int32_t *hooked;    // m: the label an L edge's union hooked (-1: none); dc_root then stores its representative
    int32_t *parent;    // m: parent edge rank (NONE: root)
    int32_t *esize;     // m: |C(e)|
    int32_t *eminid;    // m: smallest point id in C(e)
    const int32_t *orig;  // vertex label -> point id (nullptr: the label is the point id)
    int64_t n, m;         // n: vertex labels (contracted labels are n + root edge rank)
};
__device__ __forceinline__ int32_t vid(const DC &c, int32_t x) { return c.orig ? c.orig[x] : x; }

__global__ void dc_init(DC c, int b, int j, int64_t nl) {
    HDB_GRID_STRIDE(i, nl) {
        int64_t r = l_rank(i, b);
        if (r >= c.m) continue;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            int32_t x = c.lab[2 * r + s];
            c.lr[x] = LRec{x, -1, 0, NONE};  // rootedge: largest L edge of the component
            c.stamp[x] = 2 * j;
        }
    }
}

__global__ void dc_unite(DC c, int b, int64_t nl, int *__restrict__ err) {
    HDB_GRID_STRIDE(i, nl) {
        int64_t r = l_rank(i, b);
        if (r >= c.m) continue;
        const int32_t h = uf_unite(c.lr, c.lab[2 * r], c.lab[2 * r + 1], c.n);
        c.hooked[r] = h;
        if (h < 0) atomicOr(err, FE_CYCLE);  // rare: bad input
    }
}

// wave reductions (all 64 lanes call them)
__device__ __forceinline__ int32_t wave_max(int32_t v) {
    for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int32_t wave_min(int32_t v) {
    for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int32_t wave_sum(int32_t v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Per component: largest L edge, summed label sizes, smallest id.  Shallow depths put most L
// edges into a few giant components, so a workgroup first combines its lanes' contributions
// in an LDS table keyed by representative (LDS atomics), then issues one global atomic per
// distinct representative.
constexpr int ROOT_TB = 256, ROOT_SLOTS = 512;
template <int TB, int SLOTS>
__global__ __launch_bounds__(TB) void dc_root(DC c, int b, int j, int64_t nl) {
    __shared__ int32_t skey[SLOTS], smax[SLOTS], ssum[SLOTS], smin[SLOTS];
    const int t = threadIdx.x;
    for (int64_t base = (int64_t)blockIdx.x * TB; base < nl; base += (int64_t)gridDim.x * TB) {
        for (int k = t; k < SLOTS; k += TB) {
            skey[k] = -1;
            smax[k] = -1;
            ssum[k] = 0;
            smin[k] = NONE;
        }
        __syncthreads();
        const int64_t i = base + t;
        const int64_t r = i < nl ? l_rank(i, b) : c.m;
        if (r < c.m) {
            const int32_t rep = uf_find(c.lr, c.lab[2 * r]);
            // the label this edge hooked is counted once, here; the final root label is
            // added by its root edge in dc_link
            const int32_t x = c.hooked[r];
            c.hooked[r] = rep;  // dc_link reads the representative back instead of a second find
            const int32_t sz = x < 0 ? 0 : (x < c.n ? 1 : c.esize[x - c.n]);
            const int32_t mi = x < 0 ? NONE : (x < c.n ? vid(c, x) : c.eminid[x - c.n]);
            uint32_t h = uf_prio(rep, 0) & (SLOTS - 1);
            while (true) {  // <= TB distinct keys in 2x slots: always finds one
                int32_t k = atomicCAS(&skey[h], -1, rep);
                if (k == -1 || k == rep) break;
                h = (h + 1) & (SLOTS - 1);
            }
            atomicMax(&smax[h], (int32_t)r);
            if (sz) atomicAdd(&ssum[h], sz);
            if (mi != NONE) atomicMin(&smin[h], mi);
        }
        __syncthreads();
        for (int k = t; k < SLOTS; k += TB) {
            const int32_t rep = skey[k];
            if (rep < 0) continue;
            atomicMax(&c.lr[rep].rootedge, smax[k]);
            if (ssum[k]) atomicAdd(&c.lr[rep].csize, ssum[k]);
            if (smin[k] != NONE) atomicMin(&c.lr[rep].cmin, smin[k]);
        }
        __syncthreads();
    }
}

// Several batches per workgroup with the table kept across them: a component spanning the
// whole block (the shallow depths' giant ones) costs one set of global atomics per workgroup
// and flush, not per batch.  The table is flushed when the next batch might overfill it.
template <int TB, int SLOTS, int EPT>
__global__ __launch_bounds__(TB) void dc_root_multi(DC c, int b, int j, int64_t nl) {
    __shared__ int32_t skey[SLOTS], smax[SLOTS], ssum[SLOTS], smin[SLOTS];
    __shared__ int s_used;
    const int t = threadIdx.x;
    auto clear = [&]() {
        for (int k = t; k < SLOTS; k += TB) {
            skey[k] = -1;
            smax[k] = -1;
            ssum[k] = 0;
            smin[k] = NONE;
        }
        if (t == 0) s_used = 0;
    };
    auto flush = [&]() {
        for (int k = t; k < SLOTS; k += TB) {
            const int32_t rep = skey[k];
            if (rep < 0) continue;
            atomicMax(&c.lr[rep].rootedge, smax[k]);
            if (ssum[k]) atomicAdd(&c.lr[rep].csize, ssum[k]);
            if (smin[k] != NONE) atomicMin(&c.lr[rep].cmin, smin[k]);
        }
    };
    const int64_t per = (int64_t)TB * EPT;
    for (int64_t base = (int64_t)blockIdx.x * per; base < nl; base += (int64_t)gridDim.x * per) {
        clear();
        __syncthreads();
        for (int e = 0; e < EPT; e++) {
            const int64_t i = base + (int64_t)e * TB + t;
            const int64_t r = i < nl ? l_rank(i, b) : c.m;
            if (r < c.m) {
                const int32_t rep = uf_find(c.lr, c.lab[2 * r]);
                const int32_t x = c.hooked[r];
                c.hooked[r] = rep;
                const int32_t sz = x < 0 ? 0 : (x < c.n ? 1 : c.esize[x - c.n]);
                const int32_t mi = x < 0 ? NONE : (x < c.n ? vid(c, x) : c.eminid[x - c.n]);
                uint32_t h = uf_prio(rep, 0) & (SLOTS - 1);
                while (true) {  // the table is kept below SLOTS - TB keys before every batch
                    const int32_t k = atomicCAS(&skey[h], -1, rep);
                    if (k == -1) {
                        atomicAdd(&s_used, 1);
                        break;
                    }
                    if (k == rep) break;
                    h = (h + 1) & (SLOTS - 1);
                }
                atomicMax(&smax[h], (int32_t)r);
                if (sz) atomicAdd(&ssum[h], sz);
                if (mi != NONE) atomicMin(&smin[h], mi);
            }
            __syncthreads();
            if (e + 1 < EPT && s_used > SLOTS / 2 - TB) {  // the next batch could push it past 3/4
                flush();
                __syncthreads();
                clear();
                __syncthreads();
            }
        }
        flush();
        __syncthreads();
    }
}

// the same without the LDS table: one set of global atomics per L edge (A/B)
__global__ void dc_root_direct(DC c, int b, int j, int64_t nl) {
    HDB_GRID_STRIDE(i, nl) {
        const int64_t r = l_rank(i, b);
        if (r >= c.m) continue;
        const int32_t rep = uf_find(c.lr, c.lab[2 * r]);
        const int32_t x = c.hooked[r];
        c.hooked[r] = rep;
        atomicMax(&c.lr[rep].rootedge, (int32_t)r);
        if (x >= 0) {
            atomicAdd(&c.lr[rep].csize, x < c.n ? 1 : c.esize[x - c.n]);
            atomicMin(&c.lr[rep].cmin, x < c.n ? vid(c, x) : c.eminid[x - c.n]);
        }
    }
}

__global__ void dc_link(DC c, int b, int j, int64_t nl) {
    HDB_GRID_STRIDE(i, nl) {
        int64_t r = l_rank(i, b);
        if (r >= c.m) continue;
        {  // L edge: a component root records |C(e)| and its smallest id (rep from dc_root)
            const int32_t rep = c.hooked[r];
            const LRec q = c.lr[rep];
            if (q.rootedge == (int32_t)r) {
                c.esize[r] = q.csize + (rep < c.n ? 1 : c.esize[rep - c.n]);
                c.eminid[r] = min(q.cmin, rep < c.n ? vid(c, rep) : c.eminid[rep - c.n]);
            }
        }
        const int64_t u = r | (int64_t(1) << b);  // the U edge paired with this thread
        if (u >= c.m) continue;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            int32_t x = c.lab[2 * u + s];
            if (c.stamp[x] == 2 * j) {  // x lies in an L component of this block
                const int32_t R = c.lr[uf_find(c.lr, x)].rootedge;
                // lighter U edges run in earlier lanes: most see their bound already beaten
                if (uf_ld(c.parent + R) > (int32_t)u) atomicMin(&c.parent[R], (int32_t)u);
                c.lab[2 * u + s] = (int32_t)(c.n + R);
            }
        }
    }
}

// dc_link with the parent minima combined per workgroup first (LDS table keyed by the root
// edge R, several batches per workgroup): the U edges around a giant L component all target
// its root edge, and their global atomicMins on one address serialise.
template <int TB, int SLOTS, int EPT>
__global__ __launch_bounds__(TB) void dc_link_multi(DC c, int b, int j, int64_t nl) {
    __shared__ int32_t skey[SLOTS], smin[SLOTS];
    __shared__ int s_used;
    const int t = threadIdx.x;
    auto clear = [&]() {
        for (int k = t; k < SLOTS; k += TB) {
            skey[k] = -1;
            smin[k] = INT32_MAX;
        }
        if (t == 0) s_used = 0;
    };
    auto flush = [&]() {
        for (int k = t; k < SLOTS; k += TB) {
            const int32_t R = skey[k];
            if (R < 0) continue;
            if (uf_ld(c.parent + R) > smin[k]) atomicMin(&c.parent[R], smin[k]);
        }
    };
    const int64_t per = (int64_t)TB * EPT;
    for (int64_t base = (int64_t)blockIdx.x * per; base < nl; base += (int64_t)gridDim.x * per) {
        clear();
        __syncthreads();
        for (int e = 0; e < EPT; e++) {
            const int64_t i = base + (int64_t)e * TB + t;
            const int64_t r = i < nl ? l_rank(i, b) : c.m;
            if (r < c.m) {
                {  // L edge: a component root records |C(e)| and its smallest id (rep from dc_root)
                    const int32_t rep = c.hooked[r];
                    const LRec q = c.lr[rep];
                    if (q.rootedge == (int32_t)r) {
                        c.esize[r] = q.csize + (rep < c.n ? 1 : c.esize[rep - c.n]);
                        c.eminid[r] = min(q.cmin, rep < c.n ? vid(c, rep) : c.eminid[rep - c.n]);
                    }
                }
                const int64_t u = r | (int64_t(1) << b);
                if (u < c.m) {
#pragma unroll
                    for (int s = 0; s < 2; s++) {
                        const int32_t x = c.lab[2 * u + s];
                        if (c.stamp[x] == 2 * j) {
                            const int32_t R = c.lr[uf_find(c.lr, x)].rootedge;
                            uint32_t h = uf_prio(R, 0) & (SLOTS - 1);
                            while (true) {  // <= SLOTS / 2 keys before every batch's 2 TB inserts
                                const int32_t k = atomicCAS(&skey[h], -1, R);
                                if (k == -1) {
                                    atomicAdd(&s_used, 1);
                                    break;
                                }
                                if (k == R) break;
                                h = (h + 1) & (SLOTS - 1);
                            }
                            atomicMin(&smin[h], (int32_t)u);
                            c.lab[2 * u + s] = (int32_t)(c.n + R);
                        }
                    }
                }
            }
            __syncthreads();
            if (e + 1 < EPT && s_used > SLOTS / 2 - 2 * TB) {
                flush();
                __syncthreads();
                clear();
                __syncthreads();
            }
        }
        flush();
        __syncthreads();
    }
}

// Middle depths in one launch (round 6): a workgroup owns a block of 2^LM consecutive ranks and
// runs the global depths' four phases (dc_init, dc_unite, dc_root_multi, dc_link_multi: the
// same per-edge work on the same global arrays) for its block's depths b = LM-1 .. LB itself,
// one workgroup barrier between phases instead of a kernel boundary.  With rank-ordered labels
// (flat_relabel) a block's label records, stamps and edge arrays are a few hundred KB, so they
// stay in the one XCD's L2 the workgroup runs on -- a global depth spreads every block over all
// eight XCDs and streams the whole record array through the MALL.  Cross-wave visibility of the
// plain stores and the L2 atomics between phases: the workgroup barrier's workgroup-scope
// acquire/release (every wave of the workgroup shares one CU and its write-through L1; the
// compiler's gfx950 memory model needs no cache maintenance at that scope).  An agent-scope
// __threadfence here would write the XCD's L2 back at every phase (buffer_wbl2): 4x slower.
__device__ __forceinline__ void dc_phase_sync() { __syncthreads(); }

template <int TB>
__global__ __launch_bounds__(TB) void dc_mid(DC c, int J, int LM, int LB, int *__restrict__ err) {
    constexpr int RS = 4096, KS = 8192;  // LDS table slots: root phase (4 ints), link phase (2 ints)
    __shared__ int32_t tab[4 * RS > 2 * KS ? 4 * RS : 2 * KS];
    __shared__ int s_used;
    const int t = threadIdx.x;
    const int64_t blk = blockIdx.x;
    if ((blk << LM) >= c.m) return;
    int e_cyc = 0;
    for (int b = LM - 1; b >= LB; b--) {
        const int j = J - 1 - b;
        const int64_t bl = int64_t(1) << (b + 1), half = int64_t(1) << b;
        const int64_t nl = (c.m / bl) * half + std::min(c.m % bl, half);
        const int64_t i0 = blk << (LM - 1), i1 = std::min(i0 + (int64_t(1) << (LM - 1)), nl);
        // init
        for (int64_t i = i0 + t; i < i1; i += TB) {
            const int64_t r = l_rank(i, b);
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const int32_t x = c.lab[2 * r + s];
                c.lr[x] = LRec{x, -1, 0, NONE};
                c.stamp[x] = 2 * j;
            }
        }
        dc_phase_sync();
        // unite
        for (int64_t i = i0 + t; i < i1; i += TB) {
            const int64_t r = l_rank(i, b);
            const int32_t h = uf_unite(c.lr, c.lab[2 * r], c.lab[2 * r + 1], c.n);
            c.hooked[r] = h;
            if (h < 0) e_cyc = 1;
        }
        dc_phase_sync();
        // root: per component largest L edge, summed sizes, smallest id (LDS-combined)
        {
            int32_t *skey = tab, *smax = tab + RS, *ssum = tab + 2 * RS, *smin = tab + 3 * RS;
            auto clear = [&]() {
                for (int k = t; k < RS; k += TB) {
                    skey[k] = -1;
                    smax[k] = -1;
                    ssum[k] = 0;
                    smin[k] = NONE;
                }
                if (t == 0) s_used = 0;
            };
            auto flush = [&]() {
                for (int k = t; k < RS; k += TB) {
                    const int32_t rep = skey[k];
                    if (rep < 0) continue;
                    atomicMax(&c.lr[rep].rootedge, smax[k]);
                    if (ssum[k]) atomicAdd(&c.lr[rep].csize, ssum[k]);
                    if (smin[k] != NONE) atomicMin(&c.lr[rep].cmin, smin[k]);
                }
            };
            clear();
            __syncthreads();
            for (int64_t base = i0; base < i1; base += TB) {
                const int64_t i = base + t;
                if (i < i1) {
                    const int64_t r = l_rank(i, b);
                    const int32_t rep = uf_find(c.lr, c.lab[2 * r]);
                    const int32_t x = c.hooked[r];
                    c.hooked[r] = rep;
                    const int32_t sz = x < 0 ? 0 : (x < c.n ? 1 : c.esize[x - c.n]);
                    const int32_t mi = x < 0 ? NONE : (x < c.n ? vid(c, x) : c.eminid[x - c.n]);
                    uint32_t h = uf_prio(rep, 0) & (RS - 1);
                    while (true) {  // kept below RS / 2 keys before every batch of TB
                        const int32_t k = atomicCAS(&skey[h], -1, rep);
                        if (k == -1) {
                            atomicAdd(&s_used, 1);
                            break;
                        }
                        if (k == rep) break;
                        h = (h + 1) & (RS - 1);
                    }
                    atomicMax(&smax[h], (int32_t)r);
                    if (sz) atomicAdd(&ssum[h], sz);
                    if (mi != NONE) atomicMin(&smin[h], mi);
                }
                __syncthreads();
                if (base + TB < i1 && s_used > RS / 2 - TB) {
                    flush();
                    __syncthreads();
                    clear();
                    __syncthreads();
                }
            }
            flush();
        }
        dc_phase_sync();
        // link: root edges record |C(e)| / min id; U edges' parent minima (LDS-combined) + relabel
        {
            int32_t *skey = tab, *smin = tab + KS;
            auto clear = [&]() {
                for (int k = t; k < KS; k += TB) {
                    skey[k] = -1;
                    smin[k] = INT32_MAX;
                }
                if (t == 0) s_used = 0;
            };
            auto flush = [&]() {
                for (int k = t; k < KS; k += TB) {
                    const int32_t R = skey[k];
                    if (R < 0) continue;
                    if (uf_ld(c.parent + R) > smin[k]) atomicMin(&c.parent[R], smin[k]);
                }
            };
            clear();
            __syncthreads();
            for (int64_t base = i0; base < i1; base += TB) {
                const int64_t i = base + t;
                if (i < i1) {
                    const int64_t r = l_rank(i, b);
                    {
                        const int32_t rep = c.hooked[r];
                        const LRec q = c.lr[rep];
                        if (q.rootedge == (int32_t)r) {
                            c.esize[r] = q.csize + (rep < c.n ? 1 : c.esize[rep - c.n]);
                            c.eminid[r] = min(q.cmin, rep < c.n ? vid(c, rep) : c.eminid[rep - c.n]);
                        }
                    }
                    const int64_t u = r | half;
                    if (u < c.m) {
#pragma unroll
                        for (int s = 0; s < 2; s++) {
                            const int32_t x = c.lab[2 * u + s];
                            if (c.stamp[x] == 2 * j) {
                                const int32_t R = c.lr[uf_find(c.lr, x)].rootedge;
                                uint32_t h = uf_prio(R, 0) & (KS - 1);
                                while (true) {
                                    const int32_t k = atomicCAS(&skey[h], -1, R);
                                    if (k == -1) {
                                        atomicAdd(&s_used, 1);
                                        break;
                                    }
                                    if (k == R) break;
                                    h = (h + 1) & (KS - 1);
                                }
                                atomicMin(&smin[h], (int32_t)u);
                                c.lab[2 * u + s] = (int32_t)(c.n + R);
                            }
                        }
                    }
                }
                __syncthreads();
                if (base + TB < i1 && s_used > KS / 2 - 2 * TB) {
                    flush();
                    __syncthreads();
                    clear();
                    __syncthreads();
                }
            }
            flush();
        }
        dc_phase_sync();
    }
    if (e_cyc) atomicOr(err, FE_CYCLE);
}

// Deep depths in one launch, in parallel: a workgroup takes a block of 2^LB consecutive ranks
// whose labels name the components of F_{<lo} and runs the same rank divide and conquer on
// LDS (labels hashed to local ids, contracted labels = HS + local root-edge rank, an LDS
// union-find with the global kernels' randomised linking, LDS atomics for the component
// root edge / size / smallest id).  Every edge whose local bits are not all ones is a
// component root edge at exactly one local depth (trailing ones) and gets |C(e)| and min id
// there; the block's last edge got them at a global depth.  Parents inside the block are set
// here, the others were set by the global depths.
template <int LB>
struct DcBlk {
    static constexpr int B = 1 << LB, HS = 4 * B, NL = HS + B;
};

__device__ __forceinline__ int32_t lds_find(int32_t *uf, int32_t x) {
    while (true) {
        const int32_t p = ((volatile int32_t *)uf)[x];
        if (p == x) return x;
        const int32_t g = ((volatile int32_t *)uf)[p];
        if (g == p) return p;
        ((volatile int32_t *)uf)[x] = g;
        x = g;
    }
}

template <int LB, int TB>
__global__ __launch_bounds__(TB) void dc_block(DC c, int *__restrict__ err) {
    using P = DcBlk<LB>;
    __shared__ int32_t key[P::HS], bsz[P::HS], bmn[P::HS];             // hashed labels, base size / min id
    __shared__ int32_t uf[P::NL], re[P::NL], cs[P::NL], cm[P::NL];     // per label (per depth)
    __shared__ int8_t stp[P::NL];                                      // local depth stamp
    __shared__ int16_t lab[2 * P::B];                                  // endpoint labels (local ids)
    __shared__ int32_t esz[P::B], emn[P::B], lpar[P::B];
    __shared__ int16_t hk[P::B], rp[P::B];
    __shared__ int s_err;
    const int t = threadIdx.x;
    for (int64_t lo = (int64_t)blockIdx.x * P::B; lo < c.m; lo += (int64_t)gridDim.x * P::B) {
        const int cnt = (int)(c.m - lo < P::B ? c.m - lo : P::B);
        for (int k = t; k < P::HS; k += TB) key[k] = -1;
        for (int k = t; k < P::NL; k += TB) stp[k] = -1;
        for (int k = t; k < P::B; k += TB) {
            esz[k] = -1;
            lpar[k] = INT32_MAX;
        }
        if (t == 0) s_err = 0;
        __syncthreads();
        for (int k = t; k < 2 * cnt; k += TB) {
            const int32_t x = c.lab[2 * lo + k];
            uint32_t h = uf_prio(x, 0) & (P::HS - 1);
            while (true) {  // <= 2B keys in 4B slots
                const int32_t old = atomicCAS(&key[h], -1, x);
                if (old == -1) {
                    bsz[h] = x < c.n ? 1 : c.esize[x - c.n];
                    bmn[h] = x < c.n ? vid(c, x) : c.eminid[x - c.n];
                    break;
                }
                if (old == x) break;
                h = (h + 1) & (P::HS - 1);
            }
            lab[k] = (int16_t)h;
        }
        __syncthreads();
        for (int b = LB - 1; b >= 0; b--) {
            const int half = 1 << b, nl = (P::B >> 1);
            // L edges: local ranks with bit b clear
            for (int i = t; i < nl; i += TB) {
                const int k = ((i >> b) << (b + 1)) | (i & (half - 1));
                if (k >= cnt) continue;
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int x = lab[2 * k + s];
                    uf[x] = x;
                    re[x] = -1;
                    cs[x] = x < P::HS ? bsz[x] : esz[x - P::HS];
                    cm[x] = x < P::HS ? bmn[x] : emn[x - P::HS];
                    stp[x] = (int8_t)b;
                }
            }
            __syncthreads();
            for (int i = t; i < nl; i += TB) {
                const int k = ((i >> b) << (b + 1)) | (i & (half - 1));
                if (k >= cnt) continue;
                int32_t a = lab[2 * k], d = lab[2 * k + 1], hooked = -1;
                while (true) {
                    a = lds_find(uf, a);
                    d = lds_find(uf, d);
                    if (a == d) break;
                    const uint32_t pa = uf_prio(a, P::HS), pd = uf_prio(d, P::HS);
                    if (pa < pd || (pa == pd && a < d)) {
                        const int32_t tt = a;
                        a = d;
                        d = tt;
                    }
                    if (atomicCAS(&uf[d], d, a) == d) {
                        hooked = d;
                        break;
                    }
                }
                if (hooked < 0) s_err = 1;
                hk[k] = (int16_t)hooked;
            }
            __syncthreads();
            for (int i = t; i < nl; i += TB) {
                const int k = ((i >> b) << (b + 1)) | (i & (half - 1));
                if (k >= cnt) continue;
                const int32_t rep = lds_find(uf, lab[2 * k]);
                rp[k] = (int16_t)rep;
                atomicMax(&re[rep], k);
                const int32_t x = hk[k];
                if (x >= 0) {  // a hooked label is never a representative: its cs / cm are its base
                    atomicAdd(&cs[rep], cs[x]);
                    atomicMin(&cm[rep], cm[x]);
                }
            }
            __syncthreads();
            for (int i = t; i < nl; i += TB) {
                const int k = ((i >> b) << (b + 1)) | (i & (half - 1));
                if (k >= cnt) continue;
                const int32_t rep = rp[k];
                if (re[rep] == k) {
                    esz[k] = cs[rep];
                    emn[k] = cm[rep];
                }
                const int u = k | half;
                if (u >= cnt) continue;
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    const int x = lab[2 * u + s];
                    if (stp[x] == (int8_t)b) {
                        const int32_t R = re[lds_find(uf, x)];
                        atomicMin(&lpar[R], u);
                        lab[2 * u + s] = (int16_t)(P::HS + R);
                    }
                }
            }
            __syncthreads();
        }
        for (int k = t; k < cnt; k += TB) {
            if (esz[k] >= 0) {
                c.esize[lo + k] = esz[k];
                c.eminid[lo + k] = emn[k];
            }
            if (lpar[k] != INT32_MAX) c.parent[lo + k] = (int32_t)(lo + lpar[k]);
        }
        if (t == 0 && s_err) atomicOr(err, FE_CYCLE);
        __syncthreads();
    }
}

// Deep depths in one launch: a block of LOC_EDGES consecutive ranks whose labels name the
// components of F_{<lo} runs the sequential Kruskal process itself (one wave per block, the
// block's labels hashed to LDS slots, union by size, one lane walking the ranks in order):
// parents inside the block, |C(e)| and min id of C(e) for every edge.  Parents that leave the
// block were assigned by the shallower depths.
constexpr int LOC_LOG = 8, LOC_EDGES = 1 << LOC_LOG, LOC_SLOTS = 4 * LOC_EDGES;
__global__ __launch_bounds__(64) void dc_local(DC c, int *__restrict__ err) {
    __shared__ int32_t key[LOC_SLOTS], lsz[LOC_SLOTS], lmn[LOC_SLOTS];
    __shared__ int16_t luf[LOC_SLOTS], lre[LOC_SLOTS];
    __shared__ int16_t le[2 * LOC_EDGES];
    const int lane = threadIdx.x;
    for (int64_t lo = (int64_t)blockIdx.x * LOC_EDGES; lo < c.m; lo += (int64_t)gridDim.x * LOC_EDGES) {
        const int cnt = (int)(c.m - lo < LOC_EDGES ? c.m - lo : LOC_EDGES);
        for (int k = lane; k < LOC_SLOTS; k += 64) key[k] = -1;
        __syncthreads();
        for (int k = lane; k < 2 * cnt; k += 64) {
            const int32_t x = c.lab[2 * lo + k];
            uint32_t h = uf_prio(x, 0) & (LOC_SLOTS - 1);
            while (true) {  // <= 2 LOC_EDGES keys in 4x slots
                const int32_t old = atomicCAS(&key[h], -1, x);
                if (old == -1) {  // inserted: initialise the slot
                    luf[h] = (int16_t)h;
                    lre[h] = -1;
                    lsz[h] = x < c.n ? 1 : c.esize[x - c.n];
                    lmn[h] = x < c.n ? vid(c, x) : c.eminid[x - c.n];
                    break;
                }
                if (old == x) break;
                h = (h + 1) & (LOC_SLOTS - 1);
            }
            le[k] = (int16_t)h;
        }
        __syncthreads();
        if (lane == 0) {
            auto find = [&](int x) {
                while (luf[x] != x) {
                    const int g = luf[luf[x]];
                    luf[x] = (int16_t)g;
                    x = g;
                }
                return x;
            };
            for (int k = 0; k < cnt; k++) {
                int a = find(le[2 * k]), b = find(le[2 * k + 1]);
                if (a == b) {
                    atomicOr(err, FE_CYCLE);
                    break;
                }
                if (lre[a] >= 0) c.parent[lo + lre[a]] = (int32_t)(lo + k);
                if (lre[b] >= 0) c.parent[lo + lre[b]] = (int32_t)(lo + k);
                if (lsz[a] < lsz[b]) {
                    const int t = a;
                    a = b;
                    b = t;
                }
                luf[b] = (int16_t)a;
                lsz[a] += lsz[b];
                lmn[a] = min(lmn[a], lmn[b]);
                lre[a] = (int16_t)k;
                c.esize[lo + k] = lsz[a];
                c.eminid[lo + k] = lmn[a];
            }
        }
        __syncthreads();
    }
}

// -------------------------------------------------------------------- 3. nodes + clusters
__global__ void fl_tie_up(const int32_t *__restrict__ parent, const double *__restrict__ ew, int64_t m,
                          int32_t *__restrict__ up, int *__restrict__ err) {
    int e = 0;
    HDB_GRID_STRIDE(r, m) {
        int32_t p = parent[r];
        up[r] = (p != NONE && ew[p] == ew[r]) ? p : (int32_t)r;
        if (p == NONE && r != m - 1) e |= FE_ROOTS;
    }
    if (e) atomicOr(err, e);
}

// synchronous-ish pointer jumping over an upward forest (pointers only move to ancestors, so
// in-place jumps are safe); flags[k] records whether round k changed anything and round k+1
// exits at once when it did not.  ~log2(longest chain) rounds do work.
__global__ void fl_jump(int32_t *__restrict__ up, int64_t m, const int *__restrict__ flag_prev,
                        int *__restrict__ flag_next) {
    if (flag_prev && *flag_prev == 0) return;
    int ch = 0;
    HDB_GRID_STRIDE(r, m) {
        int32_t p = up[r];
        bool moved = false;
#pragma unroll 1
        for (int it = 0; it < 2; it++) {  // two hops per step, two steps per launch
            const int32_t g = up[p];
            if (g == p) break;
            p = up[g];
            moved = true;
        }
        if (moved) {
            up[r] = p;
            ch = 1;
        }
    }
    flag_or(flag_next, ch);
}

// the launch counts below are sized from the reach a launch guarantees when every read
// returns the value from the start of the launch (the writer may sit on another XCD): 5x for
// fl_jump's two 2-hop steps, 4x for three doublings; one launch more than convergence needs,
// so its flag is zero unless a chain outran the bound -- then the result is not trusted
__global__ void fl_jump_check(const int *__restrict__ flag_last, int *__restrict__ err) {
    if (threadIdx.x == 0 && *flag_last != 0) atomicOr(err, FE_JUMP);
}

struct NodeArr {
    const int32_t *parent, *top, *esize;
    int32_t *pnode;   // parent node (NONE at the root); only at node ids
    int32_t *nvalid;  // valid (>= mcs) child nodes
    int32_t *vsum;    // their total size
    int64_t m;
    int32_t mcs;
};

__global__ void fl_nodes(NodeArr a) {
    HDB_GRID_STRIDE(r, a.m) {
        if (a.top[r] != (int32_t)r) continue;  // not a node (merged into a heavier tie edge)
        int32_t p = a.parent[r];
        int32_t P = p == NONE ? NONE : a.top[p];
        a.pnode[r] = P;
        if (P != NONE && a.esize[r] >= a.mcs) {
            atomicAdd(&a.nvalid[P], 1);
            atomicAdd(&a.vsum[P], a.esize[r]);
        }
    }
}

// cluster starts: the root, and each valid child of a node with >= 2 valid children
__global__ void fl_starts(const int32_t *__restrict__ top, const int32_t *__restrict__ pnode,
                          const int32_t *__restrict__ esize, const int32_t *__restrict__ nvalid, int64_t m, int32_t mcs,
                          int32_t *__restrict__ is_start, int32_t *__restrict__ cup) {
    HDB_GRID_STRIDE(r, m) {
        int32_t s = 0, u = (int32_t)r;
        if (top[r] == (int32_t)r) {
            int32_t P = pnode[r];
            s = (P == NONE) || (esize[r] >= mcs && nvalid[P] >= 2);
            u = s ? (int32_t)r : P;
        }
        is_start[r] = s;
        cup[r] = u;
    }
}

// stability terms of the reached nodes outside the root cluster, keyed (cluster, -rank)
__global__ void fl_terms(const int32_t *__restrict__ top, const int32_t *__restrict__ pnode,
                         const int32_t *__restrict__ cs, const int32_t *__restrict__ cid,
                         const int32_t *__restrict__ esize, const int32_t *__restrict__ nvalid,
                         const int32_t *__restrict__ vsum, const double *__restrict__ ew, int64_t m, int32_t mcs,
                         uint64_t *__restrict__ key, double *__restrict__ val, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    HDB_GRID_STRIDE(r, m) {
        uint64_t k = ~uint64_t(0);
        double v = 0.0;
        const int32_t root = (int32_t)(m - 1);
        if (top[r] == (int32_t)r && esize[r] >= mcs) {  // reached (the root cluster is skipped)
            const int32_t L = cs[r];
            if (L != root) {
                const double eps = ew[r];
                const double inv_birth = 1.0 / ew[pnode[L]];
                const int32_t nv = nvalid[r];
                int64_t pts = nv == 1 ? (int64_t)esize[r] - vsum[r] : esize[r];
                if (pts > 0) {
                    v = (double)pts * (1.0 / eps - inv_birth);  // Cluster.detachPoints
                    k = ((uint64_t)(uint32_t)cid[L] << 32) | (uint32_t)(m - 1 - r);
                }
            }
        }
        key[r] = k;
        val[r] = v;
    }
}

// ssort functors of the stability terms' order: (cluster, descending level) keys, ties (the
// non-terms' all-ones keys) by position -- the stable radix order
struct TermKeyF {
    const uint64_t *key;
    __device__ SKey operator()(int64_t i) const { return SKey{key[i], (uint64_t)i}; }
};
struct TermEmitF {
    const double *val;
    uint64_t *key_out;
    double *val_out;
    __device__ void operator()(int64_t r, const SKey &k) const {
        key_out[r] = k.hi;
        val_out[r] = val[k.lo];
    }
};

// one wave per cluster: lanes stage the chain's terms through LDS (coalesced, the next chunk
// in flight), lane 0 adds them in order -- the host's sequential sum, descending level
constexpr int STAB_CHUNK = 256;
__global__ __launch_bounds__(64) void fl_stab(const double *__restrict__ val, const int32_t *__restrict__ seg_lo,
                                              const int32_t *__restrict__ seg_hi, const int32_t *__restrict__ Kp,
                                              double *__restrict__ stab, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    __shared__ double buf[STAB_CHUNK];
    const int lane = threadIdx.x;
    const int32_t nc = *Kp;
    for (int32_t c = blockIdx.x; c < nc; c += gridDim.x) {
        const int64_t lo = seg_lo[c], hi = lo < 0 ? -1 : seg_hi[c];
        double s = 0.0;
        double nxt[STAB_CHUNK / 64];
        auto load = [&](int64_t base) {
#pragma unroll
            for (int k = 0; k < STAB_CHUNK / 64; k++) {
                int64_t i = base + k * 64 + lane;
                nxt[k] = i < hi ? val[i] : 0.0;
            }
        };
        if (lo >= 0) load(lo);
        for (int64_t base = lo; lo >= 0 && base < hi; base += STAB_CHUNK) {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < STAB_CHUNK / 64; k++) buf[k * 64 + lane] = nxt[k];
            __syncthreads();
            if (base + STAB_CHUNK < hi) load(base + STAB_CHUNK);  // overlaps lane 0's adds
            if (lane == 0) {
                const int cnt = hi - base < STAB_CHUNK ? (int)(hi - base) : STAB_CHUNK;
                for (int k = 0; k < cnt; k++) s = s + buf[k];
            }
        }
        if (lane == 0) stab[c] = s;
    }
}

__global__ void fl_seg(const uint64_t *__restrict__ key, int64_t m, int32_t *__restrict__ seg_lo,
                       int32_t *__restrict__ seg_hi, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    HDB_GRID_STRIDE(i, m) {
        uint64_t k = key[i];
        if (k == ~uint64_t(0)) continue;
        int32_t c = (int32_t)(k >> 32);
        if (i == 0 || (int32_t)(key[i - 1] >> 32) != c) seg_lo[c] = (int32_t)i;
        if (i == m - 1 || (int32_t)(key[i + 1] >> 32) != c) seg_hi[c] = (int32_t)(i + 1);
    }
}

__global__ void fl_cluster_meta(const int32_t *__restrict__ is_start, const int32_t *__restrict__ cid,
                                const int32_t *__restrict__ cs, const int32_t *__restrict__ pnode,
                                const int32_t *__restrict__ eminid, const int32_t *__restrict__ esize, int64_t m,
                                int32_t *__restrict__ cpar, int32_t *__restrict__ cmin, int32_t *__restrict__ csz,
                                int32_t *__restrict__ Kp, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    HDB_GRID_STRIDE(r, m) {
        if (r == m - 1) *Kp = cid[r] + 1;  // the root (rank m-1) always starts a cluster
        if (!is_start[r]) continue;
        int32_t c = cid[r];
        int32_t P = pnode[r];
        cpar[c] = P == NONE ? -1 : cid[cs[P]];
        cmin[c] = eminid[r];
        csz[c] = esize[r];
    }
}

// ------------------------------------------------------ 5. FOSC over the cluster tree
// (HDBSCANStar.java:567-625 propagateTree / findProminentClusters with flat.cpp step 3's
// canonical rules).  Clusters 0..K-1, a child's id below its parent's, the root K-1.  The
// bottom-up pass contrib(c) = stab(c) if stab(c) >= (sum of the children's contribs, summed
// in ascending smallest point id) else that sum, must reproduce the host's floating-point
// order exactly, so it is never re-associated: the tree is cut into heavy paths (heavy child
// = most points, so a root-leaf path crosses <= log2(n) light edges) and ONE wave walks a
// path bottom-up, the running value in a register, the light children's values already
// final.  A path starts when its last light child path finishes (last-arriver continuation
// inside one launch: no level-synchronous launches).  Selection = the topmost self-selected
// cluster below the root on every chain (pointer jumping); labels 1..K by smallest point id.
__device__ __forceinline__ uint64_t pk(int32_t lo, int32_t hi) { return (uint32_t)lo | ((uint64_t)(uint32_t)hi << 32); }
__device__ __forceinline__ int32_t pk_lo(uint64_t w) { return (int32_t)(uint32_t)w; }
__device__ __forceinline__ int32_t pk_hi(uint64_t w) { return (int32_t)(uint32_t)(w >> 32); }

__global__ void fo_children(const int32_t *__restrict__ cpar, const int32_t *__restrict__ csz,
                            const int32_t *__restrict__ Kp, int32_t *__restrict__ nch,
                            unsigned long long *__restrict__ hkey, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K - 1) {
        const int32_t p = cpar[c];
        if ((uint32_t)p >= (uint32_t)K) continue;  // malformed input (reported by the caller)
        atomicAdd(&nch[p], 1);
        atomicMax(&hkey[p], (unsigned long long)pk((int32_t)c, csz[c]));  // (points, id): heavy child
    }
}

__global__ void fo_kids_fill(const int32_t *__restrict__ cpar, const int32_t *__restrict__ Kp,
                             const int32_t *__restrict__ kstart, int32_t *__restrict__ kcur, int32_t *__restrict__ kids, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K - 1) {
        const int32_t p = cpar[c];
        if ((uint32_t)p >= (uint32_t)K) continue;
        const int32_t slot = kstart[p] + atomicAdd(&kcur[p], 1);
        if (slot < K) kids[slot] = (int32_t)c;
    }
}

// multi-way nodes: children in ascending smallest point id (disjoint clusters: distinct ids);
// heavy-path word: (ancestor, distance) -- a heavy child points to its parent at distance 1
__global__ void fo_paths_init(const int32_t *__restrict__ cpar, const int32_t *__restrict__ cmin,
                              const int32_t *__restrict__ Kp, const int32_t *__restrict__ nch,
                              const unsigned long long *__restrict__ hkey, const int32_t *__restrict__ kstart,
                              int32_t *__restrict__ kids, uint64_t *__restrict__ jw, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K) {
        const int32_t p = c == K - 1 ? -1 : cpar[c];
        const bool heavy = p >= 0 && p < K && pk_lo(hkey[p]) == (int32_t)c;
        jw[c] = heavy ? pk(p, 1) : pk((int32_t)c, 0);
        const int32_t k = nch[c];
        if (k > 2) {  // insertion sort by smallest id (few, small segments)
            int32_t *s = kids + kstart[c];
            for (int32_t i = 1; i < k; i++) {
                const int32_t x = s[i], key = cmin[x];
                int32_t j = i - 1;
                while (j >= 0 && cmin[s[j]] > key) {
                    s[j + 1] = s[j];
                    j--;
                }
                s[j + 1] = x;
            }
        }
    }
}

// pointer jumping over packed (ancestor, accumulated sum) words; a word whose ancestor is
// itself is final.  Words are read and written whole, so a stale read is a valid shorter jump.
__global__ void fo_jump_sum(uint64_t *__restrict__ jw, const int32_t *__restrict__ Kp, const int *__restrict__ flag_prev,
                            int *__restrict__ flag_next, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    if (flag_prev && *flag_prev == 0) return;
    const int32_t K = *Kp;
    int ch = 0;
    HDB_GRID_STRIDE(c, K) {
        uint64_t w = jw[c];
        bool moved = false;
#pragma unroll 1
        for (int it = 0; it < 3; it++) {  // several doublings per launch (fewer launches)
            const int32_t a = pk_lo(w);
            if (a == (int32_t)c) break;
            const uint64_t w2 = jw[a];
            const int32_t a2 = pk_lo(w2);
            if (a2 == a) break;
            w = pk(a2, pk_hi(w) + pk_hi(w2));
            moved = true;
        }
        if (moved) {
            jw[c] = w;
            ch = 1;
        }
    }
    flag_or(flag_next, ch);
}

// per path (top t): length (from its bottom leaf); light-depth word of a top = (top of the
// parent's path, 1), jumped to (root path, number of light edges above it)
__global__ void fo_paths_meta(const int32_t *__restrict__ cpar, const int32_t *__restrict__ Kp,
                              const int32_t *__restrict__ nch, const uint64_t *__restrict__ jw,
                              int32_t *__restrict__ plen, uint64_t *__restrict__ lw, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K) {
        const uint64_t w = jw[c];
        const int32_t top = pk_lo(w);
        if (nch[c] == 0) plen[top] = pk_hi(w) + 1;  // every path ends at exactly one leaf
        lw[c] = top == (int32_t)c && c != K - 1 ? pk(pk_lo(jw[cpar[c]]), 1) : pk((int32_t)c, 0);
    }
}

// path node lists, by position from the top; the deepest light depth
__global__ void fo_paths_nodes(const int32_t *__restrict__ Kp, const uint64_t *__restrict__ jw,
                               const int32_t *__restrict__ poff, const uint64_t *__restrict__ lw,
                               int32_t *__restrict__ nodes, int *__restrict__ maxld, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    int32_t mx = 0;
    HDB_GRID_STRIDE(c, K) {
        const uint64_t w = jw[c];
        const int32_t top = pk_lo(w);
        const int64_t at = (int64_t)poff[top] + pk_hi(w);
        if (at >= 0 && at < K) nodes[at] = (int32_t)c;
        if (top == (int32_t)c) mx = max(mx, pk_hi(lw[c]));
    }
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0 && mx > 0) atomicMax(maxld, mx);
}

// path-ordered node records (cluster, light child / -2 leaf / -1 multi-way, stability), the
// multi-way node list, and a flag on paths holding a multi-way node wider than FO_WIDE
constexpr int FO_CHUNK = 64, FO_SHORT = 48, FO_WIDE = 8;
__global__ void fo_paths_rec(const int32_t *__restrict__ Kp, const int32_t *__restrict__ nodes,
                             const int32_t *__restrict__ nch, const unsigned long long *__restrict__ hkey,
                             const int32_t *__restrict__ kstart, const int32_t *__restrict__ kids,
                             const double *__restrict__ stab, int32_t *__restrict__ rc, int32_t *__restrict__ rl,
                             double *__restrict__ rs, int32_t *__restrict__ mlist, int32_t *__restrict__ mcount,
                             const uint64_t *__restrict__ jw, int32_t *__restrict__ pwide, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    auto top_of = [&](int32_t c) { return pk_lo(jw[c]); };
    HDB_GRID_STRIDE(i, K) {
        const int32_t c = nodes[i];
        const int32_t k = nch[c];
        int32_t lt = -2;
        if (k == 2) {
            const int32_t h = pk_lo(hkey[c]), k0 = kids[kstart[c]], k1 = kids[kstart[c] + 1];
            lt = k0 == h ? k1 : k0;
        } else if (k > 0) {
            lt = -1;
            mlist[atomicAdd(mcount, 1)] = c;
            if (k > FO_WIDE) atomicOr(&pwide[top_of(c)], 1);  // its path runs wave-cooperatively
        }
        rc[i] = c;
        rl[i] = lt;
        rs[i] = stab[c];
    }
}

// paths walked by a whole wave (long, or holding a wide multi-way node), one list for all levels
__global__ void fo_long_list(const int32_t *__restrict__ Kp, const uint64_t *__restrict__ jw,
                             const int32_t *__restrict__ plen, const int32_t *__restrict__ pwide,
                             int32_t *__restrict__ llist, int32_t *__restrict__ lcount, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K) {
        if (pk_lo(jw[c]) == (int32_t)c && (plen[c] > FO_SHORT || pwide[c])) llist[atomicAdd(lcount, 1)] = (int32_t)c;
    }
}

struct FoscArr {
    const int32_t *cpar, *nch, *kstart, *kids, *plen, *poff, *rc, *rl, *Kp, *mlist, *mcount, *pwide, *llist, *lcount;
    const double *rs;
    const uint64_t *jw, *lw;
    const unsigned long long *hkey;
    const int *maxld;
    int32_t *ssel, *hpos;      // hpos: the heavy child's place among a multi-way node's children
    double *cp, *pre, *postv;  // pre: per multi-way node; postv: aligned with kids
};

__device__ __forceinline__ double readlane_d(double x, int l) {  // l: wave-uniform
    const uint64_t u = __builtin_bit_cast(uint64_t, x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int32_t fo_level(const FoscArr &a, int32_t c) { return pk_hi(a.lw[pk_lo(a.jw[c])]); }

// multi-way nodes on the paths of light depth d: their light children are final.  The sum
// before the heavy child (from 0.0, ascending smallest id) is formed here; the values after
// it are staged for the walker, which adds them after the heavy child's value.
__global__ __launch_bounds__(64) void fo_multi_pre(FoscArr a, int d, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    if (d > *a.maxld) return;
    __shared__ double sv[64];
    const int lane = threadIdx.x;
    const int32_t M = *a.mcount;
    for (int32_t j = blockIdx.x; j < M; j += gridDim.x) {
        const int32_t c = a.mlist[j];
        if (fo_level(a, c) != d) continue;
        const int32_t k = a.nch[c], k0 = a.kstart[c], h = pk_lo(a.hkey[c]);
        double s = 0.0;
        int32_t hpos = -1;  // the heavy child's position once seen
        for (int32_t q0 = 0; q0 < k; q0 += 64) {
            const int32_t q = q0 + lane;
            const int32_t x = q < k ? a.kids[k0 + q] : -1;
            const double v = (q < k && x != h) ? a.cp[x] : 0.0;
            const uint64_t hb = __ballot(x == h);
            const int lim = hpos >= 0 ? 0 : (hb ? __ffsll((unsigned long long)hb) - 1 : min(64, k - q0));
            if (hb) hpos = q0 + __ffsll((unsigned long long)hb) - 1;
            if (hpos >= 0 && q > hpos && q < k) a.postv[k0 + q] = v;  // added after the heavy child
            sv[lane] = v;
            __syncthreads();
            if (lane == 0)
                for (int i = 0; i < lim; i++) s = s + sv[i];  // before it, from 0.0
            __syncthreads();
        }
        if (lane == 0) {
            a.pre[c] = s;
            a.hpos[c] = hpos;
        }
    }
}

__device__ __forceinline__ bool fo_nonneg(double x) { return x >= 0.0 && !signbit(x); }

// one node of the chain: the host's additions and comparison, in its order
__device__ __forceinline__ double fo_node(const FoscArr &a, int32_t c, int32_t lt, double st, double lv, double acc,
                                          int32_t &self) {
    double prop;
    if (lt == -2) {
        self = 1;
        return st;
    }
    if (lt >= 0) {
        prop = acc + lv;  // binary: a + b == b + a
    } else {              // multi-way: (sum before the heavy child) + heavy, then the ones after it
        prop = a.pre[c] + acc;
        const int32_t k = a.nch[c], k0 = a.kstart[c];
        for (int32_t q = a.hpos[c] + 1; q < k; q++) prop = prop + a.postv[k0 + q];
    }
    self = st >= prop;  // Cluster.propagate: ties keep the parent
    return self ? st : prop;
}

// paths of light depth d (launched deepest first: a path's light children are final when it
// runs).  Long paths (and paths holding a wide multi-way node) from the list: one wave each,
// 64 records at a time staged in LDS, lane 0 running the chain, the whole wave staging a
// multi-way node's values after its heavy child.  Short paths: one lane each, walking its
// records bottom-up with the next record's loads in flight.
__global__ __launch_bounds__(64) void fo_walk(FoscArr a, int d, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    if (d > *a.maxld) return;
    __shared__ double s_st[FO_CHUNK], s_lv[FO_CHUNK], s_out[FO_CHUNK];
    const int lane = threadIdx.x;
    const int32_t K = *a.Kp, NL = *a.lcount;
    for (int32_t j = blockIdx.x; j < NL; j += gridDim.x) {
        const int32_t t = a.llist[j];
        if (pk_hi(a.lw[t]) != d) continue;
        const int32_t tlen = min(a.plen[t], K), toff = a.poff[t], tstop = t == K - 1 ? 1 : 0;
        double acc = 0.0;  // the running value, the same in every lane
        for (int32_t hi = tlen - 1; hi >= tstop; hi -= FO_CHUNK) {
            const int cnt = min(FO_CHUNK, hi - tstop + 1);
            int32_t c = 0, lt = -2;
            if (lane < cnt) {  // step q of the chunk = the record q above its bottom
                const int32_t i = toff + hi - lane;
                c = a.rc[i];
                lt = a.rl[i];
                s_st[lane] = a.rs[i];
                s_lv[lane] = lt >= 0 ? a.cp[lt] : 0.0;
            }
            const uint64_t multi = __ballot(lane < cnt && lt == -1);
            // every staged value >= +0 (no NaN, no -0.0): then st >= prop ? st : prop == max(st, prop)
            // bit for bit (equal non-negative doubles have equal bits; sums of them stay >= +0)
            const bool clean = __all(lane >= cnt || (fo_nonneg(s_st[lane]) && fo_nonneg(s_lv[lane])));
            __syncthreads();
            int i = 0;
            if (hi == tlen - 1) {  // the path's bottom: a leaf, its own stability
                acc = s_st[0];
                s_out[0] = acc;
                i = 1;
            }
            while (i < cnt) {
                const uint64_t mr = i < 64 ? multi & (~0ull << i) : 0;
                const int e = mr ? min(cnt, __ffsll((unsigned long long)mr) - 1) : cnt;
                int q = i;
                if (clean && fo_nonneg(acc)) {  // two dependent ops per node (add, max) instead of four
                    for (; q + 8 <= e; q += 8) {
                        double st8[8], lv8[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            st8[u] = s_st[q + u];
                            lv8[u] = s_lv[q + u];
                        }
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            acc = fmax(st8[u], acc + lv8[u]);
                            s_out[q + u] = acc;
                        }
                    }
                }
                for (; q + 8 <= e; q += 8) {  // binary nodes: uniform LDS reads ahead of the chain
                    double st8[8], lv8[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        st8[u] = s_st[q + u];
                        lv8[u] = s_lv[q + u];
                    }
#pragma unroll
                    for (int u = 0; u < 8; u++) {
                        const double prop = acc + lv8[u];  // binary: a + b == b + a
                        const bool sq = st8[u] >= prop;    // ties keep the parent
                        acc = sq ? st8[u] : prop;
                        s_out[q + u] = acc;  // self-selected <=> out == st (st >= prop keeps st)
                    }
                }
                for (; q < e; q++) {
                    const double st1 = s_st[q], prop = acc + s_lv[q];
                    const bool sq = st1 >= prop;
                    acc = sq ? st1 : prop;
                    s_out[q] = acc;
                }
                if (e < cnt) {  // a multi-way node: (sum before the heavy child) + heavy + the rest
                    const int32_t cm = __builtin_amdgcn_readlane(c, e);
                    const double stm = s_st[e];
                    const int32_t k = a.nch[cm], k0 = a.kstart[cm];
                    double prop = a.pre[cm] + acc;
                    for (int32_t q0 = a.hpos[cm] + 1; q0 < k; q0 += 64) {
                        const int32_t qq = q0 + lane;
                        const double pv = qq < k ? a.postv[k0 + qq] : 0.0;
                        const int lim = min(64, k - q0);
                        for (int r = 0; r < lim; r++) prop = prop + readlane_d(pv, r);
                    }
                    const bool sm = stm >= prop;
                    acc = sm ? stm : prop;
                    s_out[e] = acc;
                    i = e + 1;
                } else {
                    i = e;
                }
            }
            __syncthreads();
            if (lane < cnt) {
                const double o = s_out[lane];
                a.cp[c] = o;
                // st >= prop kept st; otherwise out = prop != st (or NaN); a leaf always keeps its own
                a.ssel[c] = (o == s_st[lane]) || (lane == 0 && hi == tlen - 1);
            }
            __syncthreads();
        }
    }
    for (int32_t base = blockIdx.x * 64; base < K; base += gridDim.x * 64) {
        const int32_t me = base + lane;
        if (me >= K || pk_lo(a.jw[me]) != me || pk_hi(a.lw[me]) != d) continue;
        const int32_t len = min(a.plen[me], K), off = a.poff[me];
        if (len > FO_SHORT || a.pwide[me]) continue;  // a wave's path
        const int32_t stop = me == K - 1 ? 1 : 0;  // the root's own contribution is never used
        double acc = 0.0;
        int32_t hi = len - 1;
        int32_t c = 0, lt = -2;
        double st = 0.0, lv = 0.0;
        if (hi >= stop) {
            c = a.rc[off + hi];
            lt = a.rl[off + hi];
            st = a.rs[off + hi];
            lv = lt >= 0 ? a.cp[lt] : 0.0;
        }
        for (; hi >= stop; hi--) {
            int32_t c2 = 0, lt2 = -2;
            double st2 = 0.0, lv2 = 0.0;
            if (hi - 1 >= stop) {  // next record in flight while this one is evaluated
                c2 = a.rc[off + hi - 1];
                lt2 = a.rl[off + hi - 1];
                st2 = a.rs[off + hi - 1];
                lv2 = lt2 >= 0 ? a.cp[lt2] : 0.0;
            }
            int32_t self;
            acc = fo_node(a, c, lt, st, lv, acc, self);
            a.cp[c] = acc;
            a.ssel[c] = self;
            c = c2;
            lt = lt2;
            st = st2;
            lv = lv2;
        }
    }
}

// topmost self-selected cluster below the root on each chain: word (ancestor, best); the
// ancestor is the cluster itself once the chain reaches the root's children
__global__ void fo_sel_init(const int32_t *__restrict__ cpar, const int32_t *__restrict__ ssel,
                            const int32_t *__restrict__ Kp, uint64_t *__restrict__ tw, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K) {
        if (c == K - 1) {
            tw[c] = pk((int32_t)c, NONE);
            continue;
        }
        const int32_t p = cpar[c];
        tw[c] = pk(p == K - 1 ? (int32_t)c : p, ssel[c] ? (int32_t)c : NONE);
    }
}

__global__ void fo_sel_jump(uint64_t *__restrict__ tw, const int32_t *__restrict__ Kp, const int *__restrict__ flag_prev,
                            int *__restrict__ flag_next, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    if (flag_prev && *flag_prev == 0) return;
    const int32_t K = *Kp;
    int ch = 0;
    HDB_GRID_STRIDE(c, K) {
        uint64_t w = tw[c];
        bool moved = false;
#pragma unroll 1
        for (int it = 0; it < 3; it++) {  // several doublings per launch (fewer launches)
            const int32_t x = pk_lo(w);
            if (x == (int32_t)c) break;
            const uint64_t w2 = tw[x];
            const int32_t x2 = pk_lo(w2), v2 = pk_hi(w2);
            w = pk(x2 == x ? (int32_t)c : x2, v2 != NONE ? v2 : pk_hi(w));
            moved = true;
        }
        if (moved) {
            tw[c] = w;
            ch = 1;
        }
    }
    flag_or(flag_next, ch);
}

// chosen = its own topmost self-selected ancestor-or-self; mark its smallest point id
__global__ void fo_mark(const uint64_t *__restrict__ tw, const int32_t *__restrict__ cmin, const int32_t *__restrict__ Kp,
                        int32_t *__restrict__ mk, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K - 1) {
        if (pk_hi(tw[c]) == (int32_t)c) mk[cmin[c]] = 1;
    }
}

__global__ void fo_labels(const uint64_t *__restrict__ tw, const int32_t *__restrict__ cmin,
                          const int32_t *__restrict__ rk, const int32_t *__restrict__ Kp, int32_t *__restrict__ clab, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    const int32_t K = *Kp;
    HDB_GRID_STRIDE(c, K) {
        const int32_t v = pk_hi(tw[c]);
        clab[c] = v == NONE ? 0 : rk[cmin[v]] + 1;
    }
}

__global__ void fo_count(const int32_t *__restrict__ mk, const int32_t *__restrict__ rk, int64_t n,
                         int64_t *__restrict__ out, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = (int64_t)rk[n - 1] + mk[n - 1];
}

// labels: a point's node -> its cluster (cs) -> the label of the nearest selected ancestor
// cluster (0 = none)
__global__ void fl_point_labels(const int32_t *__restrict__ pparent, const int32_t *__restrict__ top,
                                const int32_t *__restrict__ cs, const int32_t *__restrict__ cid,
                                const int32_t *__restrict__ clab, int64_t n, int32_t *__restrict__ labels, const int *__restrict__ bad) {
    if (*bad & (FE_CYCLE | FE_ROOTS)) return;  // malformed input: reported by the caller
    HDB_GRID_STRIDE(v, n) labels[v] = clab[cid[cs[top[pparent[v]]]]];
}

// zero-initialised FOSC block: nch, kcur, plen, maxld (+ counters), pwide, a spare (m ints
// each: 24m bytes, so the u64 array after them is 8-byte aligned), hkey (m u64), 192 jump flags
inline size_t fz_layout(int64_t m) { return (size_t)m * 24 + (size_t)m * 8 + 192 * 4; }

inline int grid_for(int64_t count) { return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(count, 256), 16384)); }

struct Carver {
    char *base = nullptr;
    size_t off = 0;
    template <class T>
    T *take(int64_t count) {
        size_t o = off;
        off += ((size_t)std::max<int64_t>(count, 1) * sizeof(T) + 255) & ~size_t(255);
        return base ? (T *)(base + o) : nullptr;
    }
};

}  // namespace

void flat_labels_device(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w, int64_t ne, int64_t n,
                        int32_t mcs, int32_t *labels, int64_t *n_clusters) {
    if (n <= 0) {
        if (n_clusters) *n_clusters = 0;
        return;
    }
    if (mcs < 2) HDB_THROW(HDB_EINVAL, "flat labels: minClSize must be >= 2");
    if (n >= (int64_t(1) << 30)) HDB_THROW(HDB_EINVAL, "flat labels: too many points");
    if (ne < 0) HDB_THROW(HDB_EINVAL, "bad arguments");
    hipStream_t st = ctx->stream;
    KernelTimer tt(ctx, "flat_labels");
    const int64_t m = n - 1;  // a spanning tree has exactly n - 1 non-self edges
    int64_t *pin = pinned_words(ctx) + PINNED_WORDS - 8;  // private slice
    const int64_t mm = std::max<int64_t>(m, 1);
    // vertex labels of the divide and conquer: rank-ordered (2m of them) or the point ids.
    // Contracted labels are nv + rank: < 3m with relabelling (< 2n without, which the n guard
    // above covers), so relabelling needs 3m to fit int32 -- larger inputs keep point ids
    const bool relabel = ctx->flat_relabel && m >= 1 && flat_relabel_fits(m);
    const int64_t nv = relabel ? 2 * mm : n;

    // scratch: sizes are fixed by n and ne
    auto layout = [&](Carver &cv) {
        cv.take<int32_t>(ne);            // keep
        cv.take<int32_t>(ne);            // pos
        cv.take<int32_t>(mm);            // ca
        cv.take<int32_t>(mm);            // cb
        cv.take<double>(mm);             // cw
        cv.take<int64_t>(4);             // m_dev, err, flags
        cv.take<int32_t>(mm);            // ea
        cv.take<int32_t>(mm);            // eb
        cv.take<double>(mm);             // ew
        cv.take<int32_t>(2 * mm);        // lab
        cv.take<LRec>(nv + mm);          // label records
        cv.take<int32_t>(nv + mm);       // stamp
        cv.take<int32_t>(nv);            // orig (relabelled vertices)
        cv.take<int32_t>(mm);            // hooked
        for (int k = 0; k < 3; k++) cv.take<int32_t>(mm);      // parent esize eminid
        cv.take<int32_t>(n);             // pparent
    };
    Carver probe;
    layout(probe);
    Carver cv{(char *)arena(ctx, A_FLAT0, probe.off), 0};
    int32_t *keep = cv.take<int32_t>(ne), *pos = cv.take<int32_t>(ne);
    int32_t *ca = cv.take<int32_t>(mm), *cb = cv.take<int32_t>(mm);
    double *cw = cv.take<double>(mm);
    int64_t *words = cv.take<int64_t>(4);
    int64_t *m_dev = words;
    int *err = (int *)(words + 1), *flags = (int *)(words + 2);
    int32_t *ea = cv.take<int32_t>(mm), *eb = cv.take<int32_t>(mm);
    double *ew = cv.take<double>(mm);
    DC dc;
    dc.lab = cv.take<int32_t>(2 * mm);
    dc.lr = cv.take<LRec>(nv + mm);
    dc.stamp = cv.take<int32_t>(nv + mm);
    int32_t *orig = cv.take<int32_t>(nv);
    dc.hooked = cv.take<int32_t>(mm);
    dc.parent = cv.take<int32_t>(mm);
    dc.esize = cv.take<int32_t>(mm);
    dc.eminid = cv.take<int32_t>(mm);
    int32_t *pparent = cv.take<int32_t>(n);
    dc.n = nv;
    dc.m = m;
    dc.orig = relabel ? orig : nullptr;

    HIP_CHECK(hipMemsetAsync(words, 0, sizeof(int64_t) * 4, st));
    // ---- 1. compact, validate, order
    if (ne > 0) {
        if (ne > INT32_MAX) HDB_THROW(HDB_EINVAL, "too many edges");
        hipLaunchKernelGGL(fl_mark, dim3(grid_for(ne)), dim3(256), 0, st, va, vb, w, ne, n, keep, err);
        size_t tb = 0;
        HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, keep, pos, 0, (size_t)ne, rocprim::plus<int32_t>(), st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(rocprim::exclusive_scan(tmp, tb, keep, pos, 0, (size_t)ne, rocprim::plus<int32_t>(), st));
        hipLaunchKernelGGL(fl_compact, dim3(grid_for(ne)), dim3(256), 0, st, va, vb, w, ne, keep, pos, m, ca, cb, cw,
                           m_dev);
        // a descending list sets bit 1 in every workgroup: few workgroups, few same-address atomics
        hipLaunchKernelGGL(fl_order, dim3((unsigned)std::min<int64_t>(grid_for(ne) / 4 + 1, 256)), dim3(1024), 0, st,
                           cw, m_dev, flags);
    }
    HIP_CHECK(hipMemcpyAsync(pin, words, sizeof(int64_t) * 3, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const int64_t m_got = pin[0];
    const int e0 = (int)pin[1], order = (int)pin[2];
    if (e0 & FE_RANGE) HDB_THROW(HDB_EINVAL, "flat labels: vertex id out of range");
    if (e0 & FE_NAN) HDB_THROW(HDB_EINVAL, "flat labels: NaN edge weight");
    if (m_got != m) HDB_THROW(HDB_EINVAL, "flat labels: the edges are not a spanning tree");
    if (m == 0) {  // one point: no hierarchy below the root
        HIP_CHECK(hipMemsetAsync(labels, 0, sizeof(int32_t), st));
        if (n_clusters) *n_clusters = 0;
        return;
    }
    const int g = grid_for(m);
    const int32_t *perm = nullptr;
    int desc = !(order & 1);
    if (desc == 0 && (order & 2)) {  // neither ascending nor descending: radix sort by weight
        Carver sp;
        sp.take<double>(m);
        sp.take<double>(m);
        sp.take<int32_t>(m);
        sp.take<int32_t>(m);
        Carver sc{(char *)arena(ctx, A_FLAT1, sp.off), 0};
        double *k1 = sc.take<double>(m), *k2 = sc.take<double>(m);
        int32_t *i1 = sc.take<int32_t>(m), *i2 = sc.take<int32_t>(m);
        hipLaunchKernelGGL(fl_sort_keys, dim3(g), dim3(256), 0, st, cw, m, k1, i1);
        size_t tb = 0;
        HIP_CHECK(sort_pairs(nullptr, tb, k1, k2, i1, i2, m, 0, 64, st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(sort_pairs(tmp, tb, k1, k2, i1, i2, m, 0, 64, st));
        perm = i2;
    }
    hipLaunchKernelGGL(fl_rank, dim3(g), dim3(256), 0, st, ca, cb, cw, m, desc, perm, ea, eb, ew, dc.lab, dc.parent);
    hipLaunchKernelGGL(fill_i32, dim3(grid_for(nv + m)), dim3(256), 0, st, dc.stamp, nv + m, -1);
    hipLaunchKernelGGL(fill_i32, dim3(grid_for(n)), dim3(256), 0, st, pparent, n, NONE);
    hipLaunchKernelGGL(fl_point_parent, dim3(g), dim3(256), 0, st, ea, eb, m, pparent);
    if (relabel) {
        hipLaunchKernelGGL(fl_relabel_orig, dim3(grid_for(n)), dim3(256), 0, st, pparent, eb, n, orig);
        hipLaunchKernelGGL(fl_relabel, dim3(g), dim3(256), 0, st, ea, eb, pparent, m, dc.lab);
    }

    // ---- 2. Kruskal tree by rank divide and conquer
    int J = 0;
    while ((int64_t(1) << J) <= m) J++;  // 2^J > m: every rank < m has a clear bit below J
    // global depths split blocks down to 2^LB ranks; dc_block (dc_local) finishes each such block
    const int LB = ctx->flat_block_log >= 8 && ctx->flat_block_log <= 10 ? ctx->flat_block_log : LOC_LOG;
    // depths LM-1 .. LB per workgroup (dc_mid), the shallower ones global
    const int LM = ctx->flat_mid_log > LB ? std::max(LB, std::min(ctx->flat_mid_log, J)) : LB;
    for (int j = 0; j < J - LM; j++) {
        const int b = J - 1 - j;
        // L ranks (bit b clear) below m; every U rank is an L rank + 2^b
        const int64_t blk = int64_t(1) << (b + 1), half = int64_t(1) << b;
        const int64_t nl = (m / blk) * half + std::min(m % blk, half);
        const int gl = grid_for(nl);
        hipLaunchKernelGGL(dc_init, dim3(gl), dim3(256), 0, st, dc, b, j, nl);
        hipLaunchKernelGGL(dc_unite, dim3(gl), dim3(256), 0, st, dc, b, nl, err);
        // deep depths: small components, no hot records -- the per-workgroup LDS tables only
        // cost occupancy (the multi-batch kernels run nl / 4096 workgroups)
        const bool deep = j >= ctx->flat_deep_depth;
        switch (deep ? ctx->flat_deep_root : ctx->flat_root_variant) {
        case 1: hipLaunchKernelGGL((dc_root<1024, 4096>), dim3((unsigned)ceil_div(nl, 1024)), dim3(1024), 0, st, dc, b, j, nl); break;
        case 2: hipLaunchKernelGGL(dc_root_direct, dim3(gl), dim3(256), 0, st, dc, b, j, nl); break;
        case 3: hipLaunchKernelGGL((dc_root_multi<1024, 4096, 4>), dim3((unsigned)ceil_div(nl, 4096)), dim3(1024), 0, st, dc, b, j, nl); break;
        case 4: hipLaunchKernelGGL((dc_root_multi<1024, 8192, 4>), dim3((unsigned)ceil_div(nl, 4096)), dim3(1024), 0, st, dc, b, j, nl); break;
        case 5: hipLaunchKernelGGL((dc_root_multi<512, 4096, 4>), dim3((unsigned)ceil_div(nl, 2048)), dim3(512), 0, st, dc, b, j, nl); break;
        default: hipLaunchKernelGGL((dc_root<ROOT_TB, ROOT_SLOTS>), dim3(gl), dim3(ROOT_TB), 0, st, dc, b, j, nl);
        }
        if ((deep ? ctx->flat_deep_link : ctx->flat_link_variant) == 1)
            hipLaunchKernelGGL((dc_link_multi<1024, 8192, 2>), dim3((unsigned)ceil_div(nl, 2048)), dim3(1024), 0, st, dc,
                               b, j, nl);
        else
            hipLaunchKernelGGL(dc_link, dim3(gl), dim3(256), 0, st, dc, b, j, nl);
    }
    if (LM > LB)
        hipLaunchKernelGGL(dc_mid<1024>, dim3((unsigned)ceil_div(m, int64_t(1) << LM)), dim3(1024), 0, st, dc, J, LM, LB,
                           err);
    const unsigned nblk = (unsigned)std::min<int64_t>(ceil_div(m, int64_t(1) << LB), 65536);
    switch (ctx->flat_block_log) {
    case 8: hipLaunchKernelGGL((dc_block<8, 128>), dim3(nblk), dim3(128), 0, st, dc, err); break;
    case 9: hipLaunchKernelGGL((dc_block<9, 256>), dim3(nblk), dim3(256), 0, st, dc, err); break;
    case 10: hipLaunchKernelGGL((dc_block<10, 512>), dim3(nblk), dim3(512), 0, st, dc, err); break;
    default: hipLaunchKernelGGL(dc_local, dim3(nblk), dim3(64), 0, st, dc, err);
    }

    // ---- 3. multi-way nodes, condensation
    // reuse the union-find scratch (n + m ints each) for the node arrays
    int32_t *top = (int32_t *)dc.lr, *pnode = top + (n + m), *nvalid = pnode + (n + m), *vsum = nvalid + (n + m),
            *is_start = dc.stamp;
    Carver nc2{nullptr, 0};
    nc2.take<int32_t>(m);  // cup / cs
    nc2.take<int32_t>(m);  // cid
    nc2.take<uint64_t>(m);
    nc2.take<uint64_t>(m);
    nc2.take<double>(m);
    nc2.take<double>(m);
    nc2.take<int32_t>(m);  // seg
    nc2.take<double>(m);   // stab
    nc2.take<int32_t>(m);  // cpar
    nc2.take<int32_t>(m);  // cminid
    nc2.take<int32_t>(m);  // clab
    nc2.take<int32_t>(64);  // jump flags
    nc2.take<int64_t>(1);  // cluster count
    for (int k = 0; k < 11; k++) nc2.take<int32_t>(m);  // csz kstart kids pnodes poff ssel Kp rc rl mlist llist
    for (int k = 0; k < 7; k++) nc2.take<uint64_t>(m);  // jw tw cpv lw rs mpre postv
    nc2.take<char>(fz_layout(m));                        // zeroed block
    nc2.take<int32_t>(n);                                // mk
    nc2.take<int32_t>(n);                                // rk
    Carver cv2{(char *)arena(ctx, A_FLAT1, nc2.off), 0};
    int32_t *cs = cv2.take<int32_t>(m), *cid = cv2.take<int32_t>(m);
    uint64_t *key1 = cv2.take<uint64_t>(m), *key2 = cv2.take<uint64_t>(m);
    double *val1 = cv2.take<double>(m), *val2 = cv2.take<double>(m);
    int32_t *seg = cv2.take<int32_t>(m);
    double *stab = cv2.take<double>(m);
    int32_t *cpar = cv2.take<int32_t>(m), *cminid = cv2.take<int32_t>(m), *clab = cv2.take<int32_t>(m);
    int *jflags = cv2.take<int32_t>(64);
    cv2.take<int64_t>(1);
    int32_t *csz = cv2.take<int32_t>(m), *kstart = cv2.take<int32_t>(m), *kids = cv2.take<int32_t>(m),
            *pnodes = cv2.take<int32_t>(m), *poff = cv2.take<int32_t>(m),
            *ssel = cv2.take<int32_t>(m), *Kp = cv2.take<int32_t>(m), *rc = cv2.take<int32_t>(m),
            *rl = cv2.take<int32_t>(m), *mlist = cv2.take<int32_t>(m), *llist = cv2.take<int32_t>(m);
    uint64_t *jw = cv2.take<uint64_t>(m), *tw = cv2.take<uint64_t>(m);
    double *cpv = cv2.take<double>(m);
    uint64_t *lw = cv2.take<uint64_t>(m);
    double *rs = cv2.take<double>(m), *mpre = cv2.take<double>(m), *postv = cv2.take<double>(m);
    char *fz = cv2.take<char>(fz_layout(m));
    const size_t fz_bytes = fz_layout(m);
    int32_t *nch = (int32_t *)fz, *kcur = nch + m, *plen = kcur + m, *maxld = plen + m;  // (m ints)
    int32_t *mcount = maxld + 1, *lcount = maxld + 2, *pwide = maxld + m;
    unsigned long long *hkey = (unsigned long long *)(pwide + 2 * m);
    int *ffl = (int *)(hkey + m);  // 192 jump flags
    int32_t *mk = cv2.take<int32_t>(n), *rk = cv2.take<int32_t>(n);
    // guaranteed reach 5x per fl_jump launch (see fl_jump_check): ceil(log5 m) launches + one
    int rounds = 2;
    for (int64_t span = 5; span < m; span *= 5) rounds++;
    rounds = std::min(rounds, 64);
    // pointer-jumping grids (grid-stride): most launches only see the previous launch's zero
    // flag and return, so a grid of at most HDB_JUMP_WG workgroups (0: one element per thread;
    // 256: jump kernels 303 -> 265 us per C2 partition, profiles/r06/jump/)
#ifndef HDB_JUMP_WG
#define HDB_JUMP_WG 256
#endif
    const unsigned jump_wg = (unsigned)(HDB_JUMP_WG > 0 ? std::min<int64_t>(g / 4 + 1, HDB_JUMP_WG) : g / 4 + 1);
    auto jump_all = [&](int32_t *up) {  // roots of an upward forest, in place
        HIP_CHECK(hipMemsetAsync(jflags, 0, sizeof(int) * 64, st));
        for (int k = 0; k < rounds; k++)
            hipLaunchKernelGGL(fl_jump, dim3(jump_wg), dim3(1024), 0, st, up, m, k ? jflags + k - 1 : nullptr,
                               jflags + k);
        hipLaunchKernelGGL(fl_jump_check, dim3(1), dim3(64), 0, st, jflags + rounds - 1, err);
    };

    hipLaunchKernelGGL(fl_tie_up, dim3(g), dim3(256), 0, st, dc.parent, ew, m, top, err);
    jump_all(top);
    HIP_CHECK(hipMemsetAsync(nvalid, 0, sizeof(int32_t) * m, st));
    HIP_CHECK(hipMemsetAsync(vsum, 0, sizeof(int32_t) * m, st));
    NodeArr na{dc.parent, top, dc.esize, pnode, nvalid, vsum, m, mcs};
    hipLaunchKernelGGL(fl_nodes, dim3(g), dim3(256), 0, st, na);
    hipLaunchKernelGGL(fl_starts, dim3(g), dim3(256), 0, st, top, pnode, dc.esize, nvalid, m, mcs, is_start, cs);
    jump_all(cs);
    {
        size_t tb = 0;
        HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, is_start, cid, 0, (size_t)m, rocprim::plus<int32_t>(), st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(rocprim::exclusive_scan(tmp, tb, is_start, cid, 0, (size_t)m, rocprim::plus<int32_t>(), st));
    }
    // ---- 4. stabilities: chains grouped by cluster, descending level inside.  The cluster
    // count K stays on the device (no host round trip): kernels read it, and the key width
    // is bounded by m (the same number of radix passes at every K of this size)
    hipLaunchKernelGGL(fl_terms, dim3(g), dim3(256), 0, st, top, pnode, cs, cid, dc.esize, nvalid, vsum, ew, m, mcs,
                       key1, val1, err);
    int kb = 0;
    while ((int64_t(1) << kb) < m + 1) kb++;
    const SsPlan tpl = ss_plan(m, ctx->ssort_cap);
    if (ctx->ssort && tpl.nb) {  // the terms' keys are unique (rank in the low word); non-terms last
        ssort(tpl, (char *)arena(ctx, A_SS, tpl.bytes), TermKeyF{key1}, TermEmitF{val1, key2, val2}, st);
    } else {
        size_t tb = 0;
        // keys of non-terms are all-ones: sorting on the cluster bits + 32 keeps them last
        HIP_CHECK(sort_pairs(nullptr, tb, key1, key2, val1, val2, m, 0, 64, st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(sort_pairs(tmp, tb, key1, key2, val1, val2, m, 0, std::min(64, 32 + kb + 1), st));
    }
    int32_t *seg_hi = (int32_t *)key1;  // key1 is free after the sort
    hipLaunchKernelGGL(fill_i32, dim3(g), dim3(256), 0, st, seg, m, -1);
    hipLaunchKernelGGL(fl_seg, dim3(g), dim3(256), 0, st, key2, m, seg, seg_hi, err);
    hipLaunchKernelGGL(fl_cluster_meta, dim3(g), dim3(256), 0, st, is_start, cid, cs, pnode, dc.eminid, dc.esize, m,
                       cpar, cminid, csz, Kp, err);
    hipLaunchKernelGGL(fl_stab, dim3((int)std::min<int64_t>(m, 16384)), dim3(64), 0, st, val2, seg, seg_hi, Kp, stab, err);

    // ---- 5. FOSC on the device (heavy-path walkers), selection, labels
    // three doublings per launch: guaranteed reach 4x per launch under stale reads (8x when the
    // reads see this launch's writes); ceil(log4 m) launches + one, checked
    int jrounds = 2;
    for (int64_t span = 4; span < m; span *= 4) jrounds++;
    jrounds = std::min(jrounds, 64);
    auto jump64 = [&](auto kern, uint64_t *wd, int *flags) {  // flags: jrounds ints, zeroed below
        for (int k = 0; k < jrounds; k++)
            hipLaunchKernelGGL(kern, dim3(jump_wg), dim3(1024), 0, st, wd, Kp, k ? flags + k - 1 : nullptr, flags + k, err);
        hipLaunchKernelGGL(fl_jump_check, dim3(1), dim3(64), 0, st, flags + jrounds - 1, err);
    };
    // zero: nch, kcur, plen, maxld, hkey (contiguous) and the jump flags
    HIP_CHECK(hipMemsetAsync(fz, 0, fz_bytes, st));
    hipLaunchKernelGGL(fo_children, dim3(g), dim3(256), 0, st, cpar, csz, Kp, nch, hkey, err);
    {
        size_t tb = 0;
        HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, nch, kstart, 0, (size_t)m, rocprim::plus<int32_t>(), st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(rocprim::exclusive_scan(tmp, tb, nch, kstart, 0, (size_t)m, rocprim::plus<int32_t>(), st));
    }
    hipLaunchKernelGGL(fo_kids_fill, dim3(g), dim3(256), 0, st, cpar, Kp, kstart, kcur, kids, err);
    hipLaunchKernelGGL(fo_paths_init, dim3(g), dim3(256), 0, st, cpar, cminid, Kp, nch, hkey, kstart, kids, jw, err);
    jump64(fo_jump_sum, jw, ffl);
    hipLaunchKernelGGL(fo_paths_meta, dim3(g), dim3(256), 0, st, cpar, Kp, nch, jw, plen, lw, err);
    jump64(fo_jump_sum, lw, ffl + 128);
    {
        size_t tb = 0;
        HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, plen, poff, 0, (size_t)m, rocprim::plus<int32_t>(), st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(rocprim::exclusive_scan(tmp, tb, plen, poff, 0, (size_t)m, rocprim::plus<int32_t>(), st));
    }
    hipLaunchKernelGGL(fo_paths_nodes, dim3(g), dim3(256), 0, st, Kp, jw, poff, lw, pnodes, maxld, err);
    hipLaunchKernelGGL(fo_paths_rec, dim3(g), dim3(256), 0, st, Kp, pnodes, nch, hkey, kstart, kids, stab, rc, rl, rs,
                       mlist, mcount, jw, pwide, err);
    hipLaunchKernelGGL(fo_long_list, dim3(g), dim3(256), 0, st, Kp, jw, plen, pwide, llist, lcount, err);
    FoscArr fa{cpar, nch, kstart, kids, plen, poff, rc, rl, Kp, mlist, mcount, pwide, llist, lcount, rs, jw, lw, hkey,
               maxld, ssel, csz /* free after fo_children: heavy positions */, cpv, mpre, postv};
    // a light child has at most half its parent's points: light depth <= log2(n)
    int dmax = 0;
    while ((int64_t(1) << (dmax + 1)) <= n) dmax++;
    for (int d = dmax; d >= 0; d--) {
        hipLaunchKernelGGL(fo_multi_pre, dim3(1024), dim3(64), 0, st, fa, d, err);
        hipLaunchKernelGGL(fo_walk, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(m, 64), 8192))),
                           dim3(64), 0, st, fa, d, err);
    }
    hipLaunchKernelGGL(fo_sel_init, dim3(g), dim3(256), 0, st, cpar, ssel, Kp, tw, err);
    jump64(fo_sel_jump, tw, ffl + 64);
    HIP_CHECK(hipMemsetAsync(mk, 0, sizeof(int32_t) * n, st));
    hipLaunchKernelGGL(fo_mark, dim3(g), dim3(256), 0, st, tw, cminid, Kp, mk, err);
    {
        size_t tb = 0;
        HIP_CHECK(rocprim::exclusive_scan(nullptr, tb, mk, rk, 0, (size_t)n, rocprim::plus<int32_t>(), st));
        void *tmp = arena(ctx, A_FLAT_TMP, tb);
        HIP_CHECK(rocprim::exclusive_scan(tmp, tb, mk, rk, 0, (size_t)n, rocprim::plus<int32_t>(), st));
    }
    hipLaunchKernelGGL(fo_labels, dim3(g), dim3(256), 0, st, tw, cminid, rk, Kp, clab, err);
    hipLaunchKernelGGL(fo_count, dim3(1), dim3(64), 0, st, mk, rk, n, (int64_t *)(words + 3), err);
    hipLaunchKernelGGL(fl_point_labels, dim3(grid_for(n)), dim3(256), 0, st, pparent, top, cs, cid, clab, n,
                       labels, err);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(pin, words, sizeof(int64_t) * 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(pin + 4, Kp, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    const int e1 = (int)pin[1];
    if (e1 & FE_CYCLE) HDB_THROW(HDB_EINVAL, "flat labels: the edges contain a cycle");
    if (e1 & FE_ROOTS) HDB_THROW(HDB_EINVAL, "flat labels: the edges are not a spanning tree");
    if (e1 & FE_JUMP) HDB_THROW(HDB_EDEVICE, "flat labels: pointer jumping did not converge in its launch budget");
    if (n_clusters) *n_clusters = pin[3];
    ctx->stats["flat_clusters_total"] = *(int32_t *)(pin + 4);  // condensed-tree clusters incl. the root
}

}  // namespace hdb
