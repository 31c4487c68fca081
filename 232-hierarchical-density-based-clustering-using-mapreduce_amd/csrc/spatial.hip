// spatial.hip -- the Morton-ordered tile/BVH index over a partition and the two exact
// traversals that use it:
//   K1t  knn_tree_kernel    -- per-point k smallest distances (core distances, a3/a4) with
//                              box pruning instead of all n^2 pairs;
//   K2b  boruvka_bvh_kernel -- exact MST of the mutual-reachability graph (a5) for graphs
//                              too large for the step-serial Prim (config 2: one 1M graph).
//
// K1t contract: lists bit-identical to K1 (knn.hip).  Every evaluated pair uses the same
// FP64 expression in the reference's operation order (EuclideanDistance.java:31-33), and a
// subtree is skipped only when its box lower bound lb satisfies lb >= the lane's current
// K-th smallest squared distance.  With correctly rounded, monotone operations the computed
// squared distance of any point in the box is >= the computed lb (|fl(c-x)| >= fl(a-x) for
// c beyond the face a, squares and sums are monotone), so a skipped pair could never pass
// the strict '<' insertion test (HDBSCANStar.java:89).  The kept values form the same
// multiset as the brute-force scan's, independent of visit order.
//
// K2b contract: an MST under the strict total order (w, s, min id, max id) on edges, with
// w = max(sqrt(s), core_p, core_q) computed with exactly the reference Prim's expression
// (HDBSCANStar.java:162-168) and s the squared distance (see Best below).  Every MST has the same sorted weight sequence, so the
// weights equal the reference Prim's bit-for-bit; the topology may differ from Prim's only
// among equal-weight edges (Prim breaks ties by scan order).  Edges are returned sorted by
// (w, min id, max id).
//
// Layout: points are sorted by a Morton key over (up to) the first 8 dimensions, cut into
// 64-point tiles with a per-tile bounding box; tiles are the leaves of a fan-8 BVH whose
// node boxes are fixed and whose per-round "uniform component" tags drive K2b.  A wave owns
// one query tile (lane = point) and walks the BVH nearest-first with a wave-uniform stack in
// LDS, descending into a node only when some lane still needs it.  For K2b the bound is
// min(own best, the component's best so far), the latter read from the per-round component
// minimum that other waves publish with atomicMin (a stale read only weakens the bound,
// never prunes a winner: pruning needs LB > bound strictly).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "internal.hpp"
#include "sort.hpp"
#include "ssort.hpp"

namespace hdb {

constexpr int BT = 64;  // tile size (one wave)
#ifndef CAND_UNROLL
#define CAND_UNROLL 2  // candidate-loop unroll: LDS-broadcast latency vs VGPRs (occupancy)
#endif

template <int D>
struct Rec {
    double x[D];
    double core;
    int32_t comp;
    int32_t id;
};

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }

// A leaf tile staged in LDS: one coalesced vector load (lane l fetches record l of the tile),
// then every candidate is a broadcast LDS read at a wave-uniform address.  Replaces one
// dependent scalar load per candidate (the scalar cache serialises a leaf into many round
// trips); 16-B aligned rows so a record is a few ds_read_b128.
template <int D>
struct alignas(16) LRec {
    double x[D];
    double core;
    int32_t comp;
    int32_t id;
};

template <int D>
__device__ __forceinline__ LRec<D> fetch_rec(const Rec<D> *__restrict__ recs, int64_t n, int64_t q) {
    LRec<D> r;
    if (q < n) {
        const Rec<D> g = recs[q];
#pragma unroll
        for (int c = 0; c < D; c++) r.x[c] = g.x[c];
        r.core = g.core;
        r.comp = g.comp;
        r.id = g.id;
    } else {
#pragma unroll
        for (int c = 0; c < D; c++) r.x[c] = 0;
        r.core = 0;
        r.comp = -5;
        r.id = -5;
    }
    return r;
}

// XCD-interleaved chunks (round 6, K1t and the K2b scan; xcb > 0): the dispatcher deals blocks to the 8 XCDs round
// robin (b and b + 8 share one; placement affects only speed), so block b runs logical block
// ((q * 8) + b % 8) * xcb + o with (q, o) = divmod(b / 8, xcb): every XCD works through chunks of
// xcb consecutive blocks (4 * xcb Morton-consecutive tiles), chunks dealt round robin -- a
// tile's neighbour tiles are mostly fetched by the same XCD (its L2) while dense and sparse
// regions still spread over all XCDs (round 5's eight contiguous ranges did not).  The grid is a
// multiple of 8 * xcb (the map is then a bijection); blocks past the tiles exit.
__device__ __forceinline__ int64_t xcd_chunk_block(int64_t b, int64_t xcb) {
    if (xcb <= 0) return b;
    const int64_t j = b >> 3, q = j / xcb, o = j - q * xcb;
    return ((q << 3) + (b & 7)) * xcb + o;
}
// ---------------------------------------------------------------- morton
// bounding box of X: per-block partial min/max over rows (fmin/fmax ignore NaN), then one
// block folds the partials
constexpr int BBOX_BLOCKS = 1024;
template <int D>
__global__ __launch_bounds__(256) void bbox_partial_kernel(const double *__restrict__ X, int64_t n,
                                                           double *__restrict__ part) {
    double l[D], h[D];
#pragma unroll
    for (int c = 0; c < D; c++) {
        l[c] = INFINITY;
        h[c] = -INFINITY;
    }
    HDB_GRID_STRIDE(i, n) {
#pragma unroll
        for (int c = 0; c < D; c++) {
            const double v = X[i * D + c];
            l[c] = fmin(l[c], v);
            h[c] = fmax(h[c], v);
        }
    }
    __shared__ double sl[4][D], sh[4][D];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int c = 0; c < D; c++) {
        for (int off = 32; off >= 1; off >>= 1) {
            l[c] = fmin(l[c], __shfl_xor(l[c], off));
            h[c] = fmax(h[c], __shfl_xor(h[c], off));
        }
        if (lane == 0) {
            sl[w][c] = l[c];
            sh[w][c] = h[c];
        }
    }
    __syncthreads();
    if (threadIdx.x < D) {
        const int c = threadIdx.x;
        double a = fmin(fmin(sl[0][c], sl[1][c]), fmin(sl[2][c], sl[3][c]));
        double b = fmax(fmax(sh[0][c], sh[1][c]), fmax(sh[2][c], sh[3][c]));
        part[(int64_t)blockIdx.x * 2 * D + c] = a;
        part[(int64_t)blockIdx.x * 2 * D + D + c] = b;
    }
}
template <int D>
__global__ void bbox_final_kernel(const double *__restrict__ part, int nb, double *__restrict__ lo,
                                  double *__restrict__ hi) {
    // one wave per dimension
    const int c = blockIdx.x;
    double l = INFINITY, h = -INFINITY;
    for (int k = threadIdx.x; k < nb; k += 64) {
        l = fmin(l, part[(int64_t)k * 2 * D + c]);
        h = fmax(h, part[(int64_t)k * 2 * D + D + c]);
    }
    for (int off = 32; off >= 1; off >>= 1) {
        l = fmin(l, __shfl_xor(l, off));
        h = fmax(h, __shfl_xor(h, off));
    }
    if (threadIdx.x == 0) {
        lo[c] = l;
        hi[c] = h;
    }
}

// Morton bits per dimension: at most 16 (65,536 cells per axis is far below the point
// spacing that matters for 64-point tiles) so the key sort runs 48 bits (6 onesweep passes)
// instead of 63 (8).  The order only shapes the index; every result is order-independent.
__host__ __device__ inline int morton_bits(int d) {
    const int dk = d < 8 ? d : 8;
    const int b = 63 / dk;
    return b > 16 ? 16 : b;
}

__device__ __forceinline__ uint64_t morton_key(const double *__restrict__ x, int d, const double *__restrict__ lo,
                                               const double *__restrict__ hi) {
    const int dk = d < 8 ? d : 8;
    const int bits = morton_bits(d);
    uint64_t key = 0;
    uint32_t q[8];
    for (int c = 0; c < dk; c++) {
        double span = hi[c] - lo[c];
        double t = span > 0 ? (x[c] - lo[c]) / span : 0.0;
        t = t < 0 ? 0 : (t > 1 ? 1 : t);
        if (t != t) t = 0;
        q[c] = (uint32_t)(t * (double)((1u << bits) - 1));
    }
    for (int b = bits - 1; b >= 0; b--)
        for (int c = 0; c < dk; c++) key = (key << 1) | ((q[c] >> b) & 1u);
    return key;
}

__global__ void morton_kernel(const double *__restrict__ X, int64_t n, int d, const double *__restrict__ lo,
                              const double *__restrict__ hi, uint64_t *__restrict__ keys, int32_t *__restrict__ iota) {
    HDB_GRID_STRIDE(i, n) {
        keys[i] = morton_key(X + i * d, d, lo, hi);
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
        r.core = core ? core[o] : 0.0;
        r.comp = (int32_t)i;
        r.id = o;
        recs[i] = r;
        inv[o] = (int32_t)i;
    }
}

// ssort functors of the index build (the Morton order, ties by input position) and of the
// record build fused into the sort's last kernel (build_recs_kernel's output)
template <int D>
struct MortonKeyF {
    const double *X;
    const double *lo, *hi;
    __device__ SKey operator()(int64_t i) const { return SKey{morton_key(X + i * D, D, lo, hi), (uint64_t)i}; }
};
template <int D>
struct RecEmitF {
    const double *X;
    const double *core;
    Rec<D> *recs;
    int32_t *inv;
    __device__ void operator()(int64_t r, const SKey &k) const {
        const int32_t o = (int32_t)k.lo;
        Rec<D> rec;
        for (int c = 0; c < D; c++) rec.x[c] = X[(int64_t)o * D + c];
        rec.core = core ? core[o] : 0.0;
        rec.comp = (int32_t)r;
        rec.id = o;
        recs[r] = rec;
        inv[o] = (int32_t)r;
    }
};

// Tile boxes (coordinates fixed) and uniform-component tags (per round).  Each 64-point
// tile is also cut into 4 sub-groups of SG = 16 consecutive points with their own box and
// tag: a leaf visit skips a sub-group no lane needs (finer culling, same wave shape).
constexpr int SG = 16;
constexpr int NSG = BT / SG;
#ifndef HDB_K1T_WPE  // waves per EU the D <= 3 K1t is compiled for (82 VGPRs free-running: 5)
#define HDB_K1T_WPE 5
#endif
#ifndef HDB_BOR_WPE  // waves per EU the D <= 3 Boruvka scan is compiled for
#define HDB_BOR_WPE 4
#endif

template <int D>
__global__ void tile_box_kernel(const Rec<D> *__restrict__ recs, int64_t n, double *__restrict__ tlo,
                                double *__restrict__ thi, double *__restrict__ slo, double *__restrict__ shi) {
    const int64_t t = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t i = t * BT + lane;
    for (int c = 0; c < D; c++) {
        double v = i < n ? recs[i].x[c] : NAN;
        double l = i < n ? v : INFINITY, h = i < n ? v : -INFINITY;
        for (int off = SG / 2; off >= 1; off >>= 1) {
            l = fmin(l, __shfl_xor(l, off));
            h = fmax(h, __shfl_xor(h, off));
        }
        if ((lane & (SG - 1)) == 0) {
            slo[(t * NSG + lane / SG) * D + c] = l;
            shi[(t * NSG + lane / SG) * D + c] = h;
        }
        for (int off = BT / 2; off >= SG; off >>= 1) {
            l = fmin(l, __shfl_xor(l, off));
            h = fmax(h, __shfl_xor(h, off));
        }
        if (lane == 0) {
            tlo[t * D + c] = l;
            thi[t * D + c] = h;
        }
    }
}

// --------------------------------------------------------------- scan
// Edge order for K2b: (w, s, lo, hi) -- mutual-reachability weight, then the squared
// Euclidean distance s (bitwise symmetric: (a-b)^2 == (b-a)^2 in the same dimension
// order), then the ids.  A strict total order on edges, so Boruvka is exact; its primary
// key is w, so the tree is a minimum spanning tree by weight.  The secondary key s makes
// weight ties cheap: a lane whose best weight already equals its own core distance (the
// smallest weight any of its edges can have) needs only candidates with s <= best s, so
// its search radius shrinks to its nearest tied neighbour instead of the whole core ball.
struct Best {
    double w, s;
    int32_t lo, hi;  // original ids
};
__device__ __forceinline__ bool key_less(double w, double s, int32_t lo, int32_t hi, const Best &b) {
    if (w < b.w) return true;
    if (w > b.w) return false;
    if (s < b.s) return true;
    if (s > b.s) return false;
    if (lo != b.lo) return lo < b.lo;
    return hi < b.hi;
}

// BVH over the Morton-ordered tiles: level 0 = tiles (64 points), level L node i covers
// level L-1 nodes 8i .. 8i+7.  Node boxes are fixed; node component tags (uniform
// component id or -1) are rebuilt every round.  slo/shi/stag: the tiles' 16-point groups.
constexpr int FAN = 8;
constexpr int MAXLEV = 12;
struct Bvh {
    double *lo, *hi;      // [total_nodes][D]
    int32_t *tag;         // [total_nodes]
    double *slo, *shi;    // [ntiles * NSG][D]
    int32_t *stag;        // [ntiles * NSG]
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

// lane lower bound (squared) from point x to a box.  Monotone rounding makes it a true
// lower bound of the computed squared distance of every point in the box (see header).
// All 2D box values are loaded up front and combined without branches, so a box test is one
// memory round trip (a conditional form lets the compiler sink each load into its branch:
// 2D dependent round trips per test).  max(a - x, x - b, 0) equals the gap to [a, b]
// (x < a: a - x; x > b: x - b; else 0; NaN x or an all-NaN box: 0, i.e. "needed").
template <int D>
__device__ __forceinline__ double box_lb2(const double (&x)[D], const double *__restrict__ l,
                                          const double *__restrict__ h) {
    double a[D], b[D];
#pragma unroll
    for (int c = 0; c < D; c++) {
        a[c] = l[c];
        b[c] = h[c];
    }
    double lb = 0;
#pragma unroll
    for (int c = 0; c < D; c++) {
        const double g = fmax(fmax(a[c] - x[c], x[c] - b[c]), 0.0);
        lb = lb + g * g;
    }
    return lb;
}

// the same bound on boxes already in registers
template <int D>
__device__ __forceinline__ double box_lb2v(const double (&x)[D], const double (&a)[D], const double (&b)[D]) {
    double lb = 0;
#pragma unroll
    for (int c = 0; c < D; c++) {
        const double g = fmax(fmax(a[c] - x[c], x[c] - b[c]), 0.0);
        lb = lb + g * g;
    }
    return lb;
}

// Cooperative box staging: a run of NB consecutive boxes (lo/hi rows of D doubles, plus tags)
// is fetched with lanes loading DIFFERENT elements -- one round trip, one or two VGPRs per
// lane -- and parked in the wave's LDS area; the tests then read each box back with
// broadcast LDS reads.  (Every lane loading every box at a uniform address would hold
// NB x 2D doubles in VGPRs per lane and cut occupancy to ~3 waves/SIMD.)  Boxes past
// nvalid become empty (+inf, -inf; tag -1), so their lower bound is +inf.
constexpr int BOXBUF = 2 * FAN;  // doubles per dimension in the per-wave staging area
template <int D, int NB>
__device__ __forceinline__ void stage_boxes(const double *__restrict__ lo, const double *__restrict__ hi,
                                            const int32_t *__restrict__ tag, int nvalid, double *sb, int32_t *st,
                                            int lane) {
    constexpr int E = NB * D, R = (E + 63) / 64;
    double l[R], h[R];
    const int last = nvalid * D - 1;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int e = lane + 64 * r;
        const int ec = e < last ? e : last;  // clamped: unconditional, in-bounds loads
        l[r] = lo[ec];
        h[r] = hi[ec];
    }
    int32_t tg = tag[lane < nvalid - 1 ? lane : nvalid - 1];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < R; r++) {
        const int e = lane + 64 * r;
        if (e < E) {
            const bool ok = e / D < nvalid;
            sb[e] = ok ? l[r] : INFINITY;
            sb[E + e] = ok ? h[r] : -INFINITY;
        }
    }
    if (lane < NB) st[lane] = lane < nvalid ? tg : -1;
    __builtin_amdgcn_wave_barrier();
}
template <int D, int NB>
__device__ __forceinline__ void staged_box(const double *sb, int k, double (&a)[D], double (&b)[D]) {
#pragma unroll
    for (int c = 0; c < D; c++) {
        a[c] = sb[k * D + c];
        b[c] = sb[NB * D + k * D + c];
    }
}


// The BVH level table (offset and node count per level, as bvh_shape) rebuilt per wave in
// LDS from ntiles: reading Bvh::off/cnt with a dynamic level index from the kernel arguments
// keeps both arrays resident in SGPRs and spills them to VGPR lanes.
__device__ __forceinline__ void level_table(int64_t ntiles, int64_t *off_s, int64_t *cnt_s, int lane) {
    if (lane <= MAXLEV) {
        int64_t c = ntiles, o = 0;
        for (int l = 0; l < lane; l++) {
            o += c;
            c = (c + FAN - 1) / FAN;
        }
        off_s[lane] = o;
        cnt_s[lane] = c;
    }
    __builtin_amdgcn_wave_barrier();
}

// Per-round relabel + component tags in one launch (one wave per tile): points take their
// component's hook-tree root (parent2 after resolve_kernel), the tile and its 16-point groups
// get uniform-component tags, and lane 0 folds the tile's tag into every BVH ancestor with
// an atomic merge (EMPTY + x = x, x + x = x, else -1 "mixed") -- replacing one launch per
// level.  A tile stops at the first ancestor already mixed or already holding its tag: the
// tiles that wrote those values carry them to every higher ancestor themselves.
constexpr int32_t TAG_EMPTY = (int32_t)0x80808080;  // memset-able marker, never a component id

template <int D>
__global__ __launch_bounds__(256) void retag_kernel(Rec<D> *__restrict__ recs, int32_t *__restrict__ pcomp, int64_t n,
                                                    int64_t ntiles, int levels, const int32_t *__restrict__ parent,
                                                    int32_t *__restrict__ tag, int32_t *__restrict__ stag) {
    __shared__ int64_t lvl_s[4][2 * (MAXLEV + 1)];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t t = (int64_t)blockIdx.x * 4 + w;
    if (t >= ntiles) return;
    int64_t *off_s = lvl_s[w], *cnt_s = lvl_s[w] + MAXLEV + 1;
    if (lane <= MAXLEV) {  // level table (as bvh_shape)
        int64_t c = ntiles, o = 0;
        for (int l = 0; l < lane; l++) {
            o += c;
            c = (c + FAN - 1) / FAN;
        }
        off_s[lane] = o;
        cnt_s[lane] = c;
    }
    __builtin_amdgcn_wave_barrier();
    const int64_t i = t * BT + lane;
    int32_t c = -2;
    if (i < n) {
        c = pcomp[i];
        if (parent) {
            c = parent[c];
            recs[i].comp = c;
            pcomp[i] = c;
        }
    }
    const int32_t c0 = __shfl(c, 0);
    const bool all = __all((c == c0) || (c == -2));
    const int32_t tg = all ? c0 : -1;
    const int32_t g0 = __shfl(c, lane & ~(SG - 1));
    const unsigned long long bad = __ballot(!((c == g0) || (c == -2)));
    if ((lane & (SG - 1)) == 0) {
        const bool uni = ((bad >> (lane & ~(SG - 1))) & ((1ull << SG) - 1)) == 0;
        stag[t * NSG + lane / SG] = uni ? g0 : -1;
    }
    if (lane == 0) {
        tag[t] = tg;
        for (int L = 1; L < levels; L++) {
            int32_t *a = tag + off_s[L] + (t >> (3 * L));
            int32_t old = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool stop = false;
            while (true) {
                // already mixed, or already holding this tile's tag: the tile that wrote that
                // value carries the same value to every higher ancestor itself
                if (old == -1 || old == tg) {
                    stop = true;
                    break;
                }
                const int32_t nv = old == TAG_EMPTY ? tg : -1;
                const int32_t prev = atomicCAS(a, old, nv);
                if (prev == old) break;
                old = prev;
            }
            if (stop) break;
        }
    }
}

#ifndef HDB_BOR_REFRESH_LOG2
#define HDB_BOR_REFRESH_LOG2 3  // K2b: re-read the component bound every 2^x node visits
#endif
// K2b leaf publish: a better edge reaches the component bound at once, one DPP minimum and at
// most one atomic per wave (A/B r04: per-lane atomics 4.35 ms, never 3.90, per wave 2.84 ms)
#ifndef HDB_BOR_ROWS
#define HDB_BOR_ROWS 1  // K2b leaf groups needed by few lanes: (query, candidate) pairs in 16-lane rows
#endif
#ifndef HDB_BOR_SHFL
#define HDB_BOR_SHFL 0  // K2b rows: query values by lane shuffles instead of LDS (occupancy A/B)
#endif
#ifndef HDB_BOR_ROWS_MAX
#define HDB_BOR_ROWS_MAX 8  // ... when at most this many lanes need the group (else the candidate loop; r04 A/B scan: 2.85 ms at 4, 2.81 at 8, 2.84 at 16, 2.97 at 32, 4.1 at 64; K1t at 8: 1.58 vs 1.56 ms at 16)
#endif
// (round 4 also batched all needed groups of a leaf into one set of row passes, filtered at the
// leaf's start, each lane recomputing its passers' distances: scan 2.84 -> 2.94 ms, 2 VGPRs
// spilled at the 128-VGPR cap; removed)
#ifndef HDB_K1T_ROWS
#define HDB_K1T_ROWS 1  // K1t leaf groups needed by few lanes: (query, candidate) pairs in 16-lane rows
#endif
#ifndef HDB_K1T_SHFL
#define HDB_K1T_SHFL 1  // K1t rows: query values by lane shuffles instead of LDS (occupancy; 0: LDS)
#endif
#ifndef HDB_K1T_ROWS_MAX
#define HDB_K1T_ROWS_MAX 16
#endif
#ifndef HDB_BOR_PROF
#define HDB_BOR_PROF 0  // diagnostic build: per-wave cycle split of the K2b scan (stats boruvka_prof_*)
#endif
// Cycle split of one wave's scan (HDB_BOR_PROF, STATS instantiation only): mark(k) charges the
// shader cycles since the previous mark to phase k.  Phases: 0 setup, 1 pop + bound refresh,
// 2 internal-node box staging (the dependent global load), 3 child tests, 4 ranking + push,
// 5 leaf record/group-box staging, 6 leaf group mask, 7 leaf candidate loops, 8 bound publish,
// 9 tail (best writes, component minimum).
constexpr int BOR_PROF_N = 10;
// STATS: one record of BOR_STATS_REC words per wave (no same-address atomics: thousands of waves
// adding into one line serialise at its L2 channel and slow every load that maps there):
// [0] pair evals, [1] leaves, [2] visits, [3] lanes searching at start, [4] any such lane,
// [5] shader cycles, [6..15] cycle split (HDB_BOR_PROF); summed on the host
constexpr int BOR_STATS_REC = 16;
template <bool ON>
struct BorProf {
    unsigned long long pc[BOR_PROF_N];
    long long last;
    __device__ __forceinline__ void start() {
        if (ON) {
#pragma unroll
            for (int k = 0; k < BOR_PROF_N; k++) pc[k] = 0;
            last = clock64();
        }
    }
    __device__ __forceinline__ void mark(int k) {
        if (ON) {
            const long long now = clock64();
            pc[k] += (unsigned long long)(now - last);
            last = now;
        }
    }
};
struct NoProf {
    __device__ __forceinline__ void mark(int) {}
};

// Cross-lane helpers without the LDS crossbar (__shfl is a ds_bpermute: ~60 cycles per use on
// the traversal's dependent path): DPP within 8-lane subgroups, readlane broadcasts for ranking.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)b, (int)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// max over the lane's 8-lane subgroup: quad swaps, then the other quad (row_half_mirror)
__device__ __forceinline__ double sub8_max(double m) {
    m = fmax(m, dpp_f64<0xb1>(m));   // quad_perm [1,0,3,2]
    m = fmax(m, dpp_f64<0x4e>(m));   // quad_perm [2,3,0,1]
    return fmax(m, dpp_f64<0x141>(m));  // row_half_mirror
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Pushes the children of internal node (lev, idx) that some lane needs, farthest first
// (so the nearest is popped first), ordered by box-to-box distance from the query box.
// needs(a, b, tag): does this lane need the box [a, b] with that tag.  The per-child test
// loop is not unrolled (one child's box live at a time: low VGPR count, high occupancy);
// the ordering is lane-parallel: lane k < FAN ranks child k among the needed children and
// writes its stack slot directly.
template <int D, class Needs>
__device__ __forceinline__ void push_children(const Bvh &bvh, const int64_t *off_s, const int64_t *cnt_s, int lev,
                                              int64_t idx, const double *qlo, const double *qhi, int32_t *stk,
                                              int &sp, int lane, double *sb, int32_t *st, Needs needs) {
    const int64_t c0 = idx * FAN;
    const int64_t c1 = min(c0 + FAN, cnt_s[lev - 1]);
    const int64_t base = off_s[lev - 1] + c0;
    const int nc = (int)(c1 - c0);
    stage_boxes<D, FAN>(bvh.lo + base * D, bvh.hi + base * D, bvh.tag + base, nc, sb, st, lane);
    unsigned okmask = 0;
#pragma unroll 1
    for (int k = 0; k < nc; k++) {
        double a[D], b[D];
        staged_box<D, FAN>(sb, k, a, b);
        if (__any(needs(a, b, st[k]))) okmask |= 1u << k;
    }
    okmask = __builtin_amdgcn_readfirstlane(okmask);
    if (okmask == 0) return;
    // lane k: key of child k (box-to-box squared gap), then its rank among needed children
    double key = -1.0;
    const bool mine = lane < FAN && ((okmask >> lane) & 1u);
    if (mine) {
        double kk = 0;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const double g = fmax(fmax(sb[lane * D + d] - qhi[d], qlo[d] - sb[FAN * D + lane * D + d]), 0.0);
            kk = kk + g * g;
        }
        key = kk;
    }
    int rank = 0;
#pragma unroll
    for (int j = 0; j < FAN; j++) {
        const double kj = readlane_f64(key, j);  // (DPP/readlane, no LDS trips)
        const bool okj = (okmask >> j) & 1u;
        rank += (okj && (kj > key || (kj == key && j < lane))) ? 1 : 0;
    }
    __builtin_amdgcn_wave_barrier();
    if (mine) stk[sp + rank] = ((lev - 1) << 26) | (int32_t)(c0 + lane);
    __builtin_amdgcn_wave_barrier();
    sp += __popc(okmask);
}

// K2b child / group tests lane-parallel against 8-lane subgroup boxes (push_children_sub)
// The same push with a lane-parallel pre-filter: lane L tests child L & 7 against the box of
// its 8-lane subgroup L >> 3 (ok(a, b, tag): a superset of what the subgroup's lanes need),
// then only the children that pass are tested per lane (needs) -- the same children as
// push_children, with one wave-wide test plus one per surviving child instead of one per child.
template <int D, class SubOk, class Needs, class Prof = NoProf>
__device__ __forceinline__ void push_children_sub(const Bvh &bvh, const int64_t *off_s, const int64_t *cnt_s, int lev,
                                                  int64_t idx, const double *qlo, const double *qhi, int32_t *stk,
                                                  int &sp, int lane, double *sb, int32_t *st, SubOk ok, Needs needs,
                                                  Prof &&prof = NoProf{}) {
    const int64_t c0 = idx * FAN;
    const int64_t c1 = min(c0 + FAN, cnt_s[lev - 1]);
    const int64_t base = off_s[lev - 1] + c0;
    const int nc = (int)(c1 - c0);
    stage_boxes<D, FAN>(bvh.lo + base * D, bvh.hi + base * D, bvh.tag + base, nc, sb, st, lane);
    prof.mark(2);
    const int k = lane & (FAN - 1);
    bool need = false;
    if (k < nc) {
        double a[D], b[D];
#pragma unroll
        for (int c = 0; c < D; c++) {
            a[c] = sb[k * D + c];
            b[c] = sb[FAN * D + k * D + c];
        }
        need = ok(a, b, st[k]);
    }
    unsigned long long m = __ballot(need);
    m |= m >> 32;
    m |= m >> 16;
    m |= m >> 8;
    const unsigned pre = __builtin_amdgcn_readfirstlane((unsigned)(m & 0xffu));
    if (pre == 0) return;
    unsigned okmask = 0;
#pragma unroll 1
    for (unsigned r = pre; r; r &= r - 1) {
        const int kk = __builtin_ctz(r);
        double a[D], b[D];
        staged_box<D, FAN>(sb, kk, a, b);
        if (__any(needs(a, b, st[kk]))) okmask |= 1u << kk;
    }
    okmask = __builtin_amdgcn_readfirstlane(okmask);
    prof.mark(3);
    if (okmask == 0) return;
    double key = -1.0;
    const bool mine = lane < FAN && ((okmask >> lane) & 1u);
    if (mine) {
        double kk = 0;
#pragma unroll
        for (int d = 0; d < D; d++) {
            const double g = fmax(fmax(sb[lane * D + d] - qhi[d], qlo[d] - sb[FAN * D + lane * D + d]), 0.0);
            kk = kk + g * g;
        }
        key = kk;
    }
    int rank = 0;
#pragma unroll
    for (int j = 0; j < FAN; j++) {
        const double kj = readlane_f64(key, j);  // (DPP/readlane, no LDS trips)
        const bool okj = (okmask >> j) & 1u;
        rank += (okj && (kj > key || (kj == key && j < lane))) ? 1 : 0;
    }
    __builtin_amdgcn_wave_barrier();
    if (mine) stk[sp + rank] = ((lev - 1) << 26) | (int32_t)(c0 + lane);
    __builtin_amdgcn_wave_barrier();
    sp += __popc(okmask);
    prof.mark(4);
}

// Publishes min(v) per component into arr with few atomics: late rounds put most of the
// n lanes into a handful of components, and one atomicMin per lane on the same address
// serialises in L2.  A wave whose active lanes share one component reduces first; any
// lane skips the atomic when the stored value is already <= v.
__device__ __forceinline__ void publish_min(unsigned long long *arr, int32_t c, unsigned long long v, bool active) {
    const unsigned long long act = __ballot(active);
    if (act == 0) return;
    const int first = __ffsll((long long)act) - 1;
    const int32_t c0 = __shfl(c, first);
    if (__all(!active || c == c0)) {
        unsigned long long m = active ? v : ~0ull;
        for (int off = 32; off >= 1; off >>= 1) {
            unsigned long long o = __shfl_xor(m, off);
            m = o < m ? o : m;
        }
        if ((int)(threadIdx.x & 63) == first) {
            if (m < __hip_atomic_load(&arr[c0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&arr[c0], m);
        }
        return;
    }
    if (active && v < __hip_atomic_load(&arr[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&arr[c], v);
}

template <int D, bool STATS>
__global__ __launch_bounds__(256, (D <= 3 ? HDB_BOR_WPE : 1)) void boruvka_bvh_kernel(const Rec<D> *__restrict__ recs, int64_t n, int64_t ntiles,
                                                          Bvh bvh, unsigned long long *__restrict__ comp_w,
                                                          double *__restrict__ best_w, double *__restrict__ best_s,
                                                          int32_t *__restrict__ best_lo, int32_t *__restrict__ best_hi,
                                                          const int32_t *__restrict__ work,
                                                          const unsigned long long *__restrict__ desc,
                                                          const int32_t *__restrict__ nwaves, int pop_test,
                                                          const int32_t *__restrict__ inv,
                                                          int32_t *__restrict__ best_pos,
                                                          const unsigned long long *__restrict__ n_edges_done,
                                                          double *__restrict__ lbw, uint8_t *__restrict__ xact,
                                                          int xm, unsigned long long *__restrict__ stats) {
    __shared__ int32_t stack_s[4][MAXLEV * FAN + 8];
    __shared__ LRec<D> tile_s[4][BT];
    __shared__ double boxs_s[4][BOXBUF * D];
    __shared__ int32_t boxt_s[4][FAN];
    __shared__ int64_t lvl_s[4][2 * (MAXLEV + 1)];
    __shared__ double q_s[4][2 * D];
    __shared__ double sg_s[4][8 * 2 * D];
#if HDB_BOR_ROWS
    // row-batched leaf groups: the wave's query points (staged once) and per group the needing
    // lanes' bounds and the passing pairs' keys
#if HDB_BOR_SHFL
    // the query lanes' values come by lane shuffles (ds_bpermute) instead: 12 KB less LDS per
    // workgroup (6 instead of 4 workgroups per CU)
    __shared__ int32_t rq_lane[4][BT];
#else
    __shared__ double rq_x[4][BT * D];
    __shared__ double rq_core[4][BT], rq_sb[4][BT];
    __shared__ int32_t rq_comp[4][BT], rq_id[4][BT], rq_lane[4][BT];
#endif
    __shared__ double rk_w[4][BT], rk_s[4][BT];
    __shared__ int32_t rk_lo[4][BT], rk_hi[4][BT];
#endif
    const int w = threadIdx.x >> 6;
    double *bxs = boxs_s[w];
    int32_t *bxt = boxt_s[w];
    int64_t *off_s = lvl_s[w], *cnt_s = lvl_s[w] + MAXLEV + 1;
    // compacted work list (group_compact_kernel): wave t takes desc[t]'s run of sorted
    // positions; the grid covers the worst case (+ 8 xm blocks), waves past the count exit.
    // xm > 0: xm XCD-interleaved chunks per XCD over this round's blocks (xcd_chunk_block)
    const int64_t nw = *nwaves;
    int64_t blk = blockIdx.x;
    if (xm > 0) {
        const int64_t xcb = std::max<int64_t>(1, ceil_div(ceil_div(nw, 4), 8 * (int64_t)xm));
        if (blk >= 8 * xm * xcb) return;
        blk = xcd_chunk_block(blk, xcb);
    }
    const int64_t t = blk * 4 + w;
    if (t >= nw) return;
    if (*n_edges_done >= (unsigned long long)(n - 1)) return;  // speculative round after the last
    const long long t_start = STATS ? clock64() : 0;
    BorProf<STATS && HDB_BOR_PROF> prof;
    prof.start();
    LRec<D> *cand = tile_s[w];
    const int lane = threadIdx.x & 63;
    int32_t *stk = stack_s[w];
    const unsigned long long dsc = desc[t];
    const bool valid = lane < (int)(dsc & 255u);
    const int64_t i = valid ? work[(int64_t)(dsc >> 8) + lane] : 0;
    unsigned long long n_leaf = 0, nev = 0;
    double mx[D];
    double mcore = 0;
    double mlb = 0;  // lower bound of the lane's best weight: max(core, bound kept from earlier rounds)
    int32_t mcomp = -3, mid = 0;
    if (valid) {
        const Rec<D> r = recs[i];
#pragma unroll
        for (int c = 0; c < D; c++) mx[c] = r.x[c];
        mcore = r.core;
        mcomp = r.comp;
        mid = r.id;
        const double l = lbw[i];
        mlb = mcore > l ? mcore : l;
    } else {
#pragma unroll
        for (int c = 0; c < D; c++) mx[c] = 0;
    }
#if HDB_BOR_ROWS && !HDB_BOR_SHFL
#pragma unroll
    for (int c = 0; c < D; c++) rq_x[w][lane * D + c] = mx[c];
    rq_core[w][lane] = mcore;
    rq_comp[w][lane] = mcomp;
    rq_id[w][lane] = mid;
#endif
    Best b{INFINITY, INFINITY, INT32_MAX, INT32_MAX};
    if (valid && best_w[i] < INFINITY) b = Best{best_w[i], best_s[i], best_lo[i], best_hi[i]};  // seed_kernel
    double cb2 = INFINITY;  // padded square of the component bound
    double cwv = INFINITY;  // the component bound itself: every lane candidate has w >= mcore
    // squared-distance bound from the lane's own best: a candidate can only win with
    // s <= sb.  b.w == own core: ties need s <= b.s (exact: lb <= s by monotone rounding);
    // otherwise sqrt(s) <= b.w, i.e. s <= b.w^2 (padded: s > fl(b^2)(1+2^-48) proves
    // fl(sqrt(s)) > b).
    auto own_sb = [&]() -> double {
        if (!(b.w < INFINITY)) return INFINITY;
        return (b.w <= mcore) ? b.s : (b.w * b.w) * 1.0000000000000036;
    };
    double sb = own_sb();
    auto refresh = [&]() {
        if (valid) {
            unsigned long long cw = __hip_atomic_load(&comp_w[mcomp], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            double cwd = __longlong_as_double((long long)cw);
            double c2 = (cwd * cwd) * (1.0 + 1e-12);
            if (c2 < cb2) cb2 = c2;
            if (cwd < cwv) cwv = cwd;
        }
    };
    auto bound = [&]() -> double { return sb < cb2 ? sb : cb2; };
    const bool search = valid;  // done / dead lanes are not in the work list
    refresh();  // the seeds already bound the component (seed kernels publish before the scan)
    const bool active0 = search && !(mlb > cwv);
    // MRD >= own core (HDBSCANStar.java:164-166): a lane whose core exceeds the component
    // bound cannot supply the component's edge (false for a NaN core, which never raises MRD).
    // Branch-free so the box loads are not sunk into conditional blocks.
    auto needs_vals = [&](const double (&a)[D], const double (&b)[D], int32_t tg) -> bool {
        const double lb = box_lb2v<D>(mx, a, b);
        const double bd = bound();
        const bool same = (tg >= 0) & (tg == mcomp);
        return search & !(mlb > cwv) & !same & (!(bd < INFINITY) | !(lb > bd));
    };
    // query box = the wave's own points (orders the children nearest-first); kept in LDS
    // (only the ranking lanes read it)
    double *qlo = q_s[w], *qhi = q_s[w] + D;
#pragma unroll
    for (int c = 0; c < D; c++) {
        double l = valid ? mx[c] : INFINITY, h = valid ? mx[c] : -INFINITY;
        for (int off = 32; off >= 1; off >>= 1) {
            l = fmin(l, __shfl_xor(l, off));
            h = fmax(h, __shfl_xor(h, off));
        }
        if (lane == 0) {
            qlo[c] = l;
            qhi[c] = h;
        }
    }
    __builtin_amdgcn_wave_barrier();
    // 8-lane subgroups (consecutive work entries: Morton-close points).  Every node and group
    // test below runs once per (child, subgroup) pair on its own lane, with the box of the
    // subgroup's points, the largest bound among its searching lanes and the component they
    // all share (-2: mixed or none).  Exact: the box-to-box gap (monotone rounding) is <= the
    // gap of every point of the subgroup, so a child no subgroup needs is needed by no lane.
    // subgroup boxes parked in LDS (registers would spill): [8][lo D | hi D]
    double *sgb = sg_s[w];
#pragma unroll
    for (int c = 0; c < D; c++) {
        const bool nan = !(mx[c] == mx[c]);  // a NaN coordinate needs every box (its gaps are 0)
        double l = valid ? (nan ? -INFINITY : mx[c]) : INFINITY, h = valid ? (nan ? INFINITY : mx[c]) : -INFINITY;
#pragma unroll
        for (int off = 1; off < 8; off <<= 1) {
            l = fmin(l, __shfl_xor(l, off));
            h = fmax(h, __shfl_xor(h, off));
        }
        if ((lane & 7) == 0) {
            sgb[(lane >> 3) * 2 * D + c] = l;
            sgb[(lane >> 3) * 2 * D + D + c] = h;
        }
    }
    __builtin_amdgcn_wave_barrier();
    const double *sgl = sgb + (lane >> 3) * 2 * D, *sgh = sgl + D;
    int32_t ucomp;
    {
        int32_t cmn = search ? mcomp : INT32_MAX, cmx = search ? mcomp : INT32_MIN;
#pragma unroll
        for (int off = 1; off < 8; off <<= 1) {
            cmn = min(cmn, __shfl_xor(cmn, off));
            cmx = max(cmx, __shfl_xor(cmx, off));
        }
        ucomp = cmn == cmx ? cmn : -2;
    }
    // the subgroup's largest bound over its lanes still searching (-1: none)
    auto sub_bound = [&]() -> double {
        double m = (search & !(mlb > cwv)) ? bound() : -1.0;
        return sub8_max(m);
    };
    auto sub_ok = [&](double mb) {
        return [&, mb](const double (&a)[D], const double (&b)[D], int32_t tg) -> bool {
            double lb = 0;
#pragma unroll
            for (int c = 0; c < D; c++) {
                const double g = fmax(fmax(a[c] - sgh[c], sgl[c] - b[c]), 0.0);
                lb = lb + g * g;
            }
            return (mb >= 0.0) & !((tg >= 0) & (tg == ucomp)) & !(lb > mb);
        };
    };
    // needed 16-point groups of the staged leaf: lane L tests group L & 7 (< NSG)
    auto group_mask = [&]() -> unsigned {
        const double mb = sub_bound();
        const int k = lane & 7;
        bool need = false;
        if (k < NSG) {
            double a[D], bb[D];
            staged_box<D, NSG>(bxs, k, a, bb);
            need = sub_ok(mb)(a, bb, bxt[k]);
        }
        unsigned long long m = __ballot(need);
        m |= m >> 32;
        m |= m >> 16;
        m |= m >> 8;
        return __builtin_amdgcn_readfirstlane((unsigned)(m & ((1u << NSG) - 1)));
    };
    level_table(ntiles, off_s, cnt_s, lane);
    int sp = 0;
    if (lane == 0) stk[0] = ((bvh.levels - 1) << 26) | 0;
    sp = 1;
    int visits = 0;
    prof.mark(0);
    while (sp > 0) {
        __builtin_amdgcn_wave_barrier();
        const int32_t code = __builtin_amdgcn_readfirstlane(stk[sp - 1]);
        sp--;
        const int lev = code >> 26;
        const int64_t idx = code & ((1 << 26) - 1);
        const int64_t node = off_s[lev] + idx;
        if ((visits++ & ((1 << HDB_BOR_REFRESH_LOG2) - 1)) == 0) refresh();
        prof.mark(1);
        // re-test the popped node with the current bound (its parent tested it when pushing)
        if (pop_test & 1) {
            stage_boxes<D, 1>(bvh.lo + node * D, bvh.hi + node * D, bvh.tag + node, 1, bxs, bxt, lane);
            double a[D], bb[D];
            staged_box<D, 1>(bxs, 0, a, bb);
            if (!__any(needs_vals(a, bb, bxt[0]))) continue;
        }
        if (lev > 0) {
            push_children_sub<D>(bvh, off_s, cnt_s, lev, idx, qlo, qhi, stk, sp, lane, bxs, bxt, sub_ok(sub_bound()),
                                 needs_vals, prof);
            continue;
        }
        // leaf: tile idx, 4 groups of 16 candidates.  The tile's records are fetched with one
        // vector load together with the group boxes, then staged in LDS.
        n_leaf++;
        bool found = false;
        const LRec<D> mine = fetch_rec<D>(recs, n, idx * BT + lane);
        stage_boxes<D, NSG>(bvh.slo + idx * NSG * D, bvh.shi + idx * NSG * D, bvh.stag + idx * NSG, NSG, bxs, bxt,
                            lane);
        cand[lane] = mine;  // staged now: the record's registers die before the culling
        __builtin_amdgcn_wave_barrier();
        prof.mark(5);
        auto gneeds = [&](int gi) -> bool {
            double a[D], bb[D];
            staged_box<D, NSG>(bxs, gi, a, bb);
            return needs_vals(a, bb, bxt[gi]);
        };
        const unsigned gmask = group_mask();  // pre-filter; the per-lane test below decides
        prof.mark(6);
        if (gmask == 0) continue;
#pragma unroll 1
        for (int gi = 0; gi < NSG; gi++) {
            if (!((gmask >> gi) & 1u)) continue;
            const bool need = gneeds(gi);  // re-test in registers: the bound may have tightened
            if (!__any(need)) continue;
            const int q0 = gi * SG;
            const int nq = (int)min<int64_t>(SG, n - (idx * BT + q0));
#if HDB_BOR_ROWS
            // Few lanes need the group (typically 3-5 of 64): the wave-uniform candidate loop
            // spends 16 iterations on all 64 lanes for them.  Instead the (needing lane,
            // candidate) pairs are laid out four queries x 16 candidates per wave instruction
            // (one 16-lane row per query), the passing pairs' keys (w, s, lo, hi) parked in LDS,
            // and each needing lane folds its row's passers into its best with key_less.  The
            // filter uses the group-start bound (only looser: a candidate it rejects cannot beat
            // the lane's best then or later), and the key order is a strict total order, so the
            // best edge is the one the sequential loop finds.
            const unsigned long long M = __ballot(need);
            const int K = __popcll(M);
            if (K <= HDB_BOR_ROWS_MAX) {
                const int rank = __popcll(M & ((1ull << lane) - 1));
#if HDB_BOR_SHFL
                const double sb0 = sb;  // the group-start bound of every lane
                if (need) rq_lane[w][rank] = lane;
#else
                if (need) {
                    rq_sb[w][lane] = sb;
                    rq_lane[w][rank] = lane;
                }
#endif
                __builtin_amdgcn_wave_barrier();
                const int row = lane >> 4, c = lane & 15;
                const LRec<D> r = cand[q0 + c];  // the row's candidate (4-way LDS broadcast)
                for (int r0 = 0; r0 < K; r0 += 4) {
                    const int qr = r0 + row;
                    const bool rowact = qr < K;
                    const int ql = rq_lane[w][rowact ? qr : 0];
#if HDB_BOR_SHFL
                    // every lane shuffles (the loop is wave-uniform): a shuffle inside the
                    // divergent branch below would read inactive lanes
                    double s2 = sq_diff(__shfl(mx[0], ql), r.x[0]);
#pragma unroll
                    for (int cc = 1; cc < D; cc++) s2 = s2 + sq_diff(__shfl(mx[cc], ql), r.x[cc]);
                    const int32_t qcomp = __shfl(mcomp, ql), qid = __shfl(mid, ql);
                    const double qsb = __shfl(sb0, ql), qc = __shfl(mcore, ql);
#else
                    double s2 = sq_diff(rq_x[w][ql * D], r.x[0]);
#pragma unroll
                    for (int cc = 1; cc < D; cc++) s2 = s2 + sq_diff(rq_x[w][ql * D + cc], r.x[cc]);
                    const int32_t qcomp = rq_comp[w][ql], qid = rq_id[w][ql];
                    const double qsb = rq_sb[w][ql], qc = rq_core[w][ql];
#endif
                    const bool pair = rowact & (c < nq) & (r.comp != qcomp);
                    if (STATS) nev += pair ? 1 : 0;  // pair evaluated for a lane that needs it
                    const bool pass = pair & (s2 <= qsb);  // also drops NaN
                    if (pass) {
                        double mrd = sqrt(s2);  // HDBSCANStar.java:162-168 order
                        if (qc > mrd) mrd = qc;
                        if (r.core > mrd) mrd = r.core;
                        rk_w[w][lane] = mrd;
                        rk_s[w][lane] = s2;
                        rk_lo[w][lane] = qid < r.id ? qid : r.id;
                        rk_hi[w][lane] = qid < r.id ? r.id : qid;
                    }
                    const unsigned long long pm = __ballot(pass);
                    __builtin_amdgcn_wave_barrier();
                    if (need && rank >= r0 && rank < r0 + 4) {
                        const int rr = rank - r0;
                        unsigned bits = (unsigned)(pm >> (16 * rr)) & 0xFFFFu;
                        while (bits) {
                            const int k = 16 * rr + __builtin_ctz(bits);
                            bits &= bits - 1;
                            const double kw = rk_w[w][k], ks = rk_s[w][k];
                            const int32_t klo = rk_lo[w][k], khi = rk_hi[w][k];
                            if (key_less(kw, ks, klo, khi, b)) {
                                b = Best{kw, ks, klo, khi};
                                sb = own_sb();
                                found = true;
                            }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                continue;
            }
#endif
            const int q1 = q0 + nq;
#pragma unroll CAND_UNROLL
            for (int qq = q0; qq < q1; qq++) {
                const LRec<D> r = cand[qq];  // uniform address -> LDS broadcast
                double s = sq_diff(mx[0], r.x[0]);
#pragma unroll
                for (int c = 1; c < D; c++) s = s + sq_diff(mx[c], r.x[c]);
                if (!need || r.comp == mcomp) continue;
                if (STATS) nev++;  // pair evaluated for a lane that needs it
                if (!(s <= sb)) continue;  // also drops NaN
                double mrd = sqrt(s);  // HDBSCANStar.java:162-168 order
                if (mcore > mrd) mrd = mcore;
                if (r.core > mrd) mrd = r.core;
                const int32_t lo = mid < r.id ? mid : r.id;
                const int32_t hi = mid < r.id ? r.id : mid;
                if (key_less(mrd, s, lo, hi, b)) {
                    b = Best{mrd, s, lo, hi};
                    sb = own_sb();
                    found = true;
                }
            }
        }
        prof.mark(7);
        {
            // wave-aggregated publish: when every lane with a better edge shares one component
            // (the late rounds' common case), one DPP minimum and at most one atomic per wave
            const bool pub = found && (b.w * b.w) * (1.0 + 1e-12) < cb2;
            const unsigned long long pm = __ballot(pub);
            if (pm) {
                const int first = __ffsll((long long)pm) - 1;
                const int32_t c0 = __shfl(mcomp, first);
                if (!__any(pub && mcomp != c0)) {
                    const unsigned long long m = wave_min_u64(pub ? (unsigned long long)dbits(b.w) : ~0ull);
                    if (lane == first &&
                        m < __hip_atomic_load(&comp_w[c0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        atomicMin(&comp_w[c0], m);
                }
            }
        }
        if (found) {
            const double c2 = (b.w * b.w) * (1.0 + 1e-12);
            if (c2 < cb2) {
                cb2 = c2;
                if (b.w < cwv) cwv = b.w;
            }
        }
        prof.mark(8);
    }
    if (valid) {
        best_w[i] = b.w;
        best_s[i] = b.s;
        best_lo[i] = b.lo;
        best_hi[i] = b.hi;
        if (b.w < INFINITY) best_pos[i] = inv[b.lo == mid ? b.hi : b.lo];  // partner, for the next seed
        // Bounds carried to later rounds (a component only grows, so a point's best over the
        // shrinking outside set never decreases).  Candidates the component bound pruned have
        // w > cwv; a lane that stopped (mlb > cwv) has best >= mlb.  So best >= min(b.w, cwv)
        // always, and b is the exact (key-minimal) best iff the lane never stopped and
        // b.w <= cwv.
        const double lb = b.w < cwv ? b.w : cwv;
        if (lb > lbw[i]) lbw[i] = lb;
        xact[i] = (!(mlb > cwv) && b.w <= cwv) ? 1 : 0;
    }
    publish_min(comp_w, mcomp, dbits(b.w), valid && b.w < INFINITY);
    prof.mark(9);
    if (STATS) {
        for (int off = 32; off >= 1; off >>= 1) nev += __shfl_xor(nev, off);
        const unsigned long long act_mask = __ballot(active0);
        if (lane == 0) {
            unsigned long long *rec = stats + (size_t)t * BOR_STATS_REC;
            rec[0] = nev;
            rec[1] = n_leaf;
            rec[2] = (unsigned long long)visits;
            rec[3] = (unsigned long long)__popcll(act_mask);  // lanes searching at start
            rec[4] = (unsigned long long)(act_mask != 0);     // waves with any such lane
#if HDB_BOR_PROF
            for (int k = 0; k < BOR_PROF_N; k++) rec[6 + k] = prof.pc[k];
#endif
            rec[5] = (unsigned long long)(clock64() - t_start);  // per-wave shader cycles
        }
    }
}

// Work lists for the scan.  A lane searches unless its seed is exact (done) or its core
// already exceeds the component bound the seeds published (it cannot supply the edge; comp_w
// starts as all-ones bits, a NaN: no bound).  Searching lanes are compacted per group of
// WGRP = 512 sorted positions (one level-1 BVH node), so a wave's points stay inside one
// small Morton range: a wave takes up to P consecutive entries of one group.
constexpr int WGRP = 512;

template <int D>
__global__ __launch_bounds__(WGRP) void group_compact_kernel(const Rec<D> *__restrict__ recs, int64_t n,
                                                             const uint8_t *__restrict__ done,
                                                             const double *__restrict__ lbw,
                                                             const unsigned long long *__restrict__ comp_w, int P,
                                                             int32_t *__restrict__ work, int32_t *__restrict__ gcnt,
                                                             int32_t *__restrict__ gwaves) {
    __shared__ int wc[WGRP / 64];
    const int64_t g = blockIdx.x;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int64_t p = g * WGRP + tid;
    bool f = false;
    if (p < n) {
        const double cw = __longlong_as_double((long long)comp_w[recs[p].comp]);
        const double c = recs[p].core, l = lbw[p];
        f = !(done && done[p]) && !((c > l ? c : l) > cw);
    }
    const unsigned long long m = __ballot(f);
    const int rank = __popcll(m & ((1ull << lane) - 1));
    if (lane == 0) wc[wv] = __popcll(m);
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int k = 0; k < WGRP / 64; k++) {
        base += k < wv ? wc[k] : 0;
        total += wc[k];
    }
    if (f) work[g * WGRP + base + rank] = (int32_t)p;
    if (tid == 0) {
        gcnt[g] = total;
        gwaves[g] = (total + P - 1) / P;
    }
}

// Adjacency seeds (round 6).  From round 1 on, a component's bound comes only from last round's
// edges whose partner is still outside it -- after a merge, mostly none, so comp_w stays "no
// bound" (NaN bits), no lane is filtered and every wave walks unbounded until some wave
// publishes.  Any edge between two components is a valid candidate: consecutive sorted
// positions i, i + 1 in different components (Morton neighbours, so usually close) give one
// for both, with the scan's exact weight (HDBSCANStar.java:162-168 order).  Only valid edges
// enter comp_w, so its final value is still the true minimum; every component has such a pair
// while more than one component remains.
template <int D>
__global__ void adj_seed_kernel(const Rec<D> *__restrict__ recs, const int32_t *__restrict__ pcomp, int64_t n,
                                unsigned long long *__restrict__ comp_w) {
    HDB_GRID_STRIDE(i, n - 1) {
        const int32_t ca = pcomp[i], cb = pcomp[i + 1];
        if (ca == cb) continue;
        const Rec<D> a = recs[i], b = recs[i + 1];
        double s = sq_diff(a.x[0], b.x[0]);
#pragma unroll
        for (int c = 1; c < D; c++) s = s + sq_diff(a.x[c], b.x[c]);
        double mrd = sqrt(s);
        if (a.core > mrd) mrd = a.core;
        if (b.core > mrd) mrd = b.core;
        if (!(mrd == mrd)) continue;  // NaN coordinates: no bound
        const unsigned long long v = dbits(mrd);
        if (v < __hip_atomic_load(&comp_w[ca], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&comp_w[ca], v);
        if (v < __hip_atomic_load(&comp_w[cb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&comp_w[cb], v);
    }
}

// wave descriptors: (start in work) << 8 | count, at the group's exclusive wave offset
__global__ void wave_desc_kernel(const int32_t *__restrict__ gcnt, const int32_t *__restrict__ woff, int64_t ngroups,
                                 int P, unsigned long long *__restrict__ desc, int32_t *__restrict__ nwaves) {
    HDB_GRID_STRIDE(g, ngroups) {
        const int c = gcnt[g];
        const int64_t o = woff[g];
        for (int k = 0; k * P < c; k++) {
            const int cnt = c - k * P < P ? c - k * P : P;
            desc[o + k] = ((unsigned long long)(g * WGRP + k * P) << 8) | (unsigned long long)cnt;
        }
        if (g == ngroups - 1) *nwaves = (int32_t)(o + (c + P - 1) / P);
    }
}

// component minimum: comp_w = min w (published during the scan); then min s among the
// lanes at that weight; then min (lo, hi) among the lanes at (w, s)
__global__ void comp_s_kernel(const int32_t *__restrict__ pcomp, int64_t n, const unsigned long long *__restrict__ comp_w,
                              const double *__restrict__ best_w, const double *__restrict__ best_s,
                              unsigned long long *__restrict__ comp_s) {
    HDB_GRID_STRIDE(i, n) {
        int32_t c = pcomp[i];
        double w = best_w[i];
        if (w < INFINITY && dbits(w) == comp_w[c]) atomicMin(&comp_s[c], dbits(best_s[i]));
    }
}

__global__ void comp_key_kernel(const int32_t *__restrict__ pcomp, int64_t n, const unsigned long long *__restrict__ comp_w,
                                const unsigned long long *__restrict__ comp_s, const double *__restrict__ best_w,
                                const double *__restrict__ best_s, const int32_t *__restrict__ best_lo,
                                const int32_t *__restrict__ best_hi, unsigned long long *__restrict__ comp_key) {
    HDB_GRID_STRIDE(i, n) {
        int32_t c = pcomp[i];
        double w = best_w[i];
        if (w < INFINITY && dbits(w) == comp_w[c] && dbits(best_s[i]) == comp_s[c])
            atomicMin(&comp_key[c], ((unsigned long long)(uint32_t)best_lo[i] << 32) | (uint32_t)best_hi[i]);
    }
}

// per component root c: chosen edge -> parent pointer; record edge unless mutual-larger
__global__ void hook_kernel(const int32_t *__restrict__ pcomp, int64_t n, const int32_t *__restrict__ inv,
                            const unsigned long long *__restrict__ comp_w,
                            const unsigned long long *__restrict__ comp_key, int32_t *__restrict__ parent,
                            int32_t *__restrict__ out_a, int32_t *__restrict__ out_b, double *__restrict__ out_w,
                            unsigned long long *__restrict__ n_edges) {
    HDB_GRID_STRIDE(c, n) {
        if (pcomp[c] != (int32_t)c) continue;  // not a root
        unsigned long long k = comp_key[c];
        if (k == ~0ull) {
            parent[c] = (int32_t)c;
            continue;
        }
        int32_t lo = (int32_t)(k >> 32), hi = (int32_t)(k & 0xffffffffu);
        int32_t cl = pcomp[inv[lo]], ch = pcomp[inv[hi]];
        int32_t other = cl == (int32_t)c ? ch : cl;
        parent[c] = other;
    }
}

// One workgroup covers HF_T * HF_E consecutive ids and reserves its edge slots with ONE
// atomic: n_edges is a single hot address, and per-wave reservations (15.6k waves at 1M
// points, most holding a root in every round) serialised at the L2 (~66 us per round).
constexpr int HF_T = 1024, HF_E = 4;

template <int D>
__global__ __launch_bounds__(HF_T) void hook_fix_kernel(const int32_t *__restrict__ pcomp, int64_t n,
                                                       const unsigned long long *__restrict__ comp_w,
                                                       const unsigned long long *__restrict__ comp_key,
                                                       int32_t *__restrict__ parent, int32_t *__restrict__ parent2,
                                                       int32_t *__restrict__ out_a, int32_t *__restrict__ out_b,
                                                       double *__restrict__ out_w, unsigned long long *__restrict__ n_edges) {
    __shared__ int wcnt[HF_T / 64];
    __shared__ unsigned long long sbase;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * (HF_T * HF_E) + threadIdx.x;
    unsigned long long m[HF_E];
    int wtot = 0;
#pragma unroll
    for (int e = 0; e < HF_E; e++) {
        const int64_t c = c0 + (int64_t)e * HF_T;  // coalesced: consecutive lanes, consecutive ids
        bool emit = false;
        if (c < n) {
            if (pcomp[c] != (int32_t)c) {
                parent2[c] = -1;  // not a root: resolve skips it
            } else {
                const int32_t p = parent[c];
                if (p == (int32_t)c) {
                    parent2[c] = p;
                } else {
                    const bool mutual = parent[p] == (int32_t)c;
                    parent2[c] = (mutual && (int32_t)c < p) ? (int32_t)c : p;  // smaller id of a mutual pair is the root
                    emit = !(mutual && (int32_t)c > p);
                }
            }
        }
        m[e] = __ballot(emit);
        wtot += __popcll(m[e]);
    }
    if (lane == 0) wcnt[wv] = wtot;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int k = 0; k < HF_T / 64; k++) tot += wcnt[k];
        sbase = tot ? atomicAdd(n_edges, (unsigned long long)tot) : 0;
    }
    __syncthreads();
    unsigned long long slot = sbase;
    for (int k = 0; k < wv; k++) slot += (unsigned long long)wcnt[k];
    const unsigned long long below = (1ull << lane) - 1;
#pragma unroll
    for (int e = 0; e < HF_E; e++) {
        if ((m[e] >> lane) & 1ull) {
            const int64_t c = c0 + (int64_t)e * HF_T;
            const unsigned long long sl = slot + __popcll(m[e] & below);
            const unsigned long long k = comp_key[c];
            out_a[sl] = (int32_t)(k >> 32);
            out_b[sl] = (int32_t)(k & 0xffffffffu);
            out_w[sl] = __longlong_as_double((long long)comp_w[c]);
        }
        slot += __popcll(m[e]);
    }
}

__global__ void fill_inf_kernel(double *__restrict__ p, int64_t n) { HDB_GRID_STRIDE(i, n) p[i] = INFINITY; }

// per-round reset of the component minima (one launch instead of three memsets)
__global__ void reset_comp_kernel(unsigned long long *__restrict__ a, unsigned long long *__restrict__ b,
                                  unsigned long long *__restrict__ c, int64_t n, int32_t *__restrict__ node_tags,
                                  int64_t n_nodes) {
    HDB_GRID_STRIDE(i, n) {
        a[i] = ~0ull;
        b[i] = ~0ull;
        c[i] = ~0ull;
        if (i < n_nodes) node_tags[i] = TAG_EMPTY;
    }
}

// parent pointers -> the root of each hook tree in one launch (chains only shorten while
// other lanes write: every value read is an ancestor, so the walk always ends at the root)
__global__ void resolve_kernel(int32_t *__restrict__ parent, int64_t n) {
    HDB_GRID_STRIDE(c, n) {
        int32_t p = parent[c];
        if (p < 0) continue;
        while (true) {
            const int32_t pp = __hip_atomic_load(&parent[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (pp == p) break;
            p = pp;
        }
        parent[c] = p;
    }
}

__global__ void pos_iota_kernel(int32_t *__restrict__ a, int64_t n) { HDB_GRID_STRIDE(i, n) a[i] = (int32_t)i; }

// (lo, hi) key packed into 2B bits (ids < 2^B), so the id sort runs only 2B radix bits
__global__ void edge_idkey_kernel(const int32_t *a, const int32_t *b, int64_t m, int B, uint64_t *k, int32_t *io) {
    HDB_GRID_STRIDE(i, m) {
        k[i] = ((uint64_t)(uint32_t)a[i] << B) | (uint32_t)b[i];
        io[i] = (int32_t)i;
    }
}
__global__ void edge_wkey_kernel(const int32_t *perm_, const double *ww, int64_t m, uint64_t *k) {
    HDB_GRID_STRIDE(i, m) k[i] = (uint64_t)__double_as_longlong(ww[perm_[i]]);
}
// self edges' sort keys: the core (+0.0 for -0.0: Java's comparator ties them) and the id
__global__ void self_keys_kernel(const double *__restrict__ core, int64_t n, double *__restrict__ k,
                                 int32_t *__restrict__ id) {
    HDB_GRID_STRIDE(i, n) {
        const double c = core[i];
        k[i] = c == 0.0 ? 0.0 : c;
        id[i] = (int32_t)i;
    }
}
// the sorted self edges' weights: the cores themselves (a -0.0 core stays -0.0, as the plain
// path writes it; the sort keys normalised it to +0.0, which the merge's comparisons tie anyway)
__global__ void gather_core_kernel(const double *__restrict__ core, const int32_t *__restrict__ perm, int64_t n,
                                   double *__restrict__ w) {
    HDB_GRID_STRIDE(i, n) w[i] = core[perm[i]];
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

// ssort functors of the MST edge orders.  Keys: the weight through an order-preserving map
// of doubles to u64 (-0.0 read as +0.0, as the radix path's keys), then the tie breaker:
// tree edges (ea << 31 | eb) -- the (lo, hi) order the radix path sorts by first --, self
// edges (1 << 62 | id) after every tree edge of equal weight (the merge's "tree edges first").
__device__ __forceinline__ uint64_t dkey_asc(double x) {
    const uint64_t b = (uint64_t)__double_as_longlong(x == 0.0 ? 0.0 : x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_inv(uint64_t u) {
    return __longlong_as_double((long long)((u >> 63) ? (u & 0x7fffffffffffffffull) : ~u));
}
constexpr uint64_t EK_SELF = 1ull << 62;
struct TreeEdgeKeyF {  // desc: the reducers' merge order; asc: FirstStep's (w, lo, hi)
    const int32_t *ea, *eb;
    const double *ew;
    const double *core;  // self edges (desc only), nullable
    int64_t ne;
    bool desc;
    __device__ SKey operator()(int64_t i) const {
        if (i < ne) {
            const uint64_t k = dkey_asc(ew[i]);
            return SKey{desc ? ~k : k, ((uint64_t)(uint32_t)ea[i] << 31) | (uint32_t)eb[i]};
        }
        const int64_t j = i - ne;
        return SKey{~dkey_asc(core[j]), EK_SELF | (uint64_t)j};
    }
};
struct TreeEdgeEmitF {
    int32_t *va, *vb;
    double *w;
    const double *core;
    bool desc;
    __device__ void operator()(int64_t r, const SKey &k) const {
        if (k.lo & EK_SELF) {
            const int32_t j = (int32_t)(k.lo & 0x7fffffffu);
            va[r] = j;
            vb[r] = j;
            w[r] = core[j];
        } else {
            va[r] = (int32_t)((k.lo >> 31) & 0x7fffffffu);
            vb[r] = (int32_t)(k.lo & 0x7fffffffu);
            w[r] = dkey_inv(desc ? ~k.hi : k.hi);
        }
    }
};

// ------------------------------------------------ fused leaf: kNN-seeded round 0
template <int D>
__global__ void set_core_kernel(Rec<D> *__restrict__ recs, int64_t n, const double *__restrict__ core) {
    HDB_GRID_STRIDE(i, n) recs[i].core = core[recs[i].id];
}

// Block-level min publish for block-uniform loops: lanes reduce per wave (publish_min's
// uniform case), then, when all waves of the block target one component, a single atomic.
// Late rounds put almost every lane of a block into one huge component; one atomic per
// wave on that address serialises at its L2 channel.
__device__ __forceinline__ void block_publish_min(unsigned long long *arr, int32_t c, unsigned long long v,
                                                  bool active, int32_t *s_c, unsigned long long *s_v) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const unsigned long long act = __ballot(active);
    const int first = act ? __ffsll((long long)act) - 1 : 0;
    const int32_t c0 = __shfl(c, first);
    const bool uni = __all(!active || c == c0);
    unsigned long long m = active ? v : ~0ull;
    if (uni) {
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long o = __shfl_xor(m, off);
            m = o < m ? o : m;
        }
    }
    if (lane == 0) {
        s_c[wv] = act == 0 ? -2 : (uni ? c0 : -1);  // -2: nothing, -1: mixed
        s_v[wv] = m;
    }
    __syncthreads();
    int32_t cb = -2;
    unsigned long long mb = ~0ull;
    bool block_uni = true;
    for (int k = 0; k < nw; k++) {
        const int32_t ck = s_c[k];
        if (ck == -2) continue;
        if (ck == -1 || (cb >= 0 && ck != cb)) block_uni = false;
        cb = ck;
        mb = s_v[k] < mb ? s_v[k] : mb;
    }
    __syncthreads();
    if (block_uni) {
        if (threadIdx.x == 0 && cb >= 0 && mb < __hip_atomic_load(&arr[cb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(&arr[cb], mb);
        return;
    }
    if (uni) {
        if (lane == first && act && m < __hip_atomic_load(&arr[c0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(&arr[c0], m);
        return;
    }
    if (active && v < __hip_atomic_load(&arr[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&arr[c], v);
}

// Per-round Boruvka seed.  (1) prev: round r-1's per-point best edge, when its endpoints are
// still in different components, is a valid candidate (seed_kernel's rule).  (2) K > 0: the
// K nearest neighbours K1t found (sorted positions, squared distances): every list member
// in another component is a valid candidate.  The lane keeps the smallest key and publishes
// it to comp_w, so the scan starts with a component bound.  Only valid edges enter comp_w,
// so its final value is still the true component minimum.
// The seed is provably the lane's exact best when no point outside the list can beat it:
// every such point has s' >= s_K (the list holds every point with s' < s_K), so its weight
// is >= LB = max(fl(sqrt(s_K)), core_p); exact if w < LB, or w == LB and s < s_K.  Exact
// lanes skip the traversal (done[i] = 1).
template <int D, int K>
__global__ __launch_bounds__(256) void round_seed_kernel(const Rec<D> *__restrict__ recs, const int32_t *__restrict__ pcomp,
                                                        int64_t n, int prev, const int32_t *__restrict__ nb_pos,
                                                        const double *__restrict__ nb_s, double *__restrict__ best_w,
                                                        double *__restrict__ best_s, int32_t *__restrict__ best_lo,
                                                        int32_t *__restrict__ best_hi, int32_t *__restrict__ best_pos,
                                                        uint8_t *__restrict__ done, double *__restrict__ lbw,
                                                        uint8_t *__restrict__ xact, unsigned long long *__restrict__ comp_w) {
    __shared__ int32_t s_c[4];
    __shared__ unsigned long long s_v[4];
    const int64_t stride = (int64_t)blockDim.x * gridDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < n; base += stride) {  // block-uniform trip count
        const int64_t i = base + threadIdx.x;
        int32_t mcomp = 0;
        Best b{INFINITY, INFINITY, INT32_MAX, INT32_MAX};
        if (i < n) {
            mcomp = pcomp[i];
            int32_t bpos = -1;
            bool exact = false;
            if (prev) {
                const double w0 = best_w[i];
                if (w0 < INFINITY) {
                    const int32_t bp = best_pos[i];
                    if (pcomp[bp] != mcomp) {
                        b = Best{w0, best_s[i], best_lo[i], best_hi[i]};
                        bpos = bp;
                        // last round's exact best is still outside the component: still exact
                        // (the outside set only shrank), so the lane skips the traversal
                        exact = xact[i] != 0;
                    }
                }
            }
            if constexpr (K > 0) {
                const Rec<D> &me = recs[i];
                const double mcore = me.core;
                const int32_t mid = me.id;
                double sK = -INFINITY;
                bool full = true;
                // every neighbour's component, core and id loaded up front (unconditional,
                // clamped to the point itself): K independent random loads in flight at once
                // instead of K dependent rounds
                int32_t nj[K], ncomp[K], nid[K];
                double ns[K], ncore[K];
#pragma unroll
                for (int k = 0; k < K; k++) {
                    nj[k] = nb_pos[i * K + k];
                    ns[k] = nb_s[i * K + k];
                }
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const int64_t jc = nj[k] < 0 ? i : nj[k];
                    ncomp[k] = pcomp[jc];
                    ncore[k] = recs[jc].core;
                    nid[k] = recs[jc].id;
                }
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const int32_t j = nj[k];
                    const double s = ns[k];
                    if (j < 0 || !(s < INFINITY)) {
                        full = false;
                        continue;
                    }
                    sK = s > sK ? s : sK;
                    if (ncomp[k] == mcomp) continue;  // also the point itself (INCL lists)
                    double mrd = sqrt(s);             // HDBSCANStar.java:162-168 order, as the scan kernel
                    if (mcore > mrd) mrd = mcore;
                    const double oc = ncore[k];
                    if (oc > mrd) mrd = oc;
                    const int32_t oid = nid[k];
                    const int32_t lo = mid < oid ? mid : oid, hi = mid < oid ? oid : mid;
                    if (key_less(mrd, s, lo, hi, b)) {
                        b = Best{mrd, s, lo, hi};
                        bpos = j;
                    }
                }
                if (!exact && full && b.w < INFINITY) {
                    double lb = sqrt(sK);
                    if (mcore > lb) lb = mcore;
                    exact = (b.w < lb) || (b.w == lb && b.s < sK);
                }
            }
            if (done) done[i] = exact ? 1 : 0;
            xact[i] = exact ? 1 : 0;
            if (exact && b.w > lbw[i]) lbw[i] = b.w;
            best_w[i] = b.w;
            best_s[i] = b.s;
            best_lo[i] = b.lo;
            best_hi[i] = b.hi;
            best_pos[i] = bpos;
        }
        block_publish_min(comp_w, mcomp, dbits(b.w), i < n && b.w < INFINITY, s_c, s_v);
    }
}

// ------------------------------------------------------------ K1t: tree kNN
// chunk size for m chunks per XCD (m <= 0: off): the last chunk holds the remainder, so no XCD
// gets more than one chunk over the mean
inline int k1t_xcb(int64_t ntiles, int m) {
    return m > 0 ? (int)std::max<int64_t>(1, ceil_div(ceil_div(ntiles, 4), 8 * (int64_t)m)) : 0;
}
inline unsigned k1t_grid(int64_t ntiles, int xcb) {
    const int64_t g = ceil_div(ntiles, 4);
    return (unsigned)(xcb > 0 ? ceil_div(g, 8 * (int64_t)xcb) * 8 * xcb : g);
}
// A wave owns query tile t (lane = point).  Its own tile is scanned first (it holds the
// nearest candidates in Morton order, so the K-th bound is tight from the start), then the
// BVH is walked nearest-first, skipping any node whose box no lane can still improve on.
// A visited tile is fetched with one vector load and staged in LDS; candidates are then
// wave-uniform broadcast reads, and each lane evaluates the exact FP64 squared distance in
// the reference's order and feeds the register top-K network.
template <int D, int K, bool IDX, bool STATS>
__global__ __launch_bounds__(256, (D <= 3 ? HDB_K1T_WPE : 1)) void knn_tree_kernel(const Rec<D> *__restrict__ recs, int64_t n, int64_t ntiles,
                                                       Bvh bvh, int excl, double *__restrict__ lists,
                                                       int32_t *__restrict__ nb_pos, double *__restrict__ nb_s,
                                                       int pop_test, int xcb, unsigned long long *__restrict__ stats) {
    __shared__ int32_t stack_s[4][MAXLEV * FAN + 8];
    __shared__ LRec<D> tile_s[4][BT];
    __shared__ double boxs_s[4][BOXBUF * D];
    __shared__ int32_t boxt_s[4][FAN];
    __shared__ int64_t lvl_s[4][2 * (MAXLEV + 1)];
    __shared__ double q_s[4][2 * D];
#if HDB_K1T_ROWS
#if HDB_K1T_SHFL
    // the query lanes' coordinates, bounds and self ids come by lane shuffles (ds_bpermute): 10 KB
    // less LDS per workgroup, 8 instead of 5 workgroups per CU
    __shared__ double kq_s[4][BT];
    __shared__ int32_t kq_lane[4][BT];
#else
    __shared__ double kq_x[4][BT * D], kq_thr[4][BT], kq_s[4][BT];
    __shared__ int32_t kq_skip[4][BT], kq_lane[4][BT];
#endif
#endif
    const int w = threadIdx.x >> 6;
    int64_t *off_s = lvl_s[w], *cnt_s = lvl_s[w] + MAXLEV + 1;
    // (XCD-contiguous tile ranges were measured again in round 4: 1.56 -> 1.74 ms, not kept)
    const int64_t t = xcd_chunk_block(blockIdx.x, xcb) * 4 + w;
    if (t >= ntiles) return;
    const int lane = threadIdx.x & 63;
    int32_t *stk = stack_s[w];
    LRec<D> *cand = tile_s[w];
    double *bxs = boxs_s[w];
    int32_t *bxt = boxt_s[w];
    const int64_t i = t * BT + lane;
    const bool valid = i < n;
    double mx[D];
    int32_t mid = -1;
    if (valid) {
        const Rec<D> r = recs[i];
#pragma unroll
        for (int c = 0; c < D; c++) mx[c] = r.x[c];
        mid = r.id;
    } else {
#pragma unroll
        for (int c = 0; c < D; c++) mx[c] = 0;
    }
    double buf[K];
    int bix[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        buf[k] = INFINITY;
        bix[k] = -1;
    }
    const int32_t skip_self = excl ? mid : -2;
    unsigned long long nev = 0, n_leaf = 0, n_node = 0;
#if HDB_K1T_ROWS
#if !HDB_K1T_SHFL
#pragma unroll
    for (int c = 0; c < D; c++) kq_x[w][lane * D + c] = mx[c];
    kq_skip[w][lane] = skip_self;
#endif
#endif

    auto needs_vals = [&](const double (&a)[D], const double (&b)[D], int32_t) -> bool {
        return valid & (box_lb2v<D>(mx, a, b) < buf[K - 1]);
    };
    int sp = 0;
    auto scan_leaf = [&](int64_t tile, bool own) {
        // the tile's 64 records (one coalesced vector load) and group boxes (cooperative
        // staging), one round trip; the records are staged in LDS for broadcast reads
        const LRec<D> mine = fetch_rec<D>(recs, n, tile * BT + lane);
        stage_boxes<D, NSG>(bvh.slo + tile * NSG * D, bvh.shi + tile * NSG * D, bvh.stag + tile * NSG, NSG, bxs, bxt,
                            lane);
        cand[lane] = mine;  // staged now: the record's registers die before the culling
        __builtin_amdgcn_wave_barrier();
        auto gneeds = [&](int gi) -> bool {
            double a[D], b[D];
            staged_box<D, NSG>(bxs, gi, a, b);
            return needs_vals(a, b, 0);
        };
        unsigned gmask = 0;
#pragma unroll 1
        for (int gi = 0; gi < NSG; gi++)
            if (own || __any(gneeds(gi))) gmask |= 1u << gi;
        if (gmask == 0) return;
        n_leaf++;
#pragma unroll 1
        for (int gi = 0; gi < NSG; gi++) {
            if (!((gmask >> gi) & 1u)) continue;
            const int64_t sg = tile * NSG + gi;
            if (!own && !__any(gneeds(gi))) continue;  // re-test in registers with the current bound
            const int64_t j0 = sg * SG, j1 = min(j0 + SG, n);
            if (j1 <= j0) break;
            nev += (unsigned long long)(j1 - j0);
            const int q0 = gi * SG, q1 = q0 + (int)(j1 - j0);
#if HDB_K1T_ROWS
            // few lanes need this group (not the own tile): the (needing lane, candidate) pairs
            // in 16-lane rows against the group-start K-th values (only looser: a rejected
            // candidate fails the insertion test at its turn too), the passers inserted by their
            // query lane in candidate order -- the same lists, ties included (see K2b's rows)
            if (!own) {
                const bool need = gneeds(gi);
                const unsigned long long M = __ballot(need);
                const int Kn = __popcll(M);
                if (Kn <= HDB_K1T_ROWS_MAX) {
                    const int rank = __popcll(M & ((1ull << lane) - 1));
#if HDB_K1T_SHFL
                    const double thr0 = buf[K - 1];  // the group-start K-th value of every lane
                    if (need) kq_lane[w][rank] = lane;
#else
                    if (need) {
                        kq_thr[w][lane] = buf[K - 1];
                        kq_lane[w][rank] = lane;
                    }
#endif
                    __builtin_amdgcn_wave_barrier();
                    const int row = lane >> 4, c = lane & 15;
                    const LRec<D> r = cand[q0 + c];
                    for (int r0 = 0; r0 < Kn; r0 += 4) {
                        const int qr = r0 + row;
                        const bool rowact = qr < Kn;
                        const int ql = kq_lane[w][rowact ? qr : 0];
#if HDB_K1T_SHFL
                        double s2 = sq_diff(__shfl(mx[0], ql), r.x[0]);
#pragma unroll
                        for (int cc = 1; cc < D; cc++) s2 = s2 + sq_diff(__shfl(mx[cc], ql), r.x[cc]);
                        const bool pass = rowact & (q0 + c < q1) & (r.id != __shfl(skip_self, ql)) &
                                          (s2 < __shfl(thr0, ql));
#else
                        double s2 = sq_diff(kq_x[w][ql * D], r.x[0]);
#pragma unroll
                        for (int cc = 1; cc < D; cc++) s2 = s2 + sq_diff(kq_x[w][ql * D + cc], r.x[cc]);
                        const bool pass = rowact & (q0 + c < q1) & (r.id != kq_skip[w][ql]) & (s2 < kq_thr[w][ql]);
#endif
                        if (pass) kq_s[w][lane] = s2;
                        const unsigned long long pm = __ballot(pass);
                        __builtin_amdgcn_wave_barrier();
                        if (need && rank >= r0 && rank < r0 + 4) {
                            const int rr = rank - r0;
                            unsigned bits = (unsigned)(pm >> (16 * rr)) & 0xFFFFu;
                            while (bits) {  // ascending candidate order
                                const int k = __builtin_ctz(bits);
                                bits &= bits - 1;
                                const double sv = kq_s[w][16 * rr + k];
                                if (IDX) topk_insert_idx<K>(buf, bix, sv, (int)(tile * BT + q0 + k));
                                else topk_insert<K>(buf, sv);
                            }
                        }
                        __builtin_amdgcn_wave_barrier();
                    }
                    continue;
                }
            }
#endif
#pragma unroll CAND_UNROLL
            for (int qq = q0; qq < q1; qq++) {
                const LRec<D> r = cand[qq];  // uniform address -> LDS broadcast
                double s = sq_diff(mx[0], r.x[0]);
#pragma unroll
                for (int c = 1; c < D; c++) s = s + sq_diff(mx[c], r.x[c]);
                if (r.id == skip_self) s = INFINITY;
                if (IDX) topk_insert_idx<K>(buf, bix, s, (int)(tile * BT + qq));
                else topk_insert<K>(buf, s);
            }
        }
    };
    scan_leaf(t, true);  // own tile first: the K-th bound is tight from the start
    double *qlo = q_s[w], *qhi = q_s[w] + D;  // query box (the own tile's) in LDS
    if (lane < 2 * D) q_s[w][lane] = lane < D ? bvh.lo[t * D + lane] : bvh.hi[t * D + lane - D];
    __builtin_amdgcn_wave_barrier();
    level_table(ntiles, off_s, cnt_s, lane);
    if (lane == 0) stk[0] = ((bvh.levels - 1) << 26) | 0;
    sp = 1;
    while (sp > 0) {
        __builtin_amdgcn_wave_barrier();
        const int32_t code = __builtin_amdgcn_readfirstlane(stk[sp - 1]);
        sp--;
        const int lev = code >> 26;
        const int64_t idx = code & ((1 << 26) - 1);
        n_node++;
        if (lev == 0) {
            if (idx == t) continue;
            if (pop_test & 2) {  // re-test the popped leaf with the current K-th bound
                stage_boxes<D, 1>(bvh.lo + idx * D, bvh.hi + idx * D, bvh.tag + idx, 1, bxs, bxt, lane);
                double a[D], b[D];
                staged_box<D, 1>(bxs, 0, a, b);
                if (!__any(needs_vals(a, b, 0))) continue;
            }
            scan_leaf(idx, false);
            continue;
        }
        push_children<D>(bvh, off_s, cnt_s, lev, idx, qlo, qhi, stk, sp, lane, bxs, bxt, needs_vals);
    }
    if (valid) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double v = buf[k];
            lists[(int64_t)mid * K + k] = (v < INFINITY) ? sqrt(v) : JMAX;  // Java keeps Double.MAX_VALUE
            if (IDX) {  // sorted-position neighbour list (squared distances) for the MST seeds
                nb_pos[i * K + k] = bix[k];
                nb_s[i * K + k] = v;
            }
        }
    }
    if (STATS) {
        const unsigned long long nvalid = (unsigned long long)__popcll(__ballot(valid));
        if (lane == 0) {
            atomicAdd(&stats[0], nev * nvalid);  // (query, candidate) pairs evaluated
            atomicAdd(&stats[1], n_leaf);
            atomicAdd(&stats[2], n_node);
        }
    }
}

// ---------------------------------------------------------------- host
// The index over one partition: Morton-sorted records + BVH (level 0 = 64-point tiles).
template <int D>
struct Spatial {
    int64_t n = 0, ntiles = 0;
    Rec<D> *recs = nullptr;
    int32_t *inv = nullptr;  // original id -> sorted position
    Bvh bvh;
    // scratch reused by the callers (n entries each)
    uint64_t *keys = nullptr, *keys2 = nullptr;
    int32_t *iota = nullptr, *perm = nullptr;
};

static Bvh bvh_shape(int64_t ntiles) {
    Bvh bvh;
    int64_t c = ntiles, tot = 0;
    bvh.levels = 0;
    while (true) {
        if (bvh.levels >= MAXLEV) HDB_THROW(HDB_EINVAL, "spatial index: too many BVH levels");
        bvh.off[bvh.levels] = tot;
        bvh.cnt[bvh.levels] = c;
        tot += c;
        bvh.levels++;
        if (c == 1) break;
        c = ceil_div(c, FAN);
    }
    bvh.off[bvh.levels] = tot;
    return bvh;
}

// bump allocator over one arena slot: pass 1 sizes (base == nullptr), pass 2 assigns
struct Carve {
    char *base = nullptr;
    size_t off = 0;
    template <class T>
    T *take(size_t count) {
        size_t o = off;
        off += (sizeof(T) * count + 255) & ~size_t(255);
        return base ? (T *)(base + o) : nullptr;
    }
};

template <int D>
static void spatial_carve(Carve &cv, Spatial<D> &sp) {
    const int64_t n = sp.n, nnodes = sp.bvh.off[sp.bvh.levels];
    sp.bvh.lo = cv.take<double>((size_t)D * nnodes);
    sp.bvh.hi = cv.take<double>((size_t)D * nnodes);
    sp.bvh.tag = cv.take<int32_t>(nnodes);
    sp.bvh.slo = cv.take<double>((size_t)D * sp.ntiles * NSG);
    sp.bvh.shi = cv.take<double>((size_t)D * sp.ntiles * NSG);
    sp.bvh.stag = cv.take<int32_t>((size_t)sp.ntiles * NSG);
    sp.recs = cv.take<Rec<D>>(n);
    sp.inv = cv.take<int32_t>(n);
    sp.keys = cv.take<uint64_t>(n);
    sp.keys2 = cv.take<uint64_t>(n);
    sp.iota = cv.take<int32_t>(n);
    sp.perm = cv.take<int32_t>(n);
}

// Builds the index on ctx->stream.  core nullable (records then carry 0).  `extra` = bytes
// the caller wants carved after the index in the same arena slot (returned in *extra_ptr).
template <int D>
static Spatial<D> build_spatial(hdb_ctx *ctx, const double *X, int64_t n, const double *core, Carve &cv) {
    if (n > INT32_MAX / 2) HDB_THROW(HDB_EINVAL, "n too large");
    Spatial<D> sp;
    sp.n = n;
    sp.ntiles = ceil_div(n, BT);
    sp.bvh = bvh_shape(sp.ntiles);
    spatial_carve<D>(cv, sp);
    double *blo = cv.take<double>(64), *bhi = cv.take<double>(64);
    double *bpart = cv.take<double>((size_t)BBOX_BLOCKS * 2 * D);
    if (!cv.base) return sp;
    const int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    hipStream_t st = ctx->stream;
    const int nbb = (int)std::min<int64_t>(BBOX_BLOCKS, ceil_div(n, 256));
    hipLaunchKernelGGL(bbox_partial_kernel<D>, dim3(nbb), dim3(256), 0, st, X, n, bpart);
    hipLaunchKernelGGL(bbox_final_kernel<D>, dim3(D), dim3(64), 0, st, bpart, nbb, blo, bhi);
    const SsPlan pl = ss_plan(n, ctx->ssort_cap);
    if (ctx->ssort && pl.nb) {  // Morton order + records in one sample sort
        ssort(pl, (char *)arena(ctx, A_SS, pl.bytes), MortonKeyF<D>{X, blo, bhi},
              RecEmitF<D>{X, core, sp.recs, sp.inv}, st);
    } else {
        hipLaunchKernelGGL(morton_kernel, dim3(g), dim3(256), 0, st, X, n, D, blo, bhi, sp.keys, sp.iota);
        size_t tb = 0;
        const int kbits = (D < 8 ? D : 8) * morton_bits(D);
        HIP_CHECK(sort_pairs(nullptr, tb, sp.keys, sp.keys2, sp.iota, sp.perm, n, 0, kbits, st));
        void *tmp = arena(ctx, A_SORT, tb);
        HIP_CHECK(sort_pairs(tmp, tb, sp.keys, sp.keys2, sp.iota, sp.perm, n, 0, kbits, st));
        hipLaunchKernelGGL(build_recs_kernel<D>, dim3(g), dim3(256), 0, st, X, core, sp.perm, n, sp.recs, sp.inv);
    }
    hipLaunchKernelGGL(tile_box_kernel<D>, dim3((unsigned)sp.ntiles), dim3(64), 0, st, sp.recs, n, sp.bvh.lo,
                       sp.bvh.hi, sp.bvh.slo, sp.bvh.shi);
    for (int L = 1; L < sp.bvh.levels; L++)
        hipLaunchKernelGGL(bvh_box_kernel<D>, dim3((unsigned)std::min<int64_t>(ceil_div(sp.bvh.cnt[L], 256), 4096)),
                           dim3(256), 0, st, sp.bvh.lo, sp.bvh.hi, sp.bvh.off[L - 1], sp.bvh.cnt[L - 1], sp.bvh.off[L],
                           sp.bvh.cnt[L]);
    HIP_CHECK(hipGetLastError());
    return sp;
}

template <int D>
static Spatial<D> build_spatial_in(hdb_ctx *ctx, int slot, const double *X, int64_t n, const double *core,
                                   Carve &cv, size_t extra_bytes, char **extra) {
    Carve probe;
    build_spatial<D>(ctx, X, n, core, probe);
    char *base = (char *)arena(ctx, slot, probe.off + extra_bytes + 256);
    cv.base = base;
    cv.off = 0;
    Spatial<D> sp = build_spatial<D>(ctx, X, n, core, cv);
    if (extra) *extra = base + ((cv.off + 255) & ~size_t(255));
    return sp;
}

// ------------------------------------------------------------------- K1t host
template <int D, int K>
static void knn_tree_impl(hdb_ctx *ctx, const double *X, int64_t n, bool excl, double *lists) {
    Carve cv;
    char *extra = nullptr;
    Spatial<D> sp = build_spatial_in<D>(ctx, A_WORK1, X, n, nullptr, cv, 64, &extra);
    unsigned long long *evals = ctx->count_evals ? (unsigned long long *)extra : nullptr;
    if (evals) HIP_CHECK(hipMemsetAsync(evals, 0, 24, ctx->stream));
    {
        KernelTimer t(ctx, "knn_tree");
        const int xcb = k1t_xcb(sp.ntiles, ctx->k1t_xcd_chunks);
        if (evals)
            hipLaunchKernelGGL((knn_tree_kernel<D, K, false, true>), dim3(k1t_grid(sp.ntiles, xcb)), dim3(256),
                               0, ctx->stream, sp.recs, n, sp.ntiles, sp.bvh, excl ? 1 : 0, lists, nullptr, nullptr,
                               ctx->trav_pop_test, xcb, evals);
        else
            hipLaunchKernelGGL((knn_tree_kernel<D, K, false, false>), dim3(k1t_grid(sp.ntiles, xcb)),
                               dim3(256), 0, ctx->stream, sp.recs, n, sp.ntiles, sp.bvh, excl ? 1 : 0, lists, nullptr,
                               nullptr, ctx->trav_pop_test, xcb, evals);
        HIP_CHECK(hipGetLastError());
    }
    if (evals) {
        unsigned long long h[3];
        HIP_CHECK(hipMemcpyAsync(h, evals, 24, hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        ctx->stats["knn_tree_evals"] = (int64_t)h[0];
        ctx->stats["knn_tree_leaves"] = (int64_t)h[1];
        ctx->stats["knn_tree_nodes"] = (int64_t)h[2];
        ctx->stats["last_evals"] = (int64_t)h[0];
    }
}

template <int D>
static bool knn_tree_k(hdb_ctx *ctx, const double *X, int64_t n, int KC, bool excl, double *lists) {
    switch (KC) {
    case 1: knn_tree_impl<D, 1>(ctx, X, n, excl, lists); return true;
    case 3: knn_tree_impl<D, 3>(ctx, X, n, excl, lists); return true;
    case 7: knn_tree_impl<D, 7>(ctx, X, n, excl, lists); return true;
    case 15: knn_tree_impl<D, 15>(ctx, X, n, excl, lists); return true;
    case 31: knn_tree_impl<D, 31>(ctx, X, n, excl, lists); return true;
    default: return false;
    }
}

bool knn_tree_device(hdb_ctx *ctx, const double *X, int64_t n, int d, int KC, bool excl, double *lists) {
    switch (d) {
    case 1: return knn_tree_k<1>(ctx, X, n, KC, excl, lists);
    case 2: return knn_tree_k<2>(ctx, X, n, KC, excl, lists);
    case 3: return knn_tree_k<3>(ctx, X, n, KC, excl, lists);
    case 4: return knn_tree_k<4>(ctx, X, n, KC, excl, lists);
    case 8: return knn_tree_k<8>(ctx, X, n, KC, excl, lists);
    case 16: return knn_tree_k<16>(ctx, X, n, KC, excl, lists);
    default: return false;
    }
}

// ------------------------------------------------------------------- K2b host
// per-round Boruvka state carved after the index: comp_w, comp_key, comp_s, best_w, best_s
// (8n each), best_lo/hi, parent, parent2 (4n each), counters, edge lists
// diag: count_evals -- one BOR_STATS_REC-word record per scan wave, sized for the most waves a
// round can have (16 points per wave: boruvka_wave_pts / boruvka_early_pts may ask for it)
static size_t boruvka_extra_bytes(int64_t n, bool diag) {
    const size_t per = (size_t)n;
    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t waves_max = (size_t)ceil_div(n, (int64_t)WGRP) * (WGRP / 16);
    return 5 * rnd(8 * per) + 5 * rnd(4 * per) + 3 * 256 + 2 * rnd(4 * per) + rnd(8 * per) +
           (diag ? rnd(8 * (size_t)BOR_STATS_REC * waves_max) : 0) +
           rnd(4 * per) + 3 * rnd(4 * (per / WGRP + 1)) + rnd(8 * waves_max) + 256 +  // + work lists
           2 * rnd(4 * per) + rnd(8 * per) + rnd(per);  // + best_pos, pcomp, lbw, xact
}

// k-NN lists over the index's sorted positions (K1t with IDX): seed every Boruvka round
struct KnnLists {
    const int32_t *pos = nullptr;
    const double *s = nullptr;  // squared distances, ascending per row
    int K = 0;
    uint8_t *done = nullptr;  // n flags: the lane's seed is exact this round
};

// Boruvka rounds over a built index whose records carry the core distances.  extra: the
// boruvka_extra_bytes(n) region.  kl (nullable): k-NN lists that seed every round.
template <int D>
static void boruvka_on_index(hdb_ctx *ctx, Spatial<D> &sp, int64_t n, char *extra, const KnnLists *kl,
                             int32_t *va, int32_t *vb, double *w, bool merged = false,
                             const double *self_core = nullptr);

template <int D>
struct BoruvkaState {
    unsigned long long *comp_w, *comp_key, *comp_s;
    double *best_w, *best_s;
    int32_t *best_lo, *best_hi;
    int32_t *best_pos;  // sorted position of the best edge's partner
    int32_t *pcomp;     // component per sorted position (a compact copy of Rec::comp)
    double *lbw;        // per point: lower bound of its best outgoing weight (monotone over rounds)
    uint8_t *xact;      // per point: best_* is the exact best of the last round
};
template <int D>
static BoruvkaState<D> boruvka_state(char *extra, int64_t n, size_t *used = nullptr) {
    Carve ex;
    ex.base = extra;
    const size_t per = (size_t)n;
    BoruvkaState<D> b;
    b.best_w = ex.take<double>(per);
    b.best_s = ex.take<double>(per);
    b.best_lo = ex.take<int32_t>(per);
    b.best_hi = ex.take<int32_t>(per);
    b.comp_w = ex.take<unsigned long long>(per);
    b.comp_key = ex.take<unsigned long long>(per);
    b.comp_s = ex.take<unsigned long long>(per);
    b.best_pos = ex.take<int32_t>(per);
    b.pcomp = ex.take<int32_t>(per);
    b.lbw = ex.take<double>(per);
    b.xact = ex.take<uint8_t>(per);
    if (used) *used = ex.off;
    return b;
}

template <int D>
static void boruvka_impl(hdb_ctx *ctx, const double *X, int64_t n, const double *core, int32_t *va, int32_t *vb,
                         double *w) {
    Carve cv;
    char *extra = nullptr;
    KernelTimer tt(ctx, "boruvka_total");
    Spatial<D> sp = build_spatial_in<D>(ctx, A_WORK0, X, n, core, cv, boruvka_extra_bytes(n, ctx->count_evals), &extra);
    boruvka_on_index<D>(ctx, sp, n, extra, nullptr, va, vb, w);
}

template <int D>
static void boruvka_on_index(hdb_ctx *ctx, Spatial<D> &sp, int64_t n, char *extra, const KnnLists *kl,
                             int32_t *va, int32_t *vb, double *w, bool merged, const double *self_core) {
    const size_t per = (size_t)n;
    size_t used = 0;
    BoruvkaState<D> bs = boruvka_state<D>(extra, n, &used);
    Carve ex;  // the rest of the region, after the BoruvkaState arrays
    ex.base = extra;
    ex.off = used;
    unsigned long long *comp_w = bs.comp_w, *comp_key = bs.comp_key, *comp_s = bs.comp_s;
    double *best_w = bs.best_w, *best_s = bs.best_s;
    int32_t *best_lo = bs.best_lo, *best_hi = bs.best_hi;
    int32_t *parent = ex.take<int32_t>(per), *parent2 = ex.take<int32_t>(per);
    unsigned long long *n_edges = ex.take<unsigned long long>(1);
    int32_t *ea = ex.take<int32_t>(per), *eb = ex.take<int32_t>(per);
    double *ew = ex.take<double>(per);
    std::vector<unsigned long long> wave_cyc(ctx->count_evals ? sp.ntiles : 0);
    const int64_t ngroups = ceil_div(n, (int64_t)WGRP);
    const int P = ctx->boruvka_wave_pts;
    if (P != 16 && P != 32 && P != 64) HDB_THROW(HDB_EINVAL, "boruvka_wave_pts must be 16, 32 or 64");
    // early rounds search few lanes (few waves in flight for a latency-bound walk): optionally
    // spread their work over more, smaller waves
    const int PE = ctx->boruvka_early_pts ? ctx->boruvka_early_pts : P;
    if (PE != 16 && PE != 32 && PE != 64) HDB_THROW(HDB_EINVAL, "boruvka_early_pts must be 16, 32 or 64");
    const int64_t max_waves = ngroups * (WGRP / std::min(P, PE));
    int32_t *work = ex.take<int32_t>(per);
    int32_t *gcnt = ex.take<int32_t>(ngroups), *gwaves = ex.take<int32_t>(ngroups), *woff = ex.take<int32_t>(ngroups);
    unsigned long long *desc = ex.take<unsigned long long>(max_waves);
    int32_t *nwaves = ex.take<int32_t>(1);
    unsigned long long *evals = ctx->count_evals ? ex.take<unsigned long long>((size_t)BOR_STATS_REC * max_waves) : nullptr;
    if (ex.off > boruvka_extra_bytes(n, ctx->count_evals))
        HDB_THROW(HDB_EINVAL, "boruvka: scratch carve exceeds its reserve");
    int64_t tot_evals = 0;
    Rec<D> *recs = sp.recs;
    int32_t *inv = sp.inv;
    Bvh bvh = sp.bvh;
    const int64_t ntiles = sp.ntiles;
    int32_t *tcomp = bvh.tag;
    const int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    hipStream_t st = ctx->stream;
    HIP_CHECK(hipMemsetAsync(n_edges, 0, 8, st));
    hipLaunchKernelGGL(fill_inf_kernel, dim3(g), dim3(256), 0, st, best_w, n);
    HIP_CHECK(hipMemsetAsync(bs.lbw, 0, sizeof(double) * per, st));  // +0.0: no bound yet
    HIP_CHECK(hipMemsetAsync(bs.xact, 0, per, st));
    HIP_CHECK(hipGetLastError());
    int32_t *best_pos = bs.best_pos, *pcomp = bs.pcomp;
    hipLaunchKernelGGL(pos_iota_kernel, dim3(g), dim3(256), 0, st, pcomp, n);  // comp = own position
    auto round_seed = [&](int round) {
        const int prev = (round > 0 && ctx->boruvka_seed) ? 1 : 0;
        // the lists stop paying once components outgrow them (their points are then all
        // inside the component): seed from them only in the first list_rounds rounds
        const int K = (kl && round < ctx->leaf_list_rounds) ? kl->K : 0;
        if (!prev && K == 0) {
            if (round > 0) hipLaunchKernelGGL(fill_inf_kernel, dim3(g), dim3(256), 0, st, best_w, n);
            if (kl && kl->done) HIP_CHECK(hipMemsetAsync(kl->done, 0, (size_t)n, st));  // no exact seeds
            return;
        }
#ifndef HDB_SEED_MAX_BLOCKS
#define HDB_SEED_MAX_BLOCKS 2048
#endif
        const int gs = (int)std::min<int64_t>(ceil_div(n, 256), HDB_SEED_MAX_BLOCKS);
#define ROUND_SEED(KK)                                                                                                 \
    case KK:                                                                                                           \
        hipLaunchKernelGGL((round_seed_kernel<D, KK>), dim3(gs), dim3(256), 0, st, recs, pcomp, n, prev,              \
                           kl ? kl->pos : nullptr, kl ? kl->s : nullptr, best_w, best_s, best_lo, best_hi, best_pos,  \
                           kl ? kl->done : nullptr, bs.lbw, bs.xact, comp_w);                                          \
        break;
        switch (K) {
            ROUND_SEED(0)
            ROUND_SEED(1)
            ROUND_SEED(3)
            ROUND_SEED(7)
            ROUND_SEED(15)
            ROUND_SEED(31)
        default: HDB_THROW(HDB_EINVAL, "round seed: unsupported list length");
        }
#undef ROUND_SEED
        HIP_CHECK(hipGetLastError());
    };

    static const char *round_names[] = {"boruvka_r0", "boruvka_r1", "boruvka_r2", "boruvka_r3", "boruvka_r4",
                                        "boruvka_r5", "boruvka_r6", "boruvka_r7", "boruvka_r8+"};
    // Rounds are enqueued one ahead of the host's view of the edge count: the count after
    // round r is copied to pinned memory and read only after round r+1 is queued, so the
    // device never idles on a host round trip.  A round queued after the tree completed is a
    // no-op (its scan exits on the count; no component has an outgoing edge to hook).
    int64_t *hcnt = pinned_words(ctx);
    const int max_rounds = 64;
    std::vector<hipEvent_t> round_ev;
    auto release_events = [&]() {
        for (auto e : round_ev) (void)hipEventDestroy(e);
        round_ev.clear();
    };
    for (int round = 0; n > 1; round++) {
        if (round >= max_rounds || round >= PINNED_WORDS) {
            release_events();
            HDB_THROW(HDB_EINVAL, "boruvka did not converge (non-finite distances?)");
        }
        // internal node tags -> EMPTY, then relabel (previous round's hook roots) + tags
        const int64_t n_inner = bvh.off[bvh.levels] - bvh.off[1];
        hipLaunchKernelGGL(reset_comp_kernel, dim3(g), dim3(256), 0, st, comp_w, comp_key, comp_s, n,
                           tcomp + bvh.off[1], n_inner);
        hipLaunchKernelGGL(retag_kernel<D>, dim3((unsigned)ceil_div(ntiles, 4)), dim3(256), 0, st, recs, pcomp, n,
                           ntiles, bvh.levels, round > 0 ? parent2 : nullptr, tcomp, bvh.stag);
        if (evals) HIP_CHECK(hipMemsetAsync(evals, 0, 8 * (size_t)BOR_STATS_REC * max_waves, st));
        round_seed(round);
        {
            KernelTimer ts(ctx, "boruvka_scan");
            KernelTimer tr(ctx, round_names[round < 8 ? round : 8]);
            const int Pr = round < ctx->boruvka_early_rounds ? PE : P;
            if (ctx->boruvka_adj_seed && round > 0)
                hipLaunchKernelGGL(adj_seed_kernel<D>, dim3(g), dim3(256), 0, st, recs, pcomp, n, comp_w);
            hipLaunchKernelGGL(group_compact_kernel<D>, dim3((unsigned)ngroups), dim3(WGRP), 0, st, recs, n,
                               kl ? kl->done : nullptr, bs.lbw, comp_w, Pr, work, gcnt, gwaves);
            size_t tb = 0;
            HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, gwaves, woff, (int)ngroups, st));
            void *tmp = arena(ctx, A_SORT, tb);
            HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, gwaves, woff, (int)ngroups, st));
            hipLaunchKernelGGL(wave_desc_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(ngroups, 256), 4096)),
                               dim3(256), 0, st, gcnt, woff, ngroups, Pr, desc, nwaves);
            const int xm = ctx->bor_xcd_chunks > 0 ? ctx->bor_xcd_chunks : 0;
            const unsigned scan_grid = (unsigned)(ceil_div(max_waves, 4) + 8 * xm);
            if (evals)
                hipLaunchKernelGGL((boruvka_bvh_kernel<D, true>), dim3(scan_grid), dim3(256), 0,
                                   st, recs, n, ntiles, bvh, comp_w, best_w, best_s, best_lo, best_hi, work, desc,
                                   nwaves, ctx->trav_pop_test, inv, best_pos, n_edges, bs.lbw, bs.xact, xm, evals);
            else
                hipLaunchKernelGGL((boruvka_bvh_kernel<D, false>), dim3(scan_grid), dim3(256), 0,
                                   st, recs, n, ntiles, bvh, comp_w, best_w, best_s, best_lo, best_hi, work, desc,
                                   nwaves, ctx->trav_pop_test, inv, best_pos, n_edges, bs.lbw, bs.xact, xm, evals);
        }
        if (evals) {
            std::vector<unsigned long long> recs_h((size_t)BOR_STATS_REC * max_waves);
            HIP_CHECK(hipMemcpyAsync(recs_h.data(), evals, 8 * recs_h.size(), hipMemcpyDeviceToHost, st));
            HIP_CHECK(hipStreamSynchronize(st));
            unsigned long long h[BOR_STATS_REC] = {};
            wave_cyc.clear();
            for (int64_t t = 0; t < max_waves; t++) {
                const unsigned long long *rec = recs_h.data() + (size_t)t * BOR_STATS_REC;
                for (int k = 0; k < BOR_STATS_REC; k++) h[k] += rec[k];
                if (rec[5]) wave_cyc.push_back(rec[5]);  // waves that ran (exited waves leave 0)
            }
            const std::string r = "boruvka_r" + std::to_string(round);
            if (HDB_BOR_PROF) {
                static const char *pn[BOR_PROF_N] = {"setup", "pop", "stage", "test", "push",
                                                     "leaf_load", "leaf_mask", "leaf_eval", "publish", "tail"};
                for (int k = 0; k < BOR_PROF_N; k++) ctx->stats[r + "_prof_" + pn[k]] = (int64_t)h[6 + k];
            }
            if (wave_cyc.empty()) wave_cyc.push_back(0);
            std::sort(wave_cyc.begin(), wave_cyc.end());
            unsigned long long cs = 0;
            for (auto c : wave_cyc) cs += c;
            ctx->stats[r + "_wave_cyc_mean"] = (int64_t)(cs / wave_cyc.size());
            ctx->stats[r + "_wave_cyc_p50"] = (int64_t)wave_cyc[wave_cyc.size() / 2];
            ctx->stats[r + "_wave_cyc_p99"] = (int64_t)wave_cyc[wave_cyc.size() * 99 / 100];
            ctx->stats[r + "_wave_cyc_max"] = (int64_t)wave_cyc.back();
            ctx->stats[r + "_active_lanes"] = (int64_t)h[3];
            ctx->stats[r + "_active_waves"] = (int64_t)h[4];
            ctx->stats[r + "_evals"] = (int64_t)h[0];
            ctx->stats[r + "_leaves"] = (int64_t)h[1];
            ctx->stats[r + "_nodes"] = (int64_t)h[2];
            tot_evals += (int64_t)h[0];
            // accumulated over calls (C3/C5 lines: every forced leaf of a job): visits, executed
            // pair evals and the latency model's lower bound -- one dependent Infinity-Cache round
            // trip (227 ns) per visit over min(waves, resident wave slots) in flight
            const int64_t visits = (int64_t)(h[1] + h[2]), waves = (int64_t)h[4];
            ctx->stats["boruvka_visits_sum"] += visits;
            ctx->stats["boruvka_evals_sum"] += (int64_t)h[0];
            if (visits > 0)
                ctx->stats["boruvka_bound_ns_sum"] += visits * 227 / std::max<int64_t>(1, std::min<int64_t>(waves, 4096));
        }
        hipLaunchKernelGGL(comp_s_kernel, dim3(g), dim3(256), 0, st, pcomp, n, comp_w, best_w, best_s, comp_s);
        hipLaunchKernelGGL(comp_key_kernel, dim3(g), dim3(256), 0, st, pcomp, n, comp_w, comp_s, best_w, best_s,
                           best_lo, best_hi, comp_key);
        hipLaunchKernelGGL(hook_kernel, dim3(g), dim3(256), 0, st, pcomp, n, inv, comp_w, comp_key, parent, ea, eb,
                           ew, n_edges);
        hipLaunchKernelGGL(hook_fix_kernel<D>, dim3((unsigned)ceil_div(n, (int64_t)HF_T * HF_E)), dim3(HF_T), 0, st,
                           pcomp, n, comp_w, comp_key, parent, parent2,
                           ea, eb, ew, n_edges);
        // hook trees -> roots (one launch, no host round trip)
        hipLaunchKernelGGL(resolve_kernel, dim3(g), dim3(256), 0, st, parent2, n);
        HIP_CHECK(hipMemcpyAsync(hcnt + round, n_edges, 8, hipMemcpyDeviceToHost, st));
        hipEvent_t ev;
        HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        round_ev.push_back(ev);
        HIP_CHECK(hipEventRecord(ev, st));
        HIP_CHECK(hipGetLastError());
        if (round == 0) continue;  // keep one round in flight
        HIP_CHECK(hipEventSynchronize(round_ev[round - 1]));
        const int64_t c = hcnt[round - 1];
        if (c >= n - 1) break;  // the tree was complete: round `round` was a no-op
        if (round >= 2 && c == hcnt[round - 2]) {
            release_events();
            HDB_THROW(HDB_EINVAL, "boruvka made no progress (non-finite distances?)");
        }
    }
    release_events();
    if (evals) {
        ctx->stats["boruvka_evals"] = tot_evals;
        ctx->stats["last_evals"] = tot_evals;
    }
    // sort edges by (w, lo, hi): stable sort by (lo,hi) then stable by w
    bool sorted = false;
    if (ctx->ssort) {  // one sample sort: tree edges (+ self edges) straight into the outputs
        const int64_t ne = n - 1, tot = ne + ((merged && self_core) ? n : 0);
        const SsPlan pl = ss_plan(tot, ctx->ssort_cap);
        if (pl.nb) {
            sorted = ssort(pl, (char *)arena(ctx, A_SS, pl.bytes), TreeEdgeKeyF{ea, eb, ew, self_core, ne, merged},
                           TreeEdgeEmitF{va, vb, w, self_core, merged}, st);
        }
    }
    if (!sorted) {
        int64_t ne = n - 1;
        if (ne > 0) {
            uint64_t *k1 = sp.keys, *k2 = sp.keys2;
            int32_t *p1 = sp.iota, *p2 = sp.perm;
            int B = 1;
            while (B < 31 && ((int64_t)1 << B) < n) B++;
            hipLaunchKernelGGL(edge_idkey_kernel, dim3(g), dim3(256), 0, st, ea, eb, ne, B, k1, p1);
            size_t tb = 0;
            HIP_CHECK(sort_pairs(nullptr, tb, k1, k2, p1, p2, ne, 0, 2 * B, st));
            void *tmp = arena(ctx, A_SORT, tb);
            HIP_CHECK(sort_pairs(tmp, tb, k1, k2, p1, p2, ne, 0, 2 * B, st));
            hipLaunchKernelGGL(edge_wkey_kernel, dim3(g), dim3(256), 0, st, p2, ew, ne, k1);
            if (!merged) {
                // stable sort by w (non-negative doubles: bit order == numeric order, sign bit 0)
                HIP_CHECK(sort_pairs(nullptr, tb, k1, k2, p2, p1, ne, 0, 63, st));
                tmp = arena(ctx, A_SORT, tb);
                HIP_CHECK(sort_pairs(tmp, tb, k1, k2, p2, p1, ne, 0, 63, st));
                hipLaunchKernelGGL(edge_out_kernel, dim3(g), dim3(256), 0, st, p1, ea, eb, ew, ne, va, vb, w);
                HIP_CHECK(hipGetLastError());
            } else {
                // the reducers' merge order directly (SortMST.java:9-17, stable descending over
                // FirstStep's order): the tree edges by w DESCENDING, stable over the (lo, hi)
                // order -- exactly how a stable descending sort keeps FirstStep's (w, lo, hi)
                // tie groups -- then merged with the self edges sorted by core (descending, ids
                // ascending on ties), tree edges first on equal weights.  No 2n-1 re-sort.
                HIP_CHECK(sort_pairs_desc(nullptr, tb, k1, k2, p2, p1, ne, 0, 63, st));
                tmp = arena(ctx, A_SORT, tb);
                HIP_CHECK(sort_pairs_desc(tmp, tb, k1, k2, p2, p1, ne, 0, 63, st));
                if (!self_core) {
                    hipLaunchKernelGGL(edge_out_kernel, dim3(g), dim3(256), 0, st, p1, ea, eb, ew, ne, va, vb, w);
                    HIP_CHECK(hipGetLastError());
                } else {
                    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
                    const size_t o_tb = rnd(4 * (size_t)ne), o_tw = o_tb + rnd(4 * (size_t)ne),
                                 o_sk = o_tw + rnd(8 * (size_t)ne), o_sk2 = o_sk + rnd(8 * (size_t)n),
                                 o_si = o_sk2 + rnd(8 * (size_t)n), o_sp = o_si + rnd(4 * (size_t)n),
                                 tot = o_sp + rnd(4 * (size_t)n);
                    char *base = (char *)arena(ctx, A_WORK3, tot);
                    int32_t *ta = (int32_t *)base, *tbv = (int32_t *)(base + o_tb);
                    double *tw = (double *)(base + o_tw), *sk = (double *)(base + o_sk), *sk2 = (double *)(base + o_sk2);
                    int32_t *si = (int32_t *)(base + o_si), *sperm = (int32_t *)(base + o_sp);
                    hipLaunchKernelGGL(edge_out_kernel, dim3(g), dim3(256), 0, st, p1, ea, eb, ew, ne, ta, tbv, tw);
                    hipLaunchKernelGGL(self_keys_kernel, dim3(g), dim3(256), 0, st, self_core, n, sk, si);
                    size_t tb2 = 0;
                    HIP_CHECK(sort_pairs_desc(nullptr, tb2, sk, sk2, si, sperm, n, 0, 64, st));
                    void *tmp2 = arena(ctx, A_SORT, tb2);
                    HIP_CHECK(sort_pairs_desc(tmp2, tb2, sk, sk2, si, sperm, n, 0, 64, st));
                    hipLaunchKernelGGL(gather_core_kernel, dim3(g), dim3(256), 0, st, self_core, sperm, n, sk2);
                    merge_two_runs_device(ctx, ta, tbv, tw, ne, sperm, sperm, sk2, n, va, vb, w);
                }
            }
        }
    }
    if (merged && self_core && n - 1 <= 0) self_edges_device(ctx, self_core, n, va, vb, w);
}

__global__ void self_edges_kernel(const double *__restrict__ core, int64_t n, int32_t *__restrict__ va,
                                  int32_t *__restrict__ vb, double *__restrict__ w) {
    HDB_GRID_STRIDE(i, n) {
        va[i] = (int32_t)i;
        vb[i] = (int32_t)i;
        w[i] = core[i];
    }
}

void self_edges_device(hdb_ctx *ctx, const double *core, int64_t n, int32_t *va, int32_t *vb, double *w) {
    if (n <= 0) return;
    hipLaunchKernelGGL(self_edges_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(n, 256), 4096)), dim3(256), 0,
                       ctx->stream, core, n, va, vb, w);
    HIP_CHECK(hipGetLastError());
}


// ------------------------------------------------- fused exact leaf (a3 + a5)
// FirstStep's leaf branch for one large partition (FirstStep.java:104-108:
// calculateCoreDistances then constructMST) on ONE index: K1t also keeps each point's
// neighbour positions, the core epilogue runs on its lists, and Boruvka's round 0 starts
// from the kNN seeds (lanes whose seed is provably exact skip the traversal).
template <int D, int K>
static void exact_leaf_impl(hdb_ctx *ctx, const double *X, int64_t n, int min_pts, int semantics, double *core,
                            int self_edges, int32_t *va, int32_t *vb, double *w) {
    KernelTimer tt(ctx, "exact_leaf_total");
    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t bx = rnd(boruvka_extra_bytes(n, ctx->count_evals));
    const size_t nk = (size_t)n * K;
    const size_t more = rnd(8 * nk) + rnd(4 * nk) + rnd(8 * nk) + rnd((size_t)n) + 256;
    Carve cv;
    char *extra = nullptr;
    Spatial<D> sp = build_spatial_in<D>(ctx, A_WORK0, X, n, nullptr, cv, bx + more, &extra);
    Carve ex;
    ex.base = extra + bx;
    double *lists = ex.take<double>(nk);
    int32_t *nb_pos = ex.take<int32_t>(nk);
    double *nb_s = ex.take<double>(nk);
    uint8_t *done = ex.take<uint8_t>((size_t)n);
    unsigned long long *stats = ctx->count_evals ? ex.take<unsigned long long>(3) : nullptr;
    if (stats) HIP_CHECK(hipMemsetAsync(stats, 0, 24, ctx->stream));
    {
        KernelTimer t(ctx, "knn_tree");
        const int xcb = k1t_xcb(sp.ntiles, ctx->k1t_xcd_chunks);
        if (stats)
            hipLaunchKernelGGL((knn_tree_kernel<D, K, true, true>), dim3(k1t_grid(sp.ntiles, xcb)), dim3(256), 0,
                               ctx->stream, sp.recs, n, sp.ntiles, sp.bvh, semantics == HDB_CORE_EXCL_SELF ? 1 : 0,
                               lists, nb_pos, nb_s, ctx->trav_pop_test, xcb, stats);
        else
            hipLaunchKernelGGL((knn_tree_kernel<D, K, true, false>), dim3(k1t_grid(sp.ntiles, xcb)), dim3(256),
                               0, ctx->stream, sp.recs, n, sp.ntiles, sp.bvh, semantics == HDB_CORE_EXCL_SELF ? 1 : 0,
                               lists, nb_pos, nb_s, ctx->trav_pop_test, xcb, stats);
        HIP_CHECK(hipGetLastError());
    }
    if (stats) {
        unsigned long long h[3];
        HIP_CHECK(hipMemcpyAsync(h, stats, 24, hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        ctx->stats["knn_tree_evals"] = (int64_t)h[0];
    }
    core_epilogue_device(ctx, lists, n, K, min_pts - 1, semantics, core);
    const int g = (int)std::min<int64_t>(ceil_div(n, 256), 4096);
    hipLaunchKernelGGL(set_core_kernel<D>, dim3(g), dim3(256), 0, ctx->stream, sp.recs, n, core);
    KnnLists kl;
    kl.pos = nb_pos;
    kl.s = nb_s;
    kl.K = K;
    kl.done = done;
    const bool self = self_edges & HDB_EDGES_SELF, merged = self_edges & HDB_EDGES_MERGED;
    {
        KernelTimer tb(ctx, "boruvka_total");
        boruvka_on_index<D>(ctx, sp, n, extra, ctx->boruvka_knn_seed ? &kl : nullptr, va, vb, w, merged,
                            (merged && self) ? core : nullptr);
    }
    if (self && !merged) self_edges_device(ctx, core, n, va + (n - 1), vb + (n - 1), w + (n - 1));
}

template <int D>
static bool exact_leaf_k(hdb_ctx *ctx, const double *X, int64_t n, int min_pts, int semantics, double *core,
                         int self_edges, int32_t *va, int32_t *vb, double *w) {
    // list length: >= minPts-1; longer lists make more round-0/1 seeds provably exact
    // (measured at d = 3, 1M blobs: K = 7 cuts the scans by 1.6 ms for +0.7 ms of k-NN)
    const int seed_k = ctx->leaf_seed_k >= 0 ? ctx->leaf_seed_k : (D <= 3 ? 7 : 0);
    const int k = min_pts - 1 > seed_k ? min_pts - 1 : seed_k;
    switch (pick_kc(k)) {
    case 1: exact_leaf_impl<D, 1>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); return true;
    case 3: exact_leaf_impl<D, 3>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); return true;
    case 7: exact_leaf_impl<D, 7>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); return true;
    case 15: exact_leaf_impl<D, 15>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); return true;
    case 31: exact_leaf_impl<D, 31>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); return true;
    default: return false;
    }
}

void exact_leaf_device(hdb_ctx *ctx, const double *X, int64_t n, int d, int min_pts, int metric, int semantics,
                       double *core, int self_edges, int32_t *va, int32_t *vb, double *w) {
    if (n <= 0) return;
    if (min_pts < 1 || min_pts > 32) HDB_THROW(HDB_EINVAL, "minPts must be in 1..32");
    bool done = false;
    if (metric == HDB_METRIC_EUCLIDEAN && min_pts >= 2 && n >= 2) {
        switch (d) {
        case 1: done = exact_leaf_k<1>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); break;
        case 2: done = exact_leaf_k<2>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); break;
        case 3: done = exact_leaf_k<3>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); break;
        case 4: done = exact_leaf_k<4>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); break;
        case 8: done = exact_leaf_k<8>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); break;
        case 16: done = exact_leaf_k<16>(ctx, X, n, min_pts, semantics, core, self_edges, va, vb, w); break;
        default: break;
        }
    }
    if (done) return;
    // the two calls on separate indexes (min_pts 1, tiny n, other d)
    core_distances_device(ctx, X, n, d, min_pts, metric, semantics, core);
    boruvka_device(ctx, X, n, d, core, metric, va, vb, w);
    if (self_edges & HDB_EDGES_SELF) self_edges_device(ctx, core, n, va + (n - 1), vb + (n - 1), w + (n - 1));
    if (self_edges & HDB_EDGES_MERGED)
        sort_edges_desc_device(ctx, va, vb, w, (n - 1) + ((self_edges & HDB_EDGES_SELF) ? n : 0));
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
