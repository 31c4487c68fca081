// common.hpp -- shared internals of libhdbmi (context, staging, errors, metrics).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/hdbmi.h"

namespace hdb {

constexpr double JMAX = DBL_MAX;  // Double.MAX_VALUE

// ----------------------------------------------------------------- errors
void set_error(const std::string &msg);
struct Error {
    int code;
    std::string msg;
};
#define HDB_THROW(code, msg) throw ::hdb::Error{(code), (msg)}
#define HIP_CHECK(expr)                                                                      \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            HDB_THROW(HDB_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));       \
    } while (0)

// ---------------------------------------------------------------- context
struct TimedLaunch {
    std::string name;
    hipEvent_t a, b;
};

struct Arena {  // grow-only device scratch, stream ordered reuse
    void *ptr = nullptr;
    size_t bytes = 0;
};

struct StageChunk {  // Stager device memory: per-context chunks used as a stack
    void *ptr = nullptr;
    size_t bytes = 0, used = 0;
};

}  // namespace hdb

struct hdb_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    hipStream_t side = nullptr;  // private non-blocking stream for graph capture (the null
                                 // stream cannot be captured); fenced to `stream` by events
    bool timing = false;
    std::vector<hdb::TimedLaunch> pending;
    std::vector<hipEvent_t> event_pool;
    std::map<std::string, std::pair<double, int64_t>> acc;
    hdb::Arena arenas[16];
    std::vector<hdb::StageChunk> stage;  // Stager buffers (stack discipline, see Stager)
    int stage_depth = 0;                 // live Stagers on this context
    int64_t *pinned = nullptr;  // pinned_words(): async device -> host counters
    void *host_stage = nullptr;  // host_arena(): grow-only pinned staging
    size_t host_stage_bytes = 0;
    int num_cus = 256;
    bool force_fp64 = false;  // disable the FP32 screen in K1 (A/B and tests)
    bool knn_tree = true;     // K1t (box-pruned) for euclidean lists when the shape allows
    int64_t knn_tree_min_n = 8192;
    bool knn_mfma = true;           // K1m for euclidean lists with 16 < d <= 256
    int64_t knn_mfma_min_n = 2048;
    bool knn_mfma_two_pass = true;  // K1m two-pass kernel (fallback): upper-bound pass first (few exact re-checks)
    bool knn_mfma_single = true;    // K1m single pass: screen + candidate log, FP64 re-check of the log
    bool knn_mfma_prune = true;     // K1m single pass: k-means order + FP64-ball superblock pruning
    bool nearest_grouped = true;   // K3g: median-split sample groups + box pruning for big unkeyed scans
    bool boruvka_seed = true;      // seed Boruvka rounds from the previous round's edges
    int leaf_seed_k = -1;          // exact leaf: k-NN list length at least this (-1: by dimension)
    int leaf_list_rounds = 2;      // exact leaf: Boruvka rounds seeded from the k-NN lists (A/B: tools/seedk_ab.py)
    bool boruvka_knn_seed = true;  // exact leaf: k-NN lists seed every Boruvka round
    int boruvka_wave_pts = 64;     // points per scan wave (16/32/64), compacted per 512-position group
    int boruvka_early_pts = 0;     // points per scan wave in rounds < boruvka_early_rounds (0: as above)
    int boruvka_early_rounds = 5;
    bool boruvka_adj_seed = true;    // K2b: Morton-adjacent pairs across components bound comp_w before the scan
    int bor_xcd_chunks = 8;        // K2b scan: the same XCD-interleaved chunks over each round's waves
    int k1t_xcd_chunks = 8;        // K1t: Morton chunks per XCD (XCD-interleaved tiles; 0: dispatch order)
    int trav_pop_test = 0;         // bit 0: Boruvka re-tests a popped node, bit 1: K1t a popped leaf
    bool prim_coop = true;         // cooperative single-launch Prim for 4096 < n <= 65536
    bool prim_coop_plain = true;   // launch it as a plain kernel first (cooperative launches serialise)
    bool bubble_fold_dim = true;   // K4: one lane per (bubble, dimension) fold (0: one lane per bubble, A/B)
    bool bubble_knn_split = true;  // K5: candidate range in chunks + merge (one thread per bubble is 256 waves at 16k)
    bool prim_coop_xcd = true;     // plain attempt: working blocks on one XCD exchange through its L2 (checked at run time)
    int prim_coop_xcd_max_wg = 32;  // ... for Prims of at most this many workgroups (one XCD: 32 CUs)
    int prim_coop_bs = 1024;  // cooperative Prim (slots 4/5) workgroup size; 0: the smallest of 128..1024 that keeps
                              // the Prim within prim_coop_xcd_max_wg workgroups (more CUs share a step's relaxation)
    int prim_coop_plain_spin_log2 = 20;  // plain attempt: polls per exchange before it reports non-co-residency
    int prim_coop_slots = 4;  // cooperative Prim exchange, rows in registers (d <= 16): 1 release/acquire slots, 2 granules,
                              // 3 drained sc1 slots, 4 DPP folds + key granules (default), 5 key+row granule sweep
    bool merge_runs = false;   // merge sort: radix-sort only what follows a non-decreasing prefix, then merge (slower as built: sync + binary searches)
    int flat_link_variant = 1;  // K6 dc_link A/B: 0 direct guarded atomics, 1 LDS-combined multi-batch
    int flat_root_variant = 3;  // K6 dc_root A/B: 0 LDS table (256 threads), 1 (1024), 2 direct atomics, 3-5 multi-batch
    bool flat_relabel = true;  // K6: divide-and-conquer vertex labels in rank order (locality; false: point ids)
    int flat_block_log = 10;
    int flat_mid_log = 12;     // K6: depths below 2^flat_mid_log ranks per workgroup (dc_mid, L2-local); <= block log: off
    int flat_deep_depth = 64;  // K6: global depths >= this use flat_deep_root / flat_deep_link (A/B)
    int flat_deep_root = 3;
    int flat_deep_link = 1;   // K6: deep depths per workgroup in LDS (2^x ranks, 8-10; 0: the sequential dc_local)
    bool ssort = true;         // sample sort (ssort.hpp) for the Morton order, the edge orders and K6's term sort
                               // (false: the rocPRIM radix chains; A/B and tests)
    int ssort_cap = 0;         // ssort bucket size sorted in LDS (0: SS_CAP; tests lower it to run the merge path)
    bool count_evals = false;  // K1t counts evaluated pairs (diagnostic; costs one sync)
    std::map<std::string, int64_t> stats;  // diagnostic counters (count_evals)
};

namespace hdb {

// scratch slot ids
enum {
    A_STAGE_IN = 0, A_STAGE_OUT = 1, A_WORK0 = 2, A_WORK1 = 3, A_WORK2 = 4, A_WORK3 = 5, A_PAD = 6, A_SORT = 7,
    A_FLAT0 = 8, A_FLAT1 = 9, A_FLAT_TMP = 10, A_LOG = 11, A_ORDER = 12, A_SBKEY = 13, A_XLAY = 14,
    A_SS = 15  // ssort.hpp scratch
};

void *arena(hdb_ctx *ctx, int slot, size_t bytes);
bool hdb_prim_spec_built();  // prim.hip: the speculative Prim (slots 6) is in this build
constexpr int PINNED_WORDS = 512;
int64_t *pinned_words(hdb_ctx *ctx);
// grow-only pinned host buffer (synchronises the stream before it grows)
void *host_arena(hdb_ctx *ctx, size_t bytes);
// order `to` after all work queued so far on `from` (event record + stream wait)
void stream_fence(hdb_ctx *ctx, hipStream_t from, hipStream_t to);

// kernel timing helpers: begin/end around a launch of a named kernel
void time_begin(hdb_ctx *ctx, const char *name, TimedLaunch &t);
void time_end(hdb_ctx *ctx, TimedLaunch &t);
struct KernelTimer {
    hdb_ctx *ctx;
    TimedLaunch t;
    bool on;
    KernelTimer(hdb_ctx *c, const char *name) : ctx(c), on(c->timing) {
        if (on) time_begin(ctx, name, t);
    }
    ~KernelTimer() {
        if (on) time_end(ctx, t);
    }
};

// ---------------------------------------------------- host/device staging
bool is_device_ptr(const void *p);

// Staging of caller arrays: device pointers pass through, host pointers are copied.
// Device copies come from the context's own stage chunks, carved as a stack (a Stager frees
// what it carved when it ends; nested Stagers carve above their parent), reused stream-ordered
// on ctx->stream like the arenas.  No stream-ordered allocator (hipMallocAsync/hipFreeAsync on
// the device's shared default pool) on this path: the C3/C5 model pool calls it from many host
// threads at once, and per-context memory keeps those threads from sharing any allocator state.
class Stager {
   public:
    explicit Stager(hdb_ctx *ctx);
    ~Stager();
    // input array (nullable)
    template <class T>
    const T *in(const T *p, size_t count) {
        return static_cast<const T *>(in_raw(p, count * sizeof(T)));
    }
    // output array (nullable); copied back at finish()
    template <class T>
    T *out(T *p, size_t count) {
        return static_cast<T *>(out_raw(p, count * sizeof(T), false));
    }
    // in/out array
    template <class T>
    T *inout(T *p, size_t count) {
        return static_cast<T *>(out_raw(p, count * sizeof(T), true));
    }
    // copy host outputs back and synchronise if any host pointer was involved
    void finish();
    bool any_host() const { return any_host_; }

   private:
    const void *in_raw(const void *p, size_t bytes);
    void *out_raw(void *p, size_t bytes, bool copy_in);
    void *carve(size_t bytes);
    hdb_ctx *ctx_;
    size_t mark_chunks_ = 0, mark_used_ = 0;
    struct Buf {
        void *dev;
        void *host_dst;
        size_t bytes;
    };
    std::vector<Buf> bufs_;
    bool any_host_ = false;
    bool finished_ = false;
};

// ------------------------------------------------------------- device side
// Euclidean squared distance in the reference's exact operation order
// (EuclideanDistance.java:31-33): s = 0 + t0 + t1 + ..., t_i = (a_i - b_i) * (a_i - b_i).
// 0 + t0 == t0 bitwise because t0 >= +0 or NaN.  Built with -ffp-contract=off.
__device__ __forceinline__ double sq_diff(double a, double b) {
    double t = a - b;
    return t * t;
}

// generic metric over runtime d (reference order for each metric)
__device__ __forceinline__ double metric_distance(const double *a, const double *b, int d, int metric) {
    if (metric == HDB_METRIC_EUCLIDEAN) {
        double s = sq_diff(a[0], b[0]);
        for (int i = 1; i < d; i++) s = s + sq_diff(a[i], b[i]);
        return sqrt(s);
    } else if (metric == HDB_METRIC_COSINE) {
        double dot = 0, m1 = 0, m2 = 0;
        for (int i = 0; i < d; i++) {
            dot = dot + a[i] * b[i];
            m1 = m1 + a[i] * a[i];
            m2 = m2 + b[i] * b[i];
        }
        return 1 - (dot / sqrt(m1 * m2));
    } else if (metric == HDB_METRIC_PEARSON) {
        double mean1 = 0, mean2 = 0;
        for (int i = 0; i < d; i++) {
            mean1 = mean1 + a[i];
            mean2 = mean2 + b[i];
        }
        mean1 = mean1 / d;
        mean2 = mean2 / d;
        double cov = 0, s1 = 0, s2 = 0;
        for (int i = 0; i < d; i++) {
            cov = cov + (a[i] - mean1) * (b[i] - mean2);
            s1 = s1 + (a[i] - mean1) * (a[i] - mean1);
            s2 = s2 + (b[i] - mean2) * (b[i] - mean2);
        }
        return 1 - (cov / sqrt(s1 * s2));
    } else if (metric == HDB_METRIC_MANHATTAN) {
        double s = 0;
        for (int i = 0; i < d; i++) s = s + fabs(a[i] - b[i]);
        return s;
    } else {  // supremum
        double s = 0;
        for (int i = 0; i < d; i++) {
            double diff = fabs(a[i] - b[i]);
            if (diff > s) s = diff;
        }
        return s;
    }
}

// HdbscanDataBubbles.distanceBubbles (HdbscanDataBubbles.java:592-600), exact order.
__device__ __forceinline__ double distance_bubbles(double distance, double ep, double eq, double np_,
                                                   double nq) {
    double verify = distance - (ep + eq);
    if (verify >= 0) return (distance - (ep + eq)) + (np_ + nq);
    // Math.max: NaN if either argument is NaN
    if (np_ != np_ || nq != nq) return NAN;
    return np_ >= nq ? np_ : nq;
}

// Java Math.max(a, b) for doubles without NaN (-0.0 handling irrelevant here)
__device__ __forceinline__ double jmax_sel(double a, double b) { return (a > b) ? a : b; }

// argmin combine with the reference Prim select rule: smaller value wins, equal values ->
// the LARGER index (HDBSCANStar.java:177-180 '<=').  idx < 0 marks "no candidate".
__device__ __forceinline__ void argmin_last(double &v, int &i, double v2, int i2) {
    if (i2 < 0) return;
    if (i < 0 || v2 < v || (v2 == v && i2 > i)) {
        v = v2;
        i = i2;
    }
}

// top-K insertion network (shared by K1, K1t and the epilogues)
// Insert x into ascending buf[0..K) if x < buf[K-1] (strict, HDBSCANStar.java:89);
// the largest element drops out.  x goes after every element <= x (ties keep the earlier
// ones first), exactly where a bubble pass would put it; the K comparisons are independent
// (buf is sorted, so lt[] is monotone) and every slot takes its value from one select pair --
// no serial compare/carry chain, no dynamic indexing.
template <int K>
__device__ __forceinline__ void topk_insert(double (&buf)[K], double x) {
    if (x < buf[K - 1]) {
        bool lt[K];
#pragma unroll
        for (int i = 0; i < K; i++) lt[i] = x < buf[i];
#pragma unroll
        for (int i = K - 1; i > 0; i--) buf[i] = lt[i - 1] ? buf[i - 1] : (lt[i] ? x : buf[i]);
        buf[0] = lt[0] ? x : buf[0];
    }
}
template <int K>
__device__ __forceinline__ void topk_insert_idx(double (&buf)[K], int (&idx)[K], double x, int xi) {
    if (x < buf[K - 1]) {
        bool lt[K];
#pragma unroll
        for (int i = 0; i < K; i++) lt[i] = x < buf[i];
#pragma unroll
        for (int i = K - 1; i > 0; i--) {
            buf[i] = lt[i - 1] ? buf[i - 1] : (lt[i] ? x : buf[i]);
            idx[i] = lt[i - 1] ? idx[i - 1] : (lt[i] ? xi : idx[i]);
        }
        buf[0] = lt[0] ? x : buf[0];
        idx[0] = lt[0] ? xi : idx[0];
    }
}

// Wave-wide min of a u64 through DPP moves (quad perms, row shifts, row broadcasts): no LDS
// round trip per stage, unlike __shfl_xor.  The minimum lands in lane 63 and is broadcast.
#define HDB_DPP_MIN_STEP(x, CTRL, ROWMASK)                                                                  \
    do {                                                                                                    \
        const unsigned lo_ = (unsigned)(x), hi_ = (unsigned)((x) >> 32);                                    \
        const unsigned lo2_ = (unsigned)__builtin_amdgcn_update_dpp((int)lo_, (int)lo_, CTRL, ROWMASK, 0xf, false); \
        const unsigned hi2_ = (unsigned)__builtin_amdgcn_update_dpp((int)hi_, (int)hi_, CTRL, ROWMASK, 0xf, false); \
        const unsigned long long y_ = ((unsigned long long)hi2_ << 32) | lo2_;                              \
        (x) = y_ < (x) ? y_ : (x);                                                                          \
    } while (0)

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long x) {
    HDB_DPP_MIN_STEP(x, 0xb1, 0xf);   // quad_perm [1,0,3,2]
    HDB_DPP_MIN_STEP(x, 0x4e, 0xf);   // quad_perm [2,3,0,1]
    HDB_DPP_MIN_STEP(x, 0x114, 0xf);  // row_shr:4
    HDB_DPP_MIN_STEP(x, 0x118, 0xf);  // row_shr:8
    HDB_DPP_MIN_STEP(x, 0x142, 0xa);  // row_bcast:15
    HDB_DPP_MIN_STEP(x, 0x143, 0xc);  // row_bcast:31
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// grid-stride helper
#define HDB_GRID_STRIDE(i, n)                                                                   \
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)(n);        \
         i += (int64_t)blockDim.x * gridDim.x)

}  // namespace hdb
