// prim.hip -- K2: dense Prim on the mutual-reachability graph with the reference's exact
// tie rules (HDBSCANStar.constructMST, HDBSCANStar.java:124-205; the bubble variant
// HdbscanDataBubbles.constructMSTBubbles, HdbscanDataBubbles.java:165-254):
//   * start at vertex n-1, best[] = Double.MAX_VALUE, parent[] = 0 (Java default);
//   * update iff mrd < best[nb] (strict), parent = ids[cur];
//   * select the unattached vertex with the smallest best, ties -> LARGEST index ('<=').
// mrd = max(dist, core[cur], core[nb]) evaluated with Java's two '>' tests.
//
// Three launch shapes:
//   prim_block_kernel   one workgroup per partition (n <= BS*PPT), whole Prim in-kernel,
//                       per-step argmin = DPP/shuffle wave reduce + one LDS exchange;
//   leaf_core_kernel    FirstStep leaf branch: cumulative core distances per partition;
//   prim_step_kernel    large graphs: one launch per Prim step over many workgroups; each
//                       workgroup re-reduces the previous step's per-workgroup partials
//                       (visible across the kernel boundary), so no inter-workgroup
//                       hand-off is needed inside a launch.  Launches are replayed from a
//                       captured hipGraph chunk.
// Euclidean pairs use a squared filter: s > fl(b*b)*(1+2^-50) proves sqrt(s) >= b, so
// the exact sqrt + mrd path runs only for pairs that can improve best[nb].
#include <atomic>

#include "internal.hpp"

// The speculative cooperative Prim (prim_coop_slots 6, round 5) is built only with
// -DHDB_PRIM_SPEC=1 (HDBMI_EXTRA_FLAGS): exact and faster alone (1.91 vs 2.07 us/step at
// 16,384 x 8) but slower inside the C5 job, where several Prims share the device (DESIGN §4
// "Round 5" item 3), so the default library leaves it out; slots 6 then reports HDB_EUNSUPPORTED.
#ifndef HDB_PRIM_SPEC
#define HDB_PRIM_SPEC 0
#endif

namespace hdb {

bool hdb_prim_spec_built() { return HDB_PRIM_SPEC != 0; }

// exact mrd for (cur, nb); returns true if it improves best
__device__ __forceinline__ bool mrd_improves(const PrimIn &in, int64_t cur, int64_t nb, double best, double &mrd_out) {
    const double *a = in.X + cur * in.d;
    const double *b = in.X + nb * in.d;
    double dist;
    if (in.metric == HDB_METRIC_EUCLIDEAN && !in.eB) {
        double s = sq_diff(a[0], b[0]);
        for (int c = 1; c < in.d; c++) s = s + sq_diff(a[c], b[c]);
        double thr = (best * best) * 1.0000000000000009;  // >= best^2 exactly
        if (s > thr) return false;
        dist = sqrt(s);
    } else {
        dist = metric_distance(a, b, in.d, in.metric);
        if (in.eB) dist = distance_bubbles(dist, in.eB[cur], in.eB[nb], in.nnB[cur], in.nnB[nb]);
    }
    double mrd = dist;
    double cc = in.core[cur], cn = in.core[nb];
    if (cc > mrd) mrd = cc;
    if (cn > mrd) mrd = cn;
    mrd_out = mrd;
    return mrd < best;
}

__device__ __forceinline__ void wave_argmin_last(double &v, int &i) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        double v2 = __shfl_xor(v, off);
        int i2 = __shfl_xor(i, off);
        argmin_last(v, i, v2, i2);
    }
}


// Order-preserving u64 key of a non-negative MRD value (+-0 -> 0): min over keys = min value.
__device__ __forceinline__ unsigned long long mrd_key(double v) {
    return v == 0.0 ? 0ull : (unsigned long long)__double_as_longlong(v);
}

// highest lane whose predicate holds (-1: none)
__device__ __forceinline__ int last_lane(bool p) {
    const unsigned long long m = __ballot(p);
    return m ? 63 - __clzll(m) : -1;
}

// ---------------------------------------------------------- block kernel
// parts: partition list for this launch (indices into offsets); vertex rows of partition
// p are [offsets[p], offsets[p+1]).  Edges at eoff[p].
template <int BS, int PPT>
__global__ __launch_bounds__(BS) void prim_block_kernel(PrimIn in, const int64_t *__restrict__ offsets,
                                                        const int64_t *__restrict__ eoff,
                                                        const int32_t *__restrict__ parts, int self_edges,
                                                        int32_t *__restrict__ va, int32_t *__restrict__ vb,
                                                        double *__restrict__ w) {
    constexpr int NW = BS / 64;
    __shared__ double s_v[2][NW];
    __shared__ int s_i[2][NW];
    const int p = parts[blockIdx.x];
    const int64_t o = offsets[p];
    const int n = (int)(offsets[p + 1] - o);
    if (n <= 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    double best[PPT];
    int par[PPT];
    unsigned att = 0;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        best[k] = JMAX;
        par[k] = 0;
        int i = tid + k * BS;
        if (i == n - 1 || i >= n) att |= 1u << k;
    }
    int cur = n - 1;
    for (int step = 1; step < n; step++) {
        double lv = INFINITY;
        int li = -1;
        const int cid = L.ids[cur];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            if (att & (1u << k)) continue;
            int i = tid + k * BS;
            double mrd;
            if (mrd_improves(L, cur, i, best[k], mrd)) {
                best[k] = mrd;
                par[k] = cid;
            }
            argmin_last(lv, li, best[k], i);
        }
        wave_argmin_last(lv, li);
        if (NW > 1) {
            const int buf = step & 1;
            if (lane == 0) {
                s_v[buf][wid] = lv;
                s_i[buf][wid] = li;
            }
            __syncthreads();
            lv = s_v[buf][0];
            li = s_i[buf][0];
#pragma unroll
            for (int q = 1; q < NW; q++) argmin_last(lv, li, s_v[buf][q], s_i[buf][q]);
        }
        cur = li;  // uniform
        if (cur < 0) break;  // unreachable: an unattached vertex always exists
        if ((cur % BS) == tid) att |= 1u << (cur / BS);
    }
    const int64_t eo = eoff[p];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        int i = tid + k * BS;
        if (i < n - 1) {
            va[eo + i] = par[k];
            vb[eo + i] = L.ids[i];
            w[eo + i] = best[k];
        }
        if (self_edges && i < n) {
            va[eo + n - 1 + i] = L.ids[i];
            vb[eo + n - 1 + i] = L.ids[i];
            w[eo + n - 1 + i] = L.core[i];
        }
    }
}

// ------------------------------------------------- leaf cumulative cores
// HDBSCANStar.calculateCoreDistances inside a leaf partition (HDBSCANStar.java:79-103):
// per-row top-KC lists (self included, values as Java computes them), then the
// never-reset buffer = prefix merge over rows in row order (one lane).  KC >= K; the
// K-th smallest of a union is element K-1 of its top-KC.
template <int KC>
__device__ __forceinline__ void ins_kc(double (&buf)[KC], double x) {
    if (!(x < buf[KC - 1])) return;
#pragma unroll
    for (int i = 0; i < KC; i++) {
        double b = buf[i];
        bool lt = x < b;
        buf[i] = lt ? x : b;
        x = lt ? b : x;
    }
}

template <int BS, int KC>
__global__ __launch_bounds__(BS) void leaf_core_kernel(const double *__restrict__ X, int d, int metric,
                                                       const int64_t *__restrict__ offsets,
                                                       const int32_t *__restrict__ parts, int K,
                                                       double *__restrict__ lists /* rows*KC */,
                                                       double *__restrict__ core) {
    const int p = parts[blockIdx.x];
    const int64_t o = offsets[p];
    const int n = (int)(offsets[p + 1] - o);
    for (int i = threadIdx.x; i < n; i += BS) {
        double buf[KC];
#pragma unroll
        for (int k = 0; k < KC; k++) buf[k] = JMAX;
        const double *xi = X + (o + i) * d;
        for (int j = 0; j < n; j++) ins_kc<KC>(buf, metric_distance(xi, X + (o + j) * d, d, metric));
#pragma unroll
        for (int k = 0; k < KC; k++) lists[(o + i) * KC + k] = buf[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double buf[KC];
#pragma unroll
        for (int k = 0; k < KC; k++) buf[k] = JMAX;
        for (int i = 0; i < n; i++) {
#pragma unroll
            for (int k = 0; k < KC; k++) ins_kc<KC>(buf, lists[(o + i) * KC + k]);
            double c = buf[0];
#pragma unroll
            for (int k = 1; k < KC; k++)
                if (k == K - 1) c = buf[k];
            core[o + i] = c;
        }
    }
}

void leaf_cores_device(hdb_ctx *ctx, const double *X, int d, int metric, int P, const int64_t *d_off,
                       const int32_t *d_parts, int np, int64_t total_rows, int K, double *core) {
    if (np == 0) return;
    int KC = K <= 3 ? 3 : (K <= 7 ? 7 : (K <= 15 ? 15 : 31));
    if (K > 31) HDB_THROW(HDB_EINVAL, "minPts too large (max 32)");
    double *lists = (double *)arena(ctx, A_WORK2, sizeof(double) * (size_t)std::max<int64_t>(total_rows, 1) * KC);
    KernelTimer t(ctx, "leaf_core");
    switch (KC) {
    case 3: hipLaunchKernelGGL((leaf_core_kernel<256, 3>), dim3(np), dim3(256), 0, ctx->stream, X, d, metric, d_off, d_parts, K, lists, core); break;
    case 7: hipLaunchKernelGGL((leaf_core_kernel<256, 7>), dim3(np), dim3(256), 0, ctx->stream, X, d, metric, d_off, d_parts, K, lists, core); break;
    case 15: hipLaunchKernelGGL((leaf_core_kernel<256, 15>), dim3(np), dim3(256), 0, ctx->stream, X, d, metric, d_off, d_parts, K, lists, core); break;
    default: hipLaunchKernelGGL((leaf_core_kernel<256, 31>), dim3(np), dim3(256), 0, ctx->stream, X, d, metric, d_off, d_parts, K, lists, core); break;
    }
    HIP_CHECK(hipGetLastError());
    (void)P;
}

// ------------------------------------------------------ stepwise kernel
// State per partition (global): best[], par[], att[] over its vertices; partials
// [2][nwg_p] (value, index) double-buffered by step parity; step counter ctr[2].
struct StepState {
    double *best;
    int32_t *par;
    uint8_t *att;
    double *pv;     // [2][total_wg]
    int32_t *pidx;  // [2][total_wg]
    int32_t *cur0;  // start vertex per partition (n-1)
};

// Block b belongs to partition wg_part[b]; its local index within the partition's
// workgroups is b - wg_first[p]; partition p has wg_count[p] workgroups.
template <int BS, int PPT>
__global__ __launch_bounds__(BS) void prim_step_kernel(PrimIn in, const int64_t *__restrict__ offsets,
                                                       const int32_t *__restrict__ wg_part,
                                                       const int32_t *__restrict__ wg_first,
                                                       const int32_t *__restrict__ wg_count, StepState st,
                                                       int step, int parity) {
    constexpr int NW = BS / 64;
    __shared__ double s_v[NW];
    __shared__ int s_i[NW];
    __shared__ int s_cur;
    const int b = blockIdx.x;
    const int p = wg_part[b];
    const int64_t o = offsets[p];
    const int n = (int)(offsets[p + 1] - o);
    if (step >= n) return;  // this partition is done
    const int first = wg_first[p], cnt = wg_count[p];
    const int lb = b - first;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    // current vertex: reduce the previous step's partials (or the start vertex)
    int cur;
    if (step == 1) {
        cur = n - 1;
    } else {
        if (tid < 64) {
            double v = INFINITY;
            int i = -1;
            for (int q = lane; q < cnt; q += 64)
                argmin_last(v, i, st.pv[(parity ^ 1) * gridDim.x + first + q], st.pidx[(parity ^ 1) * gridDim.x + first + q]);
            wave_argmin_last(v, i);
            if (lane == 0) s_cur = i;
        }
        __syncthreads();
        cur = s_cur;
        if (cur < 0) return;
    }
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    // mark cur attached (owner workgroup), skip it below
    const int per_wg = BS * PPT;
    const int base = lb * per_wg;
    double lv = INFINITY;
    int li = -1;
    const int cid = L.ids[cur];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        int i = base + tid + k * BS;
        if (i >= n) continue;
        const int64_t gi = o + i;
        if (i == cur) {
            st.att[gi] = 1;
            continue;
        }
        if (st.att[gi]) continue;
        double bst = st.best[gi];
        double mrd;
        if (mrd_improves(L, cur, i, bst, mrd)) {
            bst = mrd;
            st.best[gi] = mrd;
            st.par[gi] = cid;
        }
        argmin_last(lv, li, bst, i);
    }
    wave_argmin_last(lv, li);
    if (lane == 0) {
        s_v[wid] = lv;
        s_i[wid] = li;
    }
    __syncthreads();
    if (tid == 0) {
        double v = s_v[0];
        int i = s_i[0];
        for (int q = 1; q < NW; q++) argmin_last(v, i, s_v[q], s_i[q]);
        st.pv[parity * gridDim.x + b] = v;
        st.pidx[parity * gridDim.x + b] = i;
    }
}

__global__ void prim_step_init_kernel(const int64_t *__restrict__ offsets, int P, double *best, int32_t *par,
                                      uint8_t *att, int64_t total) {
    HDB_GRID_STRIDE(g, total) {
        best[g] = JMAX;
        par[g] = 0;
        att[g] = 0;
    }
}

__global__ void prim_step_final_kernel(PrimIn in, const int64_t *__restrict__ offsets,
                                       const int64_t *__restrict__ eoff, int P, StepState st, int self_edges,
                                       int32_t *__restrict__ va, int32_t *__restrict__ vb, double *__restrict__ w) {
    // one block per partition
    const int p = blockIdx.x;
    const int64_t o = offsets[p];
    const int n = (int)(offsets[p + 1] - o);
    const int64_t eo = eoff[p];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (i < n - 1) {
            va[eo + i] = st.par[o + i];
            vb[eo + i] = in.ids[o + i];
            w[eo + i] = st.best[o + i];
        }
        if (self_edges) {
            va[eo + n - 1 + i] = in.ids[o + i];
            vb[eo + n - 1 + i] = in.ids[o + i];
            w[eo + n - 1 + i] = in.core[o + i];
        }
    }
}

// ------------------------------------------------------------------ host

// --------------------------------------------------- cooperative kernel
// One partition of 4096 < n <= 65536 vertices (bubble models of the C3/C5 configs): one
// lane per vertex over ceil(n / BS) co-resident workgroups (cooperative launch), the whole
// Prim in one launch.  Each step: update + workgroup argmin, publish the partial, one
// grid barrier (monotone counter), every workgroup folds the nwg partials (argmin_last is
// associative and commutative, so all agree on the next vertex).  Partials are double
// buffered by step parity: a workgroup can be at most one step ahead of any other.
// Partial reads use agent-scope atomic loads (bypass the non-coherent L1).
template <int BS>
__global__ __launch_bounds__(BS) void prim_coop_kernel(PrimIn in, int n, int self_edges, int32_t *__restrict__ va,
                                                       int32_t *__restrict__ vb, double *__restrict__ w,
                                                       unsigned long long *__restrict__ part, unsigned *counter,
                                                       int *err) {
    constexpr int NW = BS / 64;
    __shared__ double s_v[NW];
    __shared__ int s_i[NW];
    __shared__ int s_cur;
    const int nwg = (int)gridDim.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = (int)blockIdx.x * BS + tid;
    double best = JMAX;
    int par = -1;  // partition-local; ids[] applied once at the end (HDBSCANStar.java:137,172: 0 if never set)
    bool att = (i >= n) || (i == n - 1);
    int cur = n - 1;
    for (int step = 1; step < n; step++) {
        double lv = INFINITY;
        int li = -1;
        if (!att) {
            double mrd;
            if (mrd_improves(in, cur, i, best, mrd)) {
                best = mrd;
                par = cur;
            }
            argmin_last(lv, li, best, i);
        }
        wave_argmin_last(lv, li);
        if (lane == 0) {
            s_v[wid] = lv;
            s_i[wid] = li;
        }
        __syncthreads();
        const int buf = step & 1;
        if (tid == 0) {
            double v = s_v[0];
            int ii = s_i[0];
#pragma unroll
            for (int q = 1; q < NW; q++) argmin_last(v, ii, s_v[q], s_i[q]);
            __hip_atomic_store(&part[2 * (buf * nwg + blockIdx.x)], (unsigned long long)__double_as_longlong(v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&part[2 * (buf * nwg + blockIdx.x) + 1], (unsigned long long)(unsigned)ii,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)step * (unsigned)nwg;
            unsigned spins = 0;
            while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                if (++spins > (1u << 26)) {  // a co-residency failure must not hang the device
                    atomicExch(err, 1);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        if (wid == 0) {
            double v = INFINITY;
            int ii = -1;
            for (int k = lane; k < nwg; k += 64) {
                const unsigned long long bv =
                    __hip_atomic_load(&part[2 * (buf * nwg + k)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned long long bi =
                    __hip_atomic_load(&part[2 * (buf * nwg + k) + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                argmin_last(v, ii, __longlong_as_double((long long)bv), (int)(unsigned)bi);
            }
            wave_argmin_last(v, ii);
            if (lane == 0) s_cur = ii;
        }
        __syncthreads();
        cur = s_cur;
        if (cur < 0) break;  // unreachable (an unattached vertex always exists) -- uniform exit
        if (i == cur) att = true;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    }
    if (i < n - 1) {
        va[i] = par >= 0 ? in.ids[par] : 0;
        vb[i] = in.ids[i];
        w[i] = best;
    }
    if (self_edges && i < n) {
        va[n - 1 + i] = in.ids[i];
        vb[n - 1 + i] = in.ids[i];
        w[n - 1 + i] = in.core[i];
    }
}

// ------------------------------------------ cooperative kernel, step-tagged slots
// Same Prim (HDBSCANStar.java:124-205, select '<=' = last index, update '<'), restructured
// around the step's critical path: each lane keeps its own row (d <= DM), core and bubble
// terms in registers; a workgroup publishes its candidate TOGETHER with that candidate's row
// in a slot whose tag (the step) is stored last with release semantics; wave 0 of every
// workgroup polls the nwg tags (acquire), folds the candidates and reads the winner's row
// (one word per lane) into LDS.  No barrier counter and no dependent load of X[cur].  Slots
// are double buffered by step parity (a workgroup is at most one step ahead).  (Measured:
// 6.3 us/step at 16 workgroups vs 7.0 for the counter barrier, 7.2 vs 17.8 at 4.)  Variants
// 2-5 below; 4 is the default (3.0 us/step at 16 workgroups, 3.3 at 4, 3.9 at 64: s_memtime
// phases showed the __shfl_xor argmin folds, the dependent ids[cur] load and the single-lane
// slot stores, not the fences, held the slot version at 6.3; tools/coop_prof.py).
#ifdef HDB_COOP_PROF  // phase timestamps of steps [1024, 1088) of workgroup 0 (tools/coop_prof.py)
__device__ unsigned long long g_coop_prof[64 * 8];
#define COOP_T(k)                                                                                              \
    if (blockIdx.x == 0 && tid == 0 && step >= 1024 && step < 1088) g_coop_prof[(step - 1024) * 8 + (k)] =  \
        __builtin_amdgcn_s_memtime()
extern "C" int hdb_debug_coop_prof(unsigned long long *out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_coop_prof), sizeof(g_coop_prof));
}
#else
#define COOP_T(k)
#endif

template <int DM>
struct CoopSlot {  // written by one thread, read word-wise with agent-scope loads
    unsigned long long tag, val, idx;
    double x[DM];
    double core, eB, nnB;
};

template <int DM>
__device__ __forceinline__ double coop_mrd(const PrimIn &in, const double (&xc)[DM], double cc, double ebc, double nnc,
                                           const double (&xi)[DM], double ci, double ebi, double nni, double best,
                                           bool &improves) {
    double dist;
    if (in.metric == HDB_METRIC_EUCLIDEAN) {  // the rows stay in registers (predicated, same order)
        double s = sq_diff(xc[0], xi[0]);
#pragma unroll
        for (int c = 1; c < DM; c++)
            if (c < in.d) s = s + sq_diff(xc[c], xi[c]);
        if (!in.eB) {
            const double thr = (best * best) * 1.0000000000000009;  // >= best^2 exactly
            if (s > thr) {
                improves = false;
                return best;
            }
        } else {
            // bubbles: with E = eB_c + eB_i >= 0 and nnB_c + nnB_i >= 0, distanceBubbles(d) >=
            // fl(d - E) > best once d > (best + E)(1 + 1e-12) (the margin covers every rounding
            // of sqrt, the subtraction and the square): no improvement, skip the sqrt
            const double E = ebc + ebi, T = (best + E) * (1.0 + 1e-12);
            if (s > T * T && E >= 0.0 && nnc + nni >= 0.0) {
                improves = false;
                return best;
            }
        }
        dist = sqrt(s);
    } else {
        dist = metric_distance(xc, xi, in.d, in.metric);
    }
    if (in.eB) dist = distance_bubbles(dist, ebc, ebi, nnc, nni);
    double mrd = dist;
    if (cc > mrd) mrd = cc;
    if (ci > mrd) mrd = ci;
    improves = mrd < best;
    return mrd;
}

template <int BS, int DM, bool FAST>
__global__ __launch_bounds__(BS) void prim_coop2_kernel(PrimIn in, int n, int self_edges, int32_t *__restrict__ va,
                                                        int32_t *__restrict__ vb, double *__restrict__ w,
                                                        CoopSlot<DM> *__restrict__ slots, int *err) {
    constexpr int NW = BS / 64;
    __shared__ double s_v[NW];
    __shared__ int s_i[NW];
    __shared__ double s_row[DM + 3];  // the winner's x, core, eB, nnB
    __shared__ int s_cur;
    const int nwg = (int)gridDim.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = (int)blockIdx.x * BS + tid;
    double xi[DM], ci = 0, ebi = 0, nni = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xi[c] = (i < n && c < in.d) ? in.X[(int64_t)i * in.d + c] : 0.0;
    if (i < n) {
        ci = in.core[i];
        if (in.eB) {
            ebi = in.eB[i];
            nni = in.nnB[i];
        }
    }
    double best = JMAX;
    int par = -1;
    bool att = (i >= n) || (i == n - 1);
    // the start vertex n-1 (HDBSCANStar.java:145-147): its row from memory, once
    double xc[DM], cc, ebc = 0, nnc = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xc[c] = c < in.d ? in.X[(int64_t)(n - 1) * in.d + c] : 0.0;
    cc = in.core[n - 1];
    if (in.eB) {
        ebc = in.eB[n - 1];
        nnc = in.nnB[n - 1];
    }
    int cur = n - 1;
    for (int step = 1; step < n; step++) {
        COOP_T(0);
        double lv = INFINITY;
        int li = -1;
        if (!att) {
            bool imp;
            const double mrd = coop_mrd<DM>(in, xc, cc, ebc, nnc, xi, ci, ebi, nni, best, imp);
            if (imp) {
                best = mrd;
                par = cur;
            }
            argmin_last(lv, li, best, i);
        }
        wave_argmin_last(lv, li);
        if (lane == 0) {
            s_v[wid] = lv;
            s_i[wid] = li;
        }
        __syncthreads();
        COOP_T(1);
        double v = s_v[0];
        int ii = s_i[0];
#pragma unroll
        for (int q = 1; q < NW; q++) argmin_last(v, ii, s_v[q], s_i[q]);
        const int buf = step & 1;
        CoopSlot<DM> *my = slots + (size_t)buf * nwg + blockIdx.x;
        if ((ii >= 0) ? (ii == i) : (tid == 0)) {  // the workgroup's candidate row travels with it
            unsigned long long *wd = (unsigned long long *)my;
            __hip_atomic_store(&wd[1], (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&wd[2], (unsigned long long)(long long)ii, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int c = 0; c < DM; c++)
                __hip_atomic_store(&wd[3 + c], (unsigned long long)__double_as_longlong(xi[c]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&wd[3 + DM], (unsigned long long)__double_as_longlong(ci), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&wd[4 + DM], (unsigned long long)__double_as_longlong(ebi), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&wd[5 + DM], (unsigned long long)__double_as_longlong(nni), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            if (FAST) {  // sc1 payload drained, then the tag (Guideline 16 R1, no release fence)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&wd[0], (unsigned long long)step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(&wd[0], (unsigned long long)step, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (wid == 0) {
            COOP_T(2);
            double bv = INFINITY;
            int bi = -1, bk = -1;
            bool tmo = false;
            for (int k = lane; k < nwg; k += 64) {
                const unsigned long long *wd = (const unsigned long long *)(slots + (size_t)buf * nwg + k);
                unsigned spins = 0;
                while (__hip_atomic_load(&wd[0], FAST ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) !=
                       (unsigned long long)step) {
                    if (++spins > (1u << 26)) {  // a co-residency failure must not hang the device
                        atomicExch(err, 1);
                        tmo = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (FAST) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // every payload load is sc1
                const double kv = __longlong_as_double(
                    (long long)__hip_atomic_load(&wd[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                const int ki = (int)(long long)__hip_atomic_load(&wd[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int pi = bi;
                argmin_last(bv, bi, kv, ki);
                if (bi != pi) bk = k;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {  // fold, carrying the winner's slot
                const double v2 = __shfl_xor(bv, off);
                const int i2 = __shfl_xor(bi, off), k2 = __shfl_xor(bk, off);
                const int pi = bi;
                argmin_last(bv, bi, v2, i2);
                if (bi != pi) bk = k2;
            }
            COOP_T(3);
            if (__any(tmo)) bi = bk = -1;  // timed out: every wave leaves at the next check
            if (bk >= 0 && lane < DM + 3) {  // the winner's row: one word per lane
                const unsigned long long *wd = (const unsigned long long *)(slots + (size_t)buf * nwg + bk);
                s_row[lane] = __longlong_as_double(
                    (long long)__hip_atomic_load(&wd[3 + lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
            if (lane == 0) s_cur = bi;
            COOP_T(4);
        }
        __syncthreads();
        COOP_T(5);
        cur = s_cur;
        if (cur < 0) break;  // unreachable (an unattached vertex always exists) -- uniform exit
#pragma unroll
        for (int c = 0; c < DM; c++) xc[c] = s_row[c];
        cc = s_row[DM];
        ebc = s_row[DM + 1];
        nnc = s_row[DM + 2];
        if (i == cur) att = true;
        if (!FAST && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    }
    if (i < n - 1) {
        va[i] = par >= 0 ? in.ids[par] : 0;
        vb[i] = in.ids[i];
        w[i] = best;
    }
    if (self_edges && i < n) {
        va[n - 1 + i] = in.ids[i];
        vb[n - 1 + i] = in.ids[i];
        w[n - 1 + i] = in.core[i];
    }
}

// Variant (prim_coop_slots = 2): the same exchange as data-tagged 8-byte granules
// (cdna_hip_programming.md Guideline 16, R2): the candidate's wave stores its payload as
// {tag = step, 32-bit half} granules, one write-through (sc1) store per lane, no fence; wave 0
// of every workgroup sweeps all nwg slots flat (granule j on lane j mod 64), staging them in LDS
// until every tag matches, then folds from LDS.
typedef __attribute__((address_space(1))) unsigned long long gu64;

template <int BS, int DM>
__global__ __launch_bounds__(BS) void prim_coop3_kernel(PrimIn in, int n, int self_edges, int32_t *__restrict__ va,
                                                        int32_t *__restrict__ vb, double *__restrict__ w,
                                                        gu64 *__restrict__ gr, int *err) {
    constexpr int NW = BS / 64;
    constexpr int ND = 1 + DM + 3;  // value, row, core, eB, nnB
    constexpr int G = 2 * ND + 1;   // + the index
    constexpr int MAXWG = 64;
    __shared__ double s_v[NW];
    __shared__ int s_i[NW];
    __shared__ unsigned s_g[MAXWG * G];
    __shared__ double s_row[DM + 3];
    __shared__ int s_cur;
    const int nwg = (int)gridDim.x;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = (int)blockIdx.x * BS + tid;
    double xi[DM], ci = 0, ebi = 0, nni = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xi[c] = (i < n && c < in.d) ? in.X[(int64_t)i * in.d + c] : 0.0;
    if (i < n) {
        ci = in.core[i];
        if (in.eB) {
            ebi = in.eB[i];
            nni = in.nnB[i];
        }
    }
    double best = JMAX;
    int par = -1;
    bool att = (i >= n) || (i == n - 1);
    double xc[DM], cc, ebc = 0, nnc = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xc[c] = c < in.d ? in.X[(int64_t)(n - 1) * in.d + c] : 0.0;
    cc = in.core[n - 1];
    if (in.eB) {
        ebc = in.eB[n - 1];
        nnc = in.nnB[n - 1];
    }
    int cur = n - 1;
    const int T = nwg * G;
    for (int step = 1; step < n; step++) {
        double lv = INFINITY;
        int li = -1;
        if (!att) {
            bool imp;
            const double mrd = coop_mrd<DM>(in, xc, cc, ebc, nnc, xi, ci, ebi, nni, best, imp);
            if (imp) {
                best = mrd;
                par = cur;
            }
            argmin_last(lv, li, best, i);
        }
        wave_argmin_last(lv, li);
        if (lane == 0) {
            s_v[wid] = lv;
            s_i[wid] = li;
        }
        __syncthreads();
        double v = s_v[0];
        int ii = s_i[0];
#pragma unroll
        for (int q = 1; q < NW; q++) argmin_last(v, ii, s_v[q], s_i[q]);
        const int buf = step & 1;
        const unsigned long long tag = (unsigned long long)(unsigned)step << 32;
        const int loc = ii >= 0 ? ii - (int)blockIdx.x * BS : 0;  // the candidate's thread (empty: wave 0)
        if (wid == (loc >> 6)) {  // its wave stores the payload, one granule pair per lane
            const int src = loc & 63;
            double pay = lane == 0 ? v : 0.0;
#pragma unroll
            for (int c = 0; c < DM; c++) {
                const double t = __shfl(xi[c], src);
                if (lane == 1 + c) pay = t;
            }
            const double t1 = __shfl(ci, src), t2 = __shfl(ebi, src), t3 = __shfl(nni, src);
            if (lane == 1 + DM) pay = t1;
            if (lane == 2 + DM) pay = t2;
            if (lane == 3 + DM) pay = t3;
            if (ii < 0 && lane > 0) pay = 0.0;
            gu64 *g = gr + ((size_t)buf * nwg + blockIdx.x) * G;
            if (lane < ND) {
                const unsigned long long bits = (unsigned long long)__double_as_longlong(pay);
                __hip_atomic_store(g + 2 * lane, tag | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(g + 2 * lane + 1, tag | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (lane == ND) {
                __hip_atomic_store(g + 2 * ND, tag | (unsigned)ii, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (wid == 0) {
            const gu64 *g = gr + (size_t)buf * nwg * G;
            unsigned spins = 0;
            bool tmo = false;
            while (true) {
                bool ok = true;
                for (int j = lane; j < T; j += 64) {
                    const unsigned long long x = __hip_atomic_load(g + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok &= (x & 0xffffffff00000000ull) == tag;
                    s_g[j] = (unsigned)x;
                }
                if (__all(ok)) break;
                if (++spins > (1u << 24)) {  // a co-residency failure must not hang the device
                    if (lane == 0) atomicExch(err, 1);
                    tmo = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_wave_barrier();
            double bv = INFINITY;
            int bi = -1, bk = -1;
            if (lane < nwg) {
                const unsigned *q = s_g + lane * G;
                bv = __longlong_as_double((long long)(((unsigned long long)q[1] << 32) | q[0]));
                bi = (int)q[2 * ND];
                bk = lane;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const double v2 = __shfl_xor(bv, off);
                const int i2 = __shfl_xor(bi, off), k2 = __shfl_xor(bk, off);
                const int pi = bi;
                argmin_last(bv, bi, v2, i2);
                if (bi != pi) bk = k2;
            }
            if (tmo) bi = bk = -1;
            if (bk >= 0 && lane < DM + 3) {
                const unsigned *q = s_g + bk * G + 2 * (1 + lane);
                s_row[lane] = __longlong_as_double((long long)(((unsigned long long)q[1] << 32) | q[0]));
            }
            if (lane == 0) s_cur = bi;
        }
        __syncthreads();
        cur = s_cur;
        if (cur < 0) break;
#pragma unroll
        for (int c = 0; c < DM; c++) xc[c] = s_row[c];
        cc = s_row[DM];
        ebc = s_row[DM + 1];
        nnc = s_row[DM + 2];
        if (i == cur) att = true;
    }
    if (i < n - 1) {
        va[i] = par >= 0 ? in.ids[par] : 0;
        vb[i] = in.ids[i];
        w[i] = best;
    }
    if (self_edges && i < n) {
        va[n - 1 + i] = in.ids[i];
        vb[n - 1 + i] = in.ids[i];
        w[n - 1 + i] = in.core[i];
    }
}

template <int DM>
static bool launch_coop3(hdb_ctx *ctx, const PrimIn &in, int64_t o, int64_t n, int64_t eo, int self_edges,
                         int32_t *va, int32_t *vb, double *w) {
    constexpr int BS = 1024;
    const int nwg = (int)ceil_div(n, BS);
    if (nwg > 64) return false;
    int coop = 0, ncu = 0, per_cu = 0;
    HIP_CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, prim_coop3_kernel<BS, DM>, BS, 0));
    if (!coop || (int64_t)per_cu * ncu < nwg) return false;
    constexpr int G = 2 * (1 + DM + 3) + 1;
    const size_t gbytes = (8 * (size_t)G * 2 * nwg + 255) & ~size_t(255);
    char *base = (char *)arena(ctx, A_WORK3, gbytes + 256);
    gu64 *gr = (gu64 *)base;
    int *err = (int *)(base + gbytes);
    HIP_CHECK(hipMemsetAsync(base, 0, gbytes + 256, ctx->stream));  // tags 0: no step yet
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    int nn = (int)n;
    int32_t *pva = va + eo, *pvb = vb + eo;
    double *pw = w + eo;
    void *args[] = {&L, &nn, &self_edges, &pva, &pvb, &pw, &gr, &err};
    {
        KernelTimer t(ctx, "prim_coop");
        HIP_CHECK(hipLaunchCooperativeKernel((const void *)prim_coop3_kernel<BS, DM>, dim3(nwg), dim3(BS), args, 0,
                                             ctx->stream));
    }
    int h_err = 0;
    HIP_CHECK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (h_err) HDB_THROW(HDB_EDEVICE, "prim_coop: granule sweep timed out (workgroups not co-resident)");
    return true;
}

// Variant (prim_coop_slots = 4): one step = DPP wave minimum of order-preserving keys (the
// highest lane among equal keys is the argmin_last winner: indices grow with the lane), the
// wave's winner lane parks its row in LDS, ONE barrier, wave 0 folds the 16 waves the same way
// and publishes the workgroup's candidate as data-tagged 8-byte granules (Guideline 16 R2: 3
// key granules {value lo, value hi, index} + 2 (DM + 3) row granules, one sc1 store per lane),
// sweeps the nwg x 3 key granules flat until every tag is this step, picks the winner workgroup
// and reads its row granules straight into the LDS row; ONE barrier.  No fences, no counters.
// Same-XCD exchange (spread = 8): the grid is 8x the workgroups and only blocks b % 8 == res
// work -- blocks b and b + 8 are dealt to one XCD (res rotates per launch, so concurrent Prims
// of the model pool tend to land on different XCDs).  They check that at run time (XCC_ID): when
// every working block reports the same XCC, the granules are published with plain stores (the
// line stays in that XCD's L2, which every CU's sc1 poll reads) instead of sc1 stores (which
// drop the line from L2, so every poll crossed the fabric).  Any other placement keeps the sc1
// protocol: placement changes only speed.
template <int BS, int DM, bool FULL>
__global__ __launch_bounds__(BS) void prim_coop4_kernel(PrimIn in, int n, int self_edges, int32_t *__restrict__ va,
                                                        int32_t *__restrict__ vb, double *__restrict__ w,
                                                        gu64 *__restrict__ gkey, gu64 *__restrict__ grow, int *err,
                                                        unsigned spin_limit, int spread, int *__restrict__ xcc,
                                                        int res) {
    if ((int)(blockIdx.x % spread) != res) return;  // an idle block of a spread grid
    constexpr int NW = BS / 64;
    constexpr int ND = DM + 3;  // x, core, eB, nnB
    __shared__ double s_cand[NW][ND + 1];
    __shared__ int s_ci[NW];
    constexpr int G = 3 + 2 * ND;  // FULL: one slot of key + row granules per workgroup
    __shared__ unsigned s_key[FULL ? G * 64 : 3 * 64];
    __shared__ double s_row[ND];
    __shared__ int s_cur, s_local;
    const int nwg = (int)gridDim.x / spread;
    const int bid = (int)blockIdx.x / spread;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = bid * BS + tid;
    if (tid == 0) s_local = 0;
    if (spread > 1 && wid == 0) {  // every working block on one XCC?
        if (lane == 0) {
            unsigned x;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            __hip_atomic_store(xcc + bid, (int)(x & 15u) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool same = true;
        int first = 0;
        for (unsigned spins = 0;;) {
            bool ok = true;
            int mn = 1 << 30, mx = -1;
            for (int j = lane; j < nwg; j += 64) {
                const int v = __hip_atomic_load(xcc + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok &= v != 0;
                mn = min(mn, v);
                mx = max(mx, v);
            }
            if (__all(ok)) {
                for (int o = 32; o >= 1; o >>= 1) {
                    mn = min(mn, __shfl_xor(mn, o));
                    mx = max(mx, __shfl_xor(mx, o));
                }
                same = mn == mx;
                first = mn;
                break;
            }
            if (++spins > spin_limit) {  // not co-resident: the retry takes over
                if (lane == 0) atomicExch(err, 1);
                first = -1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) s_local = first < 0 ? -1 : (same && first > 0);
    }
    __syncthreads();
    if (s_local < 0) return;
    const bool local = s_local != 0;
    double xi[DM], ci = 0, ebi = 0, nni = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xi[c] = (i < n && c < in.d) ? in.X[(int64_t)i * in.d + c] : 0.0;
    if (i < n) {
        ci = in.core[i];
        if (in.eB) {
            ebi = in.eB[i];
            nni = in.nnB[i];
        }
    }
    double best = JMAX;
    int par = -1;
    bool att = (i >= n) || (i == n - 1);
    double xc[DM], cc, ebc = 0, nnc = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xc[c] = c < in.d ? in.X[(int64_t)(n - 1) * in.d + c] : 0.0;
    cc = in.core[n - 1];
    if (in.eB) {
        ebc = in.eB[n - 1];
        nnc = in.nnB[n - 1];
    }
    int cur = n - 1;
    constexpr unsigned long long KINF = 0x7ff0000000000000ull;  // key of +inf: nothing to offer
    // Candidate caching: a wave's candidate changes only when one of its lanes
    // improved or its parked winner was attached in the last step, and a workgroup's only when
    // one of its waves' did -- most steps relax nothing near most waves (the sqrt-free rejection
    // in coop_mrd), so the wave minimum, the parking and the workgroup fold are skipped and the
    // workgroup republishes its cached granule values under the new step's tag.
    __shared__ int s_dirty;
    if (tid == 0) s_dirty = 0;
    bool just = false;    // this lane was attached at the end of the last step
    unsigned val_c = 0u;  // wave 0: the workgroup's cached granule value (this lane's)
    for (int step = 1; step < n; step++) {
        COOP_T(0);
        bool imp = false;
        double mrd = 0.0;
        if (!att) mrd = coop_mrd<DM>(in, xc, cc, ebc, nnc, xi, ci, ebi, nni, best, imp);
        if (imp) {
            best = mrd;
            par = cur;
        }
        COOP_T(6);
        const bool dirty = step == 1 || __any(imp || just);
        just = false;
        if (dirty) {
            const unsigned long long key = att ? KINF : mrd_key(best);
            const unsigned long long wmin = wave_min_u64(key);
            const int wl = last_lane(key == wmin);
            if (lane == wl) {  // the wave's candidate parks its row
#pragma unroll
                for (int c = 0; c < DM; c++) s_cand[wid][c] = xi[c];
                s_cand[wid][DM] = ci;
                s_cand[wid][DM + 1] = ebi;
                s_cand[wid][DM + 2] = nni;
                s_cand[wid][ND] = best;
                s_ci[wid] = wmin < KINF ? i : -1;
                s_dirty = 1;
            }
        }
        COOP_T(7);
        __syncthreads();
        COOP_T(1);
        if (wid == 0) {
            const int buf = step & 1;
            const unsigned tag = (unsigned)step;
            unsigned val;
            if (s_dirty) {
                // fold the waves: lane q holds wave q's candidate
                const int qi = lane < NW ? s_ci[lane] : -1;
                const unsigned long long qk = qi >= 0 ? mrd_key(s_cand[lane < NW ? lane : 0][ND]) : KINF;
                const unsigned long long gmin = wave_min_u64(qk);
                const int q = min(last_lane(qk == gmin), NW - 1);  // all waves empty: any wave (index -1)
                const unsigned *cw = (const unsigned *)s_cand[q];
                const int gidx = __builtin_amdgcn_readlane(qi, q);  // q is wave-uniform
                // publish: lanes 0-2 the key granules, lanes 3 .. 3 + 2 ND the row granules
                if (lane < 2) val = cw[2 * ND + lane];
                else if (lane == 2) val = (unsigned)gidx;
                else val = lane < 3 + 2 * ND ? cw[lane - 3] : 0u;
                val_c = val;
            } else
                val = val_c;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) s_dirty = 0;  // every lane of wave 0 has read it; set again only after the next barrier
            const unsigned long long gv = ((unsigned long long)tag << 32) | val;
            gu64 *dst = nullptr;
            if (FULL) {
                if (lane < G) dst = gkey + ((size_t)buf * nwg + bid) * G + lane;
            } else if (lane < 3)
                dst = gkey + ((size_t)buf * nwg + bid) * 3 + lane;
            else if (lane < 3 + 2 * ND)
                dst = grow + ((size_t)buf * nwg + bid) * (2 * ND) + (lane - 3);
            if (dst) {
                // local: a plain (workgroup-scope) store -- the line stays in the XCD's L2, which
                // every CU of that XCD polls with agent-scope loads.  This relies on gfx950
                // details the HIP memory model does not promise (a write-through L1 and one L2
                // per XCD; every working block checked to be on one XCC above).  Correctness never
                // depends on it: each granule carries its step tag, and if the values were not
                // seen the plain attempt times out and the cooperative launch (agent-scope
                // stores) runs instead -- visible as prim_coop_plain_retries in the C3/C5 lines
                if (local)
                    __hip_atomic_store(dst, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                else
                    __hip_atomic_store(dst, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            COOP_T(2);
            // sweep every workgroup's key granules
            constexpr int KS = FULL ? G : 3;  // granules per workgroup in the sweep
            const gu64 *kb = gkey + (size_t)buf * nwg * KS;
            const int T = KS * nwg;
            bool tmo = false;
            for (unsigned spins = 0;;) {
                bool ok = true;
                for (int j = lane; j < T; j += 64) {
                    const unsigned long long x = __hip_atomic_load(kb + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok &= (unsigned)(x >> 32) == tag;
                    s_key[j] = (unsigned)x;
                }
                if (__all(ok)) break;
                if (++spins > spin_limit) {  // a co-residency failure must not hang the device
                    if (lane == 0) atomicExch(err, 1);
                    tmo = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            COOP_T(3);
            __builtin_amdgcn_wave_barrier();
            int kidx = -1;
            unsigned long long kk = KINF;
            if (lane < nwg) {
                kidx = (int)s_key[KS * lane + 2];
                const double kv = __longlong_as_double(
                    (long long)(((unsigned long long)s_key[KS * lane + 1] << 32) | s_key[KS * lane]));
                if (kidx >= 0) kk = mrd_key(kv);
            }
            const unsigned long long amin = wave_min_u64(kk);
            const int k = last_lane(kk == amin);
            const int win = __builtin_amdgcn_readlane(kidx, k);  // k is wave-uniform
            if (tmo || amin == KINF) {
                if (lane == 0) s_cur = -1;
            } else {
                if (FULL) {  // the winner's row is already in LDS
                    if (lane < 2 * ND) ((unsigned *)s_row)[lane] = s_key[KS * k + 3 + lane];
                }
                bool row_tmo = false;
                if (!FULL && lane < 2 * ND) {  // the winner's row granules, straight into the LDS row
                    const gu64 *rb = grow + ((size_t)buf * nwg + k) * (2 * ND) + lane;
                    unsigned long long x;
                    for (unsigned spins = 0;;) {
                        x = __hip_atomic_load(rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if ((unsigned)(x >> 32) == tag) break;
                        if (++spins > spin_limit) {  // a stale row must not be used: report, exit
                            row_tmo = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    ((unsigned *)s_row)[lane] = (unsigned)x;
                }
                if (__any(row_tmo)) {
                    if (lane == 0) {
                        atomicExch(err, 1);
                        s_cur = -1;
                    }
                } else if (lane == 0)
                    s_cur = win;
            }
            COOP_T(4);
        }
        __syncthreads();
        COOP_T(5);
        cur = s_cur;
        if (cur < 0) break;
#pragma unroll
        for (int c = 0; c < DM; c++) xc[c] = s_row[c];
        cc = s_row[DM];
        ebc = s_row[DM + 1];
        nnc = s_row[DM + 2];
        if (i == cur) {
            att = true;
            just = true;
        }
    }
    if (i < n - 1) {
        va[i] = par >= 0 ? in.ids[par] : 0;
        vb[i] = in.ids[i];
        w[i] = best;
    }
    if (self_edges && i < n) {
        va[n - 1 + i] = in.ids[i];
        vb[n - 1 + i] = in.ids[i];
        w[n - 1 + i] = in.core[i];
    }
}

template <int DM, bool FULL, int BS>
static bool launch_coop4_bs(hdb_ctx *ctx, const PrimIn &in, int64_t o, int64_t n, int64_t eo, int self_edges,
                            int32_t *va, int32_t *vb, double *w) {
    const int nwg = (int)ceil_div(n, BS);
    if (nwg > 64) return false;
    int coop = 0, ncu = 0, per_cu = 0;
    HIP_CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, prim_coop4_kernel<BS, DM, FULL>, BS, 0));
    if (!coop || (int64_t)per_cu * ncu < nwg) return false;
    constexpr int ND = DM + 3;
    const size_t kbytes = (8 * (size_t)(FULL ? 3 + 2 * ND : 3) * 2 * nwg + 255) & ~size_t(255);
    const size_t rbytes = (8 * (size_t)2 * ND * 2 * nwg + 255) & ~size_t(255);
    char *base = (char *)arena(ctx, A_WORK3, kbytes + rbytes + 512);
    gu64 *gkey = (gu64 *)base;
    gu64 *grow = (gu64 *)(base + kbytes);
    int *err = (int *)(base + kbytes + rbytes);
    int *xcc = err + 64;  // the working blocks' XCC ids (spread launch)
    HIP_CHECK(hipMemsetAsync(base, 0, kbytes + rbytes + 512, ctx->stream));  // tags 0: no step yet
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    int nn = (int)n;
    int32_t *pva = va + eo, *pvb = vb + eo;
    double *pw = w + eo;
    unsigned spin = 1u << 24;
    int spread1 = 1, res0 = 0;
    void *args[] = {&L, &nn, &self_edges, &pva, &pvb, &pw, &gkey, &grow, &err, &spin, &spread1, &xcc, &res0};
    // same-XCD exchange for the plain attempt when its blocks fit one XCD (32 CUs)
    const int spread = (ctx->prim_coop_xcd && nwg <= ctx->prim_coop_xcd_max_wg && nwg <= 32 * per_cu) ? 8 : 1;
    static std::atomic<int> launches{0};
    const int res = spread > 1 ? (launches.fetch_add(1) & 7) : 0;
    // A plain launch first: ROCm serialises cooperative launches device-wide, so the concurrent
    // local models of one level (driver model pool) would queue behind each other.  The grid
    // (<= 64 workgroups) is far below the device's capacity, and every inter-workgroup wait has
    // a timeout: if the workgroups were not co-resident the kernel reports it and exits, the
    // state is reset and the cooperative launch (guaranteed co-residency) runs instead.  The
    // plain attempt waits at most 2^prim_coop_plain_spin_log2 polls per exchange (a step takes
    // microseconds once every workgroup runs; the default 2^20 polls is ~1 s), the cooperative
    // one 2^24.
    const unsigned plain_spin = 1u << ctx->prim_coop_plain_spin_log2;
    int h_err = 0;
    for (int attempt = ctx->prim_coop_plain ? 0 : 1; attempt < 2; attempt++) {
        if (attempt == 1 && h_err) HIP_CHECK(hipMemsetAsync(base, 0, kbytes + rbytes + 512, ctx->stream));
        {
            KernelTimer t(ctx, "prim_coop");
            if (attempt == 0)
                hipLaunchKernelGGL((prim_coop4_kernel<BS, DM, FULL>), dim3(nwg * spread), dim3(BS), 0, ctx->stream, L, nn,
                                   self_edges, pva, pvb, pw, gkey, grow, err, plain_spin, spread, xcc, res);
            else
                HIP_CHECK(hipLaunchCooperativeKernel((const void *)prim_coop4_kernel<BS, DM, FULL>, dim3(nwg), dim3(BS),
                                                     args, 0, ctx->stream));
            HIP_CHECK(hipGetLastError());
        }
        h_err = 0;
        HIP_CHECK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        if (!h_err) {
            ctx->stats["prim_coop_steps"] += n - 1;  // sequential Prim steps (roofline: bench.py)
            ctx->stats["prim_coop_launches"] += 1;
            return true;
        }
        if (attempt == 0) ctx->stats["prim_coop_plain_retries"] += 1;
    }
    HDB_THROW(HDB_EDEVICE, "prim_coop: key sweep timed out (workgroups not co-resident)");
    return true;
}

// workgroup size: 1024 by default; prim_coop_bs = 0 takes the smallest of 128..1024 that keeps
// the Prim within prim_coop_xcd_max_wg workgroups (one XCD), so more CUs -- and fewer waves per
// SIMD -- share each step's relaxation
template <int DM, bool FULL>
static bool launch_coop4(hdb_ctx *ctx, const PrimIn &in, int64_t o, int64_t n, int64_t eo, int self_edges,
                         int32_t *va, int32_t *vb, double *w) {
    int bs = ctx->prim_coop_bs;
    if (bs == 0) {
        bs = 1024;
        for (int b = 128; b < 1024; b *= 2)
            if (ceil_div(n, (int64_t)b) <= ctx->prim_coop_xcd_max_wg) {
                bs = b;
                break;
            }
    }
    switch (bs) {
    case 128: return launch_coop4_bs<DM, FULL, 128>(ctx, in, o, n, eo, self_edges, va, vb, w);
    case 256: return launch_coop4_bs<DM, FULL, 256>(ctx, in, o, n, eo, self_edges, va, vb, w);
    case 512: return launch_coop4_bs<DM, FULL, 512>(ctx, in, o, n, eo, self_edges, va, vb, w);
    default: return launch_coop4_bs<DM, FULL, 1024>(ctx, in, o, n, eo, self_edges, va, vb, w);
    }
}

#if HDB_PRIM_SPEC
// ------------------------------------------ cooperative kernel, speculative steps (slots 6)
// The same Prim (HDBSCANStar.java:124-205 / HdbscanDataBubbles.java:165-254: select the
// unattached vertex with the smallest best, ties -> largest index; update iff mrd < best,
// parent = the vertex just attached), with many steps per exchange instead of one.
//
// A round starts from an exact state.  Every workgroup publishes its C = 64 / nwg best
// unattached vertices (each wave's best two, the workgroup's best C of those) with their rows;
// the union is the round's list L (<= 64 vertices), known to every workgroup.  Then every wave
// runs the Prim on its own, without barriers or exchanges: step t takes the best unattached
// member of L (its key is tracked redundantly by every wave: lane j holds member j's row and
// relaxes it exactly as the owning lane does, so the keys agree bit for bit), every lane relaxes
// against it, and the wave checks its own lanes: if a non-member of L beats the step's pick
// ((best, index) order of the select rule), step t is where the round's picks stop being the
// Prim's, and the wave stops.  One exchange then gives s* = the first such step over all waves
// and the true vertex of step s* (the best violating vertex of the waves that stop there).
// Steps < s* were the Prim's own; every lane undoes the speculation past them (a lane whose
// last improvement came at a step >= s* restores its round-start best/parent and re-relaxes
// against the picks of steps < s*; a vertex attached at a step >= s* is detached), attaches the
// true vertex of step s* and relaxes against it.  The result is the sequential Prim's state
// after s* + 1 steps, so the output is the reference's whatever the speculation did.  The list
// only decides how many steps a round commits (simulated on 16,384 8-d blob points: ~34).
// LDS hand-off between the waves of one workgroup without waiting for global loads in flight
// (a release/acquire atomic also waits for vmcnt): the writer waits for its own LDS operations
// only (s_waitcnt lgkmcnt(0)) before the flag store; the reader's compiler barrier keeps the
// payload loads behind the flag load, and LDS serves them after it
__device__ __forceinline__ void lds_publish(int *flag, int v) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt, expcnt untouched
    __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int lds_peek(int *flag) {
    const int v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    return v;
}

template <int BS, int DM>
__global__ __launch_bounds__(BS + 64) void prim_spec_kernel(PrimIn in, int n, int self_edges, int32_t *__restrict__ va,
                                                       int32_t *__restrict__ vb, double *__restrict__ w,
                                                       gu64 *__restrict__ gcand, gu64 *__restrict__ gviol, int *err,
                                                       unsigned spin_limit, int spread, int *__restrict__ xcc,
                                                       int res, unsigned long long *__restrict__ stats,
                                                       unsigned *__restrict__ gstop) {
    if ((int)(blockIdx.x % spread) != res) return;  // an idle block of a spread grid
    // wave 0 leads (the list, the picks) and owns no vertex; waves 1 .. BS/64 one vertex per lane
    constexpr int NW = BS / 64 + 1;
    constexpr int ND = DM + 3;       // x, core, eB, nnB
    constexpr int GC = 3;            // candidate granules: key lo, key hi, index (rows: read from X by index)
    constexpr int GV = 4;            // violation granules: step, key lo, key hi, index
    constexpr unsigned long long KINF = 0x7ff0000000000000ull;  // key of +inf: nothing to offer
    const int nwg = (int)gridDim.x / spread;
    const int bid = (int)blockIdx.x / spread;
    const int C = min(64 / nwg, 2 * NW);  // list entries per workgroup (nwg <= 64)
    const int NL = C * nwg;          // list size
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = tid < 64 ? n + tid : bid * BS + tid - 64;  // the leader's lanes: no vertex (>= n)

    __shared__ unsigned long long s_wck[NW * 2];  // ... keys
    __shared__ int s_wci[NW * 2];                 // ... indices
    __shared__ unsigned s_cg[64 * GC];            // swept candidate granules (values)
    __shared__ double s_lrow[64][ND];             // the list: rows, keys, indices
    __shared__ double s_lkey[64];
    __shared__ int s_lidx[64];
    __shared__ int s_inl[BS + 64];                // round tag: this lane's vertex is a list member
    __shared__ int s_pick[65];                    // wave 0's picks (list entry per step)
    __shared__ int s_vt[NW];                      // per wave: first violating step
    __shared__ unsigned long long s_vk[NW];       // ... its best violating vertex: key, index, row
    __shared__ int s_vi[NW];
    __shared__ unsigned s_vg[64 * GV];            // swept violation granules (values)
    __shared__ double s_wrow[ND];                 // the round's true vertex at s*: row
    __shared__ int s_star, s_win, s_local, s_stop;
    __shared__ int s_sel[64];
    __shared__ int s_vmin;                        // this round's first violating step in the workgroup
    __shared__ unsigned long long s_pkey[65];     // wave 0's picks: key, index; published step count
    __shared__ int s_pidx[65];
    __shared__ int s_tick, s_lstop;

    if (tid == 0) s_local = 0;
    if (spread > 1 && wid == 0) {  // every working block on one XCC?  (as prim_coop4_kernel)
        if (lane == 0) {
            unsigned x;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            __hip_atomic_store(xcc + bid, (int)(x & 15u) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool same = true;
        int first = 0;
        for (unsigned spins = 0;;) {
            bool ok = true;
            int mn = 1 << 30, mx = -1;
            for (int j = lane; j < nwg; j += 64) {
                const int v = __hip_atomic_load(xcc + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok &= v != 0;
                mn = min(mn, v);
                mx = max(mx, v);
            }
            if (__all(ok)) {
                for (int o = 32; o >= 1; o >>= 1) {
                    mn = min(mn, __shfl_xor(mn, o));
                    mx = max(mx, __shfl_xor(mx, o));
                }
                same = mn == mx;
                first = mn;
                break;
            }
            if (++spins > spin_limit) {
                if (lane == 0) atomicExch(err, 1);
                first = -1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) s_local = first < 0 ? -1 : (same && first > 0);
    }
    s_inl[tid] = 0;
    __syncthreads();
    if (s_local < 0) return;
    const bool local = s_local != 0;

    // own row and state
    double xi[DM], ci = 0, ebi = 0, nni = 0;
#pragma unroll
    for (int c = 0; c < DM; c++) xi[c] = (i < n && c < in.d) ? in.X[(int64_t)i * in.d + c] : 0.0;
    if (i < n) {
        ci = in.core[i];
        if (in.eB) {
            ebi = in.eB[i];
            nni = in.nnB[i];
        }
    }
    double best = JMAX;
    int par = -1;
    bool att = (i >= n) || (i == n - 1);
    {  // the start vertex n - 1
        double xc[DM];
#pragma unroll
        for (int c = 0; c < DM; c++) xc[c] = c < in.d ? in.X[(int64_t)(n - 1) * in.d + c] : 0.0;
        const double cc = in.core[n - 1], ebc = in.eB ? in.eB[n - 1] : 0.0, nnc = in.eB ? in.nnB[n - 1] : 0.0;
        if (!att) {
            bool imp = false;
            const double mrd = coop_mrd<DM>(in, xc, cc, ebc, nnc, xi, ci, ebi, nni, best, imp);
            if (imp) {
                best = mrd;
                par = n - 1;
            }
        }
    }
    auto put = [&](gu64 *dst, unsigned tag, unsigned val) {
        const unsigned long long gv = ((unsigned long long)tag << 32) | val;
        if (local)
            __hip_atomic_store(dst, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            __hip_atomic_store(dst, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // wave 0: read `count` granules at src until every tag is `tag`, values to dst (LDS)
    auto sweep = [&](const gu64 *src, int count, unsigned tag, unsigned *dst) -> bool {
        for (unsigned spins = 0;;) {
            bool ok = true;
            for (int b = 0; b < count; b += 64 * 8) {  // 8 loads in flight per lane, then one wait
                unsigned long long x[8];
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int j = b + k * 64 + lane;
                    x[k] = j < count ? __hip_atomic_load(src + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : ((unsigned long long)tag << 32);
                }
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const int j = b + k * 64 + lane;
                    ok &= (unsigned)(x[k] >> 32) == tag;
                    if (j < count) dst[j] = (unsigned)x[k];
                }
            }
            if (__all(ok)) return true;
            if (++spins > spin_limit) {
                if (lane == 0) atomicExch(err, 1);
                return false;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    };

    int committed = 0;  // Prim steps done (vertices attached after n - 1)
    unsigned long long n_rounds = 0, n_spec = 0, cyc[4] = {0, 0, 0, 0}, n_exec = 0;
    unsigned long long tm = __builtin_amdgcn_s_memtime();
    auto tick = [&](int k) {  // per-phase cycles of workgroup 0, thread 0 (prim_spec_cyc_* stats)
        if (tid == 0) {
            const unsigned long long x = __builtin_amdgcn_s_memtime();
            cyc[k] += x - tm;
            tm = x;
        }
    };
    for (unsigned round = 1; committed < n - 1; round++) {
        const int buf = round & 1;
        // ---- 1. the list: each wave's two best, the workgroup's best C, every workgroup's C
        {
            unsigned long long key = att ? KINF : mrd_key(best);
            const unsigned long long k1 = wave_min_u64(key);
            const int l1 = last_lane(key == k1);  // lanes grow with the vertex index: largest index
            const unsigned long long key2 = lane == l1 ? KINF : key;
            const unsigned long long k2 = wave_min_u64(key2);
            const int l2 = last_lane(key2 == k2);
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int lq = q ? l2 : l1;
                const unsigned long long kq = q ? k2 : k1;
                if (lane == lq) {
                    s_wck[2 * wid + q] = kq;
                    s_wci[2 * wid + q] = kq < KINF ? i : -1;
                }
            }
        }
        __syncthreads();
        if (wid == 0) {
            // the workgroup's best C of its 2 NW wave candidates (lane q < 2 NW holds candidate q)
            unsigned long long qk = lane < 2 * NW ? s_wck[lane] : KINF;
            const int qi = lane < 2 * NW ? s_wci[lane] : -1;
            if (qi < 0) qk = KINF;
            int sel = -1;  // lane e < C: the candidate (lane) ranked e
            for (int e = 0; e < C; e++) {
                const unsigned long long m = wave_min_u64(qk);
                int pick = -1;
                if (m < KINF) {  // largest index among the minima
                    const unsigned long long inv = (qk == m) ? (0xffffffffull - (unsigned)qi) : ~0ull;
                    const unsigned long long mi = wave_min_u64(inv);
                    pick = last_lane(inv == mi && qk == m);
                }
                if (lane == e) sel = pick;
                if (pick >= 0 && lane == pick) qk = KINF;
            }
            s_sel[lane] = sel;
            __builtin_amdgcn_wave_barrier();
            // publish: entry e's granules at [e * GC, (e + 1) * GC)
            gu64 *dst = gcand + ((size_t)buf * nwg + bid) * (size_t)(C * GC);
            for (int g = lane; g < C * GC; g += 64) {
                const int e = g / GC, f = g - e * GC;
                const int q = s_sel[e];
                unsigned val;
                if (q < 0) val = f == 2 ? 0xffffffffu : 0u;
                else if (f < 2) val = (unsigned)(s_wck[q] >> (32 * f));
                else val = (unsigned)s_wci[q];
                put(dst + g, round, val);
            }
            // sweep every workgroup's entries
            const bool ok = sweep(gcand + (size_t)buf * nwg * (size_t)(C * GC), NL * GC, round, s_cg);
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                s_vmin = 1 << 30;
                s_tick = 0;
                s_lstop = 1 << 30;
            }
            if (!ok) {
                if (lane == 0) s_stop = 1;
            } else {
                if (lane == 0) s_stop = 0;
                // list entry j = lane (j < NL): key, index, row into LDS
                if (lane < NL) {
                    const unsigned *g = s_cg + lane * GC;
                    const int li = (int)g[2];
                    s_lidx[lane] = li;
                    s_lkey[lane] = __longlong_as_double((long long)(((unsigned long long)g[1] << 32) | g[0]));
                    if (li >= 0) {  // the member's row, as its owning lane holds it
#pragma unroll
                        for (int c = 0; c < DM; c++) s_lrow[lane][c] = c < in.d ? in.X[(int64_t)li * in.d + c] : 0.0;
                        s_lrow[lane][DM] = in.core[li];
                        s_lrow[lane][DM + 1] = in.eB ? in.eB[li] : 0.0;
                        s_lrow[lane][DM + 2] = in.eB ? in.nnB[li] : 0.0;
                    }
                    if (li >= 0 && li / BS == bid) s_inl[li % BS + 64] = (int)round;
                } else if (lane < 64) {
                    s_lidx[lane] = -1;
                }
            }
        }
        __syncthreads();
        if (s_stop) break;  // a timed-out sweep (not co-resident): reported through err
        tick(0);
        const bool inl = s_inl[tid] == (int)round;

        // ---- 2. speculation.  Wave 0 tracks the list (lane j: member j's row and key) and
        // publishes each step's pick (s_pick / s_pkey / s_pidx, then the step count s_tick with
        // release order); every wave checks and relaxes its own lanes against the published picks
        // and stops at its first violation, or once the workgroup's (LDS) or anyone's (global)
        // first violation lies behind it.
        double lx[DM], lc = 0.0, le = 0.0, ln = 0.0, lk = 0.0;
        int li = -1;
        bool latt = true;
        if (wid == 0) {
#pragma unroll
            for (int c = 0; c < DM; c++) lx[c] = s_lrow[lane][c];
            lc = s_lrow[lane][DM];
            le = s_lrow[lane][DM + 1];
            ln = s_lrow[lane][DM + 2];
            lk = s_lkey[lane];
            li = s_lidx[lane];
            latt = li < 0;
        }
        const double best0 = best;
        const int par0 = par;
        double b2 = best;  // the value before the last improvement of this round (t2: its step)
        int p2 = par, t2 = -1, tstep = -1, astep = 1 << 30;
        // the first violating step anyone found this round: in this workgroup (LDS) or in any
        // (a global word min-combined as (rounds left, step): a newer round always wins), the
        // global word read 4 steps ahead so its latency overlaps the steps in between
        const unsigned rtag = (0xffffffu - round) << 7;
        unsigned gpre = __hip_atomic_load(gstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int gs = 1 << 30;
        for (int t = 0;; t++) {
            bool stop = false;
            if (t > 0) {
                if ((t & 3) == 0) {
                    gs = (gpre & ~127u) == rtag ? (int)(gpre & 127u) : (1 << 30);
                    gpre = __hip_atomic_load(gstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // past the first violating step everything is undone; that step itself is still
                // checked by every wave (its best violator may be the step's vertex)
                stop = min(gs, __hip_atomic_load(&s_vmin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < t;
            }
            unsigned long long lm = KINF;
            int vlane = -1, vidx = -1;
            if (wid == 0) {
                if (stop) {
                    if (lane == 0) lds_publish(&s_lstop, t);
                } else {
                    // the step's pick: the best unattached member ((key, index) order of the select rule)
                    const unsigned long long lkey = latt ? KINF : mrd_key(lk);
                    lm = wave_min_u64(lkey);
                    if (lm < KINF) {
                        const unsigned long long eqm = __ballot(lkey == lm);
                        if (__popcll(eqm) == 1) {  // the usual case: one member holds the minimum
                            vlane = __ffsll((long long)eqm) - 1;
                        } else {  // equal keys: the largest index
                            const unsigned long long inv = (lkey == lm) ? (0xffffffffull - (unsigned)li) : ~0ull;
                            const unsigned long long mi = wave_min_u64(inv);
                            vlane = last_lane(inv == mi && lkey == lm);
                        }
                        vidx = __builtin_amdgcn_readlane(li, vlane);
                    }
                    if (lane == 0) {
                        s_pick[t] = vlane;
                        s_pkey[t] = lm;
                        s_pidx[t] = vidx;
                        lds_publish(&s_tick, t + 1);
                    }
                }
            } else if (!stop) {
                for (;;) {  // wait for the leader's pick of step t (or its stop)
                    if (lds_peek(&s_tick) > t) break;
                    if (lds_peek(&s_lstop) <= t) {
                        stop = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(0);
                }
                if (!stop) {
                    vlane = s_pick[t];
                    lm = s_pkey[t];
                    vidx = s_pidx[t];
                }
            }
            if (tid == 0 || tid == 64) n_exec += (unsigned long long)1 << (tid ? 32 : 0);
            if (stop) {
                if (lane == 0) {
                    s_vt[wid] = 1 << 30;
                    s_vi[wid] = -1;
                    s_vk[wid] = KINF;
                }
                break;
            }
            // does one of this wave's non-members beat the pick?
            const unsigned long long mk = (att || inl) ? KINF : mrd_key(best);
            const bool viol = mk < KINF && (mk < lm || (mk == lm && i > vidx));
            if (__any(viol) || vlane < 0) {
                const unsigned long long cm = wave_min_u64(mk);
                const int cl = cm < KINF ? last_lane(mk == cm) : -1;
                if (lane == 0) {
                    s_vt[wid] = t;
                    s_vk[wid] = cm;
                    atomicMin(&s_vmin, t);
                    atomicMin(gstop, rtag | (unsigned)t);
                    if (wid == 0) lds_publish(&s_lstop, t + 1);
                }
                if (cl >= 0 && lane == cl) s_vi[wid] = i;
                if (cl < 0 && lane == 0) s_vi[wid] = -1;
                break;
            }
            // attach the pick and relax against it (own lanes; wave 0 also the list copies)
            double xv[DM];
#pragma unroll
            for (int c = 0; c < DM; c++) xv[c] = s_lrow[vlane][c];
            const double cv = s_lrow[vlane][DM], ebv = s_lrow[vlane][DM + 1], nnv = s_lrow[vlane][DM + 2];
            if (wid == 0) {
                if (lane == vlane) latt = true;
                if (!latt) {
                    bool imp = false;
                    const double mrd = coop_mrd<DM>(in, xv, cv, ebv, nnv, lx, lc, le, ln, lk, imp);
                    if (imp) lk = mrd;
                }
            }
            if (i == vidx) {
                att = true;
                astep = t;
            }
            if (!att) {
                bool imp = false;
                const double mrd = coop_mrd<DM>(in, xv, cv, ebv, nnv, xi, ci, ebi, nni, best, imp);
                if (imp) {
                    b2 = best;
                    p2 = par;
                    t2 = tstep;
                    best = mrd;
                    par = vidx;
                    tstep = t;
                }
            }
        }
        __syncthreads();
        tick(1);
        // ---- 3. exchange: first violating step over all waves, the true vertex of that step
        if (wid == 0) {
            const int qt = lane < NW ? s_vt[lane] : (1 << 30);
            int tw = qt;
            for (int o = 32; o >= 1; o >>= 1) tw = min(tw, __shfl_xor(tw, o));
            unsigned long long qk = (lane < NW && qt == tw && s_vi[lane] >= 0) ? s_vk[lane] : KINF;
            const unsigned long long m = wave_min_u64(qk);
            const int q = m < KINF ? last_lane(qk == m) : -1;  // waves hold increasing indices
            gu64 *dst = gviol + ((size_t)buf * nwg + bid) * GV;
            if (lane < GV) {
                unsigned val;
                if (lane == 0) val = (unsigned)tw;
                else if (lane < 3) val = (unsigned)(m >> (32 * (lane - 1)));
                else val = q >= 0 ? (unsigned)s_vi[q] : 0xffffffffu;
                put(dst + lane, round, val);
            }
            const bool ok = sweep(gviol + (size_t)buf * nwg * GV, nwg * GV, round, s_vg);
            __builtin_amdgcn_wave_barrier();
            if (!ok) {
                if (lane == 0) s_stop = 1;
            } else {
                const int gt = lane < nwg ? (int)s_vg[lane * GV] : (1 << 30);
                int st = gt;
                for (int o = 32; o >= 1; o >>= 1) st = min(st, __shfl_xor(st, o));
                const int gi = lane < nwg ? (int)s_vg[lane * GV + 3] : -1;
                unsigned long long gk = (lane < nwg && gt == st && gi >= 0)
                                            ? (((unsigned long long)s_vg[lane * GV + 2] << 32) | s_vg[lane * GV + 1])
                                            : KINF;
                const unsigned long long gm = wave_min_u64(gk);
                int wl = -1;
                if (gm < KINF) {  // largest index among the minima
                    const unsigned long long inv = (gk == gm) ? (0xffffffffull - (unsigned)gi) : ~0ull;
                    const unsigned long long mi = wave_min_u64(inv);
                    wl = last_lane(inv == mi && gk == gm);
                }
                if (lane == 0) {
                    s_star = st;
                    s_win = wl >= 0 ? (int)s_vg[wl * GV + 3] : -1;
                    s_stop = 0;
                }
                if (wl >= 0) {  // the winner's row from X by index
                    const int wi = (int)s_vg[wl * GV + 3];
                    if (lane < DM) s_wrow[lane] = lane < in.d ? in.X[(int64_t)wi * in.d + lane] : 0.0;
                    else if (lane == DM) s_wrow[DM] = in.core[wi];
                    else if (lane == DM + 1) s_wrow[DM + 1] = in.eB ? in.eB[wi] : 0.0;
                    else if (lane == DM + 2) s_wrow[DM + 2] = in.eB ? in.nnB[wi] : 0.0;
                }
            }
        }
        __syncthreads();
        if (s_stop) break;
        tick(2);
        const int sstar = s_star, win = s_win;
        // ---- 4. keep steps < s*, undo the rest, attach the true vertex of step s*
        if (astep != (1 << 30) && astep >= sstar) att = false;  // attached at an undone step
        // a lane whose last improvement came at an undone step takes back the value before it
        // (exact when the one before was kept); two or more undone improvements: re-relax
        const bool undo = !att && tstep >= sstar;
        const bool redo = undo && t2 >= sstar;
        if (undo && !redo) {
            best = b2;
            par = p2;
        }
        if (__any(redo)) {
            if (redo) {
                best = best0;
                par = par0;
            }
            for (int u = 0; u < sstar; u++) {
                const int vl = s_pick[u];
                double xv[DM];
#pragma unroll
                for (int c = 0; c < DM; c++) xv[c] = s_lrow[vl][c];
                if (redo) {
                    bool imp = false;
                    const double mrd = coop_mrd<DM>(in, xv, s_lrow[vl][DM], s_lrow[vl][DM + 1], s_lrow[vl][DM + 2], xi, ci,
                                                    ebi, nni, best, imp);
                    if (imp) {
                        best = mrd;
                        par = s_lidx[vl];
                    }
                }
            }
        }
        committed += sstar;
        n_spec += sstar;
        if (win >= 0) {
            if (i == win) att = true;
            else if (!att) {
                double xv[DM];
#pragma unroll
                for (int c = 0; c < DM; c++) xv[c] = s_wrow[c];
                bool imp = false;
                const double mrd = coop_mrd<DM>(in, xv, s_wrow[DM], s_wrow[DM + 1], s_wrow[DM + 2], xi, ci, ebi, nni, best, imp);
                if (imp) {
                    best = mrd;
                    par = win;
                }
            }
            committed += 1;
        } else if (sstar == 0) {
            break;  // nothing left anywhere (cannot happen before n - 1 steps: a safeguard)
        }
        n_rounds++;
        __syncthreads();  // s_pick / s_lrow / s_wrow are rewritten next round
        tick(3);
    }
    if (stats && bid == 0 && tid == 0) {
        atomicAdd(stats, n_rounds);
        atomicAdd(stats + 1, n_spec);
        for (int k = 0; k < 4; k++) atomicAdd(stats + 2 + k, cyc[k]);
    }
    if (stats && bid == 0 && (tid == 0 || tid == 64)) atomicAdd(stats + 6, n_exec);  // steps run: wave 0 | wave 1 << 32
    if (i < n - 1) {
        va[i] = par >= 0 ? in.ids[par] : 0;
        vb[i] = in.ids[i];
        w[i] = best;
    }
    if (self_edges && i < n) {
        va[n - 1 + i] = in.ids[i];
        vb[n - 1 + i] = in.ids[i];
        w[n - 1 + i] = in.core[i];
    }
}

template <int DM, int BS = 512>  // 512 threads: the registers of two waves per SIMD (1024 spills)
static bool launch_spec(hdb_ctx *ctx, const PrimIn &in, int64_t o, int64_t n, int64_t eo, int self_edges,
                        int32_t *va, int32_t *vb, double *w) {
    const int nwg = (int)ceil_div(n, BS);
    if (nwg > 64 || n < 2) return false;
    int coop = 0, ncu = 0, per_cu = 0;
    HIP_CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, prim_spec_kernel<BS, DM>, BS + 64, 0));
    if (!coop || per_cu < 1 || (int64_t)per_cu * ncu < nwg) return false;
    constexpr int GC = 3, GV = 4;
    const int C = std::min(64 / nwg, 2 * (BS / 64));
    const size_t cbytes = (8 * (size_t)C * GC * 2 * nwg + 255) & ~size_t(255);
    const size_t vbytes = (8 * (size_t)GV * 2 * nwg + 255) & ~size_t(255);
    char *base = (char *)arena(ctx, A_WORK3, cbytes + vbytes + 1024);
    gu64 *gcand = (gu64 *)base;
    gu64 *gviol = (gu64 *)(base + cbytes);
    int *err = (int *)(base + cbytes + vbytes);
    int *xcc = err + 64;
    unsigned long long *stats = (unsigned long long *)(err + 192);  // rounds, speculated steps
    unsigned *gstop = (unsigned *)(err + 224);
    HIP_CHECK(hipMemsetAsync(base, 0, cbytes + vbytes + 1024, ctx->stream));  // tags 0: no round yet
    HIP_CHECK(hipMemsetAsync(gstop, 0xff, 4, ctx->stream));                   // no violation yet
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    int nn = (int)n;
    int32_t *pva = va + eo, *pvb = vb + eo;
    double *pw = w + eo;
    unsigned spin = 1u << 24;
    int spread1 = 1, res0 = 0;
    void *args[] = {&L, &nn, &self_edges, &pva, &pvb, &pw, &gcand, &gviol, &err, &spin, &spread1, &xcc, &res0, &stats,
                    &gstop};
    const int spread = (ctx->prim_coop_xcd && nwg <= ctx->prim_coop_xcd_max_wg && nwg <= 32 * per_cu) ? 8 : 1;
    static std::atomic<int> launches{0};
    const int res = spread > 1 ? (launches.fetch_add(1) & 7) : 0;
    const unsigned plain_spin = 1u << ctx->prim_coop_plain_spin_log2;
    int h_err = 0;
    for (int attempt = ctx->prim_coop_plain ? 0 : 1; attempt < 2; attempt++) {
        if (attempt == 1 && h_err) {
            HIP_CHECK(hipMemsetAsync(base, 0, cbytes + vbytes + 1024, ctx->stream));
            HIP_CHECK(hipMemsetAsync(gstop, 0xff, 4, ctx->stream));
        }
        {
            KernelTimer t(ctx, "prim_coop");
            if (attempt == 0)
                hipLaunchKernelGGL((prim_spec_kernel<BS, DM>), dim3(nwg * spread), dim3(BS + 64), 0, ctx->stream, L, nn,
                                   self_edges, pva, pvb, pw, gcand, gviol, err, plain_spin, spread, xcc, res, stats,
                                   gstop);
            else
                HIP_CHECK(hipLaunchCooperativeKernel((const void *)prim_spec_kernel<BS, DM>, dim3(nwg), dim3(BS + 64), args, 0,
                                                     ctx->stream));
            HIP_CHECK(hipGetLastError());
        }
        int64_t *pin = pinned_words(ctx) + PINNED_WORDS - 32;  // private slice: err, rounds, steps
        HIP_CHECK(hipMemcpyAsync(pin, err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipMemcpyAsync(pin + 1, stats, 56, hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        h_err = (int)(pin[0] & 0xffffffff);
        if (!h_err) {
            ctx->stats["prim_coop_steps"] += n - 1;
            ctx->stats["prim_coop_launches"] += 1;
            ctx->stats["prim_spec_rounds"] += pin[1];
            ctx->stats["prim_spec_steps"] += pin[2];
            static const char *cn[4] = {"prim_spec_cyc_list", "prim_spec_cyc_spec", "prim_spec_cyc_exch", "prim_spec_cyc_commit"};
            for (int k = 0; k < 4; k++) ctx->stats[cn[k]] += pin[3 + k];
            ctx->stats["prim_spec_exec_w0"] += pin[7] & 0xffffffff;
            ctx->stats["prim_spec_exec_w1"] += pin[7] >> 32;
            return true;
        }
        if (attempt == 0) ctx->stats["prim_coop_plain_retries"] += 1;
    }
    HDB_THROW(HDB_EDEVICE, "prim_spec: exchange timed out (workgroups not co-resident)");
    return true;
}
#endif  // HDB_PRIM_SPEC

template <int DM, bool FAST>
static bool launch_coop2(hdb_ctx *ctx, const PrimIn &in, int64_t o, int64_t n, int64_t eo, int self_edges,
                         int32_t *va, int32_t *vb, double *w) {
    constexpr int BS = 1024;
    const int nwg = (int)ceil_div(n, BS);
    int coop = 0, ncu = 0, per_cu = 0;
    HIP_CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, prim_coop2_kernel<BS, DM, FAST>, BS, 0));
    if (!coop || (int64_t)per_cu * ncu < nwg) return false;
    const size_t sbytes = (sizeof(CoopSlot<DM>) * 2 * (size_t)nwg + 255) & ~size_t(255);
    char *base = (char *)arena(ctx, A_WORK3, sbytes + 256);
    CoopSlot<DM> *slots = (CoopSlot<DM> *)base;
    int *err = (int *)(base + sbytes);
    HIP_CHECK(hipMemsetAsync(base, 0, sbytes + 256, ctx->stream));  // tags 0: no step yet
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    int nn = (int)n;
    int32_t *pva = va + eo, *pvb = vb + eo;
    double *pw = w + eo;
    void *args[] = {&L, &nn, &self_edges, &pva, &pvb, &pw, &slots, &err};
    {
        KernelTimer t(ctx, "prim_coop");
        HIP_CHECK(hipLaunchCooperativeKernel((const void *)prim_coop2_kernel<BS, DM, FAST>, dim3(nwg), dim3(BS), args, 0,
                                             ctx->stream));
    }
    int h_err = 0;
    HIP_CHECK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (h_err) HDB_THROW(HDB_EDEVICE, "prim_coop: slot poll timed out (workgroups not co-resident)");
    return true;
}

static bool launch_coop(hdb_ctx *ctx, const PrimIn &in, int64_t o, int64_t n, int64_t eo, int self_edges,
                        int32_t *va, int32_t *vb, double *w) {
    constexpr int BS = 1024;
    const int nwg = (int)ceil_div(n, BS);
    if (n > 65536 || nwg < 1) return false;
    int coop = 0, ncu = 0, per_cu = 0;
    HIP_CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, prim_coop_kernel<BS>, BS, 0));
    if (!coop || (int64_t)per_cu * ncu < nwg) return false;
    // scratch: partials [2][nwg] x (value, index), barrier counter, error flag
    char *base = (char *)arena(ctx, A_WORK3, 16 * 2 * (size_t)nwg + 512);
    unsigned long long *part = (unsigned long long *)base;
    unsigned *counter = (unsigned *)(base + 16 * 2 * (size_t)nwg + 256);
    int *err = (int *)(counter + 16);
    HIP_CHECK(hipMemsetAsync(counter, 0, 256, ctx->stream));
    PrimIn L = in;
    L.X = in.X + o * in.d;
    L.core = in.core + o;
    L.ids = in.ids + o;
    if (in.eB) {
        L.eB = in.eB + o;
        L.nnB = in.nnB + o;
    }
    int nn = (int)n;
    int32_t *pva = va + eo, *pvb = vb + eo;
    double *pw = w + eo;
    void *args[] = {&L, &nn, &self_edges, &pva, &pvb, &pw, &part, &counter, &err};
    {
        KernelTimer t(ctx, "prim_coop");
        HIP_CHECK(hipLaunchCooperativeKernel((const void *)prim_coop_kernel<BS>, dim3(nwg), dim3(BS), args, 0,
                                             ctx->stream));
    }
    int h_err = 0;
    HIP_CHECK(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (h_err) HDB_THROW(HDB_EDEVICE, "prim_coop: grid barrier timed out (workgroups not co-resident)");
    return true;
}

template <int BS, int PPT>
static void launch_block(hdb_ctx *ctx, const PrimIn &in, const int64_t *offs, const int64_t *eoff,
                         const int32_t *parts, int np, int self_edges, int32_t *va, int32_t *vb, double *w) {
    if (np == 0) return;
    KernelTimer t(ctx, "prim_block");
    hipLaunchKernelGGL((prim_block_kernel<BS, PPT>), dim3(np), dim3(BS), 0, ctx->stream, in, offs, eoff, parts,
                       self_edges, va, vb, w);
    HIP_CHECK(hipGetLastError());
}

// size classes for the block kernel
static int block_class(int64_t n) {
    if (n <= 64) return 0;        // 64 x 1
    if (n <= 256) return 1;       // 64 x 4
    if (n <= 1024) return 2;      // 256 x 4
    if (n <= 4096) return 3;      // 1024 x 4
    return 4;                     // stepwise
}

// Batched Prim. Device pointers: X (rows), offsets (P+1, host copy h_offs), core, ids.
void prim_batched_device(hdb_ctx *ctx, const PrimIn &in, const int64_t *h_offs, int P, int self_edges,
                         int32_t *va, int32_t *vb, double *w) {
    // edge offsets + per-class partition lists (host side), then upload
    std::vector<int64_t> eoff(P + 1, 0);
    std::vector<int32_t> cls[5];
    int64_t total_v = h_offs[P] - h_offs[0];
    for (int p = 0; p < P; p++) {
        int64_t n = h_offs[p + 1] - h_offs[p];
        if (n < 0) HDB_THROW(HDB_EINVAL, "offsets must be non-decreasing");
        eoff[p + 1] = eoff[p] + (n > 0 ? (n - 1) + (self_edges ? n : 0) : 0);
        // wide rows (d >= 8): one workgroup re-reads n x d doubles per step through one CU; the
        // cooperative kernel keeps one row per lane in registers across ceil(n / 1024) CUs
        // (C3's 4,096-bubble models: 19.6 -> 7.4 us/step)
        int c = block_class(n);
        if (c == 3 && in.d >= 8 && in.d <= 16 && ctx->prim_coop && ctx->prim_coop_slots) c = 4;
        if (n > 0) cls[c].push_back(p);
    }
    size_t off = 0;
    auto carve = [&](size_t bytes) {
        size_t o = off;
        off += (bytes + 255) & ~size_t(255);
        return o;
    };
    size_t o_off = carve(sizeof(int64_t) * (P + 1)), o_eoff = carve(sizeof(int64_t) * (P + 1));
    size_t o_parts = carve(sizeof(int32_t) * (P + 1));
    // cooperative single-launch Prim for 4096 < n <= 65536 when the device allows it
    if (ctx->prim_coop) {
        std::vector<int32_t> rest;
        for (int32_t p : cls[4]) {
            int64_t n = h_offs[p + 1] - h_offs[p];
            const int64_t o = h_offs[p] - h_offs[0];
            bool ok = false;
#if HDB_PRIM_SPEC
            if (n <= 65536 && ctx->prim_coop_slots == 6) {  // speculative steps, one exchange per round
                if (in.d <= 4) ok = launch_spec<4>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 8) ok = launch_spec<8>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 16) ok = launch_spec<16>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
            }
#endif
            if (n <= 65536 && ctx->prim_coop_slots == 4) {  // DPP folds + key/row granules
                if (in.d <= 4) ok = launch_coop4<4, false>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 8) ok = launch_coop4<8, false>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 16) ok = launch_coop4<16, false>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
            }
            if (n <= 65536 && ctx->prim_coop_slots == 5) {  // ... every candidate row in the sweep
                if (in.d <= 4) ok = launch_coop4<4, true>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 8) ok = launch_coop4<8, true>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 16) ok = launch_coop4<16, true>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
            }
            if (!ok && n <= 65536 && ctx->prim_coop_slots == 2) {  // data-tagged granules
                if (in.d <= 4) ok = launch_coop3<4>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 8) ok = launch_coop3<8>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                else if (in.d <= 16) ok = launch_coop3<16>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
            }
            if (!ok && n <= 65536 && ctx->prim_coop_slots) {  // step-tagged slots, the row in registers
                if (ctx->prim_coop_slots == 3) {  // write-through payload + drained tag, relaxed poll
                    if (in.d <= 4) ok = launch_coop2<4, true>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                    else if (in.d <= 8) ok = launch_coop2<8, true>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                    else if (in.d <= 16) ok = launch_coop2<16, true>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                } else {
                    if (in.d <= 4) ok = launch_coop2<4, false>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                    else if (in.d <= 8) ok = launch_coop2<8, false>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                    else if (in.d <= 16) ok = launch_coop2<16, false>(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
                }
            }
            if (!ok) ok = launch_coop(ctx, in, o, n, eoff[p], self_edges, va, vb, w);
            if (!ok) rest.push_back(p);
        }
        cls[4].swap(rest);
    }
    // stepwise state
    std::vector<int32_t> wg_part, wg_first(P, 0), wg_count(P, 0);
    constexpr int SBS = 256, SPPT = 4;
    for (int32_t p : cls[4]) {
        int64_t n = h_offs[p + 1] - h_offs[p];
        int c = (int)ceil_div(n, SBS * SPPT);
        wg_first[p] = (int)wg_part.size();
        wg_count[p] = c;
        for (int q = 0; q < c; q++) wg_part.push_back(p);
    }
    int nwg = (int)wg_part.size();
    size_t o_wgp = carve(sizeof(int32_t) * (nwg + 1)), o_wgf = carve(sizeof(int32_t) * (P + 1)),
           o_wgc = carve(sizeof(int32_t) * (P + 1));
    size_t o_best = 0, o_par = 0, o_att = 0, o_pv = 0, o_pi = 0;
    if (nwg) {
        o_best = carve(sizeof(double) * total_v);
        o_par = carve(sizeof(int32_t) * total_v);
        o_att = carve(total_v);
        o_pv = carve(sizeof(double) * 2 * nwg);
        o_pi = carve(sizeof(int32_t) * 2 * nwg);
    }
    char *base = (char *)arena(ctx, A_WORK1, off);
    int64_t *d_off = (int64_t *)(base + o_off), *d_eoff = (int64_t *)(base + o_eoff);
    int32_t *d_parts = (int32_t *)(base + o_parts);
    std::vector<int64_t> rel(P + 1);
    for (int p = 0; p <= P; p++) rel[p] = h_offs[p] - h_offs[0];
    HIP_CHECK(hipMemcpyAsync(d_off, rel.data(), sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(d_eoff, eoff.data(), sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, ctx->stream));
    std::vector<int32_t> plist;
    int cstart[5];
    for (int c = 0; c < 5; c++) {
        cstart[c] = (int)plist.size();
        plist.insert(plist.end(), cls[c].begin(), cls[c].end());
    }
    if (!plist.empty())
        HIP_CHECK(hipMemcpyAsync(d_parts, plist.data(), sizeof(int32_t) * plist.size(), hipMemcpyHostToDevice,
                                 ctx->stream));
    launch_block<64, 1>(ctx, in, d_off, d_eoff, d_parts + cstart[0], (int)cls[0].size(), self_edges, va, vb, w);
    launch_block<64, 4>(ctx, in, d_off, d_eoff, d_parts + cstart[1], (int)cls[1].size(), self_edges, va, vb, w);
    launch_block<256, 4>(ctx, in, d_off, d_eoff, d_parts + cstart[2], (int)cls[2].size(), self_edges, va, vb, w);
    launch_block<1024, 4>(ctx, in, d_off, d_eoff, d_parts + cstart[3], (int)cls[3].size(), self_edges, va, vb, w);
    if (nwg) {
        int32_t *d_wgp = (int32_t *)(base + o_wgp), *d_wgf = (int32_t *)(base + o_wgf),
                *d_wgc = (int32_t *)(base + o_wgc);
        HIP_CHECK(hipMemcpyAsync(d_wgp, wg_part.data(), sizeof(int32_t) * nwg, hipMemcpyHostToDevice, ctx->stream));
        HIP_CHECK(hipMemcpyAsync(d_wgf, wg_first.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, ctx->stream));
        HIP_CHECK(hipMemcpyAsync(d_wgc, wg_count.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, ctx->stream));
        StepState st;
        st.best = (double *)(base + o_best);
        st.par = (int32_t *)(base + o_par);
        st.att = (uint8_t *)(base + o_att);
        st.pv = (double *)(base + o_pv);
        st.pidx = (int32_t *)(base + o_pi);
        st.cur0 = nullptr;
        hipLaunchKernelGGL(prim_step_init_kernel, dim3(1024), dim3(256), 0, ctx->stream, d_off, P, st.best, st.par,
                           st.att, total_v);
        int64_t maxn = 0;
        for (int32_t p : cls[4]) maxn = std::max(maxn, h_offs[p + 1] - h_offs[p]);
        // steps 1..maxn-1 run on the context's side stream (capturable) in chunks captured
        // into a hipGraph and replayed; fenced to/from the caller's stream by events.
        const int CH = 256;
        hipStream_t ss = ctx->side;
        stream_fence(ctx, ctx->stream, ss);
        hipGraphExec_t exec = nullptr;
        KernelTimer t(ctx, "prim_step_total");
        int step = 1;
        auto launch_one = [&](int s) {
            hipLaunchKernelGGL((prim_step_kernel<SBS, SPPT>), dim3(nwg), dim3(SBS), 0, ss, in, d_off, d_wgp, d_wgf,
                               d_wgc, st, s, s & 1);
        };
        try {
            while (step < maxn) {
                int remain = (int)(maxn - step);
                if (remain < CH) {
                    for (int s = 0; s < remain; s++) launch_one(step + s);
                    HIP_CHECK(hipGetLastError());
                    step += remain;
                    continue;
                }
                hipGraph_t graph;
                HIP_CHECK(hipStreamBeginCapture(ss, hipStreamCaptureModeThreadLocal));
                for (int s = 0; s < CH; s++) launch_one(step + s);
                hipError_t ce = hipStreamEndCapture(ss, &graph);
                HIP_CHECK(ce);
                if (!exec) {
                    HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
                } else {
                    hipGraphExecUpdateResult res;
                    hipGraphNode_t errn;
                    if (hipGraphExecUpdate(exec, graph, &errn, &res) != hipSuccess) {
                        (void)hipGetLastError();
                        HIP_CHECK(hipGraphExecDestroy(exec));
                        HIP_CHECK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
                    }
                }
                HIP_CHECK(hipGraphLaunch(exec, ss));
                HIP_CHECK(hipGraphDestroy(graph));
                step += CH;
            }
        } catch (...) {
            hipGraph_t g = nullptr;
            hipStreamCaptureStatus cs;
            if (hipStreamIsCapturing(ss, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) {
                (void)hipStreamEndCapture(ss, &g);
                if (g) (void)hipGraphDestroy(g);
            }
            if (exec) (void)hipGraphExecDestroy(exec);
            throw;
        }
        stream_fence(ctx, ss, ctx->stream);
        if (exec) {
            HIP_CHECK(hipStreamSynchronize(ss));
            HIP_CHECK(hipGraphExecDestroy(exec));
        }
        // edges for stepwise partitions
        std::vector<int32_t> big(cls[4].begin(), cls[4].end());
        for (int32_t p : big) {
            // one block per partition via a shifted offsets view
            hipLaunchKernelGGL(prim_step_final_kernel, dim3(1), dim3(256), 0, ctx->stream, in, d_off + p, d_eoff + p, 1,
                               st, self_edges, va, vb, w);
        }
        HIP_CHECK(hipGetLastError());
    }
}

}  // namespace hdb
