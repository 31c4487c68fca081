// capi.cpp -- extern "C" entry points of libhdbmi (declared in include/hdbmi.h).
// Each entry: validate, select the device, stage host arrays (Stager), run the device
// building blocks on the context stream, copy host outputs back.
#include <algorithm>
#include <vector>

#include <chrono>

#include "internal.hpp"

using namespace hdb;

namespace {

template <class F>
int guarded(hdb_ctx *ctx, F &&f) {
    try {
        if (!ctx) HDB_THROW(HDB_EINVAL, "ctx is NULL");
        HIP_CHECK(hipSetDevice(ctx->device));
        f();
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return HDB_ENOMEM;
    }
}

template <class T>
std::vector<T> to_host(hdb_ctx *ctx, const T *p, size_t count) {
    std::vector<T> v(count);
    if (!count) return v;
    if (is_device_ptr(p)) {
        HIP_CHECK(hipMemcpyAsync(v.data(), p, sizeof(T) * count, hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
    } else {
        std::copy(p, p + count, v.begin());
    }
    return v;
}

void check_metric(int metric) {
    if (metric < HDB_METRIC_EUCLIDEAN || metric > HDB_METRIC_SUPREMUM) HDB_THROW(HDB_EINVAL, "unknown metric");
}

__global__ void iota_ids_kernel(int32_t *a, int64_t n) { HDB_GRID_STRIDE(i, n) a[i] = (int32_t)i; }

const int32_t *identity_ids(hdb_ctx *ctx, int64_t n) {
    int32_t *ids = (int32_t *)arena(ctx, A_STAGE_OUT, sizeof(int32_t) * std::max<int64_t>(n, 1));
    hipLaunchKernelGGL(iota_ids_kernel, dim3(1024), dim3(256), 0, ctx->stream, ids, n);
    HIP_CHECK(hipGetLastError());
    return ids;
}

}  // namespace

extern "C" {

int hdb_distance_rows(hdb_ctx *ctx, const double *a, const double *b, int64_t n, int32_t d, int32_t metric,
                      double *out) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (n < 0 || d <= 0 || !a || !b || !out) HDB_THROW(HDB_EINVAL, "bad arguments");
        Stager s(ctx);
        const double *da = s.in(a, n * d), *db = s.in(b, n * d);
        double *dout = s.out(out, n);
        distance_rows_device(ctx, da, db, n, d, metric, dout);
        s.finish();
    });
}

int hdb_core_distances(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t min_pts, int32_t metric,
                       int32_t semantics, double *core_out) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (n < 0 || d <= 0 || !X || !core_out || min_pts < 1) HDB_THROW(HDB_EINVAL, "bad arguments");
        if (semantics < 0 || semantics > 2) HDB_THROW(HDB_EINVAL, "unknown core semantics");
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        double *dc = s.out(core_out, n);
        core_distances_device(ctx, dX, n, d, min_pts, metric, semantics, dc);
        s.finish();
    });
}

int hdb_knn(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t k, int32_t metric, int32_t excl_self,
            double *dist_out, int32_t *idx_out) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (n < 0 || d <= 0 || k < 1 || !X || !dist_out) HDB_THROW(HDB_EINVAL, "bad arguments");
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        double *dv = s.out(dist_out, n * k);
        int32_t *di = s.out(idx_out, n * k);
        int KC = 0;
        // lists with the bucket width, then compact to k columns
        int kc_guess = k <= 1 ? 1 : (k <= 3 ? 3 : (k <= 7 ? 7 : (k <= 15 ? 15 : 31)));
        double *lv = (double *)arena(ctx, A_WORK0, sizeof(double) * std::max<int64_t>(n * kc_guess, 1));
        int32_t *li = di ? (int32_t *)arena(ctx, A_WORK1, sizeof(int32_t) * std::max<int64_t>(n * kc_guess, 1)) : nullptr;
        knn_lists_device(ctx, dX, n, d, k, metric, excl_self != 0, lv, li, &KC);
        if (n > 0) {
            HIP_CHECK(hipMemcpy2DAsync(dv, sizeof(double) * k, lv, sizeof(double) * KC, sizeof(double) * k, n,
                                       hipMemcpyDeviceToDevice, ctx->stream));
            if (di)
                HIP_CHECK(hipMemcpy2DAsync(di, sizeof(int32_t) * k, li, sizeof(int32_t) * KC, sizeof(int32_t) * k, n,
                                           hipMemcpyDeviceToDevice, ctx->stream));
        }
        s.finish();
    });
}

static void prim_common(hdb_ctx *ctx, const double *X, const int64_t *offsets, int32_t P, int32_t d,
                        const double *core, const int32_t *ids, const double *eB, const double *nnB, int32_t metric,
                        int32_t self_edges, int32_t *va, int32_t *vb, double *w) {
    check_metric(metric);
    if (P < 0 || d <= 0 || !X || !core || !va || !vb || !w) HDB_THROW(HDB_EINVAL, "bad arguments");
    std::vector<int64_t> offs = to_host(ctx, offsets, (size_t)P + 1);
    if (offs[0] != 0) HDB_THROW(HDB_EINVAL, "offsets[0] must be 0");
    int64_t n = offs[P];
    int64_t ne = 0;
    for (int p = 0; p < P; p++) {
        int64_t np_ = offs[p + 1] - offs[p];
        if (np_ < 0) HDB_THROW(HDB_EINVAL, "offsets must be non-decreasing");
        if (np_ > INT32_MAX) HDB_THROW(HDB_EINVAL, "partition too large");
        if (np_ > 0) ne += (np_ - 1) + (self_edges ? np_ : 0);
    }
    Stager s(ctx);
    PrimIn in;
    in.X = s.in(X, n * d);
    in.core = s.in(core, n);
    in.ids = ids ? s.in(ids, n) : nullptr;
    in.eB = eB ? s.in(eB, n) : nullptr;
    in.nnB = nnB ? s.in(nnB, n) : nullptr;
    in.d = d;
    in.metric = metric;
    int32_t *dva = s.out(va, ne), *dvb = s.out(vb, ne);
    double *dw = s.out(w, ne);
    if (!in.ids) {
        // identity per partition: local index within each partition
        std::vector<int32_t> h(n);
        for (int p = 0; p < P; p++)
            for (int64_t i = offs[p]; i < offs[p + 1]; i++) h[i] = (int32_t)(i - offs[p]);
        int32_t *dids = (int32_t *)arena(ctx, A_STAGE_OUT, sizeof(int32_t) * std::max<int64_t>(n, 1));
        HIP_CHECK(hipMemcpyAsync(dids, h.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        in.ids = dids;
    }
    prim_batched_device(ctx, in, offs.data(), P, self_edges, dva, dvb, dw);
    s.finish();
}

int hdb_prim_mst(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const double *core, const int32_t *ids,
                 int32_t metric, int32_t self_edges, int32_t *va, int32_t *vb, double *w) {
    return guarded(ctx, [&] {
        if (n < 1) HDB_THROW(HDB_EINVAL, "n must be >= 1 (new int[n-1])");
        int64_t offs[2] = {0, n};
        prim_common(ctx, X, offs, 1, d, core, ids, nullptr, nullptr, metric, self_edges, va, vb, w);
    });
}

int hdb_prim_mst_batched(hdb_ctx *ctx, const double *X, const int64_t *offsets, int32_t P, int32_t d,
                         const double *core, const int32_t *ids, int32_t metric, int32_t self_edges, int32_t *va,
                         int32_t *vb, double *w) {
    return guarded(ctx, [&] {
        if (!offsets) HDB_THROW(HDB_EINVAL, "offsets is NULL");
        prim_common(ctx, X, offsets, P, d, core, ids, nullptr, nullptr, metric, self_edges, va, vb, w);
    });
}

int hdb_leaf_msts(hdb_ctx *ctx, const double *X, const int64_t *offsets, int32_t P, int32_t d, const int32_t *ids,
                  int32_t min_pts, int32_t metric, double *core_out, int32_t *va, int32_t *vb, double *w) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (!X || !offsets || !ids || !va || !vb || !w || P < 0 || d <= 0 || min_pts < 1)
            HDB_THROW(HDB_EINVAL, "bad arguments");
        std::vector<int64_t> offs = to_host(ctx, offsets, (size_t)P + 1);
        if (offs[0] != 0) HDB_THROW(HDB_EINVAL, "offsets[0] must be 0");
        const int64_t n = offs[P];
        int64_t ne = 0;
        std::vector<int32_t> small;
        std::vector<int32_t> large;
        for (int p = 0; p < P; p++) {
            int64_t np_ = offs[p + 1] - offs[p];
            if (np_ < 0) HDB_THROW(HDB_EINVAL, "offsets must be non-decreasing");
            if (np_ > 0) ne += 2 * np_ - 1;
            if (np_ > 0 && np_ <= 4096) small.push_back(p);
            else if (np_ > 4096) large.push_back(p);
        }
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        const int32_t *dids = s.in(ids, n);
        int32_t *dva = s.out(va, ne), *dvb = s.out(vb, ne);
        double *dw = s.out(w, ne);
        double *dcore = core_out ? s.out(core_out, n)
                                 : (double *)arena(ctx, A_STAGE_OUT, sizeof(double) * std::max<int64_t>(n, 1));
        if (min_pts == 1) {
            HIP_CHECK(hipMemsetAsync(dcore, 0, sizeof(double) * std::max<int64_t>(n, 0), ctx->stream));
        } else {
            // offsets + small list on device
            int64_t *d_off = (int64_t *)arena(ctx, A_STAGE_IN, sizeof(int64_t) * (P + 1) + sizeof(int32_t) * (P + 1) + 256);
            int32_t *d_parts = (int32_t *)((char *)d_off + ((sizeof(int64_t) * (P + 1) + 255) & ~size_t(255)));
            HIP_CHECK(hipMemcpyAsync(d_off, offs.data(), sizeof(int64_t) * (P + 1), hipMemcpyHostToDevice, ctx->stream));
            if (!small.empty())
                HIP_CHECK(hipMemcpyAsync(d_parts, small.data(), sizeof(int32_t) * small.size(), hipMemcpyHostToDevice,
                                         ctx->stream));
            leaf_cores_device(ctx, dX, d, metric, P, d_off, d_parts, (int)small.size(), n, min_pts - 1, dcore);
            HIP_CHECK(hipStreamSynchronize(ctx->stream));  // d_off/d_parts live in a reused arena
            for (int32_t p : large)
                core_distances_device(ctx, dX + offs[p] * d, offs[p + 1] - offs[p], d, min_pts, metric,
                                      HDB_CORE_INCL_SELF_CUMULATIVE, dcore + offs[p]);
        }
        PrimIn in;
        in.X = dX;
        in.core = dcore;
        in.ids = dids;
        in.eB = in.nnB = nullptr;
        in.d = d;
        in.metric = metric;
        prim_batched_device(ctx, in, offs.data(), P, 1, dva, dvb, dw);
        s.finish();
    });
}

int hdb_mst_boruvka(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const double *core, int32_t metric,
                    int32_t self_edges, int32_t *va, int32_t *vb, double *w) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (n < 1 || d <= 0 || !X || !core || !va || !vb || !w) HDB_THROW(HDB_EINVAL, "bad arguments");
        int64_t ne = (n - 1) + (self_edges ? n : 0);
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        const double *dc = s.in(core, n);
        int32_t *dva = s.out(va, ne), *dvb = s.out(vb, ne);
        double *dw = s.out(w, ne);
        boruvka_device(ctx, dX, n, d, dc, metric, dva, dvb, dw);
        if (self_edges) self_edges_device(ctx, dc, n, dva + (n - 1), dvb + (n - 1), dw + (n - 1));
        s.finish();
    });
}

int hdb_exact_mst(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t min_pts, int32_t metric,
                  int32_t semantics, int32_t self_edges, double *core_out, int32_t *va, int32_t *vb, double *w) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (n < 1 || d <= 0 || !X || !va || !vb || !w) HDB_THROW(HDB_EINVAL, "bad arguments");
        if (semantics < 0 || semantics > 2) HDB_THROW(HDB_EINVAL, "unknown core semantics");
        if (self_edges & ~(HDB_EDGES_SELF | HDB_EDGES_MERGED)) HDB_THROW(HDB_EINVAL, "unknown edge flags");
        const int64_t ne = (n - 1) + ((self_edges & HDB_EDGES_SELF) ? n : 0);
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        double *dc = core_out ? s.out(core_out, n) : (double *)arena(ctx, A_STAGE_OUT, sizeof(double) * (size_t)n);
        int32_t *dva = s.out(va, ne), *dvb = s.out(vb, ne);
        double *dw = s.out(w, ne);
        exact_leaf_device(ctx, dX, n, d, min_pts, metric, semantics, dc, self_edges, dva, dvb, dw);
        s.finish();
    });
}

int hdb_nearest_sample(hdb_ctx *ctx, const double *X, int64_t n, const double *S, int64_t m, int32_t d,
                       int32_t metric, const int32_t *x_key, const int32_t *s_key, int32_t *nearest_out,
                       double *dist_out) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (n < 0 || m < 0 || d <= 0 || !X || (!S && m > 0) || !nearest_out) HDB_THROW(HDB_EINVAL, "bad arguments");
        if ((x_key == nullptr) != (s_key == nullptr)) HDB_THROW(HDB_EINVAL, "x_key and s_key go together");
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        const double *dS = m ? s.in(S, m * d) : nullptr;
        const int32_t *dxk = s.in(x_key, n), *dsk = s.in(s_key, m);
        int32_t *dn = s.out(nearest_out, n);
        double *dd = s.out(dist_out, n);
        nearest_sample_device(ctx, dX, n, dS, m, d, metric, dxk, dsk, dn, dd);
        s.finish();
    });
}

int hdb_bubble_stats(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const int32_t *bubble_of, int64_t nb,
                     int32_t variant, double *ls, double *ss, double *rep, double *info) {
    return guarded(ctx, [&] {
        if (n < 0 || nb < 0 || d <= 0 || (!X && n) || (!bubble_of && n) || !ls || !ss || !rep || !info)
            HDB_THROW(HDB_EINVAL, "bad arguments");
        if (variant != HDB_BUBBLE_COMBINESTEP && variant != HDB_BUBBLE_CF) HDB_THROW(HDB_EINVAL, "unknown variant");
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        const int32_t *dbo = s.in(bubble_of, n);
        double *dls = s.out(ls, nb * d), *dss = s.out(ss, nb * d), *drep = s.out(rep, nb * d), *dinfo = s.out(info, nb * 3);
        bubble_stats_device(ctx, dX, n, d, dbo, nb, variant, dls, dss, drep, dinfo);
        s.finish();
    });
}

int hdb_bubble_partials(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const int32_t *bubble_of, int64_t nb,
                        const int64_t *cuts, int32_t S, double *part_ls, double *part_ss, double *part_n) {
    return guarded(ctx, [&] {
        if (n < 0 || nb < 0 || d <= 0 || (!X && n) || (!bubble_of && n) || !cuts || !part_ls || !part_ss || !part_n)
            HDB_THROW(HDB_EINVAL, "bad arguments");
        if (S < 1 || S > HDB_MAX_BUBBLE_SLICES) HDB_THROW(HDB_EINVAL, "bubble slices: 1..HDB_MAX_BUBBLE_SLICES");
        std::vector<int64_t> h_cuts = to_host(ctx, cuts, (size_t)S + 1);
        Stager s(ctx);
        const double *dX = s.in(X, n * d);
        const int32_t *dbo = s.in(bubble_of, n);
        double *pl = s.out(part_ls, (int64_t)S * nb * d), *pq = s.out(part_ss, (int64_t)S * nb * d),
               *pn = s.out(part_n, (int64_t)S * nb);
        bubble_partials_device(ctx, dX, n, d, dbo, nb, h_cuts.data(), S, pl, pq, pn);
        s.finish();
    });
}

int hdb_bubble_combine(hdb_ctx *ctx, const double *part_ls, const double *part_ss, const double *part_n, int32_t S,
                       int64_t nb, int32_t d, double *ls, double *ss, double *rep, double *info) {
    return guarded(ctx, [&] {
        if (nb < 0 || d <= 0 || S < 1 || !part_ls || !part_ss || !part_n || !ls || !ss || !rep || !info)
            HDB_THROW(HDB_EINVAL, "bad arguments");
        Stager s(ctx);
        const double *pl = s.in(part_ls, (int64_t)S * nb * d), *pq = s.in(part_ss, (int64_t)S * nb * d),
                     *pn = s.in(part_n, (int64_t)S * nb);
        double *dls = s.out(ls, nb * d), *dss = s.out(ss, nb * d), *drep = s.out(rep, nb * d), *dinfo = s.out(info, nb * 3);
        bubble_combine_device(ctx, pl, pq, pn, S, nb, d, dls, dss, drep, dinfo);
        s.finish();
    });
}

static void bubble_core_impl(hdb_ctx *ctx, const double *rep, const int32_t *nB, const double *eB, const double *nnB,
                             int64_t b, int32_t d, int32_t min_pts, int32_t metric, std::vector<double> &core_h) {
    const int K = min_pts - 1;
    core_h.assign(b, 0.0);
    if (min_pts == 1 || b == 0) return;
    Stager s(ctx);
    const double *drep = s.in(rep, b * d), *deB = s.in(eB, b), *dnnB = s.in(nnB, b);
    double *knn = (double *)arena(ctx, A_WORK0, sizeof(double) * b * K);
    int32_t *lg = (int32_t *)arena(ctx, A_WORK1, sizeof(int32_t) * b * K);
    bubble_knn_device(ctx, drep, deB, dnnB, b, d, metric, K, knn, lg);
    std::vector<double> knn_h = to_host(ctx, (const double *)knn, (size_t)(b * K));
    std::vector<int32_t> lg_h = to_host(ctx, (const int32_t *)lg, (size_t)(b * K));
    std::vector<double> rep_h = to_host(ctx, rep, (size_t)(b * d)), eB_h = to_host(ctx, eB, (size_t)b),
                        nnB_h = to_host(ctx, nnB, (size_t)b);
    std::vector<int32_t> nB_h = to_host(ctx, nB, (size_t)b);
    int rc = bubble_core_epilogue(rep_h.data(), nB_h.data(), eB_h.data(), nnB_h.data(), b, d, min_pts, metric,
                                  knn_h.data(), lg_h.data(), core_h.data());
    if (rc) HDB_THROW(rc, "calculateCoreDistancesBubbles raised a reference exception");
    s.finish();
}

int hdb_bubble_core_distances(hdb_ctx *ctx, const double *rep, const int32_t *nB, const double *eB,
                              const double *nnB, int64_t b, int32_t d, int32_t min_pts, int32_t metric,
                              double *core_out) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (b < 0 || d <= 0 || min_pts < 1 || !rep || !nB || !eB || !nnB || !core_out)
            HDB_THROW(HDB_EINVAL, "bad arguments");
        if (min_pts > 32) HDB_THROW(HDB_EINVAL, "minPts too large (max 32)");
        std::vector<double> core_h;
        bubble_core_impl(ctx, rep, nB, eB, nnB, b, d, min_pts, metric, core_h);
        if (is_device_ptr(core_out)) {
            HIP_CHECK(hipMemcpyAsync(core_out, core_h.data(), sizeof(double) * b, hipMemcpyHostToDevice, ctx->stream));
            HIP_CHECK(hipStreamSynchronize(ctx->stream));
        } else {
            std::copy(core_h.begin(), core_h.end(), core_out);
        }
    });
}

int hdb_bubble_prim_mst(hdb_ctx *ctx, const double *rep, const double *eB, const double *nnB,
                        const int32_t *id_bubbles, const double *core, int64_t b, int32_t d, int32_t metric,
                        int32_t self_edges, int32_t *va, int32_t *vb, double *w) {
    return guarded(ctx, [&] {
        if (b < 1) HDB_THROW(HDB_EINVAL, "b must be >= 1");
        if (!eB || !nnB) HDB_THROW(HDB_EINVAL, "eB/nnB required");
        int64_t offs[2] = {0, b};
        prim_common(ctx, rep, offs, 1, d, core, id_bubbles, eB, nnB, metric, self_edges, va, vb, w);
    });
}

int hdb_quicksort_edges(int32_t *va, int32_t *vb, double *w, int64_t ne) {
    if (!va || !vb || !w || ne < 0) return HDB_EINVAL;
    int rc = quicksort_edges(va, vb, w, ne);
    if (rc) set_error("quicksortByEdgeWeight: stack overflow (ArrayIndexOutOfBoundsException)");
    return rc;
}

// core_in (nullable, host, b values): the bubble core distances already computed by
// hdb_bubble_core_distances on the same (rep, nB, eB, nnB) -- the model then starts at the Prim
static int local_model_impl(hdb_ctx *ctx, const double *rep, const double *info, int64_t b, int32_t d,
                            int32_t min_pts, int32_t min_cl_size, int32_t metric, const double *core_in,
                            int32_t *labels, int32_t *mst_va, int32_t *mst_vb, double *mst_w, int32_t *ic_va,
                            int32_t *ic_vb, double *ic_w, int64_t *n_ic) {
    return guarded(ctx, [&] {
        check_metric(metric);
        if (b < 1 || d <= 0 || !rep || !info || !labels || min_pts < 1) HDB_THROW(HDB_EINVAL, "bad arguments");
        if (min_pts > 32) HDB_THROW(HDB_EINVAL, "minPts too large (max 32)");
        std::vector<double> rep_h = to_host(ctx, rep, (size_t)(b * d));
        std::vector<double> info_h = to_host(ctx, info, (size_t)(b * 3));
        std::vector<double> eB(b), nnB(b);
        std::vector<int32_t> nB(b), ids(b);
        for (int64_t i = 0; i < b; i++) {  // LocalModelReduceByKey.java:80-84
            eB[i] = info_h[i * 3 + 0];
            nnB[i] = info_h[i * 3 + 1];
            nB[i] = (int32_t)info_h[i * 3 + 2];
            ids[i] = (int32_t)i;  // D4: vertex id == position
        }
        using clk = std::chrono::steady_clock;
        auto us = [](clk::time_point a, clk::time_point b) {
            return (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
        };
        auto t0 = clk::now();
        std::vector<double> core;
        if (core_in)
            core.assign(core_in, core_in + b);
        else
            bubble_core_impl(ctx, rep_h.data(), nB.data(), eB.data(), nnB.data(), b, d, min_pts, metric, core);
        auto t1 = clk::now();
        const int64_t ne = 2 * b - 1;
        std::vector<int32_t> mva(ne), mvb(ne);
        std::vector<double> mw(ne);
        {
            int64_t offs[2] = {0, b};
            prim_common(ctx, rep_h.data(), offs, 1, d, core.data(), ids.data(), eB.data(), nnB.data(), metric, 1,
                        mva.data(), mvb.data(), mw.data());
        }
        auto t2 = clk::now();
        for (auto &v : g_lm_us) v = 0;
        std::vector<int32_t> lab(b);
        std::vector<int32_t> iva(ne), ivb(ne);
        std::vector<double> iw(ne);
        int64_t nic = 0;
        int rc = local_model_host(rep_h.data(), eB.data(), nnB.data(), nB.data(), b, d, min_cl_size, metric, mva.data(),
                                  mvb.data(), mw.data(), lab.data(), iva.data(), ivb.data(), iw.data(), &nic);
        ctx->stats["lm_core_us"] += us(t0, t1);
        ctx->stats["lm_prim_us"] += us(t1, t2);
        ctx->stats["lm_quicksort_us"] += g_lm_us[0];
        ctx->stats["lm_tree_us"] += g_lm_us[1];
        ctx->stats["lm_fosc_us"] += g_lm_us[2];
        ctx->stats["lm_fosc_select_us"] += g_lm_us[3];
        ctx->stats["lm_fosc_label_us"] += g_lm_us[4];
        ctx->stats["lm_fosc_noise_us"] += g_lm_us[5];
        ctx->stats["lm_calls"] += 1;
        if (rc == HDB_EREF_NEGATIVE_CLUSTER) HDB_THROW(rc, local_model_error_detail());
        if (rc) HDB_THROW(rc, "local model raised a reference exception");
        std::copy(lab.begin(), lab.end(), labels);
        if (mst_va) std::copy(mva.begin(), mva.end(), mst_va);
        if (mst_vb) std::copy(mvb.begin(), mvb.end(), mst_vb);
        if (mst_w) std::copy(mw.begin(), mw.end(), mst_w);
        if (ic_va) std::copy(iva.begin(), iva.begin() + nic, ic_va);
        if (ic_vb) std::copy(ivb.begin(), ivb.begin() + nic, ic_vb);
        if (ic_w) std::copy(iw.begin(), iw.begin() + nic, ic_w);
        if (n_ic) *n_ic = nic;
    });
}

int hdb_local_model(hdb_ctx *ctx, const double *rep, const double *info, int64_t b, int32_t d, int32_t min_pts,
                    int32_t min_cl_size, int32_t metric, int32_t *labels, int32_t *mst_va, int32_t *mst_vb,
                    double *mst_w, int32_t *ic_va, int32_t *ic_vb, double *ic_w, int64_t *n_ic) {
    return local_model_impl(ctx, rep, info, b, d, min_pts, min_cl_size, metric, nullptr, labels, mst_va, mst_vb,
                            mst_w, ic_va, ic_vb, ic_w, n_ic);
}

int hdb_local_model_cores(hdb_ctx *ctx, const double *rep, const double *info, int64_t b, int32_t d,
                          int32_t min_pts, int32_t min_cl_size, int32_t metric, const double *core, int32_t *labels,
                          int32_t *mst_va, int32_t *mst_vb, double *mst_w, int32_t *ic_va, int32_t *ic_vb,
                          double *ic_w, int64_t *n_ic) {
    if (!core) {
        set_error("hdb_local_model_cores: core is required");
        return HDB_EINVAL;
    }
    return local_model_impl(ctx, rep, info, b, d, min_pts, min_cl_size, metric, core, labels, mst_va, mst_vb, mst_w,
                            ic_va, ic_vb, ic_w, n_ic);
}

int hdb_sort_edges_desc(hdb_ctx *ctx, int32_t *va, int32_t *vb, double *w, int64_t ne) {
    return guarded(ctx, [&] {
        if (ne < 0 || (ne > 0 && (!va || !vb || !w))) HDB_THROW(HDB_EINVAL, "bad arguments");
        Stager s(ctx);
        int32_t *dva = s.inout(va, ne), *dvb = s.inout(vb, ne);
        double *dw = s.inout(w, ne);
        sort_edges_desc_device(ctx, dva, dvb, dw, ne);
        s.finish();
    });
}

int hdb_merge_sorted_runs(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w, const int64_t *run_off,
                          int32_t nruns, int32_t *oa, int32_t *ob, double *ow) {
    return guarded(ctx, [&] {
        if (nruns < 0 || (nruns > 0 && !run_off)) HDB_THROW(HDB_EINVAL, "bad arguments");
        std::vector<int64_t> off(run_off, run_off + nruns + 1);
        if (nruns == 0) off.assign(1, 0);
        for (int r = 0; r < nruns; r++)
            if (off[r + 1] < off[r] || off[0] != 0) HDB_THROW(HDB_EINVAL, "merge_sorted_runs: bad run offsets");
        const int64_t ne = off.back();
        if (ne > INT32_MAX) HDB_THROW(HDB_EINVAL, "too many edges");
        if (ne > 0 && (!va || !vb || !w || !oa || !ob || !ow)) HDB_THROW(HDB_EINVAL, "bad arguments");
        Stager s(ctx);
        const int32_t *da = s.in(va, ne), *db = s.in(vb, ne);
        const double *dw = s.in(w, ne);
        int32_t *xa = s.out(oa, ne), *xb = s.out(ob, ne);
        double *xw = s.out(ow, ne);
        merge_sorted_runs_device(ctx, da, db, dw, off, xa, xb, xw);
        s.finish();
    });
}

int hdb_local_mst_ids(hdb_ctx *ctx, const int32_t *ids, int64_t n, const int32_t *va, const int32_t *vb,
                      const double *w, int64_t ne, int32_t node, int32_t *fake1, int32_t *fake2, int32_t *node_out) {
    return guarded(ctx, [&] {
        if (n < 0 || ne < 0 || (ne > 0 && (!va || !vb || !fake1 || !fake2))) HDB_THROW(HDB_EINVAL, "bad arguments");
        Stager sg(ctx);
        const int32_t *di = sg.in(ids, (size_t)n);
        const int32_t *da = sg.in(va, (size_t)ne), *db = sg.in(vb, (size_t)ne);
        const double *dw = sg.in(w, (size_t)ne);
        int32_t *f1 = sg.out(fake1, (size_t)ne), *f2 = sg.out(fake2, (size_t)ne), *nd = sg.out(node_out, (size_t)ne);
        local_mst_ids_device(ctx, di, n, da, db, dw, ne, node, f1, f2, nd);
        sg.finish();
    });
}

int hdb_flat_labels(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w, int64_t ne, int64_t n,
                    int32_t min_cl_size, int32_t *labels, int64_t *n_clusters) {
    if (!ctx) {  // host-only use (all pointers in host memory): no device needed
        try {
            if (ne < 0 || n < 0 || (ne > 0 && (!va || !vb || !w)) || (n > 0 && !labels))
                HDB_THROW(HDB_EINVAL, "bad arguments");
            return flat_labels_host(va, vb, w, ne, n, min_cl_size, labels, n_clusters);
        } catch (const Error &e) {
            set_error(e.msg);
            return e.code;
        } catch (const std::bad_alloc &) {
            set_error("host allocation failed");
            return HDB_ENOMEM;
        }
    }
    return guarded(ctx, [&] {
        if (ne < 0 || n < 0 || (ne > 0 && (!va || !vb || !w)) || (n > 0 && !labels)) HDB_THROW(HDB_EINVAL, "bad arguments");
        // device algorithm (K6, flat.hip); host arrays are staged
        Stager sg(ctx);
        const int32_t *da = sg.in(va, (size_t)ne), *db = sg.in(vb, (size_t)ne);
        const double *dw = sg.in(w, (size_t)ne);
        int32_t *dl = sg.out(labels, (size_t)std::max<int64_t>(n, 0));
        flat_labels_device(ctx, da, db, dw, ne, n, min_cl_size, dl, n_clusters);
        sg.finish();
    });
}

}  // extern "C"
