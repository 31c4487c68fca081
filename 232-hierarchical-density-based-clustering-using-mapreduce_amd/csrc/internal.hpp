// internal.hpp -- device-side building blocks shared by the C-ABI layer.
#pragma once
#include "common.hpp"

namespace hdb {

struct PrimIn {
    const double *X;
    const double *core;
    const int32_t *ids;
    const double *eB;
    const double *nnB;
    int d;
    int metric;
};

void pack_rows(hdb_ctx *ctx, const double *X, int64_t n, int d, int dp, double *Xp);
void knn_lists_device(hdb_ctx *ctx, const double *X_dev, int64_t n, int d, int k, int metric, bool excl,
                      double *lists_v, int32_t *lists_i, int *KC_out);
void core_epilogue_device(hdb_ctx *ctx, const double *lists, int64_t n, int KC, int K, int semantics, double *core);
// list bucket for k neighbours (K1/K1t keep KC >= k values per row)
inline int pick_kc(int k) {
    if (k <= 1) return 1;
    if (k <= 3) return 3;
    if (k <= 7) return 7;
    if (k <= 15) return 15;
    if (k <= 31) return 31;
    return -1;
}
void core_distances_device(hdb_ctx *ctx, const double *X_dev, int64_t n, int d, int min_pts, int metric,
                           int semantics, double *core);
void prim_batched_device(hdb_ctx *ctx, const PrimIn &in, const int64_t *h_offs, int P, int self_edges, int32_t *va,
                         int32_t *vb, double *w);
void leaf_cores_device(hdb_ctx *ctx, const double *X, int d, int metric, int P, const int64_t *d_off,
                       const int32_t *d_parts, int np, int64_t total_rows, int K, double *core);
void nearest_sample_device(hdb_ctx *ctx, const double *X, int64_t n, const double *S, int64_t m, int d, int metric,
                           const int32_t *xkey, const int32_t *skey, int32_t *out_i, double *out_d);
void bubble_stats_device(hdb_ctx *ctx, const double *X, int64_t n, int d, const int32_t *bo, int64_t nb, int variant,
                         double *ls, double *ss, double *rep, double *info);
void bubble_partials_device(hdb_ctx *ctx, const double *X, int64_t n, int d, const int32_t *bo, int64_t nb,
                            const int64_t *h_cuts, int S, double *pls, double *pss, double *pn);
void bubble_combine_device(hdb_ctx *ctx, const double *pls, const double *pss, const double *pn, int S, int64_t nb,
                           int d, double *ls, double *ss, double *rep, double *info);
void bubble_knn_device(hdb_ctx *ctx, const double *rep, const double *eB, const double *nnB, int64_t b, int d,
                       int metric, int K, double *knn_out, int32_t *log_out);
void sort_edges_desc_device(hdb_ctx *ctx, int32_t *va, int32_t *vb, double *w, int64_t ne);
// stable merge of two descending runs held in separate arrays (A first on equal weights)
void merge_two_runs_device(hdb_ctx *ctx, const int32_t *aA, const int32_t *bA, const double *wA, int64_t na,
                           const int32_t *aB, const int32_t *bB, const double *wB, int64_t nb, int32_t *oa,
                           int32_t *ob, double *ow);
// CreateLocalMST record fields: local indices of each edge's vertices in `ids` (synchronises)
void merge_sorted_runs_device(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w,
                              const std::vector<int64_t> &off, int32_t *oa, int32_t *ob, double *ow);
void local_mst_ids_device(hdb_ctx *ctx, const int32_t *ids, int64_t n, const int32_t *va, const int32_t *vb,
                          const double *w, int64_t ne,
                          int32_t node, int32_t *fake1, int32_t *fake2, int32_t *node_out);
void distance_rows_device(hdb_ctx *ctx, const double *a, const double *b, int64_t n, int d, int metric, double *out);
bool knn_tree_device(hdb_ctx *ctx, const double *X, int64_t n, int d, int KC, bool excl, double *lists);
// K1m: MFMA-screened exact lists for 16 < d <= 256 (false: not applicable, use the FP64 scan)
bool knn_mfma_device(hdb_ctx *ctx, const double *X, int64_t n, int d, int KC, bool excl, double *lists);
// self edges (v, v, core[v]) as FirstStep emits them after the tree edges (HDBSCANStar.java:190-203)
void self_edges_device(hdb_ctx *ctx, const double *core, int64_t n, int32_t *va, int32_t *vb, double *w);
void exact_leaf_device(hdb_ctx *ctx, const double *X, int64_t n, int d, int min_pts, int metric, int semantics,
                       double *core, int self_edges, int32_t *va, int32_t *vb, double *w);
void boruvka_device(hdb_ctx *ctx, const double *X, int64_t n, int d, const double *core, int metric, int32_t *va,
                    int32_t *vb, double *w);

// K6 rank-order vertex labels: contracted labels reach nv + rank < 3m, stored as int32
inline bool flat_relabel_fits(int64_t m) { return m >= 0 && 3 * m < (int64_t)INT32_MAX; }
// K6: global hierarchy + flat labels over a merged MST (flat.hip); synchronises
void flat_labels_device(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w, int64_t ne, int64_t n,
                        int32_t mcs, int32_t *labels, int64_t *n_clusters);

// host logic (local_model.cpp)
int bubble_core_epilogue(const double *rep, const int32_t *nB, const double *eB, const double *nnB, int64_t b, int d,
                         int min_pts, int metric, const double *knn, const int32_t *log, double *core);
int flat_labels_host(const int32_t *va, const int32_t *vb, const double *w, int64_t ne, int64_t n, int32_t mcs,
                     int32_t *labels, int64_t *n_clusters);
int quicksort_edges(int32_t *va, int32_t *vb, double *w, int64_t ne);
// message of the last HDB_EREF_NEGATIVE_CLUSTER on this thread (cluster label, level, numPoints)
const char *local_model_error_detail();
// host phase times of local_model_host (us): quicksort, cluster tree, FOSC + noise
extern thread_local int64_t g_lm_us[6];  // + FOSC parts: selection walk, labelling, noise
int local_model_host(const double *rep, const double *eB, const double *nnB, const int32_t *nB, int64_t b, int d,
                     int32_t min_cl_size, int metric, int32_t *mva, int32_t *mvb, double *mw, int32_t *labels,
                     int32_t *ic_va, int32_t *ic_vb, double *ic_w, int64_t *n_ic);

}  // namespace hdb
