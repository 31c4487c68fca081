/*
 * hdbmi.h -- C-ABI of the MI355X-native MR-HDBSCAN* hot path.
 *
 * The reference (SZU-AdvTech-2022/232, Java 8 + Spark 2.x) keeps its driver and operator
 * surface; each entry point below is the body a JNI shim substitutes for the Java method
 * cited next to it (see INTEGRATION.md for the binding).  Plain C types only.
 *
 * Memory: every array argument may be HOST memory or DEVICE memory of the context's
 * device (detected per pointer).  Host inputs are staged to HBM on the context stream and
 * host outputs copied back before the call returns (PCIe-inclusive).  When every pointer
 * is device memory the call is stream-ordered on the context stream and returns without
 * synchronising (except where noted).  The caller allocates every output; the library
 * never retains a caller pointer after return.
 *
 * Errors: int status, 0 = OK, < 0 = error; hdb_last_error() returns a thread-local message.
 * The HDB_EREF_* codes reproduce the reference's own exceptions (a JNI shim maps them to
 * the corresponding Java RuntimeException).
 *
 * Threading: re-entrant; use one hdb_ctx per calling thread.
 */
#ifndef HDBMI_H
#define HDBMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDB_OK 0
#define HDB_EINVAL (-1)
#define HDB_EDEVICE (-2)
#define HDB_ENOMEM (-3)
#define HDB_EREF_NPE (-10)              /* java.lang.NullPointerException                    */
#define HDB_EREF_OOB (-11)              /* java.lang.ArrayIndexOutOfBoundsException          */
#define HDB_EREF_NEGATIVE_CLUSTER (-12) /* Clusters.java:45-46 "Cluster cannot have less than 0 points." */
#define HDB_EREF_DIVZERO (-13)          /* java.lang.ArithmeticException: / by zero          */
#define HDB_EREF_NUMBER_FORMAT (-14)    /* java.lang.NumberFormatException                   */
#define HDB_EUNSUPPORTED (-20)          /* a reference behaviour not emulated: a treeified
                                           java.util.HashMap bin (iteration order) or a loop the
                                           reference never leaves (NaN edge weight)            */

/* DistanceCalculator.getName() (distance/DistanceCalculator.java:20) */
#define HDB_METRIC_EUCLIDEAN 0 /* EuclideanDistance.java:28-36  */
#define HDB_METRIC_COSINE 1    /* CosineSimilarity.java:28-40   */
#define HDB_METRIC_PEARSON 2   /* PearsonCorrelation.java:28-51 */
#define HDB_METRIC_MANHATTAN 3 /* ManhattanDistance.java:28-36  */
#define HDB_METRIC_SUPREMUM 4  /* SupremumDistance.java:28-38   */

/* Core-distance semantics present in the reference */
#define HDB_CORE_INCL_SELF_CUMULATIVE 0 /* HDBSCANStar.java:71-106 (live; buffer never reset) */
#define HDB_CORE_INCL_SELF 1            /* CoreDistanceMapper.java:71-109                      */
#define HDB_CORE_EXCL_SELF 2            /* CreateLocalMST.java:138-185 (standard HDBSCAN*)     */

/* Bubble-statistics variants */
#define HDB_BUBBLE_COMBINESTEP 0 /* mappers/CombineStep.java:18-64 (live)            */
#define HDB_BUBBLE_CF 1          /* datastructure/ClusterFeatureDataBubbles.java:192-215 */
#define HDB_MAX_BUBBLE_SLICES 64 /* hdb_bubble_partials: slices per call                  */

typedef struct hdb_ctx hdb_ctx;

/* ------------------------------------------------------------------ context */
int hdb_ctx_create(int device, hdb_ctx **out);
void hdb_ctx_destroy(hdb_ctx *ctx);
/* Run on a caller-owned hipStream_t (e.g. torch's current stream); NULL = the device's default
 * (null) stream.  A fresh context owns a private non-blocking stream until this is called. */
int hdb_ctx_set_stream(hdb_ctx *ctx, void *hip_stream);
/* Per-kernel HIP-event timing (off by default). */
int hdb_ctx_set_timing(hdb_ctx *ctx, int enable);
/* Synchronises, returns the summed device time (ms) and launch count of kernel `name`
 * since the last reset, then resets that accumulator when reset != 0. */
int hdb_ctx_kernel_time(hdb_ctx *ctx, const char *name, double *ms_total, int64_t *launches, int reset);
int hdb_ctx_synchronize(hdb_ctx *ctx);
/* Tuning/diagnostic switches (results are identical under every setting):
 *   "knn_fp32_screen" (default 1): K1 screens pairs in FP32 with a rigorous bound before the
 *                                  exact FP64 test;
 *   "knn_tree"        (default 1): euclidean k-NN lists of partitions with n >= "knn_tree_min_n"
 *                                  (default 8192) and d in {1,2,3,4,8,16} use K1t, the
 *                                  box-pruned traversal of the Morton/BVH index, instead of
 *                                  the all-pairs K1;
 *   "knn_mfma"        (default 1): euclidean lists with 16 < d <= 256 and n >= "knn_mfma_min_n"
 *                                  (default 2048) use K1m (bf16-split MFMA screen, FP64 re-check);
 *                                  "knn_mfma_single" (1: one screen pass + candidate log; 0: the
 *                                  two-pass kernel, "knn_mfma_two_pass"), "knn_mfma_prune" (1:
 *                                  k-means order + FP64-ball superblock pruning);
 *   "nearest_grouped" (default 1): K3g (median-split sample groups, box pruning) for large
 *                                  euclidean nearest-sample scans;
 *   "prim_coop"       (default 1): single-launch cooperative Prim for 4096 < n <= 65536;
 *                                  "prim_coop_plain" (1: launched as a plain kernel first --
 *                                  cooperative launches serialise device-wide -- with a timed-out
 *                                  co-residency wait falling back to the cooperative launch;
 *                                  stat "prim_coop_plain_retries" counts those fallbacks),
 *                                  "prim_coop_plain_spin_log2" (default 20: polls per exchange
 *                                  before the plain attempt reports non-co-residency),
 *                                  "prim_coop_xcd" (default 1: the plain attempt's working
 *                                  workgroups, when the run-time XCC_ID check finds them on one
 *                                  XCD, exchange through that XCD's L2 -- placement changes only
 *                                  speed), "prim_coop_slots" (exchange layout; 6: the speculative
 *                                  multi-step kernel, bit-exact, faster alone, slower when several
 *                                  Prims share the GPU);
 *   "bubble_knn_split"(default 1): bubble core distances scan their candidates in chunks and
 *                                  replay the sequential insertion log exactly;
 *   "boruvka_seed"    (default 1): a Boruvka round starts from the previous round's still
 *                                  valid per-point edges;
 *   "boruvka_knn_seed"(default 1): hdb_exact_mst seeds every Boruvka round from the k-NN
 *                                  lists (lanes whose seed is provably exact skip the scan);
 *                                  "leaf_seed_k" (list length, -1: by dimension),
 *                                  "leaf_list_rounds" (default 2: rounds seeded from the lists);
 *   "boruvka_wave_pts" (default 64; 16/32/64): points per scan wave; "boruvka_early_pts" /
 *                                  "boruvka_early_rounds": another size for the first rounds;
 *   "boruvka_adj_seed"(default 1): Morton-adjacent pairs across components bound every
 *                                  component before a Boruvka scan (valid edges only);
 *   "k1t_xcd_chunks" / "bor_xcd_chunks" (default 8): K1t and the Boruvka scan deal their
 *                                  Morton-ordered workgroups to the 8 XCDs as 8 interleaved chunks
 *                                  per XCD (L2 reuse of neighbour tiles; 0: dispatch order) --
 *                                  placement only, results unchanged;
 *   "trav_pop_test"   (default 0): bit 0 Boruvka, bit 1 K1t re-test a popped node;
 *   "ssort"           (default 1): the Morton order, the MST edge orders, K6's term order and
 *                                  hdb_sort_edges_desc use the sample sort (unique 128-bit keys:
 *                                  the same orders as the rocPRIM radix path, 0); "ssort_cap"
 *                                  (default 0 = 4096: keys per bucket sorted in LDS; larger
 *                                  buckets are merged in global memory);
 *   "flat_relabel"    (default 1): hdb_flat_labels renumbers vertex labels in rank order first
 *                                  (locality of the label records; the labels are unchanged);
 *   "flat_mid_log"    (default 12): hdb_flat_labels runs the divide-and-conquer depths below
 *                                  2^flat_mid_log ranks per workgroup (<= 10: all global);
 *   "count_evals"     (default 0): K1t/K2b count the pairs they evaluate (read "last_evals"). */
int hdb_ctx_set_option(hdb_ctx *ctx, const char *name, int64_t value);
/* Diagnostic counters: "last_evals" = pair evaluations of the last K1t call (count_evals on). */
int hdb_ctx_get_stat(hdb_ctx *ctx, const char *name, int64_t *value);
const char *hdb_last_error(void);
int hdb_version(void);

/* ------------------------------------------------------- distance (a1, a2) */
/* Pairwise distance of rows a[i] and b[i], i < n -- DistanceCalculator.computeDistance. */
int hdb_distance_rows(hdb_ctx *ctx, const double *a, const double *b, int64_t n, int32_t d, int32_t metric,
                      double *out);

/* ------------------------------------------------------ core distances (a3, a4)
 * Replaces HDBSCANStar.calculateCoreDistances(double[][] dataSet, int k, DistanceCalculator)
 * (HDBSCANStar.java:71) and its variants CreateLocalMST.java:138 / CoreDistanceMapper.java:71.
 * X: n x d row-major doubles.  core_out: n doubles. */
int hdb_core_distances(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t min_pts, int32_t metric,
                       int32_t semantics, double *core_out);

/* Per-row k smallest distances, ascending (Double.MAX_VALUE padded), optional neighbour
 * indices.  The value lists are the kernel output every core semantics derives from. */
int hdb_knn(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t k, int32_t metric, int32_t excl_self,
            double *dist_out /* n*k */, int32_t *idx_out /* n*k, nullable */);

/* ----------------------------------------------------------------- MST (a5, a6)
 * Replaces HDBSCANStar.constructMST(double[][] dataSet, double[] coreDistances, boolean
 * selfEdges, DistanceCalculator, int[] indices, int totalLength) (HDBSCANStar.java:124-125).
 * Exact reference Prim: start vertex n-1, strict '<' update, '<=' select, Double.MAX_VALUE
 * init.  Edge i < n-1 = (va=parent of i, vb=ids[i], w); then n self edges if self_edges.
 * ids nullable (identity). */
int hdb_prim_mst(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const double *core, const int32_t *ids,
                 int32_t metric, int32_t self_edges, int32_t *va, int32_t *vb, double *w);

/* The same Prim for P independent partitions stored back to back: partition p = rows
 * offsets[p] .. offsets[p+1]-1 of X/core/ids.  Edges of partition p start at
 * edge_offsets[p] = sum_{q<p} (n_q - 1 + (self_edges ? n_q : 0)). */
int hdb_prim_mst_batched(hdb_ctx *ctx, const double *X, const int64_t *offsets, int32_t P, int32_t d,
                         const double *core, const int32_t *ids, int32_t metric, int32_t self_edges, int32_t *va,
                         int32_t *vb, double *w);

/* FirstStep.call leaf branch (mappers/FirstStep.java:104-120) for P partitions at once:
 * live cumulative core distances (HDBSCANStar.java:71-106) + Prim with self edges, vertex
 * ids = global point ids.  core_out nullable. */
int hdb_leaf_msts(hdb_ctx *ctx, const double *X, const int64_t *offsets, int32_t P, int32_t d, const int32_t *ids,
                  int32_t min_pts, int32_t metric, double *core_out, int32_t *va, int32_t *vb, double *w);

/* Exact minimum spanning tree of the mutual-reachability graph for large n (Boruvka,
 * K2b).  Any MST: the sorted weight sequence equals the reference Prim's exactly; the
 * topology can differ only among equal-weight edges (ties broken by (w, min id, max id)).
 * Outputs n-1 edges (va < vb, by the library's order), then n self edges if self_edges. */
int hdb_mst_boruvka(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const double *core, int32_t metric,
                    int32_t self_edges, int32_t *va, int32_t *vb, double *w);

/* FirstStep's leaf branch for one large partition in one call (FirstStep.java:104-108:
 * HDBSCANStar.calculateCoreDistances then constructMST): core distances (semantics as
 * hdb_core_distances, bit-identical) and the exact mutual-reachability MST of
 * hdb_mst_boruvka (same weights and edge order), sharing one spatial index; the k-NN lists
 * seed every Boruvka round.  core_out nullable.  Local vertex ids 0..n-1. */
#define HDB_EDGES_SELF 1   /* append the n self edges (HDBSCANStar.java:196-203)                  */
#define HDB_EDGES_MERGED 2 /* return the edges in the reducers' merge order instead: exactly what
                              hdb_sort_edges_desc returns for the plain list (UnionFindReducer.java:
                              19-69 + SortMST.java:9-17, stable descending), without the re-sort */
int hdb_exact_mst(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, int32_t min_pts, int32_t metric,
                  int32_t semantics, int32_t self_edges /* HDB_EDGES_* flags; 0/1 as before */, double *core_out,
                  int32_t *va, int32_t *vb, double *w);

/* ---------------------------------------------------------- nearest sample (a8, a9)
 * FirstStep.call non-leaf branch (FirstStep.java:74-85): the FIRST minimum over the sample
 * list (strict '<').  With x_key/s_key non-NULL only samples of the point's key are scanned
 * (D3; ClusterFeaturesByNodesMapper.java:53-61).  nearest_out = list position (0 if no
 * candidate, as the Java init), dist_out nullable (Double.MAX_VALUE if none). */
int hdb_nearest_sample(hdb_ctx *ctx, const double *X, int64_t n, const double *S, int64_t m, int32_t d,
                       int32_t metric, const int32_t *x_key, const int32_t *s_key, int32_t *nearest_out,
                       double *dist_out);

/* --------------------------------------------------------- bubble statistics (a11, a12)
 * Bulk CombineStep (CombineStep.java:18-64) over a partition: member order = ascending
 * point index (D5).  Outputs per bubble: ls, ss, rep (nb*d), info (nb*3: extent, nnDist, n).
 * Empty bubbles: all zero. */
int hdb_bubble_stats(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const int32_t *bubble_of, int64_t nb,
                     int32_t variant, double *ls, double *ss, double *rep, double *info);

/* CombineStep as Spark runs it: reduceByKey(new CombineStep()) (Main.java:236-237) folds each
 * partition map-side, then merges the partials (CombineStep.java:18-40 on two partials).  With
 * the partitions fixed (D11) the statistics shard: a rank folds the rows of its slices
 * (cuts[0..S]: S + 1 non-decreasing row offsets, cuts[0] = 0, cuts[S] = n; S <= 64) into
 * per-(slice, bubble) partials -- part_ls / part_ss: S x nb x d, part_n: S x nb member counts --
 * and hdb_bubble_combine merges the gathered partials of all slices in slice order (empty
 * partials skipped) and computes rep / extent / nnDist from the merged (LS, SS, n) with
 * CombineStep.java:42-64's formulas.  One slice is hdb_bubble_stats(HDB_BUBBLE_COMBINESTEP)
 * bit for bit. */
int hdb_bubble_partials(hdb_ctx *ctx, const double *X, int64_t n, int32_t d, const int32_t *bubble_of, int64_t nb,
                        const int64_t *cuts, int32_t S, double *part_ls, double *part_ss, double *part_n);
int hdb_bubble_combine(hdb_ctx *ctx, const double *part_ls, const double *part_ss, const double *part_n, int32_t S,
                       int64_t nb, int32_t d, double *ls, double *ss, double *rep, double *info);

/* ------------------------------------------------------------- bubble model (a13-a15)
 * HdbscanDataBubbles.calculateCoreDistancesBubbles(double[][] repB, int[] nB, double[] eB,
 * double[] nnDistB, int k, DistanceCalculator) (HdbscanDataBubbles.java:75-76). */
int hdb_bubble_core_distances(hdb_ctx *ctx, const double *rep, const int32_t *nB, const double *eB,
                              const double *nnB, int64_t b, int32_t d, int32_t min_pts, int32_t metric,
                              double *core_out);

/* HdbscanDataBubbles.constructMSTBubbles(...) (HdbscanDataBubbles.java:165-167). */
int hdb_bubble_prim_mst(hdb_ctx *ctx, const double *rep, const double *eB, const double *nnB,
                        const int32_t *id_bubbles, const double *core, int64_t b, int32_t d, int32_t metric,
                        int32_t self_edges, int32_t *va, int32_t *vb, double *w);

/* LocalModelReduceByKey.call body (LocalModelReduceByKey.java:88-104) with D4 vertex ids
 * 0..b-1: bubble cores, bubble Prim, UndirectedGraph.quicksortByEdgeWeight, cluster tree,
 * FOSC + noise reassignment, inter-cluster edges.  info = b*3 (extent, nnDist, n).
 * Outputs: labels[b]; mst_* (2b-1, quicksorted ascending, nullable); ic_* (capacity 2b-1),
 * *n_ic = number of inter-cluster edges.  Host memory only for outputs. */
int hdb_local_model(hdb_ctx *ctx, const double *rep, const double *info, int64_t b, int32_t d, int32_t min_pts,
                    int32_t min_cl_size, int32_t metric, int32_t *labels, int32_t *mst_va, int32_t *mst_vb,
                    double *mst_w, int32_t *ic_va, int32_t *ic_vb, double *ic_w, int64_t *n_ic);

/* hdb_local_model from precomputed bubble core distances (host, b values: hdb_bubble_core_distances
 * of the same rep / nB = (int) info[:, 2] / eB = info[:, 0] / nnB = info[:, 1], min_pts, metric) --
 * the same outputs; lets a caller compute every model's cores of a level before any model's Prim
 * (round 6: a Prim holds its CUs for its whole run and slows concurrent work). */
int hdb_local_model_cores(hdb_ctx *ctx, const double *rep, const double *info, int64_t b, int32_t d, int32_t min_pts,
                          int32_t min_cl_size, int32_t metric, const double *core, int32_t *labels, int32_t *mst_va,
                          int32_t *mst_vb, double *mst_w, int32_t *ic_va, int32_t *ic_vb, double *ic_w,
                          int64_t *n_ic);

/* UndirectedGraph.quicksortByEdgeWeight (UndirectedGraph.java:93-124), in place, host. */
int hdb_quicksort_edges(int32_t *va, int32_t *vb, double *w, int64_t ne);

/* ------------------------------------------------------------------- merge (a20)
 * UnionFindReducer.call + SortMST (UnionFindReducer.java:19-69, SortMST.java:9-17): stable
 * sort by DESCENDING weight of the concatenated local edge lists, in place (device radix
 * sort).  The cross-GPU all-gather feeding it runs over RCCL in the host layer. */
int hdb_sort_edges_desc(hdb_ctx *ctx, int32_t *va, int32_t *vb, double *w, int64_t ne);

/* The same result when the concatenation is made of runs that are each already sorted
 * descending (as hdb_sort_edges_desc returns them): runs r = [run_off[r], run_off[r+1]) of
 * (va, vb, w), nruns of them; output (oa, ob, ow) = the stable descending sort of their
 * concatenation -- equal weights keep run order, then their order inside the run.  The
 * stable sort of a rank-major concatenation of raw lists equals this merge of the ranks'
 * individually sorted lists, so a reducer merges instead of re-sorting (pairwise merge-path
 * tiles, O(E log nruns)).  Outputs must not alias inputs.  HDB_EINVAL on a NaN weight or a
 * run that is not descending.  Synchronises. */
int hdb_merge_sorted_runs(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w, const int64_t *run_off,
                          int32_t nruns, int32_t *oa, int32_t *ob, double *ow);

/* ---------------------------------------------- cross-GPU merge over RCCL (§8(b), §8(e))
 * One communicator per rank (one process per GPU).  The caller moves the unique id from the
 * rank that made it to the others (Spark broadcast, torch.distributed, MPI ...). */
typedef struct hdb_comm hdb_comm;
/* Writes an RCCL unique id (128 bytes) into id_out; returns its size or an error. */
int hdb_comm_unique_id(void *id_out, int32_t cap);
/* Collective over the nranks ranks; the context fixes the device and stream. */
int hdb_comm_init(hdb_ctx *ctx, int32_t nranks, int32_t rank, const void *id, hdb_comm **out);
void hdb_comm_destroy(hdb_comm *comm);
/* Frees a buffer the library allocated (hdb_merge_edges outputs). */
int hdb_free(void *p);
/* Copies bytes between any two host/device buffers on the context stream; synchronises. */
int hdb_copy(hdb_ctx *ctx, void *dst, const void *src, int64_t bytes);
/* Main.java:302-347 + UnionFindReducer.call + SortMST (UnionFindReducer.java:19-69,
 * SortMST.java:9-17): every rank passes its local edge list; all ranks receive the merged
 * list of all E edges (device memory allocated by the library, freed with hdb_free), stably
 * sorted by DESCENDING weight.  seq (nullable; on every rank that has local edges or on
 * none -- a rank with e_local == 0 is consistent with either): the canonical
 * position of each local edge in the global concatenation (a permutation of [0, E) over all
 * ranks) -- the sort then sees that concatenation, independent of which rank computed which
 * partition; NULL = rank-major concatenation.  Collective; synchronises. */
int hdb_merge_edges(hdb_comm *comm, const int32_t *va, const int32_t *vb, const double *w, const int64_t *seq,
                    int64_t e_local, int32_t **va_all, int32_t **vb_all, double **w_all, int64_t *e_all);

/* CreateLocalMST's record fields (partition/mappers/CreateLocalMST.java:242,266,276-285):
 * for a partition's edge list with global vertex ids (e.g. hdb_prim_mst / hdb_leaf_msts /
 * hdb_exact_mst output), fake1[e] / fake2[e] = the local index of va[e] / vb[e] in the
 * partition's `indices` (ids, n; NULL = identity), node_out[e] = node (nullable).  On
 * hdb_prim_mst's output this is exactly nearestneighborsID / otherVertexIndicesID, so
 * hdb_format_mst_records reproduces the reference's local-MST text.  w (nullable) = the
 * edge weights of hdb_prim_mst's layout (n - 1 tree edges first): a tree edge whose weight is
 * still Double.MAX_VALUE was never relaxed (every MRD NaN or >= MAX_VALUE), and the
 * reference keeps its Java default nearestneighborsID = 0 (CreateLocalMST.java:203,242) --
 * fake1 = 0 there, whatever va holds.  Errors: HDB_EINVAL on duplicate ids or an edge vertex
 * outside the partition.  Synchronises. */
int hdb_local_mst_ids(hdb_ctx *ctx, const int32_t *ids, int64_t n, const int32_t *va, const int32_t *vb,
                      const double *w, int64_t ne, int32_t node, int32_t *fake1, int32_t *fake2, int32_t *node_out);

/* ------------------------------------------------ global flat labels (§8(f) #1)
 * The step the reference never completes (Main.java:351-408): HDBSCAN* hierarchy over the
 * merged MST and its flat FOSC / excess-of-mass partition -- HDBSCANStar.java:208-625
 * (computeHierarchyAndClusterTree, propagateTree, findProminentClusters; commented out in the
 * reference) without constraints, canonical tie rules (DESIGN.md "flat labels").
 * va/vb/w: the merged edge list (self edges ignored; the rest must form a spanning tree of
 * the n points).  labels: n ints, 1..K by ascending smallest member id, 0 = noise.
 * min_cl_size >= 2.  ctx may be NULL when every pointer is host memory (pure host algorithm). */
int hdb_flat_labels(hdb_ctx *ctx, const int32_t *va, const int32_t *vb, const double *w, int64_t ne, int64_t n,
                    int32_t min_cl_size, int32_t *labels, int64_t *n_clusters);

/* -------------------------------------------------- record formats (§8(f) #3)
 * Host-only (no context, no device); see csrc/formats.cpp. */

/* Double.toString(v) (Java layout, shortest round-trip digits) into buf (cap bytes, NUL
 * terminated).  Returns the length (>= 0) or HDB_EINVAL when cap is too small (32 always
 * suffices).  Used by the record writer below. */
int hdb_format_double(double v, char *buf, int32_t cap);

/* MapperDataset_github.call over a text file's bytes (MapperDataset_github.java:12-20):
 * one point per line, fields Double.parseDouble'd, points numbered in file order.
 * strict = 1: s.split(" ") exactly (a doubled space or an empty line -> NumberFormatException);
 * strict = 0: deviation D1 (fields separated by runs of ' '/'\t', blank lines skipped, the
 * first d fields kept).  d = 0 takes the first line's field count.  X = NULL: count only
 * (*n_out points, *d_out columns); else X holds cap points of *d_out doubles.
 * Errors: HDB_EREF_NUMBER_FORMAT (bad field), HDB_EREF_OOB (short line). */
int hdb_parse_points(const char *text, int64_t len, int32_t d, int32_t strict, double *X, int64_t cap,
                     int64_t *n_out, int32_t *d_out);

/* CreateLocalMST's local-MST text (CreateLocalMST.java:110-123): "v1 v2 w f1 f2 node" per
 * edge, '\n'-joined, no trailing newline, w via Double.toString; fake1/fake2/node nullable
 * (written as 0).  out = NULL: *len_out = the byte length; else out (cap bytes) receives
 * the text plus a NUL. */
int hdb_format_mst_records(const int32_t *va, const int32_t *vb, const double *w, const int32_t *fake1,
                           const int32_t *fake2, const int32_t *node, int64_t ne, char *out, int64_t cap,
                           int64_t *len_out);

/* UnionFindReducer.call's record parse (UnionFindReducer.java:22-45): split("\n"),
 * split(" "), Integer.parseInt / Double.parseDouble of fields 0-5.  va = NULL: count only.
 * Errors: HDB_EREF_OOB (fewer than 6 fields), HDB_EREF_NUMBER_FORMAT. */
int hdb_parse_mst_records(const char *text, int64_t len, int32_t *va, int32_t *vb, double *w, int32_t *fake1,
                          int32_t *fake2, int32_t *node, int64_t cap, int64_t *ne_out);

#ifdef __cplusplus
}
#endif
#endif /* HDBMI_H */
