/*
 * hdb_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Line-faithful CPU restatement of the MR-HDBSCAN* hot path of the reference
 * (SZU-AdvTech-2022/232, Java 8 + Spark 2.x, /root/reference/源代码/...).  It is
 * the parity checker for the HIP product path: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product library never links it.
 *
 * Parity status: the reference cannot run here (no JVM, no Spark jars, no network),
 * so this restatement is pinned by (1) known-answer tests hand-derived from the Java
 * source, (2) independent cross-checks against scipy/sklearn for the
 * standard (EXCL_SELF) semantics, and (3) the reference's own data files
 * (数据集/dataset.txt, 数据集/Skin_NonSkin.txt) as inputs.  Reference-specific quirks
 * (cumulative cores, bubble formulas, cluster-tree tie handling) are "parity unpinned"
 * beyond those hand-derived KATs.  See DESIGN.md §Oracle.
 *
 * Build: -O2 -ffp-contract=off, no -ffast-math (Java has no FMA contraction and
 * Math.sqrt is correctly rounded).
 *
 * Every function cites the Java lines it restates.
 */
#include <math.h>
#include <float.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_EINVAL (-1)
#define ORC_ENOMEM (-3)
#define ORC_EREF_NPE (-10)              /* java.lang.NullPointerException            */
#define ORC_EREF_OOB (-11)              /* ArrayIndexOutOfBoundsException            */
#define ORC_EREF_NEGATIVE_CLUSTER (-12) /* Clusters.java:45-46 IllegalStateException */
#define ORC_EREF_DIVZERO (-13)          /* java.lang.ArithmeticException (int / 0)   */
#define ORC_EUNSUPPORTED (-20)          /* a Java behaviour not emulated: a treeified HashMap bin
                                           (its iteration order changes) or a loop the reference
                                           never leaves (NaN edge weight in the cluster tree) */

enum { M_EUCLIDEAN = 0, M_COSINE = 1, M_PEARSON = 2, M_MANHATTAN = 3, M_SUPREMUM = 4 };
enum { CORE_INCL_SELF_CUMULATIVE = 0, CORE_INCL_SELF = 1, CORE_EXCL_SELF = 2 };

#define JMAX DBL_MAX /* Double.MAX_VALUE */

/* ------------------------------------------------------------------ distance */

/* EuclideanDistance.java:28-36: distance += (a-b)*(a-b) in index order, then sqrt. */
static double d_euclid(const double *a, const double *b, int d) {
    double s = 0;
    for (int i = 0; i < d; i++) s += ((a[i] - b[i]) * (a[i] - b[i]));
    return sqrt(s);
}
/* CosineSimilarity.java:28-40 */
static double d_cosine(const double *a, const double *b, int d) {
    double dot = 0, m1 = 0, m2 = 0;
    for (int i = 0; i < d; i++) {
        dot += (a[i] * b[i]);
        m1 += (a[i] * a[i]);
        m2 += (b[i] * b[i]);
    }
    return 1 - (dot / sqrt(m1 * m2));
}
/* PearsonCorrelation.java:28-51 */
static double d_pearson(const double *a, const double *b, int d) {
    double mean1 = 0, mean2 = 0;
    for (int i = 0; i < d; i++) { mean1 += a[i]; mean2 += b[i]; }
    mean1 = mean1 / d;
    mean2 = mean2 / d;
    double cov = 0, s1 = 0, s2 = 0;
    for (int i = 0; i < d; i++) {
        cov += ((a[i] - mean1) * (b[i] - mean2));
        s1 += ((a[i] - mean1) * (a[i] - mean1));
        s2 += ((b[i] - mean2) * (b[i] - mean2));
    }
    return (1 - (cov / sqrt(s1 * s2)));
}
/* ManhattanDistance.java:28-36 */
static double d_manhattan(const double *a, const double *b, int d) {
    double s = 0;
    for (int i = 0; i < d; i++) s += fabs(a[i] - b[i]);
    return s;
}
/* SupremumDistance.java:28-38 */
static double d_supremum(const double *a, const double *b, int d) {
    double s = 0;
    for (int i = 0; i < d; i++) {
        double diff = fabs(a[i] - b[i]);
        if (diff > s) s = diff;
    }
    return s;
}

double orc_distance(const double *a, const double *b, int d, int metric) {
    switch (metric) {
    case M_EUCLIDEAN: return d_euclid(a, b, d);
    case M_COSINE: return d_cosine(a, b, d);
    case M_PEARSON: return d_pearson(a, b, d);
    case M_MANHATTAN: return d_manhattan(a, b, d);
    case M_SUPREMUM: return d_supremum(a, b, d);
    }
    return NAN;
}

/* Insertion into the sorted k-NN buffer, strict '<' (HDBSCANStar.java:88-100).
 * Returns the insert position, or K when not inserted. */
static int knn_insert(double *buf, int K, double dist) {
    int pos = K;
    while (pos >= 1 && dist < buf[pos - 1]) pos--;
    if (pos < K) {
        for (int s = K - 1; s > pos; s--) buf[s] = buf[s - 1];
        buf[pos] = dist;
    }
    return pos;
}

/* -------------------------------------------------------------- core distances
 * INCL_SELF_CUMULATIVE: HDBSCANStar.calculateCoreDistances (HDBSCANStar.java:71-106),
 *   the live path: buffer initialised ONCE (:79-82), self included (:84).
 * INCL_SELF: CoreDistanceMapper.calculateCoreDistances (CoreDistanceMapper.java:71-109),
 *   buffer per query, self included.
 * EXCL_SELF: CreateLocalMST.calculateCoreDistances (CreateLocalMST.java:138-185),
 *   buffer per point, self skipped (:153-154).
 */
int orc_core_distances(const double *X, int64_t n, int d, int min_pts, int metric, int semantics,
                       double *core) {
    if (n < 0 || d <= 0 || min_pts < 1) return ORC_EINVAL;
    int K = min_pts - 1;
    if (min_pts == 1) { /* :75-77 */
        for (int64_t i = 0; i < n; i++) core[i] = 0;
        return ORC_OK;
    }
    double *buf = (double *)malloc(sizeof(double) * K);
    if (!buf) return ORC_ENOMEM;
    for (int i = 0; i < K; i++) buf[i] = JMAX;
    for (int64_t p = 0; p < n; p++) {
        if (semantics != CORE_INCL_SELF_CUMULATIVE)
            for (int i = 0; i < K; i++) buf[i] = JMAX;
        for (int64_t q = 0; q < n; q++) {
            if (semantics == CORE_EXCL_SELF && p == q) continue;
            double dist = orc_distance(X + p * d, X + q * d, d, metric);
            knn_insert(buf, K, dist);
        }
        core[p] = buf[K - 1];
    }
    free(buf);
    return ORC_OK;
}

/* Per-point top-(minPts-1) distance lists (ascending, JMAX padded), the value-only
 * kernel output from which every semantics above is an epilogue. */
int orc_knn_lists(const double *X, int64_t n, int d, int min_pts, int metric, int excl_self,
                  double *lists /* n*K */) {
    if (min_pts < 2) return ORC_EINVAL;
    int K = min_pts - 1;
    for (int64_t p = 0; p < n; p++) {
        double *buf = lists + p * K;
        for (int i = 0; i < K; i++) buf[i] = JMAX;
        for (int64_t q = 0; q < n; q++) {
            if (excl_self && p == q) continue;
            knn_insert(buf, K, orc_distance(X + p * d, X + q * d, d, metric));
        }
    }
    return ORC_OK;
}

/* ----------------------------------------------------------------- Prim MST
 * HDBSCANStar.constructMST (HDBSCANStar.java:124-205).  Start vertex n-1 (:145-147),
 * Double.MAX_VALUE init (:140-142), mrd = max(d, core[cur], core[nb]) (:164-168),
 * strict '<' update with parent = indices[cur] (:170-173), '<=' select (:177-180).
 * Parent array defaults to Java int 0 for never-updated vertices.
 * Output edge i (i < n-1): (va=parent[i], vb=ids[i], w=best[i]); then, if self_edges,
 * n self edges (ids[v], ids[v], core[v]) (:190-203).
 * `dist_bubbles` non-NULL switches to constructMSTBubbles (HdbscanDataBubbles.java:165-254):
 * distance transformed by distanceBubbles (:208-209).
 */
static double distance_bubbles(double distance, const double *eB, const double *nnB, int64_t p, int64_t q);

static int prim_core(const double *X, int64_t n, int d, const double *core, const int32_t *ids,
                     int metric, int self_edges, const double *eB, const double *nnB, int32_t *va,
                     int32_t *vb, double *w, int32_t *parent_local) {
    if (n < 1 || d <= 0) return ORC_EINVAL;
    unsigned char *attached = (unsigned char *)calloc((size_t)n, 1);
    int32_t *parent = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    double *best = (double *)malloc(sizeof(double) * (size_t)n);
    if (!attached || !parent || !best) { free(attached); free(parent); free(best); return ORC_ENOMEM; }
    for (int64_t i = 0; i < n; i++) best[i] = JMAX;
    best[n - 1] = 0; /* Java default; never read (vertex n-1 attached first) */
    int64_t cur = n - 1;
    int64_t numAttached = 1;
    attached[n - 1] = 1;
    while (numAttached < n) {
        int64_t nearestPt = -1;
        double nearestD = JMAX;
        for (int64_t nb = 0; nb < n; nb++) {
            if (cur == nb) continue;
            if (attached[nb]) continue;
            double dist = orc_distance(X + cur * d, X + nb * d, d, metric);
            if (eB) dist = distance_bubbles(dist, eB, nnB, cur, nb);
            double mrd = dist;
            if (core[cur] > mrd) mrd = core[cur];
            if (core[nb] > mrd) mrd = core[nb];
            if (mrd < best[nb]) {
                best[nb] = mrd;
                parent[nb] = ids[cur];
                if (parent_local) parent_local[nb] = (int32_t)cur; /* CreateLocalMST.java:242 nearestneighborsID */
            }
            if (best[nb] <= nearestD) {
                nearestD = best[nb];
                nearestPt = nb;
            }
        }
        if (nearestPt < 0) { free(attached); free(parent); free(best); return ORC_EREF_OOB; }
        attached[nearestPt] = 1;
        numAttached++;
        cur = nearestPt;
    }
    for (int64_t i = 0; i < n - 1; i++) {
        va[i] = parent[i];
        vb[i] = ids[i];
        w[i] = best[i];
    }
    if (self_edges) {
        for (int64_t i = n - 1; i < 2 * n - 1; i++) {
            int64_t v = i - (n - 1);
            va[i] = ids[v];
            vb[i] = ids[v];
            w[i] = core[v];
        }
    }
    free(attached);
    free(parent);
    free(best);
    return ORC_OK;
}

int orc_prim_mst(const double *X, int64_t n, int d, const double *core, const int32_t *ids, int metric,
                 int self_edges, int32_t *va, int32_t *vb, double *w) {
    return prim_core(X, n, d, core, ids, metric, self_edges, NULL, NULL, va, vb, w, NULL);
}

/* CreateLocalMST.constructMST (partition/mappers/CreateLocalMST.java:187-292): the Prim above
 * plus the record fields it keeps -- fake1 = nearestneighborsID (the parent's local index,
 * :242), fake2 = otherVertexIndicesID (the vertex's local index, :266), node (:285); self
 * edges carry (vertex, vertex, node) (:276-282). */
int orc_create_local_mst(const double *X, int64_t n, int d, const double *core, const int32_t *ids, int metric,
                         int self_edges, int32_t node, int32_t *va, int32_t *vb, double *w, int32_t *fake1,
                         int32_t *fake2, int32_t *node_out) {
    if (n < 1) return ORC_EINVAL;
    int32_t *pl = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    if (!pl) return ORC_ENOMEM;
    int rc = prim_core(X, n, d, core, ids, metric, self_edges, NULL, NULL, va, vb, w, pl);
    if (rc == ORC_OK) {
        const int64_t ne = (n - 1) + (self_edges ? n : 0);
        for (int64_t i = 0; i < ne; i++) {
            const int64_t v = i < n - 1 ? i : i - (n - 1);
            fake1[i] = i < n - 1 ? pl[i] : (int32_t)v;
            fake2[i] = (int32_t)v;
            node_out[i] = node;
        }
    }
    free(pl);
    return rc;
}

/* ---------------------------------------------------------- nearest sample
 * FirstStep.call non-leaf branch (FirstStep.java:74-85): for each point, scan the
 * whole sample list in order, strict '<' => the FIRST minimum wins; init
 * minDistance = Double.MAX_VALUE, nearest = 0.  With keys (D3 deviation, the
 * ClusterFeaturesByNodesMapper.java:53-61 filter) only samples whose key equals the
 * point's key are considered.  Returns the list position of the winning sample.
 */
int orc_nearest_sample(const double *X, int64_t n, const double *S, int64_t m, int d, int metric,
                       const int32_t *x_key, const int32_t *s_key, int32_t *nearest, double *dist_out) {
    for (int64_t p = 0; p < n; p++) {
        double minD = JMAX;
        int64_t nn = 0;
        for (int64_t j = 0; j < m; j++) {
            if (x_key && s_key && x_key[p] != s_key[j]) continue;
            double dist = orc_distance(X + p * d, S + j * d, d, metric);
            if (dist < minD) {
                minD = dist;
                nn = j;
            }
        }
        nearest[p] = (int32_t)nn;
        if (dist_out) dist_out[p] = minD;
    }
    return ORC_OK;
}

/* ------------------------------------------------------------ bubble stats
 * CombineStep (CombineStep.java:18-64) as the sequential fold Spark's reduceByKey
 * performs with the D5 canonical order (ascending point id within a bubble).
 * The first member seeds (rep=ls=x, ss=x*x, info=[0,0,1]) (FirstStep.java:87-101);
 * each further member: ls += x, ss += x*x (:24-27), n += 1 (:28), rep = ls/n (:58-64),
 * extent (:46-56), nnDist = pow(1/n, (int)(1/d)) * extent (:42-44).
 * Outputs per bubble: ls[nb*d], ss[nb*d], rep[nb*d], info[nb*3] = (extent, nnDist, n).
 * Empty bubbles: all zeros, info n = 0 (D4).
 */
static double combine_extent(const double *ls, const double *ss, double n, int d) {
    double extent = 0.0;
    if (n > 1) {
        for (int i = 0; i < d; i++) {
            double v = ((2 * n * ss[i]) - (2 * (ls[i] * ls[i])));
            if (v >= 0) extent += sqrt(((2 * n * ss[i]) - (2 * (ls[i] * ls[i]))) / (n * (n - 1)));
        }
    }
    return extent / d;
}

int orc_bubble_stats_combine(const double *X, int64_t n, int d, const int32_t *bubble_of, int64_t nb,
                             double *ls, double *ss, double *rep, double *info) {
    memset(ls, 0, sizeof(double) * (size_t)(nb * d));
    memset(ss, 0, sizeof(double) * (size_t)(nb * d));
    memset(rep, 0, sizeof(double) * (size_t)(nb * d));
    memset(info, 0, sizeof(double) * (size_t)(nb * 3));
    for (int64_t p = 0; p < n; p++) {
        int64_t b = bubble_of[p];
        if (b < 0 || b >= nb) return ORC_EINVAL;
        const double *x = X + p * d;
        double *L = ls + b * d, *Q = ss + b * d, *R = rep + b * d, *I = info + b * 3;
        if (I[2] == 0) { /* seed: FirstStep.java:87-94 */
            I[0] = 0; I[1] = 0; I[2] = 1;
            for (int i = 0; i < d; i++) { L[i] = x[i]; Q[i] = x[i] * x[i]; R[i] = x[i]; }
            continue;
        }
        for (int i = 0; i < d; i++) {
            L[i] = L[i] + x[i];
            Q[i] = Q[i] + (x[i] * x[i]);
        }
        I[2] += 1;
        for (int i = 0; i < d; i++) R[i] = L[i] / I[2];
        I[0] = combine_extent(L, Q, I[2], d);
        /* Math.pow((k / n), (1 / numberOfAttributes)) * extent, k = 1 (int), n double */
        I[1] = pow((1 / I[2]), (double)(1 / d)) * I[0];
    }
    return ORC_OK;
}

/* CombineStep over SLICES (D11): the rows are cut into S contiguous slices (cuts[0..S], the
 * driver's fixed slicing of a level's rows -- one or more slices per rank); every slice folds
 * its members exactly as orc_bubble_stats_combine does (its partial: ls, ss, n), and the
 * partials of a bubble are then combined in slice order, skipping slices without members:
 * ls = ((p_a + p_b) + p_c) ..., ss likewise, n = the member count.  This is Spark's own shape
 * for CombineStep (reduceByKey combines map-side per partition, Main.java:236-237, then merges
 * the partials) with the partitions fixed, so the result does not depend on the rank count.
 * rep / extent / nnDist come from the final (ls, ss, n) with CombineStep.java:42-64's formulas
 * -- what its last call computes.  S = 1 is orc_bubble_stats_combine bit for bit. */
int orc_bubble_stats_combine_sliced(const double *X, int64_t n, int d, const int32_t *bubble_of, int64_t nb,
                                    const int64_t *cuts, int S, double *ls, double *ss, double *rep, double *info) {
    if (S < 1 || cuts[0] != 0 || cuts[S] != n) return ORC_EINVAL;
    for (int s = 0; s < S; s++)
        if (cuts[s + 1] < cuts[s]) return ORC_EINVAL;
    double *pl = (double *)malloc(sizeof(double) * (size_t)(nb * d));
    double *pq = (double *)malloc(sizeof(double) * (size_t)(nb * d));
    double *pr = (double *)malloc(sizeof(double) * (size_t)(nb * d));
    double *pi = (double *)malloc(sizeof(double) * (size_t)(nb * 3));
    if (!pl || !pq || !pr || !pi) {
        free(pl), free(pq), free(pr), free(pi);
        return ORC_EINVAL;
    }
    memset(ls, 0, sizeof(double) * (size_t)(nb * d));
    memset(ss, 0, sizeof(double) * (size_t)(nb * d));
    memset(info, 0, sizeof(double) * (size_t)(nb * 3));
    int rc = ORC_OK;
    for (int s = 0; s < S && rc == ORC_OK; s++) {
        rc = orc_bubble_stats_combine(X + cuts[s] * d, cuts[s + 1] - cuts[s], d, bubble_of + cuts[s], nb, pl, pq, pr, pi);
        for (int64_t b = 0; b < nb && rc == ORC_OK; b++) {
            const double cnt = pi[b * 3 + 2];
            if (cnt == 0) continue;
            double *L = ls + b * d, *Q = ss + b * d;
            if (info[b * 3 + 2] == 0) {
                for (int i = 0; i < d; i++) { L[i] = pl[b * d + i]; Q[i] = pq[b * d + i]; }
            } else {
                for (int i = 0; i < d; i++) { L[i] = L[i] + pl[b * d + i]; Q[i] = Q[i] + pq[b * d + i]; }
            }
            info[b * 3 + 2] += cnt;
        }
    }
    free(pl), free(pq), free(pr), free(pi);
    if (rc != ORC_OK) return rc;
    for (int64_t b = 0; b < nb; b++) {
        double *L = ls + b * d, *Q = ss + b * d, *R = rep + b * d, *I = info + b * 3;
        if (I[2] == 0) {
            for (int i = 0; i < d; i++) R[i] = 0;
            continue;
        }
        for (int i = 0; i < d; i++) R[i] = L[i] / I[2];  /* n = 1: x / 1 == x, the seed's rep */
        I[0] = combine_extent(L, Q, I[2], d);           /* 0 when n = 1 */
        I[1] = pow((1 / I[2]), (double)(1 / d)) * I[0];
    }
    return ORC_OK;
}

/* ClusterFeatureDataBubbles.calculateRep/Extent/Nndist (ClusterFeatureDataBubbles.java:192-215)
 * driven by ConstructDataBubblesReducer.call (ConstructDataBubblesReducer.java:74-90):
 * n = n1 + n2 (int), extent = sqrt(sum_i (2n*ss - 2ls^2) / (n*(n-1)))  with the int
 * product n*(n-1) (overflows past 46,341), nnDist = pow(1/n, 1/col) * extent (real exponent).
 * Singleton bubbles keep (rep = x, extent 0, nnDist 0, n 1).
 */
int orc_bubble_stats_cf(const double *X, int64_t n, int d, const int32_t *bubble_of, int64_t nb,
                        double *ls, double *ss, double *rep, double *info) {
    memset(ls, 0, sizeof(double) * (size_t)(nb * d));
    memset(ss, 0, sizeof(double) * (size_t)(nb * d));
    memset(rep, 0, sizeof(double) * (size_t)(nb * d));
    memset(info, 0, sizeof(double) * (size_t)(nb * 3));
    for (int64_t p = 0; p < n; p++) {
        int64_t b = bubble_of[p];
        if (b < 0 || b >= nb) return ORC_EINVAL;
        const double *x = X + p * d;
        double *L = ls + b * d, *Q = ss + b * d, *R = rep + b * d, *I = info + b * 3;
        if (I[2] == 0) {
            I[2] = 1;
            for (int i = 0; i < d; i++) { L[i] = x[i]; Q[i] = x[i] * x[i]; R[i] = x[i]; }
            continue;
        }
        for (int i = 0; i < d; i++) {
            L[i] = L[i] + x[i];
            Q[i] = Q[i] + (x[i] * x[i]);
        }
        int32_t nn = (int32_t)I[2] + 1;
        I[2] = nn;
        for (int i = 0; i < d; i++) R[i] = L[i] / nn;
        int32_t prod = (int32_t)((uint32_t)nn * (uint32_t)(nn - 1)); /* Java int overflow */
        double sum = 0.0;
        for (int i = 0; i < d; i++) sum = sum + (((2 * nn * Q[i]) - (2 * (L[i] * L[i]))) / prod);
        I[0] = sqrt(sum);
        double xx = (double)1 / nn, yy = (double)1 / d;
        I[1] = (pow(xx, yy) * I[0]);
    }
    return ORC_OK;
}

/* -------------------------------------------------------- bubble distance
 * HdbscanDataBubbles.distanceBubbles (HdbscanDataBubbles.java:592-600). */
static double distance_bubbles(double distance, const double *eB, const double *nnB, int64_t p, int64_t q) {
    double verify = distance - (eB[p] + eB[q]);
    if (verify >= 0) {
        distance = (distance - (eB[p] + eB[q])) + (nnB[p] + nnB[q]);
    } else {
        distance = fmax(nnB[p], nnB[q]);
        /* Math.max: NaN if either is NaN (fmax would drop it) */
        if (isnan(nnB[p]) || isnan(nnB[q])) distance = NAN;
    }
    return distance;
}
double orc_distance_bubbles(double distance, const double *eB, const double *nnB, int64_t p, int64_t q) {
    return distance_bubbles(distance, eB, nnB, p, q);
}

/* ---------------------------------------------------- bubble core distances
 * HdbscanDataBubbles.calculateCoreDistancesBubbles (HdbscanDataBubbles.java:75-146),
 * including: self skipped (:98), buffer reset per point (:92-95), indexBubbles written
 * only at the insert position and never reset (:79-83,118), int-division pow exponents
 * (:122,142), and repB[i] with the loop counter i used as a bubble index (:135,142). */
static int64_t jpow_int_div_base(int32_t num, int32_t den) { return num / den; }

int orc_bubble_core_distances(const double *rep, const int32_t *nB, const double *eB, const double *nnB,
                              int64_t b, int d, int min_pts, int metric, double *core) {
    if (min_pts < 1 || d <= 0) return ORC_EINVAL;
    int K = min_pts - 1;
    for (int64_t i = 0; i < b; i++) core[i] = 0;
    if (min_pts == 1) return ORC_OK;
    int32_t *indexB = (int32_t *)calloc((size_t)K, sizeof(int32_t));
    double *knn = (double *)malloc(sizeof(double) * K);
    if (!indexB || !knn) { free(indexB); free(knn); return ORC_ENOMEM; }
    int rc = ORC_OK;
    int32_t inv_d = 1 / d; /* (1 / repB[point].length), int */
    for (int64_t p = 0; p < b; p++) {
        for (int i = 0; i < K; i++) knn[i] = JMAX;
        for (int64_t q = 0; q < b; q++) {
            if (p == q) continue;
            double dist = orc_distance(rep + p * d, rep + q * d, d, metric);
            dist = distance_bubbles(dist, eB, nnB, p, q);
            int pos = knn_insert(knn, K, dist);
            if (pos < K) indexB[pos] = (int32_t)q;
        }
        if (nB[p] >= K) {
            if (nB[p] == 0) { rc = ORC_EREF_DIVZERO; break; }
            core[p] = pow((double)jpow_int_div_base(K, nB[p]), (double)inv_d) * eB[p];
        } else {
            int32_t nX = nB[p];
            int i = 0;
            while (nX < K) {
                if (i >= K) { rc = ORC_EREF_OOB; goto done; }
                nX += nB[indexB[i]];
                i += 1;
            }
            int32_t sum = nB[p];
            int32_t aux = 0;
            if (i >= b) { rc = ORC_EREF_OOB; goto done; } /* repB[i] */
            for (int j = 0; j < i; j++) {
                double dc = orc_distance(rep + (int64_t)indexB[j] * d, rep + (int64_t)i * d, d, metric);
                dc = distance_bubbles(dc, eB, nnB, indexB[j], i);
                if (sum < K && knn[j] < dc) aux = K - sum;
                sum += nB[indexB[j]];
            }
            if (i >= K) { rc = ORC_EREF_OOB; goto done; } /* kNNDistances[i] */
            if (nB[i] == 0) { rc = ORC_EREF_DIVZERO; goto done; }
            core[p] = knn[i] + pow((double)(aux / nB[i]), (double)inv_d) * eB[i];
        }
    }
done:
    free(indexB);
    free(knn);
    return rc;
}

int orc_bubble_prim_mst(const double *rep, const double *eB, const double *nnB, const int32_t *id_bubbles,
                        const double *core, int64_t b, int d, int metric, int self_edges, int32_t *va,
                        int32_t *vb, double *w) {
    return prim_core(rep, b, d, core, id_bubbles, metric, self_edges, eB, nnB, va, vb, w, NULL);
}

/* ------------------------------------------------------------- quicksort
 * UndirectedGraph.quicksortByEdgeWeight (UndirectedGraph.java:93-124) with
 * selectPivotIndex always returning startIndex (the `startIndex - endIndex <= 1`
 * test at :158 is always true) and the Lomuto partition on '<' (:194-208).
 * The explicit stacks have length numEdges/2 (:97-98): overflow => ORC_EREF_OOB. */
static void swap_edges(int32_t *a, int32_t *b, double *w, int64_t i, int64_t j) {
    if (i == j) return;
    int32_t ta = a[i], tb = b[i];
    double tw = w[i];
    a[i] = a[j]; b[i] = b[j]; w[i] = w[j];
    a[j] = ta; b[j] = tb; w[j] = tw;
}
int orc_quicksort_edges(int32_t *va, int32_t *vb, double *w, int64_t ne) {
    if (ne <= 1) return ORC_OK;
    int64_t cap = ne / 2;
    int64_t *ss = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    int64_t *es = (int64_t *)malloc(sizeof(int64_t) * (size_t)cap);
    if (!ss || !es) { free(ss); free(es); return ORC_ENOMEM; }
    ss[0] = 0;
    es[0] = ne - 1;
    int64_t top = 0;
    int rc = ORC_OK;
    while (top >= 0) {
        int64_t s = ss[top], e = es[top];
        top--;
        int64_t pivot = s; /* selectPivotIndex: always startIndex */
        double pv = w[pivot];
        swap_edges(va, vb, w, pivot, e);
        int64_t low = s;
        for (int64_t i = s; i < e; i++) {
            if (w[i] < pv) {
                swap_edges(va, vb, w, i, low);
                low++;
            }
        }
        swap_edges(va, vb, w, low, e);
        pivot = low;
        if (pivot > s + 1) {
            if (top + 1 >= cap) { rc = ORC_EREF_OOB; break; }
            ss[top + 1] = s; es[top + 1] = pivot - 1; top++;
        }
        if (pivot < e - 1) {
            if (top + 1 >= cap) { rc = ORC_EREF_OOB; break; }
            ss[top + 1] = pivot + 1; es[top + 1] = e; top++;
        }
    }
    free(ss);
    free(es);
    return rc;
}

/* ------------------------------------------------------------ merge edges
 * UnionFindReducer.call (UnionFindReducer.java:19-69): concatenate the edge lists in
 * order and Collections.sort with SortMST (SortMST.java:9-17): DESCENDING by weight,
 * stable (TimSort).  Implemented as a stable merge sort. */
typedef struct { int32_t a, b; double w; } edge_t;
static void msort(edge_t *x, edge_t *tmp, int64_t n) {
    if (n < 2) return;
    int64_t h = n / 2;
    msort(x, tmp, h);
    msort(x + h, tmp, n - h);
    int64_t i = 0, j = h, k = 0;
    while (i < h && j < n) {
        /* take right only if strictly greater (descending, stable) */
        if (x[j].w > x[i].w) tmp[k++] = x[j++];
        else tmp[k++] = x[i++];
    }
    while (i < h) tmp[k++] = x[i++];
    while (j < n) tmp[k++] = x[j++];
    memcpy(x, tmp, sizeof(edge_t) * (size_t)n);
}
int orc_merge_edges(int32_t *va, int32_t *vb, double *w, int64_t ne) {
    edge_t *e = (edge_t *)malloc(sizeof(edge_t) * (size_t)(ne > 0 ? ne : 1));
    edge_t *t = (edge_t *)malloc(sizeof(edge_t) * (size_t)(ne > 0 ? ne : 1));
    if (!e || !t) { free(e); free(t); return ORC_ENOMEM; }
    for (int64_t i = 0; i < ne; i++) { e[i].a = va[i]; e[i].b = vb[i]; e[i].w = w[i]; }
    msort(e, t, ne);
    for (int64_t i = 0; i < ne; i++) { va[i] = e[i].a; vb[i] = e[i].b; w[i] = e[i].w; }
    free(e);
    free(t);
    return ORC_OK;
}

/* ============================================================ local model
 * LocalModelReduceByKey.call (LocalModelReduceByKey.java:88-104) once every bubble of a
 * subset is present: bubble cores -> bubble Prim (self edges) -> quicksort ->
 * constructClusterTree -> findProminentClustersAndClassificationNoiseBubbles ->
 * findInterClusterEdges.  D4: vertex ids are the compacted positions 0..b-1.
 */

/* ---- small dynamic int vector */
typedef struct { int32_t *v; int64_t n, cap; } ivec;
static int iv_push(ivec *x, int32_t val) {
    if (x->n == x->cap) {
        int64_t nc = x->cap ? x->cap * 2 : 4;
        int32_t *nv = (int32_t *)realloc(x->v, sizeof(int32_t) * (size_t)nc);
        if (!nv) return -1;
        x->v = nv;
        x->cap = nc;
    }
    x->v[x->n++] = val;
    return 0;
}
static int iv_remove_first(ivec *x, int32_t val) { /* ArrayList.remove(Object) */
    for (int64_t i = 0; i < x->n; i++)
        if (x->v[i] == val) {
            memmove(x->v + i, x->v + i + 1, sizeof(int32_t) * (size_t)(x->n - i - 1));
            x->n--;
            return 1;
        }
    return 0;
}

/* ---- Clusters (Clusters.java:27-47) */
typedef struct {
    int32_t label, parent;
    double birth, death, stability;
    int32_t numPoints;
    int hasChildren;
    int32_t *members; /* sorted vertex ids (TreeSet), NULL for root */
    int64_t nmembers;
} cl_t;
typedef struct { cl_t *c; int64_t n, cap; } clvec;
static int cl_push(clvec *x, cl_t c) {
    if (x->n == x->cap) {
        int64_t nc = x->cap ? x->cap * 2 : 8;
        cl_t *nv = (cl_t *)realloc(x->c, sizeof(cl_t) * (size_t)nc);
        if (!nv) return -1;
        x->c = nv;
        x->cap = nc;
    }
    x->c[x->n++] = c;
    return 0;
}
/* the state at the last "Cluster cannot have less than 0 points." (test diagnostics) */
static __thread int32_t g_neg_label, g_neg_points;
static __thread double g_neg_level;
int orc_last_negative_cluster(int32_t *label, double *level, int32_t *num_points) {
    *label = g_neg_label;
    *level = g_neg_level;
    *num_points = g_neg_points;
    return ORC_OK;
}
static int cl_detach(cl_t *c, int32_t numPoints, int32_t countMembers, double level) {
    c->numPoints -= numPoints;
    c->stability += ((double)(numPoints + countMembers) * (1 / level - 1 / c->birth));
    if (c->numPoints == 0) c->death = level;
    else if (c->numPoints < 0) {
        g_neg_label = c->label;
        g_neg_level = level;
        g_neg_points = c->numPoints;
        return ORC_EREF_NEGATIVE_CLUSTER;
    }
    return ORC_OK;
}

/* ---- java.util.HashMap<Integer, ...> key iteration order emulation:
 * bucket = spread(h) & (cap-1) with spread(h) = h ^ (h >>> 16); buckets ascending,
 * insertion order within a bucket (resizes split buckets order-preservingly).  The final
 * capacity replays the puts: 16 at the first put, doubled when size > 0.75*cap, and doubled
 * when a 9th key lands in one bucket of a table smaller than 64 (treeifyBin resizes instead);
 * at >= 64 buckets that bin becomes a tree bin, whose iteration order is not emulated:
 * ORC_EUNSUPPORTED. */
static uint32_t jhash(int32_t k) { uint32_t h = (uint32_t)k; return h ^ (h >> 16); }
static int64_t jmap_cap(const int32_t *keys, int64_t n) { /* keys in insertion order */
    int64_t cap = 16;
    int64_t *cnt = (int64_t *)calloc((size_t)cap, sizeof(int64_t));
    if (!cnt) return -1;
    for (int64_t i = 0; i < n; i++) {
        for (int pass = 0; pass < 2; pass++) {
            const int64_t before = cnt[jhash(keys[i]) & (uint32_t)(cap - 1)];
            int grow = 0;
            if (pass == 0) {
                cnt[jhash(keys[i]) & (uint32_t)(cap - 1)]++;
                if (before >= 8) {
                    if (cap >= 64) { free(cnt); return -2; }
                    grow = 1;
                }
            } else if (i + 1 > (cap * 3) / 4) {
                grow = 1;
            }
            if (grow) {
                cap *= 2;
                int64_t *nc = (int64_t *)calloc((size_t)cap, sizeof(int64_t));
                if (!nc) { free(cnt); return -1; }
                for (int64_t j = 0; j <= i; j++) nc[jhash(keys[j]) & (uint32_t)(cap - 1)]++;
                free(cnt);
                cnt = nc;
            }
        }
    }
    free(cnt);
    return cap;
}

static int cmp_i32(const void *a, const void *b) {
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

typedef struct {
    int32_t label;
    int64_t order; /* insertion order */
    int32_t *verts; /* TreeSet<Integer> of affected vertices, kept sorted unique */
    int64_t nverts, cap;
} aff_t;

static int aff_add(aff_t *a, int32_t v) {
    /* sorted unique insert */
    int64_t lo = 0, hi = a->nverts;
    while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (a->verts[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    if (lo < a->nverts && a->verts[lo] == v) return 0;
    if (a->nverts == a->cap) {
        int64_t nc = a->cap ? a->cap * 2 : 4;
        int32_t *nv = (int32_t *)realloc(a->verts, sizeof(int32_t) * (size_t)nc);
        if (!nv) return -1;
        a->verts = nv;
        a->cap = nc;
    }
    memmove(a->verts + lo + 1, a->verts + lo, sizeof(int32_t) * (size_t)(a->nverts - lo));
    a->verts[lo] = v;
    a->nverts++;
    return 0;
}

static int64_t g_cap_for_sort;
static int cmp_aff(const void *x, const void *y) {
    const aff_t *a = (const aff_t *)x, *b = (const aff_t *)y;
    uint32_t ba = jhash(a->label) & (uint32_t)(g_cap_for_sort - 1);
    uint32_t bb = jhash(b->label) & (uint32_t)(g_cap_for_sort - 1);
    if (ba != bb) return ba < bb ? -1 : 1;
    return (a->order > b->order) - (a->order < b->order);
}

/* HdbscanDataBubbles.constructClusterTree (HdbscanDataBubbles.java:256-375).
 * Edges must be the quicksorted MST (ascending); processed from the highest index. */
static int construct_cluster_tree(int64_t b, const int32_t *ea, const int32_t *eb, const double *ew,
                                  int64_t ne, int32_t mcl, const int32_t *nB, clvec *clusters) {
    int rc = ORC_OK;
    /* adjacency (UndirectedGraph.java:51-84): keyed by vertex, self loop added once */
    ivec *adj = (ivec *)calloc((size_t)b, sizeof(ivec));
    int32_t *label = (int32_t *)malloc(sizeof(int32_t) * (size_t)b);
    unsigned char *visited = (unsigned char *)malloc((size_t)b);
    int32_t *queue = (int32_t *)malloc(sizeof(int32_t) * (size_t)b);
    unsigned char *inq = (unsigned char *)malloc((size_t)b);
    if (!adj || !label || !visited || !queue || !inq) { rc = ORC_ENOMEM; goto out; }
    for (int64_t i = 0; i < ne; i++) {
        int32_t v1 = ea[i], v2 = eb[i];
        if (v1 < 0 || v1 >= b || v2 < 0 || v2 >= b) { rc = ORC_EREF_OOB; goto out; }
        if (iv_push(&adj[v1], v2)) { rc = ORC_ENOMEM; goto out; }
        if (v1 != v2)
            if (iv_push(&adj[v2], v1)) { rc = ORC_ENOMEM; goto out; }
    }
    for (int64_t i = 0; i < b; i++) label[i] = 1;
    int32_t nextLabel = 2;
    int64_t allMembers = 0;
    for (int64_t i = 0; i < b; i++) allMembers += nB[i];
    cl_t root = {1, -1, NAN, JMAX, 0, (int32_t)allMembers, 0, NULL, 0};
    if (cl_push(clusters, root)) { rc = ORC_ENOMEM; goto out; }

    int64_t cur = ne - 1;
    while (cur >= 0) {
        aff_t *aff = NULL;
        int64_t naff = 0, affcap = 0;
        double cw = ew[cur];
        if (cw != cw) { rc = ORC_EUNSUPPORTED; goto out; } /* the Java loop never advances */
        while (cur >= 0 && ew[cur] == cw) {
            int32_t f = ea[cur], s = eb[cur];
            iv_remove_first(&adj[f], s);
            iv_remove_first(&adj[s], f);
            if (label[f] == 0) { cur--; continue; }
            int64_t k;
            for (k = 0; k < naff; k++) if (aff[k].label == label[f]) break;
            if (k == naff) {
                if (naff == affcap) {
                    affcap = affcap ? affcap * 2 : 4;
                    aff = (aff_t *)realloc(aff, sizeof(aff_t) * (size_t)affcap);
                }
                aff_t na = {label[f], naff, NULL, 0, 0};
                aff[naff++] = na;
            }
            aff_add(&aff[k], f);
            aff_add(&aff[k], s);
            cur--;
        }
        if (naff == 0) { free(aff); continue; }
        {
            int32_t *keys = (int32_t *)malloc(sizeof(int32_t) * (size_t)naff);
            if (!keys) { free(aff); rc = ORC_ENOMEM; goto out; }
            for (int64_t k = 0; k < naff; k++) keys[k] = aff[k].label;
            g_cap_for_sort = jmap_cap(keys, naff);
            free(keys);
            if (g_cap_for_sort < 0) {
                for (int64_t k = 0; k < naff; k++) free(aff[k].verts);
                free(aff);
                rc = g_cap_for_sort == -2 ? ORC_EUNSUPPORTED : ORC_ENOMEM;
                goto out;
            }
        }
        qsort(aff, (size_t)naff, sizeof(aff_t), cmp_aff);

        for (int64_t ai = 0; ai < naff && rc == ORC_OK; ai++) {
            int32_t parentLabel = aff[ai].label;
            /* newClusters (ArrayList) */
            cl_t *newc = NULL;
            int64_t nnew = 0, newcap = 0;
            int64_t head = 0; /* pollFirst over the sorted affected set */
            while (head < aff[ai].nverts) {
                int32_t rootV = aff[ai].verts[head++];
                memset(visited, 0, (size_t)b);
                memset(inq, 0, (size_t)b);
                /* BFS; the component set equals the reachable set regardless of order */
                int64_t qh = 0, qt = 0;
                visited[rootV] = 1;
                queue[qt++] = rootV;
                while (qh < qt) {
                    int32_t v = queue[qh++];
                    for (int64_t a = 0; a < adj[v].n; a++) {
                        int32_t u = adj[v].v[a];
                        if (!visited[u]) { visited[u] = 1; queue[qt++] = u; }
                    }
                }
                int32_t *comp = (int32_t *)malloc(sizeof(int32_t) * (size_t)qt);
                memcpy(comp, queue, sizeof(int32_t) * (size_t)qt);
                qsort(comp, (size_t)qt, sizeof(int32_t), cmp_i32);
                int64_t countMembers = 0;
                for (int64_t i = 0; i < qt; i++) countMembers += nB[comp[i]];
                if (countMembers >= mcl) {
                    cl_t c = {parentLabel, parentLabel, cw, JMAX, 0, (int32_t)countMembers, 0, comp, qt};
                    if (nnew == newcap) {
                        newcap = newcap ? newcap * 2 : 4;
                        newc = (cl_t *)realloc(newc, sizeof(cl_t) * (size_t)newcap);
                    }
                    newc[nnew++] = c;
                } else {
                    for (int64_t i = 0; i < qt; i++) label[comp[i]] = 0;
                    free(comp);
                    for (int64_t i = 0; i < clusters->n; i++) {
                        if (clusters->c[i].label == parentLabel && clusters->c[i].death == JMAX) {
                            int r2 = cl_detach(&clusters->c[i], (int32_t)countMembers, 0, cw);
                            if (r2) rc = r2;
                            break;
                        }
                    }
                    if (rc) break;
                }
            }
            if (rc == ORC_OK && nnew >= 2) {
                for (int64_t k = 0; k < nnew; k++) {
                    cl_t c = newc[k];
                    c.label = nextLabel;
                    for (int64_t i = 0; i < c.nmembers; i++) label[c.members[i]] = nextLabel;
                    nextLabel++;
                    for (int64_t i = 0; i < clusters->n; i++) {
                        if (clusters->c[i].label == c.parent && clusters->c[i].death == JMAX) {
                            clusters->c[i].hasChildren = 1;
                            int r2 = cl_detach(&clusters->c[i], c.numPoints, 0, c.birth);
                            if (r2) rc = r2;
                            break;
                        }
                    }
                    if (cl_push(clusters, c)) rc = ORC_ENOMEM;
                    newc[k].members = NULL;
                    if (rc) break;
                }
            }
            for (int64_t k = 0; k < nnew; k++) free(newc[k].members);
            free(newc);
        }
        for (int64_t k = 0; k < naff; k++) free(aff[k].verts);
        free(aff);
        if (rc) break;
    }
out:
    if (adj) for (int64_t i = 0; i < b; i++) free(adj[i].v);
    free(adj);
    free(label);
    free(visited);
    free(queue);
    free(inq);
    return rc;
}

/* adjacency record double[5] = {parentStability, childLabel, childStability, 1.0, parentParent} */
typedef struct { double v[5]; } rec_t;
typedef struct { int32_t key; rec_t *r; int64_t n, cap; int present; } adjnode_t;

static adjnode_t *adjnode_get(adjnode_t *m, int64_t nm, int32_t key) {
    for (int64_t i = 0; i < nm; i++) if (m[i].key == key && m[i].present) return &m[i];
    return NULL;
}

/* findProminentClustersAndClassificationNoiseBubbles (HdbscanDataBubbles.java:377-504). */
static int find_prominent(clvec *cl, const double *rep, const int32_t *nB, const double *eB,
                          const double *nnB, int64_t b, int d, int metric, const int32_t *id_bubbles,
                          int32_t *flat_label) {
    int rc = ORC_OK;
    /* clusterTree.remove(0): drop root */
    int64_t nt = cl->n - 1;
    cl_t *tree = cl->c + 1;
    /* adjacency lists (:391-412) */
    adjnode_t *m = (adjnode_t *)calloc((size_t)(nt + 1), sizeof(adjnode_t));
    int64_t nm = 0;
    for (int64_t pi = 0; pi < nt; pi++) {
        cl_t *par = &tree[pi];
        if (!par->hasChildren) {
            if (!adjnode_get(m, nm, par->label)) { m[nm].key = par->label; m[nm].present = 1; nm++; }
        }
        for (int64_t ci = 0; ci < nt; ci++) {
            cl_t *ch = &tree[ci];
            if (par->label == ch->parent) {
                adjnode_t *a = adjnode_get(m, nm, par->label);
                if (!a) { m[nm].key = par->label; m[nm].present = 1; a = &m[nm]; nm++; }
                if (a->n == a->cap) {
                    a->cap = a->cap ? a->cap * 2 : 4;
                    a->r = (rec_t *)realloc(a->r, sizeof(rec_t) * (size_t)a->cap);
                }
                rec_t r = {{par->stability, (double)ch->label, ch->stability, 1.0, (double)par->parent}};
                a->r[a->n++] = r;
            }
        }
    }
    /* stable sort of the tree by birth level (:414) -- insertion sort keeps stability */
    int64_t *ord = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nt > 0 ? nt : 1));
    for (int64_t i = 0; i < nt; i++) ord[i] = i;
    for (int64_t i = 1; i < nt; i++) {
        int64_t x = ord[i];
        int64_t j = i - 1;
        while (j >= 0) {
            double a = tree[ord[j]].birth, bb = tree[x].birth;
            if (a > bb) { ord[j + 1] = ord[j]; j--; } /* compare(o_j, x) > 0 => move */
            else break;
        }
        ord[j + 1] = x;
    }
    for (int64_t o = 0; o < b; o++) flat_label[o] = 0;
    /* solution TreeSet: represented as a membership flag by label */
    int32_t maxlab = 1;
    for (int64_t i = 0; i < nt; i++) if (tree[i].label > maxlab) maxlab = tree[i].label;
    unsigned char *sol = (unsigned char *)calloc((size_t)maxlab + 1, 1);
    for (int64_t i = 0; i < nt; i++) sol[tree[ord[i]].label] = 1;
    int32_t *q = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxlab + 2));
    unsigned char *vis = (unsigned char *)malloc((size_t)maxlab + 2);
    for (int64_t oi = 0; oi < nt; oi++) {
        int32_t key = tree[ord[oi]].label;
        adjnode_t *a = adjnode_get(m, nm, key);
        if (!a) { rc = ORC_EREF_NPE; break; }
        double childStab = 0.0;
        if (a->n > 0) {
            for (int64_t i = 0; i < a->n; i++) childStab += a->r[i].v[2];
            if (childStab <= a->r[0].v[0]) {
                for (int64_t i = 0; i < a->n; i++) {
                    memset(vis, 0, (size_t)maxlab + 2);
                    int32_t rootV = (int32_t)a->r[i].v[1];
                    /* TreeSet queue: pollFirst = smallest; the set of removals is
                     * order independent, so a plain worklist suffices */
                    int64_t qh = 0, qt = 0;
                    vis[rootV] = 1;
                    q[qt++] = rootV;
                    a->r[i].v[3] = 0.0;
                    sol[rootV] = 0;
                    while (qh < qt) {
                        int32_t v = q[qh++];
                        adjnode_t *av = adjnode_get(m, nm, v);
                        if (av) {
                            for (int64_t k = 0; k < av->n; k++) {
                                sol[v] = 0;
                                int32_t c = (int32_t)av->r[k].v[1];
                                if (!vis[c]) { q[qt++] = c; vis[c] = 1; }
                            }
                        }
                    }
                }
            } else {
                a->r[0].v[0] = childStab;
                adjnode_t *gp = adjnode_get(m, nm, (int32_t)a->r[0].v[4]);
                if (gp)
                    for (int64_t k = 0; k < gp->n; k++)
                        if ((int32_t)gp->r[k].v[1] == key) gp->r[k].v[2] = childStab;
            }
        } else {
            sol[key] = 0;
        }
    }
    if (rc == ORC_OK) {
        /* (:472-480) ascending-birth order; ascending solution labels inside */
        for (int64_t oi = 0; oi < nt; oi++) {
            cl_t *c = &tree[ord[oi]];
            if (c->label <= maxlab && sol[c->label]) {
                for (int64_t k = 0; k < c->nmembers; k++) {
                    int32_t mem = c->members[k];
                    if (mem < 0 || mem >= b) { rc = ORC_EREF_OOB; break; }
                    flat_label[mem] = c->label;
                }
            }
            if (rc) break;
        }
    }
    if (rc == ORC_OK) {
        /* noise reassignment (:485-502) */
        for (int64_t p = 0; p < b; p++) {
            double minD = JMAX;
            for (int64_t nb = 0; nb < b; nb++) {
                if (p == nb) continue;
                if (flat_label[p] == 0 && flat_label[nb] != 0) {
                    double dist = orc_distance(rep + p * d, rep + nb * d, d, metric);
                    dist = distance_bubbles(dist, eB, nnB, p, nb);
                    if (dist < minD) {
                        minD = dist;
                        flat_label[p] = flat_label[nb];
                    }
                }
            }
        }
    }
    (void)id_bubbles;
    for (int64_t i = 0; i < nm; i++) free(m[i].r);
    free(m);
    free(ord);
    free(sol);
    free(q);
    free(vis);
    return rc;
}

/* LocalModelReduceByKey.call (LocalModelReduceByKey.java:76-104).
 * info[b*3] = (extent, nnDist, n); nB = (int) info[:,2] (:80-84).
 * Outputs: labels[b]; sorted MST (ascending, quicksorted) in mst_va/vb/w (2b-1 each);
 * inter-cluster edges (:506-527) in ic_va/ic_vb/ic_w (capacity 2b-1), count in *n_ic. */
int orc_local_model(const double *rep, const double *info, int64_t b, int d, int min_pts, int min_cl_size,
                    int metric, int32_t *labels, int32_t *mst_va, int32_t *mst_vb, double *mst_w,
                    int32_t *ic_va, int32_t *ic_vb, double *ic_w, int64_t *n_ic) {
    if (b < 1) return ORC_EINVAL;
    int rc;
    double *eB = (double *)malloc(sizeof(double) * (size_t)b);
    double *nnB = (double *)malloc(sizeof(double) * (size_t)b);
    int32_t *nB = (int32_t *)malloc(sizeof(int32_t) * (size_t)b);
    int32_t *ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)b);
    double *core = (double *)malloc(sizeof(double) * (size_t)b);
    clvec cl = {NULL, 0, 0};
    for (int64_t i = 0; i < b; i++) {
        eB[i] = info[i * 3 + 0];
        nnB[i] = info[i * 3 + 1];
        nB[i] = (int32_t)info[i * 3 + 2];
        ids[i] = (int32_t)i;
    }
    int64_t ne = 2 * b - 1;
    rc = orc_bubble_core_distances(rep, nB, eB, nnB, b, d, min_pts, metric, core);
    if (rc) goto out;
    rc = orc_bubble_prim_mst(rep, eB, nnB, ids, core, b, d, metric, 1, mst_va, mst_vb, mst_w);
    if (rc) goto out;
    rc = orc_quicksort_edges(mst_va, mst_vb, mst_w, ne);
    if (rc) goto out;
    rc = construct_cluster_tree(b, mst_va, mst_vb, mst_w, ne, min_cl_size, nB, &cl);
    if (rc) goto out;
    rc = find_prominent(&cl, rep, nB, eB, nnB, b, d, metric, ids, labels);
    if (rc) goto out;
    {
        int64_t k = 0;
        for (int64_t i = 0; i < ne; i++) {
            if (labels[mst_va[i]] != labels[mst_vb[i]]) {
                ic_va[k] = mst_va[i];
                ic_vb[k] = mst_vb[i];
                ic_w[k] = mst_w[i];
                k++;
            }
        }
        *n_ic = k;
    }
out:
    for (int64_t i = 0; i < cl.n; i++) free(cl.c[i].members);
    free(cl.c);
    free(eB);
    free(nnB);
    free(nB);
    free(ids);
    free(core);
    return rc;
}

/* Per-row core distances (INCL/EXCL semantics) for a subset of query rows against all n
 * points -- the bounded CPU-baseline sample of bench.py (same loop as orc_core_distances). */
int orc_core_rows(const double *X, int64_t n, int d, const int64_t *rows, int64_t nr, int min_pts, int metric,
                  int excl_self, double *core) {
    if (min_pts < 2) return ORC_EINVAL;
    int K = min_pts - 1;
    double *buf = (double *)malloc(sizeof(double) * K);
    if (!buf) return ORC_ENOMEM;
    for (int64_t r = 0; r < nr; r++) {
        int64_t p = rows[r];
        for (int i = 0; i < K; i++) buf[i] = JMAX;
        for (int64_t q = 0; q < n; q++) {
            if (excl_self && p == q) continue;
            knn_insert(buf, K, orc_distance(X + p * d, X + q * d, d, metric));
        }
        core[r] = buf[K - 1];
    }
    free(buf);
    return ORC_OK;
}

/* ------------------------------------------------ CPU-all baseline (bench.py only)
 * the line-faithful loops above, with OpenMP over independent units standing
 * in for Spark local[*].  Results are identical to the serial functions: each query row is
 * independent (orc_core_rows), and the Prim step's parallel scan combines per-thread
 * candidates with the reference select rule (smaller value; equal values -> larger index,
 * HDBSCANStar.java:177-180 '<='), the update rule (:170-173) being per-vertex. */
#ifdef _OPENMP
#include <omp.h>
#endif

int orc_core_rows_par(const double *X, int64_t n, int d, const int64_t *rows, int64_t nr, int min_pts, int metric,
                      int excl_self, int nthreads, double *core) {
    if (min_pts < 2 || nthreads < 1) return ORC_EINVAL;
    int K = min_pts - 1;
    int rc = ORC_OK;
#pragma omp parallel num_threads(nthreads)
    {
        double *buf = (double *)malloc(sizeof(double) * K);
        if (!buf) {
#pragma omp atomic write
            rc = ORC_ENOMEM;
        }
#pragma omp for schedule(dynamic, 4)
        for (int64_t r = 0; r < nr; r++) {
            if (!buf) continue;
            int64_t p = rows[r];
            for (int i = 0; i < K; i++) buf[i] = JMAX;
            for (int64_t q = 0; q < n; q++) {
                if (excl_self && p == q) continue;
                knn_insert(buf, K, orc_distance(X + p * d, X + q * d, d, metric));
            }
            core[r] = buf[K - 1];
        }
        free(buf);
    }
    return rc;
}

int orc_prim_mst_par(const double *X, int64_t n, int d, const double *core, int metric, int nthreads, int32_t *va,
                     int32_t *vb, double *w) {
    if (n < 1 || d <= 0 || nthreads < 1) return ORC_EINVAL;
    unsigned char *attached = (unsigned char *)calloc((size_t)n, 1);
    int32_t *parent = (int32_t *)calloc((size_t)n, sizeof(int32_t));
    double *best = (double *)malloc(sizeof(double) * (size_t)n);
    double *cand_d = (double *)malloc(sizeof(double) * (size_t)nthreads);
    int64_t *cand_i = (int64_t *)malloc(sizeof(int64_t) * (size_t)nthreads);
    if (!attached || !parent || !best || !cand_d || !cand_i) {
        free(attached); free(parent); free(best); free(cand_d); free(cand_i);
        return ORC_ENOMEM;
    }
    for (int64_t i = 0; i < n; i++) best[i] = JMAX;
    best[n - 1] = 0;
    int64_t cur = n - 1;
    attached[n - 1] = 1;
    int rc = ORC_OK;
#pragma omp parallel num_threads(nthreads)
    {
        int t = 0, T = 1;
#ifdef _OPENMP
        t = omp_get_thread_num();
        T = omp_get_num_threads();
#endif
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        for (int64_t step = 1; step < n; step++) {
            const int64_t c = cur;  /* read after the previous step's barrier */
            double nd = JMAX;
            int64_t np = -1;
            for (int64_t nb = lo; nb < hi; nb++) {
                if (c == nb || attached[nb]) continue;
                double mrd = orc_distance(X + c * d, X + nb * d, d, metric);
                if (core[c] > mrd) mrd = core[c];
                if (core[nb] > mrd) mrd = core[nb];
                if (mrd < best[nb]) {
                    best[nb] = mrd;
                    parent[nb] = (int32_t)c;
                }
                if (best[nb] <= nd) {
                    nd = best[nb];
                    np = nb;
                }
            }
            cand_d[t] = nd;
            cand_i[t] = np;
#pragma omp barrier
#pragma omp single
            {
                double bd = JMAX;
                int64_t bi = -1;
                for (int k = 0; k < T; k++)  /* ascending ranges: '<=' keeps the last minimum */
                    if (cand_i[k] >= 0 && cand_d[k] <= bd) {
                        bd = cand_d[k];
                        bi = cand_i[k];
                    }
                if (bi < 0) rc = ORC_EREF_OOB;
                else {
                    attached[bi] = 1;
                    cur = bi;
                }
            } /* implicit barrier */
            if (rc != ORC_OK) break;
        }
    }
    if (rc == ORC_OK)
        for (int64_t i = 0; i < n - 1; i++) {
            va[i] = parent[i];
            vb[i] = (int32_t)i;
            w[i] = best[i];
        }
    free(attached); free(parent); free(best); free(cand_d); free(cand_i);
    return rc;
}
