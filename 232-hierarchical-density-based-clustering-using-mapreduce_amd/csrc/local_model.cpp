// local_model.cpp -- host side of LocalModelReduceByKey (LocalModelReduceByKey.java:88-104).
//
// The b^2 work (bubble k-NN, bubble Prim) runs in the HIP kernels; what stays here is the
// O(b)-state logic whose result depends on Java collection semantics:
//   * the bubble-core formula over the never-reset indexBubbles[] (HdbscanDataBubbles.java:121-143),
//   * UndirectedGraph.quicksortByEdgeWeight (UndirectedGraph.java:93-208),
//   * constructClusterTree (HdbscanDataBubbles.java:256-375) incl. java.util.HashMap key order,
//   * findProminentClustersAndClassificationNoiseBubbles (:377-504),
//   * findInterClusterEdges (:506-527).
// Host C++ built with -ffp-contract=off so the few host distance evaluations match Java.
#include <cstdio>
#include <algorithm>
#include <deque>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

#include "internal.hpp"

namespace hdb {

// ------------------------------------------------------------- host metrics
static double host_distance(const double *a, const double *b, int d, int metric) {
    switch (metric) {
    case HDB_METRIC_EUCLIDEAN: {
        double s = 0;
        for (int i = 0; i < d; i++) s += ((a[i] - b[i]) * (a[i] - b[i]));
        return std::sqrt(s);
    }
    case HDB_METRIC_COSINE: {
        double dot = 0, m1 = 0, m2 = 0;
        for (int i = 0; i < d; i++) {
            dot += (a[i] * b[i]);
            m1 += (a[i] * a[i]);
            m2 += (b[i] * b[i]);
        }
        return 1 - (dot / std::sqrt(m1 * m2));
    }
    case HDB_METRIC_PEARSON: {
        double mean1 = 0, mean2 = 0;
        for (int i = 0; i < d; i++) {
            mean1 += a[i];
            mean2 += b[i];
        }
        mean1 = mean1 / d;
        mean2 = mean2 / d;
        double cov = 0, s1 = 0, s2 = 0;
        for (int i = 0; i < d; i++) {
            cov += ((a[i] - mean1) * (b[i] - mean2));
            s1 += ((a[i] - mean1) * (a[i] - mean1));
            s2 += ((b[i] - mean2) * (b[i] - mean2));
        }
        return (1 - (cov / std::sqrt(s1 * s2)));
    }
    case HDB_METRIC_MANHATTAN: {
        double s = 0;
        for (int i = 0; i < d; i++) s += std::fabs(a[i] - b[i]);
        return s;
    }
    default: {
        double s = 0;
        for (int i = 0; i < d; i++) {
            double df = std::fabs(a[i] - b[i]);
            if (df > s) s = df;
        }
        return s;
    }
    }
}

static double host_distance_bubbles(double distance, const double *eB, const double *nnB, int64_t p, int64_t q) {
    double verify = distance - (eB[p] + eB[q]);
    if (verify >= 0) return (distance - (eB[p] + eB[q])) + (nnB[p] + nnB[q]);
    if (std::isnan(nnB[p]) || std::isnan(nnB[q])) return NAN;
    return nnB[p] >= nnB[q] ? nnB[p] : nnB[q];
}

// ------------------------------------------- bubble core formula (epilogue)
// knn/log from bubble_knn_kernel; indexBubbles state carried across points in order.
int bubble_core_epilogue(const double *rep, const int32_t *nB, const double *eB, const double *nnB, int64_t b, int d,
                         int min_pts, int metric, const double *knn, const int32_t *log, double *core) {
    const int K = min_pts - 1;
    for (int64_t i = 0; i < b; i++) core[i] = 0;
    if (min_pts == 1) return HDB_OK;
    std::vector<int32_t> idx(K, 0);  // indexBubbles, zero-initialised once (:79-83)
    const int inv_d = 1 / d;
    for (int64_t p = 0; p < b; p++) {
        for (int k = 0; k < K; k++)
            if (log[p * K + k] >= 0) idx[k] = log[p * K + k];
        const double *kn = knn + p * K;
        if (nB[p] >= K) {
            core[p] = std::pow((double)(K / nB[p]), (double)inv_d) * eB[p];
        } else {
            int32_t nX = nB[p];
            int i = 0;
            while (nX < K) {
                if (i >= K) return HDB_EREF_OOB;
                nX += nB[idx[i]];
                i += 1;
            }
            int32_t sum = nB[p];
            int32_t aux = 0;
            if (i >= b) return HDB_EREF_OOB;
            for (int j = 0; j < i; j++) {
                double dc = host_distance(rep + (int64_t)idx[j] * d, rep + (int64_t)i * d, d, metric);
                dc = host_distance_bubbles(dc, eB, nnB, idx[j], i);
                if (sum < K && kn[j] < dc) aux = K - sum;
                sum += nB[idx[j]];
            }
            if (i >= K) return HDB_EREF_OOB;
            if (nB[i] == 0) return HDB_EREF_DIVZERO;
            core[p] = kn[i] + std::pow((double)(aux / nB[i]), (double)inv_d) * eB[i];
        }
    }
    return HDB_OK;
}

// --------------------------------------------------------------- quicksort
int quicksort_edges(int32_t *va, int32_t *vb, double *w, int64_t ne) {
    if (ne <= 1) return HDB_OK;
    const int64_t cap = ne / 2;  // new int[edgeWeights.length / 2] (:97-98)
    std::vector<int64_t> ss(cap), es(cap);
    // the three parallel arrays as one array of 16-byte records while sorting: the same
    // comparisons and swaps in the same order (so the same unstable result), one line per swap
    // instead of three (round 6: the 16,384-bubble models' 32,767-edge sorts, C5's critical path)
    struct E {
        double w;
        int32_t a, b;
    };
    std::vector<E> r((size_t)ne);
    for (int64_t i = 0; i < ne; i++) r[i] = E{w[i], va[i], vb[i]};
    struct Out {  // writes the records back however the sort ends
        E *r;
        int32_t *va, *vb;
        double *w;
        int64_t ne;
        ~Out() {
            for (int64_t i = 0; i < ne; i++) {
                w[i] = r[i].w;
                va[i] = r[i].a;
                vb[i] = r[i].b;
            }
        }
    } out{r.data(), va, vb, w, ne};
    auto swp = [&](int64_t i, int64_t j) {
        if (i == j) return;
        std::swap(r[i], r[j]);
    };
    auto wt = [&](int64_t i) { return r[i].w; };
    ss[0] = 0;
    es[0] = ne - 1;
    int64_t top = 0;
    while (top >= 0) {
        const int64_t s = ss[top], e = es[top];
        top--;
        const double pv = wt(s);  // selectPivotIndex always returns startIndex (:158)
        swp(s, e);
        int64_t low = s;
        E *R = r.data();
        for (int64_t i = s; i < e; i++) {  // if (w[i] < pv) swap(i, low++), without the branch
            const E x = R[i];
            const bool c = x.w < pv;
            const int64_t dst = c ? low : i;  // not taken: R[i] rewritten with itself
            R[i] = R[dst];
            R[dst] = x;
            low += c;
        }
        swp(low, e);
        const int64_t pivot = low;
        if (pivot > s + 1) {
            if (top + 1 >= cap) return HDB_EREF_OOB;
            ss[top + 1] = s;
            es[top + 1] = pivot - 1;
            top++;
        }
        if (pivot < e - 1) {
            if (top + 1 >= cap) return HDB_EREF_OOB;
            ss[top + 1] = pivot + 1;
            es[top + 1] = e;
            top++;
        }
    }
    return HDB_OK;
}

// ------------------------------------------------------------ cluster tree
struct Cl {
    int32_t label, parent;
    double birth, death = JMAX, stability = 0;
    int32_t numPoints;
    bool hasChildren = false;
    std::vector<int32_t> members;  // TreeSet order (BFS path)
    int32_t node = -1;             // fast path: members = leaves of this dendrogram node
    int32_t any_member = -1;       // fast path, while a candidate: one member (locates its group)
};

// Component dendrogram of the (quicksorted) MST edge list, built bottom-up: the component a
// vertex belongs to after the top-down walk has removed edges [j, ne) is the union-find
// state after edges [0, j).  Leaves 0..b-1 are the vertices; node k >= b merges l, r.
struct Dendro {
    int64_t b = 0;
    std::vector<int32_t> l, r;     // children of internal node b + k
    std::vector<int64_t> sum_nb;   // sum of nB over the node's vertices
    std::vector<int32_t> size;     // vertex count
    template <class F>
    void leaves(int32_t node, std::vector<int32_t> &stk, F &&f) const {
        stk.assign(1, node);
        while (!stk.empty()) {
            int32_t x = stk.back();
            stk.pop_back();
            if (x < b) {
                f(x);
                continue;
            }
            stk.push_back(r[x - b]);
            stk.push_back(l[x - b]);
        }
    }
};

thread_local char g_lm_detail[160];  // the reference's exception message + where it arose

const char *local_model_error_detail() { return g_lm_detail; }

static int detach(Cl &c, int32_t numPoints, double level) {  // Clusters.java:39-47
    c.numPoints -= numPoints;
    c.stability += ((double)(numPoints + 0) * (1 / level - 1 / c.birth));
    if (c.numPoints == 0) c.death = level;
    else if (c.numPoints < 0) {
        snprintf(g_lm_detail, sizeof(g_lm_detail),
                 "Cluster cannot have less than 0 points. (label %d, level %.17g, numPoints %d)", (int)c.label, level,
                 (int)c.numPoints);
        return HDB_EREF_NEGATIVE_CLUSTER;
    }
    return HDB_OK;
}

static uint32_t jhash(int32_t k) {
    uint32_t h = (uint32_t)k;
    return h ^ (h >> 16);
}

// Final capacity of a java.util.HashMap<Integer, ...> after putting `labels` (insertion
// order) into a fresh map: 16 at the first put, doubled when size > 0.75 cap, and doubled
// when a 9th key lands in one bucket of a table below 64 buckets (treeifyBin resizes
// instead).  At >= 64 buckets such a bin becomes a tree bin, whose iteration order is not
// emulated: -1 (HDB_EUNSUPPORTED).  Resizes split buckets order-preservingly, so the keySet
// order is (bucket at the final capacity, insertion order).
template <class T>
static int32_t jlabel(const T &x) { return x.label; }
template <class T>
static int32_t jlabel(T *const &x) { return x->label; }
template <class Label>
static int64_t jmap_capacity(const std::vector<Label> &aff) {
    int64_t cap = 16;
    thread_local std::vector<int32_t> cnt;  // reused across calls (one call per weight run)
    cnt.assign(cap, 0);
    auto recount = [&](size_t upto) {
        cnt.assign(cap, 0);
        for (size_t j = 0; j <= upto; j++) cnt[jhash(jlabel(aff[j])) & (uint32_t)(cap - 1)]++;
    };
    for (size_t i = 0; i < aff.size(); i++) {
        const int32_t before = cnt[jhash(jlabel(aff[i])) & (uint32_t)(cap - 1)]++;
        if (before >= 8) {
            if (cap >= 64) return -1;
            cap *= 2;
            recount(i);
        }
        if ((int64_t)(i + 1) > cap * 3 / 4) {
            cap *= 2;
            recount(i);
        }
    }
    return cap;
}


// Fast equivalent of construct_cluster_tree_bfs below: the same top-down control flow
// (tie runs from the heaviest, HashMap order of affected labels, TreeSet order of affected
// vertices, one "BFS" per affected vertex including the reference's re-processing of an
// already-explored component), but a component is read off the dendrogram instead of
// being re-explored: Sigma nB and the vertex set come from the pre-run union-find node.
// Labels are kept per component group (every live component owns one group; on a split all
// pieces but the largest move to fresh groups -- small-to-large, O(b log b) moves), so
// labelling a component noise or a new cluster is O(1).  Returns 1 (not an error) when the
// edges are not a forest plus self edges; the caller then runs the BFS version.
static int construct_cluster_tree_fast(int64_t b, const int32_t *ea, const int32_t *eb, const double *ew, int64_t ne,
                                       int32_t mcl, const int32_t *nB, std::vector<Cl> &clusters, Dendro &D) {
    for (int64_t i = 0; i < ne; i++) {
        if (ea[i] < 0 || ea[i] >= b || eb[i] < 0 || eb[i] >= b) return HDB_EREF_OOB;
        if (ew[i] != ew[i]) return HDB_EUNSUPPORTED;  // NaN level: the reference's walk never advances
    }
    // ---- bottom-up: pre-run component node of every edge endpoint
    D.b = b;
    D.l.clear();
    D.r.clear();
    D.sum_nb.assign((size_t)b, 0);
    D.size.assign((size_t)b, 1);
    for (int64_t v = 0; v < b; v++) D.sum_nb[v] = nB[v];
    std::vector<int32_t> uf((size_t)b), node_of((size_t)b);
    for (int64_t v = 0; v < b; v++) uf[v] = node_of[v] = (int32_t)v;
    auto find = [&](int32_t x) {
        while (uf[x] != x) {
            uf[x] = uf[uf[x]];
            x = uf[x];
        }
        return x;
    };
    std::vector<int32_t> pre_a((size_t)ne), pre_b((size_t)ne);
    for (int64_t lo = 0; lo < ne;) {
        int64_t hi = lo;
        while (hi + 1 < ne && ew[hi + 1] == ew[lo]) hi++;  // a run, as the top-down walk groups it
        for (int64_t i = lo; i <= hi; i++) {
            pre_a[i] = node_of[find(ea[i])];
            pre_b[i] = node_of[find(eb[i])];
        }
        for (int64_t i = lo; i <= hi; i++) {
            if (ea[i] == eb[i]) continue;
            int32_t x = find(ea[i]), y = find(eb[i]);
            if (x == y) return 1;  // a cycle: not a tree
            const int32_t nx = node_of[x], ny = node_of[y];
            const int32_t k = (int32_t)(b + (int64_t)D.l.size());
            D.l.push_back(nx);
            D.r.push_back(ny);
            D.sum_nb.push_back(D.sum_nb[nx] + D.sum_nb[ny]);
            D.size.push_back(D.size[nx] + D.size[ny]);
            uf[y] = x;
            node_of[x] = k;
        }
        lo = hi + 1;
    }
    // ---- top-down replay
    std::vector<int32_t> group((size_t)b, 0), gsize(1, (int32_t)b), glabel(1, 1);
    auto lab = [&](int32_t v) { return glabel[group[v]]; };
    int32_t nextLabel = 2;
    int64_t all = 0;
    for (int64_t i = 0; i < b; i++) all += nB[i];
    {
        Cl root;
        root.label = 1;
        root.parent = -1;
        root.birth = NAN;
        root.numPoints = (int32_t)all;
        clusters.push_back(root);
    }
    std::vector<int32_t> idx_of(2, -1);
    idx_of.reserve((size_t)b + 2);
    idx_of[1] = 0;
    std::vector<int32_t> pre((size_t)b, -1);  // pre-run node of an endpoint (this run)
    std::vector<int32_t> stk;
    struct Aff {
        int32_t label;
        int64_t order;
        std::vector<int32_t> verts;
    };
    struct Piece {
        int32_t g, node;
    };
    std::vector<Piece> pieces;
    std::vector<int32_t> best_of_group;  // scratch: group -> index of its largest piece
    // per-run scratch kept across runs (one run per distinct weight: ~b runs, so per-run
    // vectors cost several heap allocations each); entries [0, naff) are live
    std::deque<Aff> aff_pool;  // a deque: growing it keeps the pointers in `aff` valid
    std::vector<Aff *> aff;
    std::vector<Cl> newc;
    int64_t cur = ne - 1;
    while (cur >= 0) {
        aff.clear();
        size_t naff = 0;
        const double cw = ew[cur];
        const int64_t run_hi = cur;
        while (cur >= 0 && ew[cur] == cw) {
            const int32_t f = ea[cur], s = eb[cur];
            pre[f] = pre_a[cur];
            pre[s] = pre_b[cur];
            if (lab(f) == 0) {
                cur--;
                continue;
            }
            size_t k = 0;
            for (; k < aff.size(); k++)
                if (aff[k]->label == lab(f)) break;
            if (k == aff.size()) {
                if (naff == aff_pool.size()) aff_pool.emplace_back();
                Aff &A = aff_pool[naff++];
                A.label = lab(f);
                A.order = (int64_t)aff.size();
                A.verts.clear();
                aff.push_back(&A);
            }
            for (int32_t v : {f, s}) {
                auto &vs = aff[k]->verts;
                auto it = std::lower_bound(vs.begin(), vs.end(), v);
                if (it == vs.end() || *it != v) vs.insert(it, v);
            }
            cur--;
        }
        // the run split live components into pieces: keep each component's largest piece in
        // its group, move the others to fresh groups (labels unchanged)
        pieces.clear();
        for (int64_t i = cur + 1; i <= run_hi; i++) {
            if (ea[i] == eb[i]) continue;
            for (int32_t v : {ea[i], eb[i]}) {
                const int32_t nd = (v == ea[i]) ? pre_a[i] : pre_b[i];
                if (lab(v) == 0) continue;  // noise components are never relabelled
                pieces.push_back(Piece{group[v], nd});
            }
        }
        if (!pieces.empty()) {
            if (pieces.size() > 1)
                std::sort(pieces.begin(), pieces.end(), [](const Piece &x, const Piece &y) {
                    return x.g < y.g || (x.g == y.g && x.node < y.node);
                });
            pieces.erase(std::unique(pieces.begin(), pieces.end(),
                                     [](const Piece &x, const Piece &y) { return x.g == y.g && x.node == y.node; }),
                         pieces.end());
            for (size_t a = 0; a < pieces.size();) {
                size_t e = a;
                size_t big = a;
                while (e < pieces.size() && pieces[e].g == pieces[a].g) {
                    if (D.size[pieces[e].node] > D.size[pieces[big].node]) big = e;
                    e++;
                }
                for (size_t q = a; q < e; q++) {
                    if (q == big) continue;
                    const int32_t ng = (int32_t)glabel.size();
                    glabel.push_back(glabel[pieces[q].g]);
                    gsize.push_back(D.size[pieces[q].node]);
                    gsize[pieces[q].g] -= D.size[pieces[q].node];
                    D.leaves(pieces[q].node, stk, [&](int32_t v) { group[v] = ng; });
                }
                a = e;
            }
        }
        if (aff.empty()) continue;
        const int64_t cap = jmap_capacity(aff);
        if (cap < 0) return HDB_EUNSUPPORTED;
        // keySet order: (bucket, insertion order) -- a stable insertion sort (a run touches few
        // labels; std::stable_sort would allocate a buffer per run)
        for (size_t i = 1; i < aff.size(); i++) {
            Aff *x = aff[i];
            const uint32_t bx = jhash(x->label) & (uint32_t)(cap - 1);
            size_t j = i;
            while (j > 0 && (jhash(aff[j - 1]->label) & (uint32_t)(cap - 1)) > bx) {
                aff[j] = aff[j - 1];
                j--;
            }
            aff[j] = x;
        }
        for (const Aff *Ap : aff) {
            const Aff &A = *Ap;
            const int32_t parentLabel = A.label;
            newc.clear();
            for (int32_t rootV : A.verts) {
                const int32_t nd = pre[rootV];
                const int64_t countMembers = D.sum_nb[nd];
                if (countMembers >= mcl) {
                    Cl c;
                    c.label = parentLabel;
                    c.parent = parentLabel;
                    c.birth = cw;
                    c.numPoints = (int32_t)countMembers;
                    c.node = nd;
                    c.any_member = rootV;  // locates the piece's group
                    newc.push_back(std::move(c));
                } else {
                    glabel[group[rootV]] = 0;  // the piece is exactly this group
                    const int32_t ci = parentLabel < (int32_t)idx_of.size() ? idx_of[parentLabel] : -1;
                    if (ci >= 0 && clusters[ci].death == JMAX) {
                        int rc = detach(clusters[ci], (int32_t)countMembers, cw);
                        if (rc) return rc;
                    }
                }
            }
            if (newc.size() >= 2) {
                for (auto &c : newc) {
                    c.label = nextLabel;
                    glabel[group[c.any_member]] = nextLabel;
                    c.any_member = -1;
                    nextLabel++;
                    const int32_t pi = c.parent < (int32_t)idx_of.size() ? idx_of[c.parent] : -1;
                    if (pi >= 0 && clusters[pi].death == JMAX) {
                        clusters[pi].hasChildren = true;
                        int rc = detach(clusters[pi], c.numPoints, c.birth);
                        if (rc) return rc;
                    }
                    if ((int32_t)idx_of.size() <= c.label) idx_of.resize((size_t)c.label + 1, -1);
                    idx_of[c.label] = (int32_t)clusters.size();
                    clusters.push_back(std::move(c));
                }
            }
        }
    }
    return HDB_OK;
}

static int construct_cluster_tree_bfs(int64_t b, const int32_t *ea, const int32_t *eb, const double *ew, int64_t ne,
                                  int32_t mcl, const int32_t *nB, std::vector<Cl> &clusters) {
    std::vector<std::vector<int32_t>> adj(b);
    for (int64_t i = 0; i < ne; i++) {
        int32_t v1 = ea[i], v2 = eb[i];
        if (v1 < 0 || v1 >= b || v2 < 0 || v2 >= b) return HDB_EREF_OOB;
        adj[v1].push_back(v2);
        if (v1 != v2) adj[v2].push_back(v1);
    }
    auto remove_first = [](std::vector<int32_t> &v, int32_t x) {
        auto it = std::find(v.begin(), v.end(), x);
        if (it != v.end()) v.erase(it);
    };
    std::vector<int32_t> label(b, 1);
    int32_t nextLabel = 2;
    int64_t all = 0;
    for (int64_t i = 0; i < b; i++) all += nB[i];
    {
        Cl root;
        root.label = 1;
        root.parent = -1;
        root.birth = NAN;
        root.numPoints = (int32_t)all;
        clusters.push_back(root);
    }
    std::vector<int32_t> idx_of(2, -1);  // cluster label -> index in `clusters`
    idx_of[1] = 0;
    std::vector<uint32_t> stamp(b, 0);
    uint32_t gen = 0;
    std::vector<int32_t> queue;
    queue.reserve(b);

    struct Aff {
        int32_t label;
        int64_t order;
        std::vector<int32_t> verts;  // sorted unique (TreeSet)
    };
    int64_t cur = ne - 1;
    while (cur >= 0) {
        std::vector<Aff> aff;
        const double cw = ew[cur];
        while (cur >= 0 && ew[cur] == cw) {
            const int32_t f = ea[cur], s = eb[cur];
            remove_first(adj[f], s);
            remove_first(adj[s], f);
            if (label[f] == 0) {
                cur--;
                continue;
            }
            size_t k = 0;
            for (; k < aff.size(); k++)
                if (aff[k].label == label[f]) break;
            if (k == aff.size()) aff.push_back(Aff{label[f], (int64_t)aff.size(), {}});
            for (int32_t v : {f, s}) {
                auto &vs = aff[k].verts;
                auto it = std::lower_bound(vs.begin(), vs.end(), v);
                if (it == vs.end() || *it != v) vs.insert(it, v);
            }
            cur--;
        }
        if (aff.empty()) continue;
        // java.util.HashMap key iteration: bucket order, insertion order inside a bucket
        const int64_t cap = jmap_capacity(aff);
        if (cap < 0) return HDB_EUNSUPPORTED;
        std::stable_sort(aff.begin(), aff.end(), [&](const Aff &x, const Aff &y) {
            uint32_t bx = jhash(x.label) & (uint32_t)(cap - 1), by = jhash(y.label) & (uint32_t)(cap - 1);
            if (bx != by) return bx < by;
            return x.order < y.order;
        });
        for (auto &A : aff) {
            const int32_t parentLabel = A.label;
            std::vector<Cl> newc;
            for (int32_t rootV : A.verts) {  // pollFirst over the TreeSet
                if (++gen == 0) {
                    std::fill(stamp.begin(), stamp.end(), 0);
                    gen = 1;
                }
                queue.clear();
                stamp[rootV] = gen;
                queue.push_back(rootV);
                for (size_t h = 0; h < queue.size(); h++) {
                    int32_t v = queue[h];
                    for (int32_t u : adj[v])
                        if (stamp[u] != gen) {
                            stamp[u] = gen;
                            queue.push_back(u);
                        }
                }
                int64_t countMembers = 0;
                for (int32_t v : queue) countMembers += nB[v];
                if (countMembers >= mcl) {
                    Cl c;
                    c.label = parentLabel;
                    c.parent = parentLabel;
                    c.birth = cw;
                    c.numPoints = (int32_t)countMembers;
                    c.members = queue;
                    std::sort(c.members.begin(), c.members.end());
                    newc.push_back(std::move(c));
                } else {
                    for (int32_t v : queue) label[v] = 0;
                    // first live cluster with that label (labels are unique in `clusters`)
                    const int32_t ci = parentLabel < (int32_t)idx_of.size() ? idx_of[parentLabel] : -1;
                    if (ci >= 0 && clusters[ci].death == JMAX) {
                        int rc = detach(clusters[ci], (int32_t)countMembers, cw);
                        if (rc) return rc;
                    }
                }
            }
            if (newc.size() >= 2) {
                for (auto &c : newc) {
                    c.label = nextLabel;
                    for (int32_t v : c.members) label[v] = nextLabel;
                    nextLabel++;
                    const int32_t pi = c.parent < (int32_t)idx_of.size() ? idx_of[c.parent] : -1;
                    if (pi >= 0 && clusters[pi].death == JMAX) {
                        clusters[pi].hasChildren = true;
                        int rc = detach(clusters[pi], c.numPoints, c.birth);
                        if (rc) return rc;
                    }
                    if ((int32_t)idx_of.size() <= c.label) idx_of.resize((size_t)c.label + 1, -1);
                    idx_of[c.label] = (int32_t)clusters.size();
                    clusters.push_back(std::move(c));
                }
            }
        }
    }
    return HDB_OK;
}

static int find_prominent(std::vector<Cl> &cl, const double *rep, const double *eB, const double *nnB, int64_t b,
                          int d, int metric, int32_t *flat, const Dendro *D) {
    // clusterTree.remove(0)
    std::vector<Cl *> tree;
    for (size_t i = 1; i < cl.size(); i++) tree.push_back(&cl[i]);
    // adjListNodes: label -> list of double[5] (kept as a map in insertion-independent form)
    struct Rec {
        double v[5];
    };
    struct Span {  // one label's list in the flat record array
        Rec *b_, *e_;
        bool empty() const { return b_ == e_; }
        Rec &operator[](size_t i) { return b_[i]; }
        Rec *begin() { return b_; }
        Rec *end() { return e_; }
    };
    // label -> slot index (labels are small ints; dense lookup table)
    int32_t maxlab = 1;
    for (auto *c : tree) maxlab = std::max(maxlab, c->label);
    std::vector<int> slot(maxlab + 2, -1);
    int nslots = 0;
    auto put = [&](int32_t key) {
        if (key >= 0 && key <= maxlab && slot[key] < 0) slot[key] = nslots++;
    };
    // for par in tree: for ch in tree: par.label == ch.parent -> adj[par] += ch (tree order);
    // labels are unique, so one pass over the children builds the same lists -- laid out as one
    // flat array (counted, then filled in tree order: each list keeps the child order)
    std::vector<Cl *> by_label(maxlab + 2, nullptr);
    for (auto *c : tree) by_label[c->label] = c;
    auto parent_of = [&](const Cl *ch) -> Cl * {
        if (ch->parent < 0 || ch->parent > maxlab) return nullptr;
        return by_label[ch->parent];
    };
    for (auto *par : tree)
        if (!par->hasChildren) put(par->label);
    for (auto *ch : tree)
        if (Cl *par = parent_of(ch)) put(par->label);
    std::vector<int64_t> roff((size_t)nslots + 1, 0);
    for (auto *ch : tree)
        if (Cl *par = parent_of(ch)) roff[(size_t)slot[par->label] + 1]++;
    for (int i = 0; i < nslots; i++) roff[i + 1] += roff[i];
    std::vector<Rec> recs((size_t)roff[nslots]);
    std::vector<int64_t> rpos(roff.begin(), roff.end() - 1);
    for (auto *ch : tree)
        if (Cl *par = parent_of(ch))
            recs[(size_t)rpos[slot[par->label]]++] =
                Rec{{par->stability, (double)ch->label, ch->stability, 1.0, (double)par->parent}};
    std::vector<Span> spans((size_t)nslots);
    for (int i = 0; i < nslots; i++) spans[i] = Span{recs.data() + roff[i], recs.data() + roff[i + 1]};
    auto get = [&](int32_t key) -> Span * {
        if (key < 0 || key > maxlab || slot[key] < 0) return nullptr;
        return &spans[slot[key]];
    };
    // Collections.sort by birth level (stable)
    using fclk = std::chrono::steady_clock;
    auto fus = [](fclk::time_point a, fclk::time_point b) {
        return (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
    };
    const auto f0 = fclk::now();
    // (birth, position) pairs sorted with the same comparison on a copy of the key: the same
    // stable order without chasing a Cl pointer per comparison
    std::vector<std::pair<double, int32_t>> kb(tree.size());
    for (size_t i = 0; i < tree.size(); i++) kb[i] = {tree[i]->birth, (int32_t)i};
    std::stable_sort(kb.begin(), kb.end(),
                     [](const std::pair<double, int32_t> &a, const std::pair<double, int32_t> &b) { return a.first < b.first; });
    std::vector<Cl *> sorted(tree.size());
    for (size_t i = 0; i < tree.size(); i++) sorted[i] = tree[kb[i].second];
    for (int64_t o = 0; o < b; o++) flat[o] = 0;
    std::vector<char> sol(maxlab + 2, 0);
    for (auto *c : sorted) sol[c->label] = 1;
    std::vector<uint32_t> vis(maxlab + 2, 0);  // generation stamps (one BFS per record)
    uint32_t vgen = 0;
    std::vector<int32_t> q;
    // A node some earlier BFS visited has had its whole subtree walked: the walk only clears
    // sol (never sets it), so walking that subtree again changes nothing -- it is not
    // re-entered (the reference's repeated BFS is O(clusters^2) on deep trees).
    std::vector<char> walked(maxlab + 2, 0);
    for (auto *c : sorted) {
        const int32_t key = c->label;
        auto *A = get(key);
        if (!A) return HDB_EREF_NPE;
        double childStab = 0.0;
        if (!A->empty()) {
            for (auto &r : *A) childStab += r.v[2];
            if (childStab <= (*A)[0].v[0]) {
                for (auto &r : *A) {
                    if (++vgen == 0) {
                        std::fill(vis.begin(), vis.end(), 0);
                        vgen = 1;
                    }
                    int32_t rootV = (int32_t)r.v[1];
                    r.v[3] = 0.0;
                    sol[rootV] = 0;
                    if (rootV < 0 || rootV > maxlab + 1 || walked[rootV]) continue;
                    q.clear();
                    vis[rootV] = vgen;
                    q.push_back(rootV);
                    for (size_t h = 0; h < q.size(); h++) {
                        int32_t v = q[h];
                        walked[v] = 1;
                        auto *Av = get(v);
                        if (Av)
                            for (auto &rr : *Av) {
                                sol[v] = 0;
                                int32_t cc = (int32_t)rr.v[1];
                                if (vis[cc] != vgen && !walked[cc]) {
                                    q.push_back(cc);
                                    vis[cc] = vgen;
                                }
                            }
                    }
                }
            } else {
                (*A)[0].v[0] = childStab;
                auto *G = get((int32_t)(*A)[0].v[4]);
                if (G)
                    for (auto &rr : *G)
                        if ((int32_t)rr.v[1] == key) rr.v[2] = childStab;
            }
        } else {
            sol[key] = 0;
        }
    }
    const auto f1 = fclk::now();
    // The reference labels the selected clusters in birth order, a later one overwriting an
    // earlier one's members (nested selections happen: the BFS above does not clear childless
    // descendants).  Equivalently, in reverse order the first cluster to reach a point keeps
    // it -- and a dendrogram subtree walked once is never re-entered, so the labelling is
    // O(b) instead of O(b x nested selections).
    std::vector<int32_t> stk;
    for (auto *c : sorted)
        if (sol[c->label] && !(c->node >= 0 && D))
            for (int32_t m : c->members)
                if (m < 0 || m >= b) return HDB_EREF_OOB;
    std::vector<char> got((size_t)b, 0), claimed(D ? (size_t)(2 * b) : 0, 0);
    for (auto it = sorted.rbegin(); it != sorted.rend(); ++it) {
        const Cl *c = *it;
        if (!sol[c->label]) continue;
        if (c->node >= 0 && D) {
            stk.assign(1, c->node);
            while (!stk.empty()) {
                const int32_t x = stk.back();
                stk.pop_back();
                if (claimed[x]) continue;
                claimed[x] = 1;
                if (x < b) {
                    if (!got[x]) {
                        got[x] = 1;
                        flat[x] = c->label;
                    }
                    continue;
                }
                stk.push_back(D->r[x - b]);
                stk.push_back(D->l[x - b]);
            }
            continue;
        }
        for (int32_t m : c->members)
            if (!got[m]) {
                got[m] = 1;
                flat[m] = c->label;
            }
    }
    const auto f2 = fclk::now();
    g_lm_us[3] += fus(f0, f1);
    g_lm_us[4] += fus(f1, f2);
    struct NoiseTimer {
        fclk::time_point t = fclk::now();
        ~NoiseTimer() {
            g_lm_us[5] += (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(fclk::now() - t).count();
        }
    } noise_timer;
    // noise -> first later-valid neighbour in index order (:485-502).  With no labelled bubble
    // at all the reference's double loop changes nothing: skip its b^2 scan.
    bool any_label = false;
    for (int64_t p = 0; p < b && !any_label; p++) any_label = flat[p] != 0;
    if (!any_label) return HDB_OK;
    for (int64_t p = 0; p < b; p++) {
        double minD = JMAX;
        for (int64_t nb = 0; nb < b; nb++) {
            if (p == nb) continue;
            if (flat[p] == 0 && flat[nb] != 0) {
                double dist = host_distance(rep + p * d, rep + nb * d, d, metric);
                dist = host_distance_bubbles(dist, eB, nnB, p, nb);
                if (dist < minD) {
                    minD = dist;
                    flat[p] = flat[nb];
                }
            } else if (flat[p] != 0) {
                break;  // the condition can never hold again for this p
            }
        }
    }
    return HDB_OK;
}

thread_local int64_t g_lm_us[6];

int local_model_host(const double *rep, const double *eB, const double *nnB, const int32_t *nB, int64_t b, int d,
                     int32_t min_cl_size, int metric, int32_t *mva, int32_t *mvb, double *mw, int32_t *labels,
                     int32_t *ic_va, int32_t *ic_vb, double *ic_w, int64_t *n_ic) {
    using clk = std::chrono::steady_clock;
    auto us = [](clk::time_point a, clk::time_point b) {
        return (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
    };
    const int64_t ne = 2 * b - 1;
    auto t0 = clk::now();
    int rc = quicksort_edges(mva, mvb, mw, ne);
    if (rc) return rc;
    auto t1 = clk::now();
    std::vector<Cl> cl;
    Dendro D;
    rc = construct_cluster_tree_fast(b, mva, mvb, mw, ne, min_cl_size, nB, cl, D);
    const bool fast = rc != 1;
    if (!fast) {  // not a forest: the reference's BFS walk
        cl.clear();
        rc = construct_cluster_tree_bfs(b, mva, mvb, mw, ne, min_cl_size, nB, cl);
    }
    auto t2 = clk::now();
    g_lm_us[0] += us(t0, t1);
    g_lm_us[1] += us(t1, t2);
    if (rc) return rc;
    rc = find_prominent(cl, rep, eB, nnB, b, d, metric, labels, fast ? &D : nullptr);
    g_lm_us[2] += us(t2, clk::now());
    if (rc) return rc;
    int64_t k = 0;
    for (int64_t i = 0; i < ne; i++)
        if (labels[mva[i]] != labels[mvb[i]]) {
            if (ic_va) {
                ic_va[k] = mva[i];
                ic_vb[k] = mvb[i];
                ic_w[k] = mw[i];
            }
            k++;
        }
    if (n_ic) *n_ic = k;
    return HDB_OK;
}

}  // namespace hdb
