// flat.cpp -- global HDBSCAN* hierarchy and flat (FOSC / excess-of-mass) labels over the
// merged MST: SURVEY.md §8(f) #1, the step the reference never completes (Main.java:351-408
// exits inside its first level).  Semantics: the canonical top-down procedure of
// HDBSCANStar.computeHierarchyAndClusterTree / propagateTree / findProminentClusters
// (HDBSCANStar.java:208-625, commented out in the reference) with the canonical choices
// listed in oracle/flat_labels.py (tie groups removed together, one stability term per
// (cluster, level), children summed in ascending smallest point id, labels 1..K by smallest
// point id, 0 = noise).
//
// Implementation: bottom-up instead of the Java's repeated BFS (O(levels * n)):
//   1. sort the tree edges by weight; union-find over tie groups builds a multi-way
//      dendrogram (a node = the merge of the components a tie group joins);
//   2. one top-down pass over the dendrogram condenses it (valid child = >= minClSize points)
//      and accumulates each cluster's stability in descending level order, exactly the
//      order the top-down Java visits them;
//   3. FOSC propagation children-before-parents, then one pass labels the points.
// O(E log E + n) host work; the inputs may live in HBM (staged once).
#include <algorithm>
#include <numeric>
#include <vector>

#include "internal.hpp"

namespace hdb {

namespace {

struct UF {
    std::vector<int32_t> p;
    explicit UF(int64_t n) : p((size_t)n) { std::iota(p.begin(), p.end(), 0); }
    int32_t find(int32_t x) {
        while (p[x] != x) {
            p[x] = p[p[x]];
            x = p[x];
        }
        return x;
    }
};

struct Node {  // dendrogram node; ids 0..n-1 are the points
    double level;
    int64_t size;
    int32_t minid;
    int32_t first_child, n_children;  // into child_pool
};

struct Clu {
    double birth;
    int32_t parent;
    int32_t node;   // dendrogram node at birth
    int32_t minid;
    double stab = 0.0;
    std::vector<int32_t> kids;  // ascending minid
};

}  // namespace

int flat_labels_host(const int32_t *va, const int32_t *vb, const double *w, int64_t ne, int64_t n, int32_t mcs,
                     int32_t *labels, int64_t *n_clusters) {
    if (n <= 0) {
        if (n_clusters) *n_clusters = 0;
        return HDB_OK;
    }
    if (mcs < 2) HDB_THROW(HDB_EINVAL, "flat labels: minClSize must be >= 2");
    std::vector<int64_t> e;
    e.reserve((size_t)std::max<int64_t>(ne, 0));
    for (int64_t i = 0; i < ne; i++) {
        if (va[i] == vb[i]) continue;  // self edges (core distances) carry no split for minClSize >= 2
        if (va[i] < 0 || vb[i] < 0 || va[i] >= n || vb[i] >= n) HDB_THROW(HDB_EINVAL, "flat labels: vertex id out of range");
        if (w[i] != w[i]) HDB_THROW(HDB_EINVAL, "flat labels: NaN edge weight");
        e.push_back(i);
    }
    if ((int64_t)e.size() != n - 1) HDB_THROW(HDB_EINVAL, "flat labels: the edges are not a spanning tree");
    std::sort(e.begin(), e.end(), [&](int64_t a, int64_t b) { return w[a] < w[b] || (w[a] == w[b] && a < b); });

    // ---- 1. multi-way dendrogram over tie groups
    std::vector<Node> nodes((size_t)n);
    for (int64_t i = 0; i < n; i++) nodes[i] = Node{0.0, 1, (int32_t)i, -1, 0};
    std::vector<int32_t> pool;
    pool.reserve((size_t)(2 * n));
    UF uf(n);
    std::vector<int32_t> comp_node((size_t)n);  // UF root -> current dendrogram node
    std::iota(comp_node.begin(), comp_node.end(), 0);
    std::vector<int32_t> pre_a, pre_b, stamp((size_t)(2 * n), -1), root_slot((size_t)n, -1);  // stamp: node ids < 2n
    std::vector<std::vector<int32_t>> groups;
    for (size_t g0 = 0; g0 < e.size();) {
        size_t g1 = g0;
        const double lev = w[e[g0]];
        while (g1 < e.size() && w[e[g1]] == lev) g1++;
        const size_t m = g1 - g0;
        pre_a.resize(m);
        pre_b.resize(m);
        for (size_t k = 0; k < m; k++) {  // components before the group
            pre_a[k] = comp_node[uf.find(va[e[g0 + k]])];
            pre_b[k] = comp_node[uf.find(vb[e[g0 + k]])];
        }
        for (size_t k = 0; k < m; k++) {
            int32_t ra = uf.find(va[e[g0 + k]]), rb = uf.find(vb[e[g0 + k]]);
            if (ra == rb) HDB_THROW(HDB_EINVAL, "flat labels: the edges contain a cycle");
            uf.p[rb] = ra;
        }
        // one new node per resulting component, children = distinct pre-group nodes
        groups.clear();
        std::vector<int32_t> roots;
        for (size_t k = 0; k < m; k++) {
            const int32_t r = uf.find(va[e[g0 + k]]);
            if (root_slot[r] < 0) {
                root_slot[r] = (int32_t)groups.size();
                groups.emplace_back();
                roots.push_back(r);
            }
            auto &kids = groups[(size_t)root_slot[r]];
            for (int32_t c : {pre_a[k], pre_b[k]}) {
                if (stamp[c] != (int32_t)g0) {
                    stamp[c] = (int32_t)g0;
                    kids.push_back(c);
                }
            }
        }
        for (size_t gi = 0; gi < roots.size(); gi++) {
            auto &kids = groups[gi];
            Node nd{lev, 0, INT32_MAX, (int32_t)pool.size(), (int32_t)kids.size()};
            for (int32_t c : kids) {
                nd.size += nodes[c].size;
                nd.minid = std::min(nd.minid, nodes[c].minid);
                pool.push_back(c);
            }
            comp_node[roots[gi]] = (int32_t)nodes.size();
            nodes.push_back(nd);
            root_slot[roots[gi]] = -1;
        }
        g0 = g1;
    }
    const int32_t root = n == 1 ? 0 : (int32_t)nodes.size() - 1;

    // ---- 2. condense top-down; stability terms in descending level per cluster
    std::vector<Clu> cl;
    cl.push_back(Clu{NAN, -1, root, nodes[root].minid});
    std::vector<std::pair<int32_t, int32_t>> stack;  // (node, cluster)
    if (n > 1) stack.push_back({root, 0});
    std::vector<int32_t> valid;
    while (!stack.empty()) {
        auto [x, L] = stack.back();
        stack.pop_back();
        const Node &X = nodes[x];
        const double eps = X.level;
        valid.clear();
        int64_t invalid_pts = 0;
        for (int32_t k = 0; k < X.n_children; k++) {
            int32_t c = pool[X.first_child + k];
            if (nodes[c].size >= mcs) valid.push_back(c);
            else invalid_pts += nodes[c].size;
        }
        const double inv_birth = 1.0 / cl[L].birth;
        if (valid.size() >= 2) {
            cl[L].stab += (double)X.size * (1.0 / eps - inv_birth);  // Cluster.detachPoints
            std::sort(valid.begin(), valid.end(), [&](int32_t a, int32_t b) { return nodes[a].minid < nodes[b].minid; });
            for (int32_t c : valid) {
                cl[L].kids.push_back((int32_t)cl.size());
                cl.push_back(Clu{eps, L, c, nodes[c].minid});
            }
            // push in reverse so the smallest-minid child is condensed first (order-free)
            for (size_t k = valid.size(); k-- > 0;) stack.push_back({valid[k], cl[L].kids[cl[L].kids.size() - valid.size() + k]});
        } else if (valid.size() == 1) {
            if (invalid_pts > 0) cl[L].stab += (double)invalid_pts * (1.0 / eps - inv_birth);
            stack.push_back({valid[0], L});
        } else {
            cl[L].stab += (double)X.size * (1.0 / eps - inv_birth);
        }
    }

    // ---- 3. FOSC propagation (children were created after their parent)
    const int64_t nc = (int64_t)cl.size();
    std::vector<double> contrib((size_t)nc, 0.0);
    std::vector<char> self_sel((size_t)nc, 0);
    for (int64_t c = nc - 1; c >= 1; c--) {
        double prop = 0.0;
        for (int32_t k : cl[c].kids) prop = prop + contrib[k];
        if (cl[c].kids.empty() || cl[c].stab >= prop) {  // Cluster.propagate: ties keep the parent
            contrib[c] = cl[c].stab;
            self_sel[c] = 1;
        } else {
            contrib[c] = prop;
        }
    }
    std::vector<int32_t> sel, todo(cl[0].kids.begin(), cl[0].kids.end());
    while (!todo.empty()) {
        int32_t c = todo.back();
        todo.pop_back();
        if (self_sel[c]) sel.push_back(c);
        else todo.insert(todo.end(), cl[c].kids.begin(), cl[c].kids.end());
    }
    std::sort(sel.begin(), sel.end(), [&](int32_t a, int32_t b) { return cl[a].minid < cl[b].minid; });
    std::fill(labels, labels + n, 0);
    std::vector<int32_t> dfs;
    for (size_t i = 0; i < sel.size(); i++) {
        dfs.assign(1, cl[sel[i]].node);
        while (!dfs.empty()) {
            int32_t x = dfs.back();
            dfs.pop_back();
            if (x < n) {
                labels[x] = (int32_t)(i + 1);
                continue;
            }
            for (int32_t k = 0; k < nodes[x].n_children; k++) dfs.push_back(pool[nodes[x].first_child + k]);
        }
    }
    if (n_clusters) *n_clusters = (int64_t)sel.size();
    return HDB_OK;
}

}  // namespace hdb
