/* ASan/UBSan driver for the CPU oracle (oracle/hdb_oracle.c) -- SURVEY.md §5 "race
 * detection / sanitizers".  Built by tests/sanitize/Makefile with
 * -fsanitize=address,undefined and run by tests/test_sanitizers.py: every oracle routine on
 * tie-heavy seeded inputs (rounded blobs, duplicates), all core semantics and metrics, the
 * bubble chain and the local model.  Exit status 0 = no sanitizer report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

double orc_distance(const double *a, const double *b, int d, int metric);
int orc_core_distances(const double *X, int64_t n, int d, int min_pts, int metric, int semantics, double *core);
int orc_knn_lists(const double *X, int64_t n, int d, int min_pts, int metric, int excl_self, double *out);
int orc_prim_mst(const double *X, int64_t n, int d, const double *core, const int32_t *ids, int metric,
                 int self_edges, int32_t *va, int32_t *vb, double *w);
int orc_nearest_sample(const double *X, int64_t n, const double *S, int64_t m, int d, int metric,
                       const int32_t *xk, const int32_t *sk, int32_t *nn, double *dist);
int orc_bubble_stats_combine(const double *X, int64_t n, int d, const int32_t *bo, int64_t nb, double *ls,
                             double *ss, double *rep, double *info);
int orc_bubble_stats_cf(const double *X, int64_t n, int d, const int32_t *bo, int64_t nb, double *ls, double *ss,
                        double *rep, double *info);
int orc_bubble_core_distances(const double *rep, const int32_t *nB, const double *eB, const double *nnB, int64_t b,
                              int d, int min_pts, int metric, double *core);
int orc_bubble_prim_mst(const double *rep, const double *eB, const double *nnB, const int32_t *ids,
                        const double *core, int64_t b, int d, int metric, int self_edges, int32_t *va, int32_t *vb,
                        double *w);
int orc_quicksort_edges(int32_t *va, int32_t *vb, double *w, int64_t ne);
int orc_merge_edges(int32_t *va, int32_t *vb, double *w, int64_t ne);
int orc_local_model(const double *rep, const double *info, int64_t b, int d, int min_pts, int min_cl_size,
                    int metric, int32_t *labels, int32_t *mva, int32_t *mvb, double *mw, int32_t *iva,
                    int32_t *ivb, double *iw, int64_t *nic);
int orc_core_rows(const double *X, int64_t n, int d, const int64_t *rows, int64_t nr, int min_pts, int metric,
                  int excl_self, double *out);

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static double urand(void) {
    rs ^= rs << 13, rs ^= rs >> 7, rs ^= rs << 17;
    return (double)(rs >> 11) / 9007199254740992.0;
}

static void run(int n, int d, int centers, double round_to, int min_pts) {
    double *X = malloc(sizeof(double) * n * d), *C = malloc(sizeof(double) * centers * d);
    for (int i = 0; i < centers * d; i++) C[i] = 40.0 * urand() - 20.0;
    for (int i = 0; i < n; i++) {
        int c = (int)(urand() * centers);
        for (int j = 0; j < d; j++) {
            double v = C[c * d + j] + 2.0 * (urand() + urand() + urand() - 1.5);
            X[i * d + j] = round_to > 0 ? round(v / round_to) * round_to : v;
        }
    }
    double *core = malloc(sizeof(double) * n), *lists = malloc(sizeof(double) * n * min_pts);
    int32_t *va = malloc(sizeof(int32_t) * 2 * n), *vb = malloc(sizeof(int32_t) * 2 * n);
    double *w = malloc(sizeof(double) * 2 * n);
    int32_t *ids = malloc(sizeof(int32_t) * n);
    for (int i = 0; i < n; i++) ids[i] = 3 * i + 1;
    for (int metric = 0; metric < 5; metric++) {
        for (int sem = 0; sem < 3; sem++) orc_core_distances(X, n, d, min_pts, metric, sem, core);
        orc_knn_lists(X, n, d, min_pts, metric, 1, lists);
        orc_prim_mst(X, n, d, core, ids, metric, 1, va, vb, w);
        if (n >= 2) (void)orc_distance(X, X + d, d, metric);
    }
    orc_quicksort_edges(va, vb, w, 2 * n - 1);
    orc_merge_edges(va, vb, w, 2 * n - 1);
    if (n >= 2) {
        int64_t rows[5] = {0, 1, n / 2, n - 2, n - 1};
        double out5[5];
        orc_core_rows(X, n, d, rows, 5, min_pts, 0, 1, out5);
    }
    /* recursive-sampling level: samples, keyed nearest sample, bubbles, local model */
    int m = n / 5 + 1;
    double *S = malloc(sizeof(double) * m * d);
    int32_t *xk = malloc(sizeof(int32_t) * n), *sk = malloc(sizeof(int32_t) * m), *nn = malloc(sizeof(int32_t) * n);
    double *dist = malloc(sizeof(double) * n);
    for (int s = 0; s < m; s++) {
        memcpy(S + s * d, X + (size_t)(s * 5 % n) * d, sizeof(double) * d);
        sk[s] = s & 1;
    }
    for (int i = 0; i < n; i++) xk[i] = i & 1;
    orc_nearest_sample(X, n, S, m, d, 0, NULL, NULL, nn, dist);
    orc_nearest_sample(X, n, S, m, d, 0, xk, sk, nn, dist);
    orc_nearest_sample(X, n, S, m, d, 0, NULL, NULL, nn, dist);
    double *ls = malloc(sizeof(double) * m * d), *ss = malloc(sizeof(double) * m * d),
           *rep = malloc(sizeof(double) * m * d), *info = malloc(sizeof(double) * m * 3);
    orc_bubble_stats_cf(X, n, d, nn, m, ls, ss, rep, info);
    orc_bubble_stats_combine(X, n, d, nn, m, ls, ss, rep, info);
    /* compact the non-empty bubbles (D4) */
    int b = 0;
    for (int s = 0; s < m; s++)
        if (info[s * 3 + 2] > 0) {
            memmove(rep + b * d, rep + s * d, sizeof(double) * d);
            memmove(info + b * 3, info + s * 3, sizeof(double) * 3);
            b++;
        }
    if (b >= 2) {
        int32_t *nB = malloc(sizeof(int32_t) * b), *bid = malloc(sizeof(int32_t) * b);
        double *eB = malloc(sizeof(double) * b), *nnB = malloc(sizeof(double) * b), *bc = malloc(sizeof(double) * b);
        for (int i = 0; i < b; i++) {
            eB[i] = info[i * 3], nnB[i] = info[i * 3 + 1], nB[i] = (int32_t)info[i * 3 + 2], bid[i] = i;
        }
        orc_bubble_core_distances(rep, nB, eB, nnB, b, d, min_pts, 0, bc);
        int32_t *bva = malloc(sizeof(int32_t) * 2 * b), *bvb = malloc(sizeof(int32_t) * 2 * b);
        double *bw = malloc(sizeof(double) * 2 * b);
        orc_bubble_prim_mst(rep, eB, nnB, bid, bc, b, d, 0, 1, bva, bvb, bw);
        int32_t *lab = malloc(sizeof(int32_t) * b), *iva = malloc(sizeof(int32_t) * 2 * b),
                *ivb = malloc(sizeof(int32_t) * 2 * b);
        double *iw = malloc(sizeof(double) * 2 * b);
        int64_t nic = 0;
        for (int mcs = 2; mcs <= 8; mcs += 3)
            orc_local_model(rep, info, b, d, min_pts, mcs, 0, lab, bva, bvb, bw, iva, ivb, iw, &nic);
        free(nB), free(bid), free(eB), free(nnB), free(bc), free(bva), free(bvb), free(bw), free(lab), free(iva),
            free(ivb), free(iw);
    }
    free(S), free(xk), free(sk), free(nn), free(dist), free(ls), free(ss), free(rep), free(info);
    free(X), free(C), free(core), free(lists), free(va), free(vb), free(w), free(ids);
}

int main(void) {
    int cases[][5] = {{1, 3, 1, 0, 4}, {2, 2, 1, 0, 4}, {150, 4, 3, 0, 4}, {600, 3, 5, 1, 4},
                      {900, 2, 6, 1, 8}, {400, 8, 4, 0, 16}, {700, 3, 2, 1, 2}, {300, 1, 3, 1, 4}};
    for (size_t c = 0; c < sizeof cases / sizeof cases[0]; c++)
        run(cases[c][0], cases[c][1], cases[c][2], cases[c][3] ? 0.5 : 0.0, cases[c][4]);
    printf("oracle asan ok\n");
    return 0;
}
