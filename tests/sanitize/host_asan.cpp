// ASan/UBSan driver for the product's host C++: csrc/flat.cpp (global flat
// labels), csrc/formats.cpp (record formats), csrc/local_model.cpp (bubble core epilogue,
// UndirectedGraph quicksort, cluster tree, FOSC + noise reassignment).  Built by
// tests/sanitize/Makefile (hipcc --cuda-host-only -fsanitize=address,undefined) and run by
// tests/test_sanitizers.py on tie-heavy seeded inputs and malformed records.  The library's
// error setter lives in context.cpp (HIP runtime); a host stub stands in for it here.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "internal.hpp"

namespace hdb {
void set_error(const std::string &) {}
}  // namespace hdb

// the library's C-ABI wrapper (guarded) turns hdb::Error into a status code; do the same
template <class F>
static int guarded(F &&f) {
    try {
        return f();
    } catch (const hdb::Error &e) {
        return e.code;
    }
}

static uint64_t rs = 0x2545F4914F6CDD1Dull;
static uint64_t next() {
    rs ^= rs << 13, rs ^= rs >> 7, rs ^= rs << 17;
    return rs;
}
static double urand() { return (double)(next() >> 11) / 9007199254740992.0; }
static int irand(int n) { return (int)(next() % (uint64_t)n); }

static void random_tree(int n, int wmax, std::vector<int32_t> &va, std::vector<int32_t> &vb, std::vector<double> &w) {
    std::vector<int32_t> perm(n);
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int i = n - 1; i > 0; i--) std::swap(perm[i], perm[irand(i + 1)]);
    va.clear(), vb.clear(), w.clear();
    for (int i = 1; i < n; i++) {
        va.push_back(perm[irand(i)]);
        vb.push_back(perm[i]);
        w.push_back(wmax ? (double)irand(wmax + 1) : urand());
    }
}

static void flat() {
    for (int t = 0; t < 40; t++) {
        int n = 1 + irand(2000);
        std::vector<int32_t> va, vb;
        std::vector<double> w;
        random_tree(n, t % 4 == 0 ? 0 : 3 * (t % 5), va, vb, w);
        std::vector<int32_t> lab(n);
        int64_t k = 0;
        for (int mcs = 2; mcs <= 30; mcs += 7)
            guarded([&] { return hdb::flat_labels_host(va.data(), vb.data(), w.data(), n - 1, n, mcs, lab.data(), &k); });
        if (n > 2) {  // not spanning / cycle / bad ids: error paths
            auto fl = [&](int64_t ne) {
                return guarded([&] { return hdb::flat_labels_host(va.data(), vb.data(), w.data(), ne, n, 4, lab.data(), &k); });
            };
            fl(n - 2);
            va[0] = vb[0];
            fl(n - 1);
            va[1] = n + 5;
            fl(n - 1);
        }
    }
}

static void formats() {
    char buf[64];
    for (int i = 0; i < 20000; i++) {
        uint64_t bits = next();
        double v;
        memcpy(&v, &bits, 8);
        hdb_format_double(v, buf, sizeof buf);
        hdb_format_double(std::ldexp(1.0, irand(2098) - 1074), buf, sizeof buf);
    }
    hdb_format_double(1.0, buf, 2);  // too small
    const char *texts[] = {"1 2 3\n4 5 6\n", "1 2 3", "1  2\n", "\n\n", "", "0x1.8p1 2F 1e+2D\n", "1 2\n3\n",
                           "74\t85\t123\t1\n74\t85\t124\t1", "a b c", "1e 2", "+ -", "1 2 3   \r\n4 5 6 \n"};
    for (const char *t : texts)
        for (int strict = 0; strict < 2; strict++)
            for (int d = 0; d < 4; d++) {
                int64_t n = 0;
                int32_t dd = 0;
                hdb_parse_points(t, (int64_t)strlen(t), d, strict, nullptr, 0, &n, &dd);
                std::vector<double> X((size_t)std::max<int64_t>(n * std::max(dd, 1), 1));
                hdb_parse_points(t, (int64_t)strlen(t), d, strict, X.data(), n, &n, &dd);
                hdb_parse_points(t, (int64_t)strlen(t), d, strict, X.data(), 0, &n, &dd);  // capacity error
            }
    std::vector<int32_t> va, vb;
    std::vector<double> w;
    random_tree(500, 0, va, vb, w);
    std::vector<int32_t> f((size_t)va.size(), -7);
    int64_t len = 0;
    hdb_format_mst_records(va.data(), vb.data(), w.data(), f.data(), nullptr, f.data(), (int64_t)va.size(), nullptr, 0, &len);
    std::string s((size_t)len + 1, '\0');
    hdb_format_mst_records(va.data(), vb.data(), w.data(), f.data(), nullptr, f.data(), (int64_t)va.size(), &s[0], len + 1, &len);
    hdb_format_mst_records(va.data(), vb.data(), w.data(), nullptr, nullptr, nullptr, (int64_t)va.size(), &s[0], len / 2, &len);
    s.resize((size_t)len);
    std::vector<int32_t> a(va.size()), b(va.size()), c(va.size());
    std::vector<double> ww(va.size());
    int64_t ne = 0;
    hdb_parse_mst_records(s.data(), (int64_t)s.size(), a.data(), b.data(), ww.data(), c.data(), c.data(), c.data(),
                          (int64_t)a.size(), &ne);
    hdb_parse_mst_records(s.data(), (int64_t)s.size(), a.data(), b.data(), ww.data(), nullptr, nullptr, nullptr, 3, &ne);
    const char *bad[] = {"", "1 2 x", "1 2 0.5", "1 2 0.5 0 0 2147483648", "1 2 1.0E-5 0 0 0\n3 4 5.0 0 0 1\n\n", "\n",
                         " 1 2 3 4 5 6", "1 2 3 4 5 6 7 8"};
    for (const char *t : bad) hdb_parse_mst_records(t, (int64_t)strlen(t), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, &ne);
}

static void local_model() {
    for (int t = 0; t < 60; t++) {
        const int b = 2 + irand(400), d = 1 + irand(4), min_pts = 2 + irand(6), K = min_pts - 1;
        std::vector<double> rep((size_t)b * d), eB(b), nnB(b), knn((size_t)b * K), core(b);
        std::vector<int32_t> nB(b), log((size_t)b * K);
        for (auto &x : rep) x = std::round(urand() * 20.0);
        for (int i = 0; i < b; i++) {
            nB[i] = irand(6);  // zeros included: the reference's divide-by-zero path
            eB[i] = irand(3) * 0.5;
            nnB[i] = eB[i];
            double acc = 0;
            for (int k = 0; k < K; k++) {
                acc += irand(3);
                knn[(size_t)i * K + k] = acc;
                log[(size_t)i * K + k] = irand(3) == 0 ? -1 : irand(b);
            }
        }
        guarded([&] { return hdb::bubble_core_epilogue(rep.data(), nB.data(), eB.data(), nnB.data(), b, d, min_pts, 0, knn.data(), log.data(),
                                  core.data()); });
        // MST over the bubbles (random tree) + self edges, as constructMSTBubbles emits them
        std::vector<int32_t> va, vb;
        std::vector<double> w;
        random_tree(b, t % 3 == 0 ? 0 : 4, va, vb, w);
        for (int i = 0; i < b; i++) {
            va.push_back(i), vb.push_back(i), w.push_back(core[i]);
            if (nB[i] == 0) nB[i] = 1;
        }
        std::vector<int32_t> labels(b), iva(2 * b), ivb(2 * b);
        std::vector<double> iw(2 * b);
        int64_t nic = 0;
        for (int mcs = 2; mcs <= 8; mcs += 3) {
            std::vector<int32_t> a = va, bb = vb;
            std::vector<double> ww = w;
            guarded([&] { return hdb::local_model_host(rep.data(), eB.data(), nnB.data(), nB.data(), b, d, mcs, t % 5, a.data(), bb.data(),
                                  ww.data(), labels.data(), iva.data(), ivb.data(), iw.data(), &nic); });
        }
        std::vector<int32_t> a = va, bb = vb;
        std::vector<double> ww = w;
        guarded([&] { return hdb::quicksort_edges(a.data(), bb.data(), ww.data(), (int64_t)ww.size()); });
    }
}

int main() {
    // K6 relabel limit (flat.hip): contracted labels nv + rank < 3m must fit int32
    if (!hdb::flat_relabel_fits(715827882) || hdb::flat_relabel_fits(715827883) || !hdb::flat_relabel_fits(0)) {
        printf("flat_relabel_fits limit wrong\n");
        return 1;
    }
    flat();
    formats();
    local_model();
    printf("host asan ok\n");
    return 0;
}
