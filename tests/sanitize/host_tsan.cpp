// ThreadSanitizer driver for the host code the C3/C5 model pool runs concurrently (VERDICT r05
// item 1): the driver's local-model threads each call hdb_local_model, whose host half is
// csrc/local_model.cpp (bubble core epilogue, UndirectedGraph quicksort, cluster tree, FOSC +
// noise reassignment, thread_local phase timers and exception detail), plus the host flat labels
// (csrc/flat.cpp) and the record formats (csrc/formats.cpp).  T threads run the same seeded
// workloads at once; every thread's result digest must equal the one a serial run of the same
// seed gives (state leaking between threads changes a digest even where TSan sees no race), and
// TSan aborts on any data race (halt_on_error).  Built by tests/sanitize/Makefile (hipcc
// --cuda-host-only -fsanitize=thread), run by tests/test_sanitizers.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "internal.hpp"

namespace hdb {
void set_error(const std::string &) {}
}  // namespace hdb

template <class F>
static int guarded(F &&f) {
    try {
        return f();
    } catch (const hdb::Error &e) {
        return e.code;
    }
}

namespace {

struct Rng {
    uint64_t s;
    uint64_t next() {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        return s;
    }
    double urand() { return (double)(next() >> 11) / 9007199254740992.0; }
    int irand(int n) { return (int)(next() % (uint64_t)n); }
};

struct Digest {
    uint64_t h = 1469598103934665603ull;
    void add(const void *p, size_t n) {
        const unsigned char *c = (const unsigned char *)p;
        for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
    }
    template <class T>
    void vec(const std::vector<T> &v) { add(v.data(), v.size() * sizeof(T)); }
    void i64(int64_t x) { add(&x, sizeof x); }
};

void random_tree(Rng &r, int n, int wmax, std::vector<int32_t> &va, std::vector<int32_t> &vb, std::vector<double> &w) {
    std::vector<int32_t> perm(n);
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int i = n - 1; i > 0; i--) std::swap(perm[i], perm[r.irand(i + 1)]);
    va.clear(), vb.clear(), w.clear();
    for (int i = 1; i < n; i++) {
        va.push_back(perm[r.irand(i)]);
        vb.push_back(perm[i]);
        w.push_back(wmax ? (double)r.irand(wmax + 1) : r.urand());
    }
}

// one thread's workload for `seed`: tie-heavy local models (the C5 pool's host work), flat
// labels, quicksort, formats; returns the digest of every output and status code
uint64_t workload(uint64_t seed, int reps) {
    Rng r{seed * 0x9E3779B97F4A7C15ull + 1};
    Digest dg;
    for (int t = 0; t < reps; t++) {
        const int b = 2 + r.irand(600), d = 1 + r.irand(4), min_pts = 2 + r.irand(6), K = min_pts - 1;
        std::vector<double> rep((size_t)b * d), eB(b), nnB(b), knn((size_t)b * K), core(b);
        std::vector<int32_t> nB(b), log((size_t)b * K);
        for (auto &x : rep) x = std::round(r.urand() * 20.0);
        for (int i = 0; i < b; i++) {
            nB[i] = r.irand(6);
            eB[i] = r.irand(3) * 0.5;
            nnB[i] = eB[i];
            double acc = 0;
            for (int k = 0; k < K; k++) {
                acc += r.irand(3);
                knn[(size_t)i * K + k] = acc;
                log[(size_t)i * K + k] = r.irand(3) == 0 ? -1 : r.irand(b);
            }
        }
        dg.i64(guarded([&] {
            return hdb::bubble_core_epilogue(rep.data(), nB.data(), eB.data(), nnB.data(), b, d, min_pts, 0, knn.data(),
                                             log.data(), core.data());
        }));
        dg.vec(core);
        std::vector<int32_t> va, vb;
        std::vector<double> w;
        random_tree(r, b, t % 3 == 0 ? 0 : 4, va, vb, w);
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
            const int rc = guarded([&] {
                return hdb::local_model_host(rep.data(), eB.data(), nnB.data(), nB.data(), b, d, mcs, t % 5, a.data(),
                                             bb.data(), ww.data(), labels.data(), iva.data(), ivb.data(), iw.data(), &nic);
            });
            dg.i64(rc);
            if (rc == HDB_EREF_NEGATIVE_CLUSTER) {  // the thread_local exception detail of this call
                const char *m = hdb::local_model_error_detail();
                dg.add(m, strlen(m));
            }
            if (rc == 0) {
                dg.vec(labels);
                dg.i64(nic);
                dg.add(iva.data(), sizeof(int32_t) * nic);
                dg.add(iw.data(), sizeof(double) * nic);
            }
        }
        std::vector<int32_t> a = va, bb = vb;
        std::vector<double> ww = w;
        dg.i64(guarded([&] { return hdb::quicksort_edges(a.data(), bb.data(), ww.data(), (int64_t)ww.size()); }));
        dg.vec(a), dg.vec(ww);
        // the host flat labels over the tree part
        std::vector<int32_t> fa(va.begin(), va.begin() + (b - 1)), fb(vb.begin(), vb.begin() + (b - 1));
        std::vector<double> fw(w.begin(), w.begin() + (b - 1));
        std::vector<int32_t> lab(b);
        int64_t k = 0;
        dg.i64(guarded([&] { return hdb::flat_labels_host(fa.data(), fb.data(), fw.data(), b - 1, b, 4, lab.data(), &k); }));
        dg.vec(lab), dg.i64(k);
        char buf[64];
        for (int i = 0; i < 64; i++) {
            const double v = std::ldexp(r.urand(), r.irand(80) - 40);
            hdb_format_double(v, buf, sizeof buf);
            dg.add(buf, strlen(buf));
        }
    }
    return dg.h;
}

}  // namespace

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 8, reps = argc > 2 ? atoi(argv[2]) : 12;
    std::vector<uint64_t> serial(T), par(T);
    for (int i = 0; i < T; i++) serial[i] = workload(i, reps);
    for (int round = 0; round < 2; round++) {
        std::vector<std::thread> th;
        for (int i = 0; i < T; i++) th.emplace_back([&, i] { par[i] = workload(i, reps); });
        for (auto &x : th) x.join();
        for (int i = 0; i < T; i++)
            if (par[i] != serial[i]) {
                printf("thread %d digest %016llx != serial %016llx\n", i, (unsigned long long)par[i],
                       (unsigned long long)serial[i]);
                return 1;
            }
    }
    printf("host tsan ok (%d threads x %d models)\n", T, reps);
    return 0;
}
