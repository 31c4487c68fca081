// Host half of one bubble local model (csrc/local_model.cpp: quicksort, cluster tree, FOSC) at
// C5's model size, on the CPU: b bubbles of 8-d blob data, a Prim MST of their mutual-
// reachability graph (max(core_p, core_q, distance)) plus self edges, then local_model_host.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --cuda-host-only -x hip -I<csrc> tools/lm_host_bench.cpp
//        <csrc>/local_model.cpp <csrc>/flat.cpp <csrc>/formats.cpp -o lm_host_bench
// Usage: lm_host_bench [b] [reps]  |  lm_host_bench <dump dir> [b] [d] [reps]  (tools/lm_dump.py)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "internal.hpp"

namespace hdb {
void set_error(const std::string &) {}
}  // namespace hdb

template <class T>
static bool load(const std::string &dir, const char *name, std::vector<T> &v, size_t n) {
    v.resize(n);
    FILE *f = fopen((dir + "/" + name + ".bin").c_str(), "rb");
    if (!f) return false;
    const size_t got = fread(v.data(), sizeof(T), n, f);
    fclose(f);
    return got == n;
}

int main(int argc, char **argv) {
    // a directory argument: the inputs tools/lm_dump.py wrote (a real bubble model and its Prim MST)
    if (argc > 1 && argv[1][0] != '-' && !(argv[1][0] >= '0' && argv[1][0] <= '9')) {
        const std::string dir = argv[1];
        const int b = argc > 2 ? atoi(argv[2]) : 16384, d = argc > 3 ? atoi(argv[3]) : 8, reps = argc > 4 ? atoi(argv[4]) : 5;
        const size_t ne = 2 * (size_t)b - 1;
        std::vector<double> rep, eB, nnB, w;
        std::vector<int32_t> nB, va, vb;
        if (!load(dir, "rep", rep, (size_t)b * d) || !load(dir, "eB", eB, b) || !load(dir, "nnB", nnB, b) ||
            !load(dir, "nB", nB, b) || !load(dir, "va", va, ne) || !load(dir, "vb", vb, ne) || !load(dir, "w", w, ne)) {
            fprintf(stderr, "cannot read %s\n", dir.c_str());
            return 1;
        }
        std::vector<int32_t> labels(b), iva(ne), ivb(ne);
        std::vector<double> iw(ne);
        for (int r = 0; r < reps; r++) {
            std::vector<int32_t> a = va, bb = vb;
            std::vector<double> ww = w;
            int64_t nic = 0;
            for (int k = 0; k < 6; k++) hdb::g_lm_us[k] = 0;
            const auto t0 = std::chrono::steady_clock::now();
            int rc = -99;
            try {
                rc = hdb::local_model_host(rep.data(), eB.data(), nnB.data(), nB.data(), b, d, 4, 0, a.data(), bb.data(),
                                           ww.data(), labels.data(), iva.data(), ivb.data(), iw.data(), &nic);
            } catch (const hdb::Error &e) {
                rc = e.code;
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            uint64_t h = 1469598103934665603ull;  // digest of the outputs (labels, inter-cluster edges)
            auto mix = [&](const void *p, size_t n) {
                for (size_t i = 0; i < n; i++) h = (h ^ ((const unsigned char *)p)[i]) * 1099511628211ull;
            };
            mix(labels.data(), sizeof(int32_t) * b);
            mix(iva.data(), sizeof(int32_t) * nic);
            mix(ivb.data(), sizeof(int32_t) * nic);
            mix(iw.data(), sizeof(double) * nic);
            printf("b %d rc %d  %.3f ms  (quicksort %.3f tree %.3f fosc %.3f = select %.3f label %.3f noise %.3f)  ic %lld  digest %016llx\n",
                   b, rc, ms, hdb::g_lm_us[0] / 1e3, hdb::g_lm_us[1] / 1e3, hdb::g_lm_us[2] / 1e3, hdb::g_lm_us[3] / 1e3,
                   hdb::g_lm_us[4] / 1e3, hdb::g_lm_us[5] / 1e3, (long long)nic, (unsigned long long)h);
        }
        return 0;
    }
    const int b = argc > 1 ? atoi(argv[1]) : 16384, reps = argc > 2 ? atoi(argv[2]) : 5, d = 8, C = 20;
    uint64_t s = 88172645463325252ull;
    auto nxt = [&]() { s ^= s << 13, s ^= s >> 7, s ^= s << 17; return s; };
    auto ur = [&]() { return (double)(nxt() >> 11) / 9007199254740992.0; };
    auto gs = [&]() { return std::sqrt(-2.0 * std::log(ur() + 1e-300)) * std::cos(6.283185307179586 * ur()); };
    std::vector<double> ctr((size_t)C * d), rep((size_t)b * d), eB(b), nnB(b), core(b);
    std::vector<int32_t> nB(b);
    for (auto &x : ctr) x = ur() * 200.0 - 100.0;
    for (int i = 0; i < b; i++) {
        const int c = (int)(nxt() % C);
        for (int k = 0; k < d; k++) rep[(size_t)i * d + k] = ctr[(size_t)c * d + k] + gs() * 3.0;
        nB[i] = 1 + (int)(nxt() % 200);
        eB[i] = 0.05 + 0.1 * ur();
        nnB[i] = eB[i] * 0.5;
    }
    auto dist = [&](int p, int q) {
        double a = 0;
        for (int k = 0; k < d; k++) {
            const double t = rep[(size_t)p * d + k] - rep[(size_t)q * d + k];
            a = a + t * t;
        }
        return std::sqrt(a);
    };
    for (int i = 0; i < b; i++) {  // 4th nearest neighbour
        double best[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
        for (int j = 0; j < b; j++) {
            if (j == i) continue;
            double x = dist(i, j);
            for (int k = 0; k < 4; k++)
                if (x < best[k]) std::swap(x, best[k]);
        }
        core[i] = best[3];
    }
    std::vector<int32_t> va, vb;
    std::vector<double> w;
    {  // Prim from b - 1
        std::vector<double> bw(b, INFINITY);
        std::vector<int32_t> par(b, 0);
        std::vector<char> in(b, 0);
        int cur = b - 1;
        in[cur] = 1;
        for (int step = 1; step < b; step++) {
            int nxtv = -1;
            double nb = INFINITY;
            for (int j = 0; j < b; j++) {
                if (in[j]) continue;
                double m = dist(cur, j);
                if (core[cur] > m) m = core[cur];
                if (core[j] > m) m = core[j];
                if (m < bw[j]) bw[j] = m, par[j] = cur;
                if (bw[j] <= nb) nb = bw[j], nxtv = j;
            }
            in[nxtv] = 1;
            va.push_back(par[nxtv]), vb.push_back(nxtv), w.push_back(bw[nxtv]);
            cur = nxtv;
        }
        for (int i = 0; i < b; i++) va.push_back(i), vb.push_back(i), w.push_back(core[i]);
    }
    std::vector<int32_t> labels(b), iva(2 * b), ivb(2 * b);
    std::vector<double> iw(2 * b);
    for (int r = 0; r < reps; r++) {
        std::vector<int32_t> a = va, bb = vb;
        std::vector<double> ww = w;
        int64_t nic = 0;
        const auto t0 = std::chrono::steady_clock::now();
        int rc = -99;
        try {
            rc = hdb::local_model_host(rep.data(), eB.data(), nnB.data(), nB.data(), b, d, 4, 0, a.data(), bb.data(),
                                       ww.data(), labels.data(), iva.data(), ivb.data(), iw.data(), &nic);
        } catch (const hdb::Error &e) {
            rc = e.code;
        }
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        int64_t nl = 0;
        for (int i = 0; i < b; i++) nl = nl > labels[i] ? nl : labels[i];
        printf("b %d rc %d  %.3f ms  (quicksort %.3f tree %.3f fosc %.3f = select %.3f label %.3f noise %.3f)  clusters %lld ic %lld\n",
               b, rc, ms, hdb::g_lm_us[0] / 1e3, hdb::g_lm_us[1] / 1e3, hdb::g_lm_us[2] / 1e3, hdb::g_lm_us[3] / 1e3,
               hdb::g_lm_us[4] / 1e3, hdb::g_lm_us[5] / 1e3, (long long)nl, (long long)nic);
    }
    return 0;
}
