// Host-only developer tool: supernode / level statistics of the factor plan
// of a synthetic LP (BASELINE configs[3] banded) or an MPS file, and what a
// relaxed amalgamation of parent chains would give (columns j, j+1 share a
// panel when parent(j) = j+1 and the merged panel stays within `zfrac`
// explicit zeros).
//   g++ -O2 -std=c++17 -I linear-programming-vanderbei_amd/csrc tools/plan_levels.cpp \
//       linear-programming-vanderbei_amd/csrc/kkt_symbolic.cpp linear-programming-vanderbei_amd/csrc/lp_io.cpp \
//       linear-programming-vanderbei_amd/csrc/kkt_order_nd.cpp linear-programming-vanderbei_amd/csrc/synth.cpp \
//       -o tools/plan_levels -lz
//   (the order is build_kkt_plan's: IPO_HIP_ORDER=md|nd|auto, IPO_HIP_ND_LEAF)
//   tools/plan_levels banded 200000 1000000 256      |  tools/plan_levels mps file.mps.gz
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kkt_plan.h"
#include "lp_io.h"
#include "synth.h"

using namespace ipo;

static void levels_of(const KktOrdering& o, int tc, double zfrac, int maxw) {
    const int T = o.T;
    std::vector<int> cnt(T);
    for (int j = 0; j < T; j++) cnt[j] = o.Lp[j + 1] - o.Lp[j];
    std::vector<int> col0{0};
    double zeros = 0, ent = 0;   // of the current panel
    double tz = 0, tent = 0;
    auto close = [&]() { tz += zeros; tent += ent; };
    for (int j = 0; j + 1 < tc; j++) {
        const int c = col0.back();
        const int width = j + 1 - c;
        const bool chain = cnt[j] > 0 && o.Li[o.Lp[j]] == j + 1;
        bool join = false;
        if (chain && width < maxw) {
            // panel [c, j+2): rows = struct(j+1) below; entries per column k: (j+1 - k) + cnt[j+1]
            const int w2 = width + 1;
            double e2 = 0, nz2 = 0;
            for (int k = c; k <= j + 1; k++) { e2 += (j + 1 - k) + cnt[j + 1]; nz2 += cnt[k]; }
            (void)w2;
            if (e2 - nz2 <= zfrac * e2) { join = true; zeros = e2 - nz2; ent = e2; }
        }
        if (!join) {
            close();
            col0.push_back(j + 1);
            zeros = 0; ent = cnt[j + 1];
        }
    }
    close();
    col0.push_back(tc);
    const int ns = (int)col0.size() - 1;
    std::vector<int> sup_of(T, -1), level(ns, 0);
    for (int s = 0; s < ns; s++) for (int j = col0[s]; j < col0[s + 1]; j++) sup_of[j] = s;
    int nl = 0;
    std::vector<int> wh(65, 0);
    for (int s = 0; s < ns; s++) {
        const int last = col0[s + 1] - 1;
        if (cnt[last] > 0) {
            const int r = o.Li[o.Lp[last]];
            if (r < tc) level[sup_of[r]] = std::max(level[sup_of[r]], level[s] + 1);
        }
        nl = std::max(nl, level[s] + 1);
        wh[std::min(64, col0[s + 1] - col0[s])]++;
    }
    std::vector<int> per(nl, 0);
    for (int s = 0; s < ns; s++) per[level[s]]++;
    std::printf("zfrac %.2f maxw %d: nsup %d levels %d  zeros %.3g of %.3g entries (%.1f%%)\n", zfrac, maxw, ns, nl, tz,
                tent, 100.0 * tz / std::max(1.0, tent));
    std::printf("  width hist:");
    for (int w = 1; w <= 64; w++) if (wh[w]) std::printf(" %d:%d", w, wh[w]);
    std::printf("\n  sups per level (first 8, last 8):");
    for (int l = 0; l < std::min(nl, 8); l++) std::printf(" %d", per[l]);
    std::printf(" ...");
    for (int l = std::max(8, nl - 8); l < nl; l++) std::printf(" %d", per[l]);
    std::printf("\n");
}

int main(int argc, char** argv) {
    int m, n;
    std::vector<int> kA, iA;
    if (argc > 1 && !std::strcmp(argv[1], "mps")) {
        MpsProblem mp;
        std::string err;
        if (read_mps(argv[2], mp, &err)) { std::printf("read: %s\n", err.c_str()); return 1; }
        SolverForm sf;
        to_solver_form(mp, sf);
        m = sf.m; n = sf.n; kA = sf.kA; iA = sf.iA;
    } else {
        m = argc > 2 ? std::atoi(argv[2]) : 200000;
        n = argc > 3 ? std::atoi(argv[3]) : 1000000;
        const int band = argc > 4 ? std::atoi(argv[4]) : 256;
        SynthLP lp;
        synth_random(m, n, 4, band, 20251121ull, lp);
        kA = lp.kA; iA = lp.iA;
    }
    std::vector<int> kAt, iAt;
    std::vector<double> A(iA.size(), 1.0), At;
    csc_transpose(m, n, kA.data(), iA.data(), A.data(), kAt, iAt, At);
    const bool nd = use_nested_dissection(m + n);
    int leaf = kNdLeafRows;
    if (const char* e = std::getenv("IPO_HIP_ND_LEAF")) leaf = std::atoi(e);
    auto t0 = std::chrono::steady_clock::now();
    KktOrdering o = nd ? order_nested_dissection(m, n, kA.data(), iA.data(), kAt.data(), iAt.data(), 0, leaf, std::getenv("IPO_HIP_ND_RELAX") ? std::atof(std::getenv("IPO_HIP_ND_RELAX")) : kNdRelax)
                       : order_tiered_min_degree(m, n, kA.data(), iA.data(), kAt.data(), iAt.data());
    std::printf("%s ordering %.2f s, narth %.3g\n", nd ? "nested-dissection" : "minimum-degree",
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), o.narth);
    {
        unsigned long long h = 1469598103934665603ull;
        for (const std::vector<int>* v : {&o.perm, &o.Lp, &o.Li})
            for (int x : *v) { h ^= static_cast<unsigned>(x); h *= 1099511628211ull; }
        std::printf("pattern hash %016llx\n", h);
    }
    int tc = o.T;
    while (tc > 0 && o.Lp[tc] - o.Lp[tc - 1] == o.T - tc) tc--;
    std::printf("m %d n %d T %d lnz %d dense window %d\n", m, n, o.T, o.Lp[o.T], o.T - tc);
    const double zf[] = {0.0, 0.05, 0.1, 0.2, 0.3};
    for (double z : zf) levels_of(o, tc, z, 64);
    if (argc > 5 || (argc > 1 && !std::strcmp(argv[1], "mps"))) {
        t0 = std::chrono::steady_clock::now();
        KktPlan P = build_kkt_plan(m, n, kA.data(), iA.data(), kAt.data(), iAt.data(), 0, kTailDensity);
        std::printf("plan: nsup %d levels %d nt %d lnz %lld flops %.3g (%.2f s)\n", P.nsup, P.nlevels, P.nt,
                    (long long)P.lnz, P.flops_factor,
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        // per level: units, slots, slots whose source is on the level just below
        long tot = 0, recent = 0;
        for (int l = 1; l < P.nlevels; l++) {
            long sl = 0, rc = 0, mx = 0;
            const int u0 = P.unit_level_ptr[l], u1 = P.unit_level_ptr[l + 1];
            for (int u = u0; u < u1; u++) {
                long k = 0, kr = 0;
                for (int i = P.kslot_ptr[u]; i < P.kslot_ptr[u + 1]; i++) {
                    const int s = P.kslot[i];
                    if (s < 0) continue;
                    k++;
                    if (P.level[P.utasks[s >> 6].src] == l - 1) kr++;
                }
                sl += k; rc += kr; mx = std::max(mx, k);
            }
            tot += sl; recent += rc;
            if (l < 12 || l % 200 == 0 || l > P.nlevels - 4)
                std::printf("L%4d sups %6d units %7d slots %9ld from l-1 %9ld max/unit %ld\n", l,
                            P.level_ptr[l + 1] - P.level_ptr[l], u1 - u0, sl, rc, mx);
        }
        std::printf("all levels: slots %ld, from the level below %ld (%.1f%%)\n", tot, recent, 100.0 * recent / tot);
        // distance (target level - source level) histogram of slots, levels >= 2
        long h[8] = {0};
        const char* nm[8] = {"src lvl 0", "d=1", "d=2", "d=3-4", "d=5-8", "d=9-32", "d=33-128", "d>128"};
        for (int l = 2; l < P.nlevels; l++)
            for (int u = P.unit_level_ptr[l]; u < P.unit_level_ptr[l + 1]; u++)
                for (int i = P.kslot_ptr[u]; i < P.kslot_ptr[u + 1]; i++) {
                    const int s = P.kslot[i];
                    if (s < 0) continue;
                    const int sl = P.level[P.utasks[s >> 6].src], d = l - sl;
                    h[sl == 0 ? 0 : d == 1 ? 1 : d == 2 ? 2 : d <= 4 ? 3 : d <= 8 ? 4 : d <= 32 ? 5 : d <= 128 ? 6 : 7]++;
                }
        for (int k = 0; k < 8; k++) std::printf("  %s: %ld\n", nm[k], h[k]);
    }
    return 0;
}
