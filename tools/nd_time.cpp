// Host-only developer tool: wall time of each setup phase of the factor plan
// for the synthetic banded LP (BASELINE configs[3]) or a block-angular one,
// and a hash of the permutation / pattern so speed-ups can be checked to
// leave the plan unchanged.
//   g++ -O2 -std=c++17 -I linear-programming-vanderbei_amd/csrc tools/nd_time.cpp \
//       linear-programming-vanderbei_amd/csrc/kkt_symbolic.cpp linear-programming-vanderbei_amd/csrc/lp_io.cpp \
//       linear-programming-vanderbei_amd/csrc/kkt_order_nd.cpp linear-programming-vanderbei_amd/csrc/synth.cpp \
//       -o tools/nd_time -lz -lpthread
//   tools/nd_time [m n band]
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kkt_plan.h"
#include "lp_io.h"
#include "synth.h"

using namespace ipo;

static uint64_t fnv(const std::vector<int>& v, uint64_t h = 1469598103934665603ull) {
    for (int x : v) { h ^= static_cast<uint32_t>(x); h *= 1099511628211ull; }
    return h;
}

int main(int argc, char** argv) {
    const int m = argc > 1 ? std::atoi(argv[1]) : 200000;
    const int n = argc > 2 ? std::atoi(argv[2]) : 1000000;
    const int band = argc > 3 ? std::atoi(argv[3]) : 256;
    SynthLP lp;
    synth_random(m, n, 4, band, 20251121ull, lp);
    std::vector<int> kAt, iAt;
    std::vector<double> At;
    csc_transpose(m, n, lp.kA.data(), lp.iA.data(), lp.A.data(), kAt, iAt, At);
    using clk = std::chrono::steady_clock;
    auto sec = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
    auto t0 = clk::now();
    KktOrdering o;
    o.m = m; o.n = n; o.T = m + n;
    o.perm = nested_dissection_perm(m, n, lp.kA.data(), lp.iA.data(), kAt.data(), iAt.data(), 0, kNdLeafRows);
    std::printf("perm      %.3f s  hash %016llx\n", sec(t0), (unsigned long long)fnv(o.perm));
    t0 = clk::now();
    symbolic_from_perm(o, lp.kA.data(), lp.iA.data(), kAt.data(), iAt.data(), 0);
    std::printf("symbolic  %.3f s  lnz %d hash %016llx\n", sec(t0), o.Lp[o.T], (unsigned long long)fnv(o.Li, fnv(o.Lp)));
    int tc = o.T;
    while (tc > 0 && o.Lp[tc] - o.Lp[tc - 1] == o.T - tc) tc--;
    t0 = clk::now();
    relax_supernodes(o, tc, kNdRelax);
    std::printf("relax     %.3f s  lnz %d\n", sec(t0), o.Lp[o.T]);
    t0 = clk::now();
    KktPlan P = build_kkt_plan(m, n, lp.kA.data(), lp.iA.data(), kAt.data(), iAt.data(), 0, kTailDensity);
    const double all = sec(t0);
    std::printf("plan      %.3f s  (whole build_kkt_plan)  nsup %d levels %d nt %d hash %016llx\n", all, P.nsup,
                P.nlevels, P.nt, (unsigned long long)fnv(P.rel, fnv(P.kslot, fnv(P.perm))));
    return 0;
}
