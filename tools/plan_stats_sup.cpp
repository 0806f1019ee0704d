// plan_stats: print the symbolic plan of an MPS problem (developer tool).
#include <chrono>
#include <cstdio>
#include <string>
#include <algorithm>
#include "kkt_plan.h"
#include "lp_io.h"
#include "synth.h"
#include <cstdlib>

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: plan_stats file.mps | synth m n band | blockang K mb nb l lnz\n"); return 1; }
    ipo::SolverForm s;
    if (std::string(argv[1]) == "synth" || std::string(argv[1]) == "blockang") {
        ipo::SynthLP o;
        if (argv[1][0] == 's') ipo::synth_random(std::atoi(argv[2]), std::atoi(argv[3]), 4, std::atoi(argv[4]), 20251121, o);
        else ipo::synth_block_angular(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), 4, 256,
                                      std::atoi(argv[5]), std::atoi(argv[6]), 20251121, o);
        s.m = o.m; s.n = o.n; s.nz = o.kA[o.n]; s.kA = o.kA; s.iA = o.iA; s.A = o.A;
        argc = 2;
    } else {
    ipo::MpsProblem p; std::string err;
    if (ipo::read_mps(argv[1], p, &err)) { std::fprintf(stderr, "read error: %s\n", err.c_str()); return 1; }
    if (ipo::to_solver_form(p, s)) { std::printf("free variable -> status 3\n"); return 0; }
    }
    std::vector<int> kat, iat; std::vector<double> at;
    ipo::csc_transpose(s.m, s.n, s.kA.data(), s.iA.data(), s.A.data(), kat, iat, at);
    auto t0 = std::chrono::steady_clock::now();
    ipo::KktPlan P = ipo::build_kkt_plan(s.m, s.n, s.kA.data(), s.iA.data(), kat.data(), iat.data());
    double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("m=%d n=%d nz=%d T=%d pdf=%d lnz=%lld narth=%.4e denwin=%d\n", s.m, s.n, s.nz, P.T, P.pdf,
                (long long)P.lnz, P.narth, P.denwin);
    std::printf("nsup=%d nlevels=%d lx=%lld (%.1f MB) max_h=%d max_nc=%d pairs=%zu rel=%zu flops=%.4e symbolic=%.3fs\n",
                P.nsup, P.nlevels, (long long)P.lx_size, P.lx_size * 8e-6, P.max_h, P.max_nc, P.upd_src.size(),
                P.rel.size(), P.flops_factor, dt);
    std::printf("tail: c0=%d nt=%d blocks=%d tasks=%zu flops_tail_update=%.3e flops_tail_factor=%.3e flops_update=%.3e\n",
                P.tail_c0, P.nt, P.ntb, P.tail_tasks.size(), P.flops_tail_update, P.flops_tail_factor, P.flops_update);
    if (argc > 2) {
        for (int l = 0; l < P.nlevels; l++) {
            int cnt = P.level_ptr[l + 1] - P.level_ptr[l];
            long work = 0; int maxh = 0;
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                int s2 = P.level_sups[q]; int h = P.col0[s2+1]-P.col0[s2] + P.rowptr[s2+1]-P.rowptr[s2];
                if (h > maxh) maxh = h; work += h;
            }
            std::printf("L%d: sups=%d rows=%ld maxh=%d\n", l, cnt, work, maxh);
        }
    }
    if (argc > 2 && std::string(argv[2]) == "units") {
        // per level: units, tasks, useful flops, and the critical path of the
        // mask gather = max over units of max over threads of sum ncd*cols
        double tot_crit = 0;
        for (int l = 0; l < P.nlevels; l++) {
            int u0 = P.unit_level_ptr[l], u1 = P.unit_level_ptr[l + 1];
            long ntask = 0, maxtask = 0; double flops = 0, crit = 0, sumcrit = 0;
            for (int u = u0; u < u1; u++) {
                long nt = P.task_ptr[u + 1] - P.task_ptr[u];
                ntask += nt; if (nt > maxtask) maxtask = nt;
                double thr[256] = {0};
                for (int t = P.task_ptr[u]; t < P.task_ptr[u + 1]; t++) {
                    const ipo::TailTask& tk = P.utasks[t];
                    int d = tk.src; int ncd = P.col0[d + 1] - P.col0[d];
                    int nr = __builtin_popcountll(tk.rmask), ncl = __builtin_popcountll(tk.cmask);
                    flops += 2.0 * nr * ncl * ncd;
                    for (int r = 0; r < 64; r++) if ((tk.rmask >> r) & 1)
                        for (int g = 0; g < 4; g++) thr[r + 64 * g] += ncd * __builtin_popcountll((tk.cmask >> (16 * g)) & 0xFFFF);
                }
                double mx = 0; for (int i = 0; i < 256; i++) mx = std::max(mx, thr[i]);
                crit = std::max(crit, mx); sumcrit += mx;
            }
            tot_crit += crit;
            std::printf("L%2d units=%6d tasks=%8ld maxtasks=%6ld flops=%.3e crit=%.0f mean=%.0f\n", l, u1 - u0, ntask, maxtask, flops, crit, (u1 > u0) ? sumcrit / (u1 - u0) : 0.0);
        }
        std::printf("sum of per-level critical paths = %.0f fma steps\n", tot_crit);
        double dense = 0, tot_maxk = 0; long totk = 0;
        for (int l = 0; l < P.nlevels; l++) {
            long mk = 0, sk = 0;
            for (int u = P.unit_level_ptr[l]; u < P.unit_level_ptr[l + 1]; u++) {
                long k = 0;
                for (int t = P.task_ptr[u]; t < P.task_ptr[u + 1]; t++) { int d = P.utasks[t].src; k += P.col0[d + 1] - P.col0[d]; }
                mk = std::max(mk, k); sk += k;
            }
            dense += 8192.0 * sk; tot_maxk += mk; totk += sk;
            std::printf("L%2d sumK=%ld maxK=%ld\n", l, sk, mk);
        }
        std::printf("dense-equivalent flops %.3e, sum K %ld, sum of per-level max K %.0f\n", dense, totk, tot_maxk);
    }
    // print perm hash for comparison
    unsigned long long hsh = 1469598103934665603ull;
    for (int v : P.perm) { hsh ^= (unsigned)v; hsh *= 1099511628211ull; }
    std::printf("perm_hash=%016llx\n", hsh);
    return 0;
}
