// Host-only table of the dense tail's structurally zero 64 x 64 blocks
// (developer tool, VERDICT r04 "next" 2(a)): for every (row block bi, column
// block b) of the tail's lower triangle, whether the factor's pattern has an
// entry there; then how many of the visits' and pre-updates' tile x block
// products L(bi, b) W(bj, b)' have a structurally zero operand block, and
// the tail's share of narth against the dense count nt^3 / 3.
//   g++ -O2 -std=c++17 -I linear-programming-vanderbei_amd/csrc tools/tail_blocks.cpp \
//       linear-programming-vanderbei_amd/csrc/kkt_symbolic.cpp linear-programming-vanderbei_amd/csrc/kkt_order_nd.cpp \
//       linear-programming-vanderbei_amd/csrc/lp_io.cpp -lpthread -o tools/tail_blocks && \
//   tools/tail_blocks tests/golden/netlib/dfl001.mps.gz
#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

#include "kkt_plan.h"
#include "lp_io.h"

using namespace ipo;

int main(int argc, char** argv) {
    if (argc < 2) { std::printf("usage: tail_blocks file.mps[.gz] [density]\n"); return 2; }
    const double rho = argc > 2 ? std::atof(argv[2]) : kTailDensity;
    MpsProblem mp;
    std::string err;
    if (read_mps(argv[1], mp, &err)) { std::printf("read: %s\n", err.c_str()); return 1; }
    SolverForm sf;
    to_solver_form(mp, sf);
    std::vector<int> kAt, iAt;
    std::vector<double> At;
    csc_transpose(sf.m, sf.n, sf.kA.data(), sf.iA.data(), sf.A.data(), kAt, iAt, At);
    KktOrdering o = order_tiered_min_degree(sf.m, sf.n, sf.kA.data(), sf.iA.data(), kAt.data(), iAt.data());
    KktPlan P = build_kkt_plan(sf.m, sf.n, sf.kA.data(), sf.iA.data(), kAt.data(), iAt.data(), 0, rho);
    const int T = o.T, tc = P.tail_c0, nt = P.nt, ntb = P.ntb, B = kTileRows;
    std::printf("T %d tail_c0 %d nt %d ntb %d narth %.4e\n", T, tc, nt, ntb, o.narth);
    std::vector<char> occ(static_cast<size_t>(ntb) * ntb, 0);   // occ[bi * ntb + b], bi >= b
    double tail_na = 0, tail_nnz = 0;
    for (int j = tc; j < T; j++) {
        const double c = o.Lp[j + 1] - o.Lp[j];
        tail_na += c * c;
        tail_nnz += c;
        const int b = (j - tc) / B;
        occ[static_cast<size_t>(b) * ntb + b] = 1;               // the diagonal block always
        for (int k = o.Lp[j]; k < o.Lp[j + 1]; k++) {
            const int r = o.Li[k];
            if (r < tc) { std::printf("row %d above the tail in tail column %d\n", r, j); return 1; }
            occ[static_cast<size_t>((r - tc) / B) * ntb + b] = 1;
        }
    }
    const double tail_work = tail_na + 3.0 * tail_nnz + nt;
    std::printf("tail share of narth: sum c^2 %.4e + 3 nnz %.4e + nt %d = %.4e (%.1f %% of narth); dense nt^3/3 %.4e\n",
                tail_na, 3.0 * tail_nnz, nt, tail_work, 100.0 * tail_work / o.narth, double(nt) * nt * nt / 3.0);
    long zb = 0, allb = 0;
    for (int b = 0; b < ntb; b++)
        for (int bi = b; bi < ntb; bi++) { allb++; zb += !occ[static_cast<size_t>(bi) * ntb + b]; }
    std::printf("lower-triangle blocks: %ld, structurally zero %ld (%.1f %%)\n", allb, zb, 100.0 * zb / allb);
    // trailing-update products (bi, bj, b), b < bj <= bi: the tile (bi, bj)
    // receives L(bi, b) W(bj, b)'; zero when either operand block is
    long prod = 0, prod_nz = 0, tiles = 0, tiles_nz = 0;
    for (int bj = 1; bj < ntb; bj++)
        for (int bi = bj; bi < ntb; bi++) {
            long nzp = 0;
            for (int b = 0; b < bj; b++) {
                prod++;
                const bool nz = occ[static_cast<size_t>(bi) * ntb + b] && occ[static_cast<size_t>(bj) * ntb + b];
                nzp += nz;
            }
            prod_nz += nzp;
            tiles++;
            tiles_nz += nzp > 0;
        }
    std::printf("update products: %ld, with both operand blocks nonzero %ld (%.1f %%); executed/algorithmic "
                "%.2f dense -> %.2f skipping\n",
                prod, prod_nz, 100.0 * prod_nz / prod, double(prod) * 2.0 * B * B * B / tail_work,
                double(prod_nz) * 2.0 * B * B * B / tail_work);
    std::printf("tiles receiving updates: %ld, with a nonzero product %ld\n", tiles, tiles_nz);
    // finer: MFMA instructions (16 rows x 16 columns x kg k) of the visits
    // whose row or column fragment has no entry in any of their kg k columns
    {
        const int F = 16;
        const int nf = (nt + F - 1) / F;
        for (int kg : {4, 16, 64}) {
            const int nkg = (nt + kg - 1) / kg;
            std::vector<char> fo(static_cast<size_t>(nf) * nkg, 0);   // row fragment x k group occupancy
            for (int j = tc; j < T; j++) {
                const int g = (j - tc) / kg;
                fo[static_cast<size_t>((j - tc) / F) * nkg + g] = 1;
                for (int k = o.Lp[j]; k < o.Lp[j + 1]; k++) fo[static_cast<size_t>((o.Li[k] - tc) / F) * nkg + g] = 1;
            }
            double all = 0, need = 0, useful = 0;
            for (int fj = 0; fj < nf; fj++)
                for (int fi = fj; fi < nf; fi++)
                    for (int g = 0; g < nkg && (g + 1) * kg <= (fj / 4) * 64; g++) {  // blocks left of column fj's block
                        all++;
                        need += fo[static_cast<size_t>(fi) * nkg + g] && fo[static_cast<size_t>(fj) * nkg + g];
                    }
            (void)useful;
            std::printf("fragments 16x16 x k-group %2d: %.3e products, %.3e needed (%.1f %%): executed/algorithmic %.2f\n",
                        kg, all, need, 100.0 * need / all, need * 2.0 * F * F * kg / tail_work);
        }
    }
    // per-column-block profile: first nonzero row block
    std::printf("column block: first-zero-free fraction (nonzero blocks / blocks below)\n");
    for (int b = 0; b < ntb; b++) {
        int nzb = 0;
        for (int bi = b; bi < ntb; bi++) nzb += occ[static_cast<size_t>(bi) * ntb + b];
        std::printf("%3d:%2d/%2d%s", b, nzb, ntb - b, (b % 8 == 7) ? "\n" : "  ");
    }
    std::printf("\n");
    return 0;
}
