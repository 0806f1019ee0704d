// kkt_emul.cpp -- developer tool: host emulation of the GPU supernodal
// factor/solve (same plan, same per-kernel arithmetic) to debug numerics on
// a machine without a GPU.  Compares against the oracle when linked with it.
//   build: see tools/README or the Makefile target `emul`
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../kkt_plan.h"
#include "../lp_io.h"

extern "C" {
#include "../../../oracle/orc.h"
}

using namespace ipo;

struct Emul {
    const KktPlan& P;
    int m, n, T;
    std::vector<double> Lx, dg, dscale, dinit;
    double tau = getenv("TAU") ? atof(getenv("TAU")) : 1e-30;
    std::vector<int> live;
    double epsdiag = 1e-14;
    int ndep = 0;
    Emul(const KktPlan& p) : P(p), m(p.m), n(p.n), T(p.T) {
        Lx.assign(P.lx_size, 0.0);
        dg.assign(T, 0.0);
        dscale.assign(T, 0.0);
        dinit.assign(T, 0.0);
        live.assign(T, 1);
    }
    int h_of(int s) const { return P.col0[s + 1] - P.col0[s] + P.rowptr[s + 1] - P.rowptr[s]; }

    void factor(const std::vector<double>& A, const std::vector<double>& E, const std::vector<double>& D) {
        std::fill(Lx.begin(), Lx.end(), 0.0);
        for (size_t k = 0; k < A.size(); k++) Lx[P.amap[k]] = A[k];
        for (int v = 0; v < T; v++) {
            int o = P.perm[v];
            Lx[P.dslot[v]] = o < m ? -(E[o] > epsdiag ? E[o] : epsdiag) : (D[o - m] > epsdiag ? D[o - m] : epsdiag);
            dscale[v] = std::fabs(Lx[P.dslot[v]]);
            dinit[v] = Lx[P.dslot[v]];
            live[v] = 1;
        }
        ndep = 0;
        for (int l = 0; l < P.nlevels; l++) {
            // update
            for (int u = P.unit_level_ptr[l]; u < P.unit_level_ptr[l + 1]; u++) {
                int s = P.unit_sup[u], t = P.unit_tile[u];
                int nc = P.col0[s + 1] - P.col0[s], h = h_of(s), rbase = t * kTileRows;
                int nrow = std::min(kTileRows, h - rbase);
                std::vector<double> acc(kTileRows * 64, 0.0);
                for (int task = P.task_ptr[u]; task < P.task_ptr[u + 1]; task++) {
                    int q = P.task_pair[task], i0 = P.task_i0[task], i1 = P.task_i1[task];
                    int d = P.upd_src[q], cd0 = P.col0[d], ncd = P.col0[d + 1] - cd0, hd = h_of(d);
                    int r0 = P.upd_r0[q], ncols = P.upd_r1[q] - r0;
                    const double* Ld = Lx.data() + P.off[d] + ncd + r0;
                    const int* rl = P.rel.data() + P.relptr[q];
                    for (int jj = 0; jj < ncols; jj++)
                        for (int ii = i0; ii < i1; ii++) {
                            int prow = rl[ii], pcol = rl[jj];
                            if (prow < pcol) continue;
                            double sum = 0.0, asum = 0.0;
                            for (int k = 0; k < ncd; k++) {
                                double t = Ld[ii + (size_t)k * hd] * (dg[cd0 + k] * Ld[jj + (size_t)k * hd]);
                                sum += t; asum += std::fabs(t);
                            }
                            acc[(prow - rbase) * 64 + pcol] += sum;
                            if (prow == pcol) dscale[P.col0[s] + pcol] += asum;
                        }
                }
                double* panel = Lx.data() + P.off[s];
                for (int c = 0; c < nc; c++)
                    for (int r = 0; r < nrow; r++)
                        if (rbase + r >= c) panel[(rbase + r) + (size_t)c * h] -= acc[r * 64 + c];
            }
            // diag (reference arithmetic form: l = a/d, update l_r * (l_c * d))
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                int s = P.level_sups[q], c0 = P.col0[s], nc = P.col0[s + 1] - c0, h = h_of(s);
                double* panel = Lx.data() + P.off[s];
                std::vector<double> B(64 * 64, 0.0);
                for (int c = 0; c < nc; c++) for (int r = c; r < nc; r++) B[r * 64 + c] = panel[r + (size_t)c * h];
                for (int k = 0; k < nc; k++) {
                    double dk = B[k * 64 + k];
                    int alive = 1;
                    if (std::fabs(dk) <= tau * dscale[c0 + k]) {
                        ndep++;
                        if (getenv("EMUL_DBG")) std::fprintf(stderr, "dep col %d d=%.3e scale=%.3e init=%.3e\n", c0 + k, dk, dscale[c0 + k], dinit[c0 + k]);
                        double mx = 0.0;
                        for (int r = k + 1; r < nc; r++) mx = std::max(mx, std::fabs(B[r * 64 + k]));
                        for (int rr = nc; rr < h; rr++) {
                            double w[64];
                            for (int c = 0; c <= k; c++) w[c] = panel[rr + (size_t)c * h];
                            for (int j = 0; j < k; j++) {
                                double lj = live[c0 + j] ? w[j] / dg[c0 + j] : 0.0;
                                for (int c = j + 1; c <= k; c++) w[c] -= lj * (B[c * 64 + j] * dg[c0 + j]);
                            }
                            mx = std::max(mx, std::fabs(w[k]));
                        }
                        if (mx < 1e-2) alive = 0;
                        else dk = (P.dsign[c0 + k] < 0 ? -1.0 : 1.0) * 1e-8;
                    }
                    dg[c0 + k] = dk;
                    live[c0 + k] = alive;
                    for (int r = k + 1; r < nc; r++) B[r * 64 + k] = alive ? B[r * 64 + k] / dk : 0.0;
                    for (int c = k + 1; c < nc; c++)
                        for (int r = c; r < nc; r++) {
                            double t = B[r * 64 + k] * (B[c * 64 + k] * dk);
                            B[r * 64 + c] -= t;
                            if (r == c) dscale[c0 + c] += std::fabs(t);
                        }
                }
                for (int r = 0; r < nc; r++) for (int c = 0; c < r; c++) panel[c + (size_t)r * h] = B[r * 64 + c];
            }
            // trsm
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                int s = P.level_sups[q], c0 = P.col0[s], nc = P.col0[s + 1] - c0, h = h_of(s);
                double* panel = Lx.data() + P.off[s];
                for (int rr = nc; rr < h; rr++) {
                    std::vector<double> R(nc);
                    for (int c = 0; c < nc; c++) R[c] = panel[rr + (size_t)c * h];
                    for (int k = 0; k < nc; k++) {
                        double lk = live[c0 + k] ? R[k] / dg[c0 + k] : 0.0;
                        R[k] = lk;
                        for (int c = k + 1; c < nc; c++) R[c] -= lk * (panel[k + (size_t)c * h] * dg[c0 + k]);
                    }
                    for (int c = 0; c < nc; c++) panel[rr + (size_t)c * h] = R[c];
                }
            }
        }
        if (P.nt > 0) tail_factor();
        double mn = HUGE_VAL;
        for (int v = 0; v < T; v++) mn = std::min(mn, std::fabs(dg[v]));
        if (mn < 1e-14) epsdiag *= 10;
    }

    // dense tail: gather (tile tasks) then right-looking blocked LDL' in the
    // same arithmetic form as the kernels (MFMA sums emulated in k order)
    void tail_factor() {
        const int nt = P.nt, tc = P.tail_c0, nb = P.ntb;
        double* S = Lx.data() + P.off_tail;
        for (int bi = 0; bi < nb; bi++)
            for (int bj = 0; bj <= bi; bj++) {
                int tile = bi * (bi + 1) / 2 + bj;
                std::vector<double> acc(64 * 64, 0.0), dab(64, 0.0);
                for (int t = P.tail_task_ptr[tile]; t < P.tail_task_ptr[tile + 1]; t++) {
                    const TailTask& tk = P.tail_tasks[t];
                    int d = tk.src, cd0 = P.col0[d], ncd = P.col0[d + 1] - cd0, hd = h_of(d);
                    const double* Ld = Lx.data() + P.off[d] + ncd;
                    for (int r = 0; r < 64; r++) {
                        if (!((tk.rmask >> r) & 1ull)) continue;
                        int ri = __builtin_popcountll(tk.rmask & ((1ull << r) - 1ull));
                        for (int c = 0; c < 64; c++) {
                            if (!((tk.cmask >> c) & 1ull)) continue;
                            if (bi == bj && c > r) continue;
                            int cj = __builtin_popcountll(tk.cmask & ((1ull << c) - 1ull));
                            double sum = 0.0, as = 0.0;
                            for (int k = 0; k < ncd; k++) {
                                double t2 = Ld[tk.rbase + ri + (size_t)k * hd] * (dg[cd0 + k] * Ld[tk.cbase + cj + (size_t)k * hd]);
                                sum += t2; as += std::fabs(t2);
                            }
                            acc[r * 64 + c] += sum;
                            if (bi == bj && c == r) dab[r] += as;
                        }
                    }
                }
                for (int r = 0; r < 64; r++)
                    for (int c = 0; c < 64; c++) {
                        int rg = bi * 64 + r, cg = bj * 64 + c;
                        if (rg >= nt || cg >= nt || (bi == bj && c > r)) continue;
                        S[rg + (size_t)cg * nt] -= acc[r * 64 + c];
                        if (bi == bj && c == r) dscale[tc + rg] += dab[r];
                    }
            }
        std::vector<double> W((size_t)nt * 64);
        for (int kb = 0; kb < nb; kb++) {
            int k0 = kb * 64, nc = std::min(64, nt - k0);
            diag_block(S + k0 + (size_t)k0 * nt, nt, nc, nt - k0, tc + k0);
            for (int rr = k0 + nc; rr < nt; rr++) {
                std::vector<double> R(nc);
                for (int c = 0; c < nc; c++) R[c] = S[rr + (size_t)(k0 + c) * nt];
                for (int k = 0; k < nc; k++) {
                    double lk = live[tc + k0 + k] ? R[k] / dg[tc + k0 + k] : 0.0;
                    R[k] = lk;
                    for (int c = k + 1; c < nc; c++) R[c] -= lk * (S[(k0 + k) + (size_t)(k0 + c) * nt] * dg[tc + k0 + k]);
                }
                for (int c = 0; c < nc; c++) { S[rr + (size_t)(k0 + c) * nt] = R[c]; W[(rr - k0) + (size_t)c * nt] = R[c] * dg[tc + k0 + c]; }
            }
            for (int cg = k0 + nc; cg < nt; cg++)
                for (int rg = cg; rg < nt; rg++) {
                    double acc = 0.0, as = 0.0;
                    for (int k = 0; k < nc; k++) {
                        double t2 = S[rg + (size_t)(k0 + k) * nt] * W[(cg - k0) + (size_t)k * nt];
                        if (getenv("EMUL_MFMA")) acc = std::fma(S[rg + (size_t)(k0 + k) * nt], W[(cg - k0) + (size_t)k * nt], acc);
                        else acc += t2;
                        as += std::fabs(t2);
                    }
                    S[rg + (size_t)cg * nt] -= acc;
                    if (rg == cg) dscale[tc + rg] += as;
                }
        }
    }

    // factor_diag_block of the kernels
    void diag_block(double* panel, int ld, int nc, int h, int c0) {
        std::vector<double> B(64 * 64, 0.0);
        for (int c = 0; c < nc; c++) for (int r = c; r < nc; r++) B[r * 64 + c] = panel[r + (size_t)c * ld];
        for (int k = 0; k < nc; k++) {
            double dk = B[k * 64 + k];
            int alive = 1;
            if (std::fabs(dk) <= tau * dscale[c0 + k]) {
                ndep++;
                if (getenv("EMUL_DBG")) std::fprintf(stderr, "dep col %d d=%.3e scale=%.3e init=%.3e\n", c0 + k, dk, dscale[c0 + k], dinit[c0 + k]);
                double mx = 0.0;
                for (int r = k + 1; r < nc; r++) mx = std::max(mx, std::fabs(B[r * 64 + k]));
                for (int rr = nc; rr < h; rr++) {
                    double w[64];
                    for (int c = 0; c <= k; c++) w[c] = panel[rr + (size_t)c * ld];
                    for (int j = 0; j < k; j++) {
                        double lj = live[c0 + j] ? w[j] / dg[c0 + j] : 0.0;
                        for (int c = j + 1; c <= k; c++) w[c] -= lj * (B[c * 64 + j] * dg[c0 + j]);
                    }
                    mx = std::max(mx, std::fabs(w[k]));
                }
                if (mx < 1e-2) alive = 0;
                else dk = (P.dsign[c0 + k] < 0 ? -1.0 : 1.0) * 1e-8;
            }
            dg[c0 + k] = dk;
            live[c0 + k] = alive;
            for (int r = k + 1; r < nc; r++) B[r * 64 + k] = alive ? B[r * 64 + k] / dk : 0.0;
            for (int c = k + 1; c < nc; c++)
                for (int r = c; r < nc; r++) {
                    double t2 = B[r * 64 + k] * (B[c * 64 + k] * dk);
                    B[r * 64 + c] -= t2;
                    if (r == c) dscale[c0 + c] += std::fabs(t2);
                }
        }
        for (int r = 0; r < nc; r++) for (int c = 0; c < r; c++) panel[c + (size_t)r * ld] = B[r * 64 + c];
    }

    bool zero_always = getenv("EMUL_ZERO_ALWAYS") && atoi(getenv("EMUL_ZERO_ALWAYS"));
    double eps_cur = 0.0;
    void nl(double& v) { if (zero_always || std::fabs(v) <= eps_cur) v = 0.0; }   // non-live rule of rawsolve
    void rawsolve(std::vector<double>& z) {
        eps_cur = 0.0;
        if (ndep) { double mx = 0; for (int i = 0; i < n; i++) mx = std::max(mx, std::fabs(z[i])); eps_cur = 1e-6 * mx; }
        for (int l = 0; l < P.nlevels; l++)
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                int s = P.level_sups[q], c0 = P.col0[s], nc = P.col0[s + 1] - c0, h = h_of(s);
                const double* panel = Lx.data() + P.off[s];
                std::vector<double> zl(nc);
                for (int k = 0; k < nc; k++) {
                    int v = c0 + k;
                    double acc = 0.0;
                    for (int e = P.frow_ptr[v]; e < P.frow_ptr[v + 1]; e++) acc += Lx[P.frow_pos[e]] * z[P.frow_col[e]];
                    zl[k] = z[v] - acc;
                }
                for (int j = 0; j < nc; j++) {
                    if (!live[c0 + j]) { nl(zl[j]); continue; }
                    for (int r = j + 1; r < nc; r++) zl[r] -= panel[j + (size_t)r * h] * zl[j];
                }
                for (int k = 0; k < nc; k++) z[c0 + k] = zl[k];
            }
        if (P.nt > 0) {
            const int nt = P.nt, tc = P.tail_c0;
            const double* S = Lx.data() + P.off_tail;
            for (int i = 0; i < nt; i++) {
                int v = tc + i; double acc = 0.0;
                for (int e = P.frow_ptr[v]; e < P.frow_ptr[v + 1]; e++) acc += Lx[P.frow_pos[e]] * z[P.frow_col[e]];
                z[v] -= acc;
            }
            for (int kb = 0; kb < P.ntb; kb++) {
                int k0 = kb * 64, nc = std::min(64, nt - k0);
                for (int j = 0; j < nc; j++) {
                    if (!live[tc + k0 + j]) { nl(z[tc + k0 + j]); continue; }
                    for (int r = j + 1; r < nc; r++) z[tc + k0 + r] -= S[(k0 + j) + (size_t)(k0 + r) * nt] * z[tc + k0 + j];
                }
                for (int r = k0 + nc; r < nt; r++) {
                    double acc = 0.0;
                    for (int k = 0; k < nc; k++) acc += S[r + (size_t)(k0 + k) * nt] * z[tc + k0 + k];
                    z[tc + r] -= acc;
                }
            }
            for (int i = 0; i < nt; i++) { int v = tc + i; if (live[v]) z[v] = z[v] / dg[v]; else nl(z[v]); }
            for (int kb = P.ntb - 1; kb >= 0; kb--) {
                int k0 = kb * 64, nc = std::min(64, nt - k0);
                std::vector<double> zl(nc);
                for (int k = 0; k < nc; k++) {
                    double acc = 0.0;
                    for (int r = k0 + nc; r < nt; r++) acc += S[r + (size_t)(k0 + k) * nt] * z[tc + r];
                    zl[k] = z[tc + k0 + k] - acc;
                }
                for (int j = nc - 1; j >= 0; j--) {
                    if (!live[tc + k0 + j]) { nl(zl[j]); continue; }
                    for (int r = 0; r < j; r++) zl[r] -= S[(k0 + r) + (size_t)(k0 + j) * nt] * zl[j];
                }
                for (int k = 0; k < nc; k++) z[tc + k0 + k] = zl[k];
            }
        }
        for (int l = P.nlevels - 1; l >= 0; l--)
            for (int q = P.level_ptr[l]; q < P.level_ptr[l + 1]; q++) {
                int s = P.level_sups[q], c0 = P.col0[s], nc = P.col0[s + 1] - c0, h = h_of(s);
                int hb = h - nc;
                const double* panel = Lx.data() + P.off[s];
                const int* rows = P.rows.data() + P.rowptr[s];
                std::vector<double> zl(nc);
                for (int k = 0; k < nc; k++) {
                    double acc = 0.0;
                    for (int i = 0; i < hb; i++) acc += panel[(size_t)k * h + nc + i] * z[rows[i]];
                    double zv = z[c0 + k];
                    if (live[c0 + k]) zv = zv / dg[c0 + k]; else nl(zv);
                    zl[k] = zv - acc;
                }
                for (int j = nc - 1; j >= 0; j--) {
                    if (!live[c0 + j]) { nl(zl[j]); continue; }
                    for (int r = 0; r < j; r++) zl[r] -= panel[r + (size_t)j * h] * zl[j];
                }
                for (int k = 0; k < nc; k++) z[c0 + k] = zl[k];
            }
    }
};

// refined solve exactly as ldlt.c:327-425 with the emulated rawsolve
static int emul_solve(Emul& em, const SolverForm& sf, const std::vector<int>& kat, const std::vector<int>& iat,
                      const std::vector<double>& at, const double* E, const double* D, double* fy, double* fx) {
    int m = sf.m, n = sf.n, T = m + n;
    std::vector<double> z(T), dy(m), dx(n), ry(m), rx(n);
    double bc = std::max(orc_maxabs(fx, n), orc_maxabs(fy, m)) + 1;
    double rs = HUGE_VAL, rs_old;
    int pass = 0;
    do {
        for (int v = 0; v < T; v++) { int o = em.P.perm[v]; z[v] = o < m ? (pass ? ry[o] : fy[o]) : (pass ? rx[o - m] : fx[o - m]); }
        em.rawsolve(z);
        for (int o = 0; o < T; o++) { double v = z[em.P.iperm[o]]; if (o < m) dy[o] = pass ? dy[o] + v : v; else dx[o - m] = pass ? dx[o - m] + v : v; }
        orc_spmv(n, m, at.data(), kat.data(), iat.data(), dy.data(), rx.data());
        orc_spmv(m, n, sf.A.data(), sf.kA.data(), sf.iA.data(), dx.data(), ry.data());
        for (int j = 0; j < m; j++) ry[j] = fy[j] - (ry[j] - E[j] * dy[j]);
        for (int i = 0; i < n; i++) rx[i] = fx[i] - (rx[i] + D[i] * dx[i]);
        rs_old = rs;
        rs = std::max(orc_maxabs(rx.data(), n), orc_maxabs(ry.data(), m));
        pass++;
    } while (rs > 1e-10 * bc && rs < rs_old / 2);
    if (rs > rs_old && pass > 1)
        for (int o = 0; o < T; o++) { double v = z[em.P.iperm[o]]; if (o < m) dy[o] -= v; else dx[o - m] -= v; }
    for (int j = 0; j < m; j++) fy[j] = dy[j];
    for (int i = 0; i < n; i++) fx[i] = dx[i];
    return pass;
}

static int emul_hsd(const char* path, bool verbose) {
    MpsProblem p; std::string err;
    if (read_mps(path, p, &err)) return -1;
    SolverForm sf;
    if (to_solver_form(p, sf)) return -3;
    int m = sf.m, n = sf.n;
    std::vector<int> kat, iat; std::vector<double> at;
    csc_transpose(m, n, sf.kA.data(), sf.iA.data(), sf.A.data(), kat, iat, at);
    KktPlan P = build_kkt_plan(m, n, sf.kA.data(), sf.iA.data(), kat.data(), iat.data());
    Emul em(P);
    const double* b = sf.b.data(); const double* c = sf.c.data();
    std::vector<double> x(n, 1), z(n, 1), y(m, 1), w(m, 1), rho(m), sig(n), D(n), E(m), fx(n), fy(m), gx(n), gy(m), dx(n), dy(m), dz(n), dw(m);
    double phi = 1, psi = 1;
    int iter;
    for (iter = 0; iter < 200; iter++) {
        double mu = (orc_dot(z.data(), x.data(), n) + orc_dot(w.data(), y.data(), m) + phi * psi) / (n + m + 1);
        double delta = iter % 2 ? 1.0 : 0.0;
        double pobj = orc_dot(c, x.data(), n), dobj = orc_dot(b, y.data(), m);
        if (mu < 1e-12) break;
        orc_spmv(m, n, sf.A.data(), sf.kA.data(), sf.iA.data(), x.data(), rho.data());
        for (int i = 0; i < m; i++) rho[i] = rho[i] - b[i] * phi + w[i];
        double normr = std::sqrt(orc_dot(rho.data(), rho.data(), m)) / phi;
        for (int i = 0; i < m; i++) rho[i] = -(1 - delta) * rho[i] + w[i] - delta * mu / y[i];
        orc_spmv(n, m, at.data(), kat.data(), iat.data(), y.data(), sig.data());
        for (int j = 0; j < n; j++) sig[j] = -sig[j] + c[j] * phi + z[j];
        double norms = std::sqrt(orc_dot(sig.data(), sig.data(), n)) / phi;
        for (int j = 0; j < n; j++) sig[j] = -(1 - delta) * sig[j] + z[j] - delta * mu / x[j];
        double gamma = -(1 - delta) * (dobj - pobj + psi) + psi - delta * mu / phi;
        if (verbose) std::fprintf(stderr, "FT %d %.17g %.17g %.17g %.17g %.17g %.17g\n", iter, pobj, dobj, mu, phi, psi, normr);
        for (int j = 0; j < n; j++) D[j] = z[j] / x[j];
        for (int i = 0; i < m; i++) E[i] = w[i] / y[i];
        em.factor(sf.A, E, D);
        if (verbose) std::fprintf(stderr, "FT   ndep=%d eps=%.1e\n", em.ndep, em.epsdiag);
        for (int j = 0; j < n; j++) fx[j] = -sig[j];
        for (int i = 0; i < m; i++) fy[i] = rho[i];
        emul_solve(em, sf, kat, iat, at, E.data(), D.data(), fy.data(), fx.data());
        for (int j = 0; j < n; j++) gx[j] = -c[j];
        for (int i = 0; i < m; i++) gy[i] = -b[i];
        emul_solve(em, sf, kat, iat, at, E.data(), D.data(), gy.data(), gx.data());
        double dphi = (orc_dot(c, fx.data(), n) - orc_dot(b, fy.data(), m) + gamma) / (orc_dot(c, gx.data(), n) - orc_dot(b, gy.data(), m) - psi / phi);
        for (int j = 0; j < n; j++) dx[j] = fx[j] - gx[j] * dphi;
        for (int i = 0; i < m; i++) dy[i] = fy[i] - gy[i] * dphi;
        for (int j = 0; j < n; j++) dz[j] = delta * mu / x[j] - z[j] - D[j] * dx[j];
        for (int i = 0; i < m; i++) dw[i] = delta * mu / y[i] - w[i] - E[i] * dy[i];
        double dpsi = delta * mu / phi - psi - (psi / phi) * dphi;
        double theta = 0;
        for (int j = 0; j < n; j++) { if (theta < -dx[j] / x[j]) theta = -dx[j] / x[j]; if (theta < -dz[j] / z[j]) theta = -dz[j] / z[j]; }
        for (int i = 0; i < m; i++) { if (theta < -dy[i] / y[i]) theta = -dy[i] / y[i]; if (theta < -dw[i] / w[i]) theta = -dw[i] / w[i]; }
        if (theta < -dphi / phi) theta = -dphi / phi;
        if (theta < -dpsi / psi) theta = -dpsi / psi;
        theta = (0.95 / theta > 1.0) ? 1.0 : 0.95 / theta;
        for (int j = 0; j < n; j++) { x[j] += theta * dx[j]; z[j] += theta * dz[j]; }
        for (int i = 0; i < m; i++) { y[i] += theta * dy[i]; w[i] += theta * dw[i]; }
        phi += theta * dphi; psi += theta * dpsi;
    }
    return iter;
}

int main(int argc, char** argv) {
    if (argc > 2 && !std::strcmp(argv[1], "hsd")) {
        for (int a = 2; a < argc; a++) {
            int it = emul_hsd(argv[a], getenv("VERBOSE") != nullptr);
            std::printf("%s %d\n", argv[a], it);
        }
        return 0;
    }
    const char* path = argc > 1 ? argv[1] : "/tmp/mps/blend.mps";
    MpsProblem p; std::string err;
    if (read_mps(path, p, &err)) { std::printf("read: %s\n", err.c_str()); return 1; }
    SolverForm s;
    to_solver_form(p, s);
    std::vector<int> kat, iat; std::vector<double> at;
    csc_transpose(s.m, s.n, s.kA.data(), s.iA.data(), s.A.data(), kat, iat, at);
    KktPlan P = build_kkt_plan(s.m, s.n, s.kA.data(), s.iA.data(), kat.data(), iat.data());
    Emul em(P);
    orc_kkt* K = orc_kkt_create(s.m, s.n, s.kA.data(), s.iA.data(), s.A.data(), kat.data(), iat.data(), at.data());
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(-1, 1);
    double lo = argc > 2 ? atof(argv[2]) : -1, hi = argc > 3 ? atof(argv[3]) : 1;
    std::uniform_real_distribution<double> EX(lo, hi);
    std::vector<double> E(s.m), D(s.n), fy(s.m), fx(s.n);
    for (auto& v : E) v = std::pow(10.0, EX(rng));
    for (auto& v : D) v = std::pow(10.0, EX(rng));
    for (auto& v : fy) v = U(rng);
    for (auto& v : fx) v = U(rng);
    if (argc > 4) {   // captured state from ORC_DUMP_ED
        FILE* f = std::fopen(argv[4], "rb");
        int mm, nn; double eps;
        std::fread(&mm, sizeof(int), 1, f); std::fread(&nn, sizeof(int), 1, f);
        std::fread(E.data(), sizeof(double), mm, f); std::fread(D.data(), sizeof(double), nn, f);
        std::fread(&eps, sizeof(double), 1, f); std::fclose(f);
        em.epsdiag = eps; orc_kkt_set_epsdiag(K, eps);
    }
    em.factor(s.A, E, D);
    orc_kkt_factor(K, E.data(), D.data());
    int dropped = 0; for (int v = 0; v < P.T; v++) dropped += !em.live[v];
    std::printf("emul ndep=%d dropped=%d | oracle ndep=%d\n", em.ndep, dropped, orc_kkt_ndep(K));
    std::vector<double> od(P.T);
    orc_kkt_diag(K, od.data());
    double maxrel = 0; int worst = -1;
    for (int v = 0; v < P.T; v++) {
        double r = std::fabs(em.dg[v] - od[v]) / std::max(1e-300, std::fabs(od[v]));
        if (r > maxrel) { maxrel = r; worst = v; }
    }
    if (getenv("EMUL_DBG")) for (int v = 0; v < P.T; v++) if (od[v] == 0.0 || !em.live[v] || em.dg[v] == 0.0) {
        int sp = P.sup_of[v];
        std::printf("  v=%d old=%d(%c) sup=%d c0=%d nc=%d h=%d | emul d=%.6e live=%d | oracle d=%.6e\n", v, P.perm[v],
                    P.perm[v] < s.m ? 'y' : 'x', sp, P.col0[sp], P.col0[sp+1]-P.col0[sp], em.h_of(sp), em.dg[v], em.live[v], od[v]);
    }
    std::printf("diag max rel diff %.3e at %d (emul %.6e oracle %.6e)\n", maxrel, worst, worst >= 0 ? em.dg[worst] : 0.0,
                worst >= 0 ? od[worst] : 0.0);
    // one raw solve on the same permuted rhs
    std::vector<double> z(P.T), z2(P.T);
    for (int v = 0; v < P.T; v++) { int o = P.perm[v]; z[v] = o < s.m ? fy[o] : fx[o - s.m]; }
    z2 = z;
    em.rawsolve(z);
    orc_kkt_rawsolve(K, z2.data());
    double md = 0, mz = 0;
    for (int v = 0; v < P.T; v++) { md = std::max(md, std::fabs(z[v] - z2[v])); mz = std::max(mz, std::fabs(z2[v])); }
    std::printf("rawsolve max abs diff %.3e (|z| %.3e)\n", md, mz);
    return 0;
}
