/*
 * orc_ipm.c -- ORACLE (test infrastructure only, see orc.h).
 *
 * Restatements of the three solver() methods that ipo can link:
 *   orc_hsd    homogeneous self-dual predictor-corrector, src/ipo/hsd.c:27-311
 *   orc_intpt  primal-dual path following,               src/ipo/intpt.c:33-261
 *   orc_hsdls  homogeneous self-dual long step,          src/ipo/hsdls.c:38-336
 * plus the BLAS-1 / SpMV helpers of src/common/linalg.c:17-116 and the
 * driver of src/common/main.c:16-58 (banner, read, solvelp, status text).
 * Every expression is written in the reference's evaluation order.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "orc.h"

double orc_dot(const double *x, const double *y, int n)
{
    double s = 0.0e0;
    for (int i = 0; i < n; i++) s += x[i] * y[i];
    return s;
}

void orc_spmv(int m, int n, const double *a, const int *ka, const int *ia, const double *x, double *y)
{
    for (int i = 0; i < m; i++) y[i] = 0.0e0;
    for (int j = 0; j < n; j++)
        for (int k = ka[j]; k < ka[j + 1]; k++) y[ia[k]] += a[k] * x[j];
}

void orc_transpose(int m, int n, const int *ka, const int *ia, const double *a, int *kat, int *iat, double *at)
{
    int *cnt = calloc((size_t)(m > 0 ? m : 1), sizeof(int));
    for (int k = 0; k < ka[n]; k++) cnt[ia[k]]++;
    kat[0] = 0;
    for (int i = 0; i < m; i++) { kat[i + 1] = kat[i] + cnt[i]; cnt[i] = 0; }
    for (int j = 0; j < n; j++)
        for (int k = ka[j]; k < ka[j + 1]; k++) {
            int r = ia[k], dst = kat[r] + cnt[r]++;
            iat[dst] = j; at[dst] = a[k];
        }
    free(cnt);
}

double orc_maxabs(const double *x, int n)
{
    double v = 0.0e0;
    for (int i = 0; i < n; i++) { double ax = x[i] > 0 ? x[i] : -x[i]; v = v > ax ? v : ax; }
    return v;
}

static double now_s(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }
static double *vec(int n) { return malloc(sizeof(double) * (size_t)(n > 0 ? n : 1)); }

static void print_small(FILE *tr, int m, int n, const int *kA, const int *iA, const double *A, const double *b, const double *c)
{
    /* hsd.c:70-92 / intpt.c:70-92 */
    double AA[20][20];
    for (int j = 0; j < n; j++) for (int i = 0; i < m; i++) AA[i][j] = 0;
    for (int j = 0; j < n; j++) for (int k = kA[j]; k < kA[j + 1]; k++) AA[iA[k]][j] = A[k];
    fprintf(tr, "A <= b: \n");
    for (int i = 0; i < m; i++) {
        for (int j = 0; j < n; j++) fprintf(tr, " %5.1f", AA[i][j]);
        fprintf(tr, "<= %5.1f \n", b[i]);
    }
    fprintf(tr, "\n");
    fprintf(tr, "c: \n");
    for (int j = 0; j < n; j++) fprintf(tr, " %5.1f", c[j]);
    fprintf(tr, "\n");
}

int orc_hsd(int m, int n, int nz, const int *iA, const int *kA, const double *A,
            const double *b, const double *c, double f,
            double *x, double *y, double *w, double *z, orc_run *run)
{
    FILE *tr = run ? run->trace : NULL;
    int maxit = run && run->max_iter > 0 ? run->max_iter : 200;
    const double eps = 1.0e-12;
    double t0 = now_s();
    double *dx = vec(n), *dw = vec(m), *dy = vec(m), *dz = vec(n);
    double *rho = vec(m), *sig = vec(n), *D = vec(n), *E = vec(m);
    double *fx = vec(n), *fy = vec(m), *gx = vec(n), *gy = vec(m);
    double *At = vec(nz); int *iAt = malloc(sizeof(int) * (size_t)(nz ? nz : 1)), *kAt = malloc(sizeof(int) * (size_t)(m + 1));
    int status = 5, iter;
    double phi, psi, dphi, dpsi, normr, norms, gamma, delta, mu, theta, pobj, dobj;
    orc_kkt *K = NULL;

    if (tr && m < 20 && n < 20) print_small(tr, m, n, kA, iA, A, b, c);
    for (int j = 0; j < n; j++) { x[j] = 1.0; z[j] = 1.0; }
    for (int i = 0; i < m; i++) { w[i] = 1.0; y[i] = 1.0; }
    phi = 1.0; psi = 1.0;
    orc_transpose(m, n, kA, iA, A, kAt, iAt, At);
    if (tr) {
        fprintf(tr, "m = %d,n = %d,nz = %d\n", m, n, nz);
        fprintf(tr,
"--------------------------------------------------------------------------\n"
"         |           Primal          |            Dual           |       |\n"
"  Iter   |  Obj Value       Infeas   |  Obj Value       Infeas   |  mu   |\n"
"- - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - \n");
        fflush(tr);
    }
    const int dbg_step = getenv("ORC_DEBUG_STEP") != NULL;
    for (iter = 0; iter < maxit; iter++) {
        mu = (orc_dot(z, x, n) + orc_dot(w, y, m) + phi * psi) / (n + m + 1);
        delta = (iter % 2 == 0) ? 0.0 : 1.0;
        pobj = orc_dot(c, x, n);
        dobj = orc_dot(b, y, m);
        if (mu < eps) {
            if (phi > psi) status = 0;
            else if (dobj < 0.0) status = 2;
            else if (pobj > 0.0) status = 4;
            else { if (tr) fprintf(tr, "Trouble in river city \n"); status = 4; }
            break;
        }
        orc_spmv(m, n, A, kA, iA, x, rho);
        for (int i = 0; i < m; i++) rho[i] = rho[i] - b[i] * phi + w[i];
        normr = sqrt(orc_dot(rho, rho, m)) / phi;
        for (int i = 0; i < m; i++) rho[i] = -(1 - delta) * rho[i] + w[i] - delta * mu / y[i];

        orc_spmv(n, m, At, kAt, iAt, y, sig);
        for (int j = 0; j < n; j++) sig[j] = -sig[j] + c[j] * phi + z[j];
        norms = sqrt(orc_dot(sig, sig, n)) / phi;
        for (int j = 0; j < n; j++) sig[j] = -(1 - delta) * sig[j] + z[j] - delta * mu / x[j];

        gamma = -(1 - delta) * (dobj - pobj + psi) + psi - delta * mu / phi;

        if (tr) {
            fprintf(tr, "%8d   %14.7e  %8.1e    %14.7e  %8.1e  %8.1e \n",
                    iter, pobj / phi + f, normr, dobj / phi + f, norms, mu);
            fflush(tr);
        }
        if (run) { run->final_mu = mu; run->final_pobj = pobj / phi + f; run->final_dobj = dobj / phi + f; run->final_pinf = normr; run->final_dinf = norms; }

        for (int j = 0; j < n; j++) D[j] = z[j] / x[j];
        for (int i = 0; i < m; i++) E[i] = w[i] / y[i];

        if (!K) {
            double ts = now_s();
            K = orc_kkt_create(m, n, kA, iA, A, kAt, iAt, At);
            if (run) run->t_setup = now_s() - ts;
        }
        orc_kkt_factor(K, E, D);

        for (int j = 0; j < n; j++) fx[j] = -sig[j];
        for (int i = 0; i < m; i++) fy[i] = rho[i];
        orc_kkt_solve(K, E, D, fy, fx);
        int dbg_p1 = orc_kkt_last_passes(K);
        double dbg_r1 = orc_kkt_last_resid(K);
        for (int j = 0; j < n; j++) gx[j] = -c[j];
        for (int i = 0; i < m; i++) gy[i] = -b[i];
        orc_kkt_solve(K, E, D, gy, gx);

        dphi = (orc_dot(c, fx, n) - orc_dot(b, fy, m) + gamma) /
               (orc_dot(c, gx, n) - orc_dot(b, gy, m) - psi / phi);
        for (int j = 0; j < n; j++) dx[j] = fx[j] - gx[j] * dphi;
        for (int i = 0; i < m; i++) dy[i] = fy[i] - gy[i] * dphi;
        for (int j = 0; j < n; j++) dz[j] = delta * mu / x[j] - z[j] - D[j] * dx[j];
        for (int i = 0; i < m; i++) dw[i] = delta * mu / y[i] - w[i] - E[i] * dy[i];
        dpsi = delta * mu / phi - psi - (psi / phi) * dphi;

        theta = 0.0;
        for (int j = 0; j < n; j++) {
            if (theta < -dx[j] / x[j]) theta = -dx[j] / x[j];
            if (theta < -dz[j] / z[j]) theta = -dz[j] / z[j];
        }
        for (int i = 0; i < m; i++) {
            if (theta < -dy[i] / y[i]) theta = -dy[i] / y[i];
            if (theta < -dw[i] / w[i]) theta = -dw[i] / w[i];
        }
        if (theta < -dphi / phi) theta = -dphi / phi;
        if (theta < -dpsi / psi) theta = -dpsi / psi;
        if (dbg_step) {   /* diagnostics (ORC_DEBUG_STEP): the step and the KKT solves behind it */
            int bk = -1, bi = -1;
            double bt = 0.0;
            for (int j = 0; j < n; j++) {
                if (-dx[j] / x[j] > bt) { bt = -dx[j] / x[j]; bk = 0; bi = j; }
                if (-dz[j] / z[j] > bt) { bt = -dz[j] / z[j]; bk = 1; bi = j; }
            }
            for (int i = 0; i < m; i++) {
                if (-dy[i] / y[i] > bt) { bt = -dy[i] / y[i]; bk = 2; bi = i; }
                if (-dw[i] / w[i] > bt) { bt = -dw[i] / w[i]; bk = 3; bi = i; }
            }
            if (-dphi / phi > bt) { bt = -dphi / phi; bk = 4; bi = 0; }
            if (-dpsi / psi > bt) { bt = -dpsi / psi; bk = 5; bi = 0; }
            static const char *kn[] = {"x", "z", "y", "w", "phi", "psi"};
            fprintf(stderr, "step %3d: theta %.3e by %s[%d] ndep %d epsdiag %.0e passes %d/%d resid %.1e/%.1e "
                            "phi %.3e psi %.3e dphi %.3e\n", iter, 0.95 / theta > 1.0 ? 1.0 : 0.95 / theta,
                    bk >= 0 ? kn[bk] : "-", bi, orc_kkt_ndep(K), orc_kkt_epsdiag(K), dbg_p1,
                    orc_kkt_last_passes(K), dbg_r1, orc_kkt_last_resid(K), phi, psi, dphi);
        }
        theta = (0.95 / theta > 1.0) ? 1.0 : 0.95 / theta;   /* MIN(0.95/theta, 1.0) */

        for (int j = 0; j < n; j++) { x[j] = x[j] + theta * dx[j]; z[j] = z[j] + theta * dz[j]; }
        for (int i = 0; i < m; i++) { y[i] = y[i] + theta * dy[i]; w[i] = w[i] + theta * dw[i]; }
        phi = phi + theta * dphi;
        psi = psi + theta * dpsi;
    }
    for (int j = 0; j < n; j++) { x[j] /= phi; z[j] /= phi; }
    for (int i = 0; i < m; i++) { y[i] /= phi; w[i] /= phi; }

    if (run) { run->iters = iter; run->t_total = now_s() - t0; }
    orc_kkt_destroy(K);
    free(dx); free(dw); free(dy); free(dz); free(rho); free(sig); free(D); free(E);
    free(fx); free(fy); free(gx); free(gy); free(At); free(iAt); free(kAt);
    return status;
}

int orc_intpt(int m, int n, int nz, const int *iA, const int *kA, const double *A,
              const double *b, const double *c, double f,
              double *x, double *y, double *w, double *z, orc_run *run)
{
    FILE *tr = run ? run->trace : NULL;
    int maxit = run && run->max_iter > 0 ? run->max_iter : 200;
    const double eps = 1.0e-6;
    double t0 = now_s();
    double *dx = vec(n), *dw = vec(m), *dy = vec(m), *dz = vec(n);
    double *rho = vec(m), *sig = vec(n), *D = vec(n), *E = vec(m);
    double *At = vec(nz); int *iAt = malloc(sizeof(int) * (size_t)(nz ? nz : 1)), *kAt = malloc(sizeof(int) * (size_t)(m + 1));
    int status = 5, iter;
    double normr0, norms0, gamma, delta, mu, theta, r;
    float pobj, dobj, normr, norms;      /* intpt.c:47 -- single precision */
    orc_kkt *K = NULL;

    if (tr && m < 20 && n < 20) print_small(tr, m, n, kA, iA, A, b, c);
    for (int j = 0; j < n; j++) { x[j] = 1000.0; z[j] = 1000.0; }
    for (int i = 0; i < m; i++) { w[i] = 1000.0; y[i] = 1000.0; }
    orc_transpose(m, n, kA, iA, A, kAt, iAt, At);
    delta = 0.02; r = 0.9;
    normr0 = HUGE_VAL; norms0 = HUGE_VAL;
    if (tr) {
        fprintf(tr, "m = %d,n = %d,nz = %d\n", m, n, nz);
        fprintf(tr,
"------------------------------------------------------------------\n"
"         |           Primal          |            Dual           |\n"
"  Iter   |  Obj Value       Infeas   |  Obj Value       Infeas   |\n"
"- - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - \n");
        fflush(tr);
    }
    for (iter = 0; iter < maxit; iter++) {
        orc_spmv(m, n, A, kA, iA, x, rho);
        for (int i = 0; i < m; i++) rho[i] = b[i] - rho[i] - w[i];
        normr = sqrt(orc_dot(rho, rho, m));
        orc_spmv(n, m, At, kAt, iAt, y, sig);
        for (int j = 0; j < n; j++) sig[j] = c[j] - sig[j] + z[j];
        norms = sqrt(orc_dot(sig, sig, n));
        gamma = orc_dot(z, x, n) + orc_dot(y, w, m);
        pobj = orc_dot(c, x, n) + f;
        dobj = orc_dot(b, y, m) + f;
        if (tr) {
            fprintf(tr, "%8d   %14.7e  %8.1e    %14.7e  %8.1e \n", iter, pobj, normr, dobj, norms);
            fflush(tr);
        }
        if (run) { run->final_mu = gamma; run->final_pobj = pobj; run->final_dobj = dobj; run->final_pinf = normr; run->final_dinf = norms; }
        if (normr < eps && norms < eps && gamma < eps) { status = 0; break; }
        if (normr > 10 * normr0) { status = 2; break; }
        if (norms > 10 * norms0) { status = 4; break; }

        mu = delta * gamma / (n + m);
        for (int j = 0; j < n; j++) D[j] = z[j] / x[j];
        for (int i = 0; i < m; i++) E[i] = w[i] / y[i];
        if (!K) {
            double ts = now_s();
            K = orc_kkt_create(m, n, kA, iA, A, kAt, iAt, At);
            if (run) run->t_setup = now_s() - ts;
        }
        orc_kkt_factor(K, E, D);
        for (int j = 0; j < n; j++) dx[j] = sig[j] - z[j] + mu / x[j];
        for (int i = 0; i < m; i++) dy[i] = rho[i] + w[i] - mu / y[i];
        orc_kkt_solve(K, E, D, dy, dx);
        for (int j = 0; j < n; j++) dz[j] = mu / x[j] - z[j] - D[j] * dx[j];
        for (int i = 0; i < m; i++) dw[i] = mu / y[i] - w[i] - E[i] * dy[i];

        theta = 0.0;
        for (int j = 0; j < n; j++) {
            if (theta < -dx[j] / x[j]) theta = -dx[j] / x[j];
            if (theta < -dz[j] / z[j]) theta = -dz[j] / z[j];
        }
        for (int i = 0; i < m; i++) {
            if (theta < -dy[i] / y[i]) theta = -dy[i] / y[i];
            if (theta < -dw[i] / w[i]) theta = -dw[i] / w[i];
        }
        theta = (r / theta > 1.0) ? 1.0 : r / theta;
        for (int j = 0; j < n; j++) { x[j] = x[j] + theta * dx[j]; z[j] = z[j] + theta * dz[j]; }
        for (int i = 0; i < m; i++) { y[i] = y[i] + theta * dy[i]; w[i] = w[i] + theta * dw[i]; }
        normr0 = normr;
        norms0 = norms;
    }
    if (run) { run->iters = iter; run->t_total = now_s() - t0; }
    orc_kkt_destroy(K);
    free(dx); free(dw); free(dy); free(dz); free(rho); free(sig); free(D); free(E);
    free(At); free(iAt); free(kAt);
    return status;
}

/* hsdls.c:298-336 -- largest step keeping x z >= (1-beta) mu along the
 * centred direction: root of a t^2 + b t + c = 0, HUGE_VAL when unbounded */
double orc_linesearch(double xj, double zj, double dxj, double dzj, double beta, double delta, double mu)
{
    double a = dxj * dzj;
    double b = zj * dxj + xj * dzj + (1 - beta) * (1 - delta) * mu;
    double c = xj * zj - (1 - beta) * mu;
    double d = b * b - 4 * a * c;
    if (a == 0.0) return -c / b;
    if (a > 0) {
        if (b < 0) {
            if (d >= 0) return 2 * c / (-b + sqrt(d));
            return HUGE_VAL;
        }
        return HUGE_VAL;
    }
    if (b < 0) return 2 * c / (-b + sqrt(d));
    return (-b - sqrt(d)) / (2 * a);
}

int orc_hsdls(int m, int n, int nz, const int *iA, const int *kA, const double *A,
              const double *b, const double *c, double f,
              double *x, double *y, double *w, double *z, orc_run *run)
{
    FILE *tr = run ? run->trace : NULL;
    int maxit = run && run->max_iter > 0 ? run->max_iter : 600;      /* hsdls.c:25 */
    const double eps = 1.0e-12;
    double t0 = now_s();
    double *dx = vec(n), *dw = vec(m), *dy = vec(m), *dz = vec(n);
    double *rho = vec(m), *sig = vec(n), *D = vec(n), *E = vec(m);
    double *fx = vec(n), *fy = vec(m), *gx = vec(n), *gy = vec(m);
    double *At = vec(nz); int *iAt = malloc(sizeof(int) * (size_t)(nz ? nz : 1)), *kAt = malloc(sizeof(int) * (size_t)(m + 1));
    int status = 5, iter;
    double phi, psi, dphi, dpsi, normr, norms, gamma, beta, delta, mu, theta, pobj, dobj;
    orc_kkt *K = NULL;

    for (int j = 0; j < n; j++) { x[j] = 1.0; z[j] = 1.0; }
    for (int i = 0; i < m; i++) { w[i] = 1.0; y[i] = 1.0; }
    phi = 1.0; psi = 1.0;
    orc_transpose(m, n, kA, iA, A, kAt, iAt, At);
    if (tr) {
        fprintf(tr, "m = %d,n = %d,nz = %d\n", m, n, nz);
        fprintf(tr,
"--------------------------------------------------------------------------\n"
"         |           Primal          |            Dual           |       |\n"
"  Iter   |  Obj Value       Infeas   |  Obj Value       Infeas   |  mu   |\n"
"- - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - \n");
        fflush(tr);
    }
    beta = 0.80;
    delta = 2 * (1 - beta);
    for (iter = 0; iter < maxit; iter++) {
        mu = (orc_dot(z, x, n) + orc_dot(w, y, m) + phi * psi) / (n + m + 1);
        pobj = orc_dot(c, x, n);
        dobj = orc_dot(b, y, m);
        if (mu < eps) {
            if (phi > eps) status = 0;
            else if (dobj < 0.0) status = 2;
            else if (pobj > 0.0) status = 4;
            else status = 7;
            break;
        }
        orc_spmv(m, n, A, kA, iA, x, rho);
        for (int i = 0; i < m; i++) rho[i] = rho[i] - b[i] * phi + w[i];
        normr = sqrt(orc_dot(rho, rho, m)) / phi;
        for (int i = 0; i < m; i++) rho[i] = -(1 - delta) * rho[i] + w[i] - delta * mu / y[i];

        orc_spmv(n, m, At, kAt, iAt, y, sig);
        for (int j = 0; j < n; j++) sig[j] = -sig[j] + c[j] * phi + z[j];
        norms = sqrt(orc_dot(sig, sig, n)) / phi;
        for (int j = 0; j < n; j++) sig[j] = -(1 - delta) * sig[j] + z[j] - delta * mu / x[j];

        gamma = -(1 - delta) * (dobj - pobj + psi) + psi - delta * mu / phi;

        if (tr) {
            fprintf(tr, "%8d   %14.7e  %8.1e    %14.7e  %8.1e  %8.1e \n",
                    iter, pobj / phi + f, normr, dobj / phi + f, norms, mu);
            fflush(tr);
        }
        if (run) { run->final_mu = mu; run->final_pobj = pobj / phi + f; run->final_dobj = dobj / phi + f; run->final_pinf = normr; run->final_dinf = norms; }

        for (int j = 0; j < n; j++) D[j] = z[j] / x[j];
        for (int i = 0; i < m; i++) E[i] = w[i] / y[i];
        if (!K) {
            double ts = now_s();
            K = orc_kkt_create(m, n, kA, iA, A, kAt, iAt, At);
            if (run) run->t_setup = now_s() - ts;
        }
        orc_kkt_factor(K, E, D);
        for (int j = 0; j < n; j++) fx[j] = -sig[j];
        for (int i = 0; i < m; i++) fy[i] = rho[i];
        orc_kkt_solve(K, E, D, fy, fx);
        for (int j = 0; j < n; j++) gx[j] = -c[j];
        for (int i = 0; i < m; i++) gy[i] = -b[i];
        orc_kkt_solve(K, E, D, gy, gx);

        dphi = (orc_dot(c, fx, n) - orc_dot(b, fy, m) + gamma) /
               (orc_dot(c, gx, n) - orc_dot(b, gy, m) - psi / phi);
        for (int j = 0; j < n; j++) dx[j] = fx[j] - gx[j] * dphi;
        for (int i = 0; i < m; i++) dy[i] = fy[i] - gy[i] * dphi;
        for (int j = 0; j < n; j++) dz[j] = delta * mu / x[j] - z[j] - D[j] * dx[j];
        for (int i = 0; i < m; i++) dw[i] = delta * mu / y[i] - w[i] - E[i] * dy[i];
        dpsi = delta * mu / phi - psi - (psi / phi) * dphi;

        theta = 1.0;
        for (int j = 0; j < n; j++) {
            double t = orc_linesearch(x[j], z[j], dx[j], dz[j], beta, delta, mu);
            theta = theta < t ? theta : t;                         /* MIN(theta, t) */
        }
        for (int i = 0; i < m; i++) {
            double t = orc_linesearch(y[i], w[i], dy[i], dw[i], beta, delta, mu);
            theta = theta < t ? theta : t;
        }
        {
            double t = orc_linesearch(phi, psi, dphi, dpsi, beta, delta, mu);
            theta = theta < t ? theta : t;
        }
        if (theta < 1.0) theta *= 0.9999;

        for (int j = 0; j < n; j++) { x[j] = x[j] + theta * dx[j]; z[j] = z[j] + theta * dz[j]; }
        for (int i = 0; i < m; i++) { y[i] = y[i] + theta * dy[i]; w[i] = w[i] + theta * dw[i]; }
        phi = phi + theta * dphi;
        psi = psi + theta * dpsi;
    }
    for (int j = 0; j < n; j++) { x[j] /= phi; z[j] /= phi; }
    for (int i = 0; i < m; i++) { y[i] /= phi; w[i] /= phi; }

    if (run) { run->iters = iter; run->t_total = now_s() - t0; }
    orc_kkt_destroy(K);
    free(dx); free(dw); free(dy); free(dz); free(rho); free(sig); free(D); free(E);
    free(fx); free(fy); free(gx); free(gy); free(At); free(iAt); free(kAt);
    return status;
}

static const char *status_text[] = {
    "optimal solution", "primal unbounded", "primal infeasible", "dual unbounded",
    "dual infeasible", "iteration limit", "infinite lower bounds - not implemented",
    "suboptimal solution"
};

/* writesol of an MPS file from solver()-form x, y, z (tests) */
int orc_writesol_mps(const char *mps, const double *x, const double *y, const double *z, const char *solfile)
{
    orc_mps P;
    int rc = orc_mps_read(mps, &P, NULL);
    if (rc) return rc;
    orc_std S;
    int st = orc_stdform(&P, &S, NULL);
    if (st == 0) st = orc_writesol(solfile, &P, &S, x, y, z);
    orc_std_free(&S);
    orc_mps_free(&P);
    return st;
}

int orc_ipo_run(const char *path, int method, FILE *out, orc_run *run)
{
    orc_run local; memset(&local, 0, sizeof(local));
    if (!run) run = &local;
    run->trace = out;
    if (out) {
        fprintf(out, "%s\n%s\n%s%5s%s\n%s\n%s\n",
                "\t+-------------------------------------------------+",
                "\t                                                   ",
                "\t   ", "./ipo", ":   Version 1.00 : (Copyright) 1995        ",
                "\t                                                   ",
                "\t+-------------------------------------------------+");
        fflush(out);
    }
    orc_mps P;
    int rc = orc_mps_read(path, &P, out);
    if (rc) return -rc;
    orc_std S;
    int status;
    if (getenv("ORC_FREE")) {   /* free-variable extension (orc_split_free) */
        orc_mps Q; int *cm; double *sh;
        orc_split_free(&P, &Q, &cm, &sh);
        if (out) fprintf(out, "m = %d,n = %d,nz = %d \n", P.m, P.n, P.nz);   /* the problem as read */
        status = orc_stdform_quiet(&Q, &S, out);
        orc_split_free_release(&Q, cm, sh);
    } else
        status = orc_stdform(&P, &S, out);
    if (status == 0) {
        int m = S.m, n = S.n;
        double *x = calloc((size_t)(n + m), sizeof(double)), *y = calloc((size_t)(n + m), sizeof(double));
        double *w = calloc((size_t)(m ? m : 1), sizeof(double)), *z = calloc((size_t)(n ? n : 1), sizeof(double));
        if (method == 1)      status = orc_intpt(m, n, S.nz, S.rowind, S.colptr, S.val, S.b, S.c, S.f, x, y, w, z, run);
        else if (method == 2) status = orc_hsdls(m, n, S.nz, S.rowind, S.colptr, S.val, S.b, S.c, S.f, x, y, w, z, run);
        else                  status = orc_hsd(m, n, S.nz, S.rowind, S.colptr, S.val, S.b, S.c, S.f, x, y, w, z, run);
        if (getenv("ORC_SOLFILE") && !getenv("ORC_FREE")) orc_writesol(getenv("ORC_SOLFILE"), &P, &S, x, y, z);
        free(x); free(y); free(w); free(z);
    }
    if (out) { fprintf(out, "%s \n", status_text[status]); fflush(out); }
    orc_std_free(&S);
    orc_mps_free(&P);
    return status;
}
