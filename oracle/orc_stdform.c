/*
 * orc_stdform.c -- ORACLE (test infrastructure only, see orc.h).
 *
 * Restates solvelp() of src/common/solve.c:28-205: turn
 *     optimise c'x  s.t.  b <= Ax <= b+r,  l <= x <= u
 * into the form solver() expects,
 *     maximise c'x + f  s.t.  A'x <= b',  x >= 0
 * Row order of the result (parity-critical, the traces depend on it):
 *   rows 0..m0-1      every original row, negated          (solve.c:127-147)
 *   then one row per original row with finite r, in order   (+row, b+r)
 *   then one row  x_j <= u_j - l_j  per finite upper bound  (solve.c:152-174)
 * The CSC matrix is rebuilt by a transpose so row indices ascend in each
 * column (solve.c:189).  c and f are negated for MIN problems (:202-205).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "orc.h"

int orc_stdform(const orc_mps *P, orc_std *S, FILE *log)
{
    if (log) fprintf(log, "m = %d,n = %d,nz = %d \n", P->m, P->n, P->nz);
    return orc_stdform_quiet(P, S, log);
}

/* orc_stdform without the solve.c:62 dimension line (the free-variable
 * extension prints the dimensions of the problem as read, then normalises
 * its split form) */
int orc_stdform_quiet(const orc_mps *P, orc_std *S, FILE *log)
{
    memset(S, 0, sizeof(*S));
    int m = P->m, n = P->n, nz = P->nz;

    S->m0 = m; S->n0 = n; S->sense = P->sense;
    for (int j = 0; j < n; j++)
        if (P->lo[j] == -HUGE_VAL) { S->n = n; S->m = m; return 3; }

    double *u = malloc(sizeof(double) * (size_t)(n ? n : 1));
    double *b = malloc(sizeof(double) * (size_t)(2 * m + n + 1));
    double *c = malloc(sizeof(double) * (size_t)(n ? n : 1));
    double *lshift = malloc(sizeof(double) * (size_t)(n ? n : 1));
    memcpy(c, P->obj, sizeof(double) * (size_t)n);
    memcpy(lshift, P->lo, sizeof(double) * (size_t)n);
    memcpy(b, P->rhs, sizeof(double) * (size_t)m);

    /* shift lower bounds to zero (solve.c:103-110) */
    for (int j = 0; j < n; j++) u[j] = P->hi[j] != HUGE_VAL ? P->hi[j] - P->lo[j] : P->hi[j];
    {
        double *Al = malloc(sizeof(double) * (size_t)(m ? m : 1));
        orc_spmv(m, n, P->val, P->colptr, P->rowind, P->lo, Al);
        for (int i = 0; i < m; i++) b[i] -= Al[i];
        free(Al);
    }
    double f = P->fixed + orc_dot(c, P->lo, n);

    /* row-wise copy, room for duplicated rows and bound rows */
    int nub = 0;
    for (int j = 0; j < n; j++) if (u[j] < HUGE_VAL) nub++;
    int *rp = malloc(sizeof(int) * (size_t)(2 * m + nub + 1));
    int *ci = malloc(sizeof(int) * (size_t)(2 * nz + nub + 1));
    double *rv = malloc(sizeof(double) * (size_t)(2 * nz + nub + 1));
    orc_transpose(m, n, P->colptr, P->rowind, P->val, rp, ci, rv);

    int mm = m, nnz = rp[m];
    for (int i = 0; i < m; i++) {
        int finite = P->range[i] < HUGE_VAL;
        for (int k = rp[i]; k < rp[i + 1]; k++) {
            if (finite) { ci[nnz] = ci[k]; rv[nnz] = rv[k]; nnz++; }
            rv[k] *= -1;
        }
        if (finite) { b[mm] = b[i] + P->range[i]; mm++; rp[mm] = nnz; }
        b[i] *= -1;
    }
    for (int j = 0; j < n; j++) {
        if (u[j] < HUGE_VAL) {
            b[mm] = u[j];
            ci[nnz] = j; rv[nnz] = 1.0; nnz++;
            mm++; rp[mm] = nnz;
        }
    }

    S->m = mm; S->n = n; S->nz = nnz;
    S->colptr = malloc(sizeof(int) * (size_t)(n + 1));
    S->rowind = malloc(sizeof(int) * (size_t)(nnz ? nnz : 1));
    S->val = malloc(sizeof(double) * (size_t)(nnz ? nnz : 1));
    orc_transpose(n, mm, rp, ci, rv, S->colptr, S->rowind, S->val);

    if (P->sense == 1) {   /* MIN: solver maximises */
        for (int j = 0; j < n; j++) c[j] *= -1;
        f *= -1;
    }
    S->b = b; S->c = c; S->f = f; S->lo = lshift;

    if (mm < 7 && n < 7 && log) {   /* solve.c:210-222 */
        fprintf(log, "A: \n");
        for (int j = 0; j < n; j++) {
            for (int k = S->colptr[j]; k < S->colptr[j + 1]; k++) fprintf(log, "%5d %10.5f \n", S->rowind[k], S->val[k]);
            fprintf(log, "\n");
        }
        fprintf(log, "\n");
        fprintf(log, "b: \n");
        for (int i = 0; i < mm; i++) fprintf(log, "%10.5f \n", b[i]);
        fprintf(log, "\n");
        fprintf(log, "c: \n");
        for (int j = 0; j < n; j++) fprintf(log, "%10.5f \n", c[j]);
        fprintf(log, "\n");
    }
    free(u); free(rp); free(ci); free(rv);
    return 0;
}

/*
 * Free-variable extension (not in the reference, which aborts with status 3,
 * solve.c:79-87): an equivalent problem whose every
 * column has a finite lower bound, for the normalisation above.
 *   l = -inf, u = +inf : x = x+ - x-  -> column j keeps (a_j, c_j) with
 *                        l = 0, and a column (-a_j, -c_j), l = 0, is appended
 *                        (appended columns in order of j, after column n-1);
 *   l = -inf, u finite : x = u - x'   -> column j becomes (-a_j, -c_j),
 *                        l = 0, u = inf; b -= a_j u (rows b <= Ax <= b+r
 *                        keep their range), f += c_j u.
 * colmap[j'] (n' entries): +(j+1) / -(j+1) for x_j = +x_j' / -x_j' terms,
 * shift[j] = the constant u of a reflected column (0 otherwise); x_j =
 * shift[j] + sum of the signed x_j' mapped to j.  Returns the number of
 * free columns.
 */
int orc_split_free(const orc_mps *P, orc_mps *Q, int **colmap, double **shift)
{
    int n = P->n, m = P->m, nfree = 0, nsplit = 0;
    for (int j = 0; j < n; j++)
        if (P->lo[j] == -HUGE_VAL) { nfree++; if (P->hi[j] == HUGE_VAL) nsplit++; }
    int n2 = n + nsplit, nz2 = P->nz;
    for (int j = 0; j < n; j++)
        if (P->lo[j] == -HUGE_VAL && P->hi[j] == HUGE_VAL) nz2 += P->colptr[j + 1] - P->colptr[j];
    *Q = *P;
    Q->n = n2; Q->nz = nz2;
    Q->colptr = malloc(sizeof(int) * (size_t)(n2 + 1));
    Q->rowind = malloc(sizeof(int) * (size_t)(nz2 ? nz2 : 1));
    Q->val = malloc(sizeof(double) * (size_t)(nz2 ? nz2 : 1));
    Q->obj = malloc(sizeof(double) * (size_t)(n2 ? n2 : 1));
    Q->lo = malloc(sizeof(double) * (size_t)(n2 ? n2 : 1));
    Q->hi = malloc(sizeof(double) * (size_t)(n2 ? n2 : 1));
    Q->rhs = malloc(sizeof(double) * (size_t)(m ? m : 1));
    Q->range = malloc(sizeof(double) * (size_t)(m ? m : 1));
    memcpy(Q->rhs, P->rhs, sizeof(double) * (size_t)m);
    memcpy(Q->range, P->range, sizeof(double) * (size_t)m);
    *colmap = malloc(sizeof(int) * (size_t)(n2 ? n2 : 1));
    *shift = calloc((size_t)(n ? n : 1), sizeof(double));
    int k = 0, jn = n;
    Q->colptr[0] = 0;
    for (int j = 0; j < n; j++) {
        int refl = P->lo[j] == -HUGE_VAL && P->hi[j] < HUGE_VAL;
        double sg = refl ? -1.0 : 1.0;
        for (int q = P->colptr[j]; q < P->colptr[j + 1]; q++) {
            Q->rowind[k] = P->rowind[q]; Q->val[k] = sg * P->val[q]; k++;
            if (refl) Q->rhs[P->rowind[q]] -= P->val[q] * P->hi[j];
        }
        Q->colptr[j + 1] = k;
        Q->obj[j] = sg * P->obj[j];
        (*colmap)[j] = refl ? -(j + 1) : (j + 1);
        if (refl) {
            Q->fixed += P->obj[j] * P->hi[j];
            (*shift)[j] = P->hi[j];
            Q->lo[j] = 0.0; Q->hi[j] = HUGE_VAL;
        } else {
            Q->lo[j] = P->lo[j] == -HUGE_VAL ? 0.0 : P->lo[j];
            Q->hi[j] = P->hi[j];
        }
    }
    for (int j = 0; j < n; j++) {
        if (!(P->lo[j] == -HUGE_VAL && P->hi[j] == HUGE_VAL)) continue;
        for (int q = P->colptr[j]; q < P->colptr[j + 1]; q++) {
            Q->rowind[k] = P->rowind[q]; Q->val[k] = -P->val[q]; k++;
        }
        Q->colptr[jn + 1] = k;
        Q->obj[jn] = -P->obj[j];
        Q->lo[jn] = 0.0; Q->hi[jn] = HUGE_VAL;
        (*colmap)[jn] = -(j + 1);
        jn++;
    }
    return nfree;
}

void orc_split_free_release(orc_mps *Q, int *colmap, double *shift)
{
    free(Q->colptr); free(Q->rowind); free(Q->val); free(Q->obj); free(Q->lo); free(Q->hi);
    free(Q->rhs); free(Q->range); free(colmap); free(shift);
}

/* writesol, iolp.c:976-1045, on the LP as solvelp leaves it: x + l
 * (solve.c:241), y negated for MIN (:247-250), b shifted by A l and negated
 * and u shifted by l in place (:103-109, :145), row activity of the rebuilt
 * matrix whose first m rows are the negated originals (:142-146). */
int orc_writesol(const char *path, const orc_mps *P, const orc_std *S, const double *xs, const double *ys,
                 const double *zs)
{
    int m = P->m, n = P->n;
    FILE *fp = fopen(path, "w");
    if (!fp) return 2;
    double eps = 1.0e-5 * 1.2;
    double *x = malloc(sizeof(double) * (size_t)(n ? n : 1)), *u = malloc(sizeof(double) * (size_t)(n ? n : 1));
    double *b = malloc(sizeof(double) * (size_t)(m ? m : 1)), *ract = calloc((size_t)(m ? m : 1), sizeof(double));
    double *al = malloc(sizeof(double) * (size_t)(m ? m : 1));
    for (int j = 0; j < n; j++) {
        x[j] = xs[j] + P->lo[j];
        u[j] = P->hi[j] != HUGE_VAL ? P->hi[j] - P->lo[j] : P->hi[j];
    }
    orc_spmv(m, n, P->val, P->colptr, P->rowind, P->lo, al);
    for (int i = 0; i < m; i++) b[i] = -(P->rhs[i] - al[i]);
    for (int j = 0; j < n; j++)
        for (int k = P->colptr[j]; k < P->colptr[j + 1]; k++) ract[P->rowind[k]] += x[j] * -P->val[k];
    fprintf(fp, "COLUMNS SECTION\n");
    fprintf(fp, "   index       label  primal_val reduced_cst");
    fprintf(fp, "    lower_bd    upper_bd   OB_flag\n");
    for (int j = 0; j < n; j++) {
        double l = P->lo[j];
        if (l > -HUGE_VAL && u[j] < HUGE_VAL)
            fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e %11.4e", j, P->collab[j], x[j], zs[j], l, u[j]);
        else if (l > -HUGE_VAL)
            fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e    Infinity", j, P->collab[j], x[j], zs[j], l);
        else if (u[j] < HUGE_VAL)
            fprintf(fp, "%8d  %10s %11.4e %11.4e   -Infinity %11.4e", j, P->collab[j], x[j], zs[j], u[j]);
        else
            fprintf(fp, "%8d  %10s %11.4e %11.4e   -Infinity    Infinity", j, P->collab[j], x[j], zs[j]);
        if (x[j] < l - eps || x[j] > u[j] + eps) fprintf(fp, "      OB\n");
        else fprintf(fp, "\n");
    }
    fprintf(fp, "ROWS SECTION\n");
    fprintf(fp, "   index       label    dual_val  row_actvty");
    fprintf(fp, " rght_hnd_sd       range   OB_flag\n");
    for (int i = 0; i < m; i++) {
        double y = S->sense == 1 ? -ys[i] : ys[i], r = P->range[i];
        if (r < HUGE_VAL)
            fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e %11.4e", i, P->rowlab[i], y, ract[i], b[i], r);
        else
            fprintf(fp, "%8d  %10s %11.4e %11.4e %11.4e    Infinity", i, P->rowlab[i], y, ract[i], b[i]);
        if (ract[i] < b[i] - eps || ract[i] > b[i] + r + eps) fprintf(fp, "     OB\n");
        else fprintf(fp, "\n");
    }
    fprintf(fp, "ENDOUT\n");
    fclose(fp);
    free(x); free(u); free(b); free(ract); free(al);
    return 0;
}

void orc_std_free(orc_std *p)
{
    free(p->colptr); free(p->rowind); free(p->val); free(p->b); free(p->c); free(p->lo);
    memset(p, 0, sizeof(*p));
}
