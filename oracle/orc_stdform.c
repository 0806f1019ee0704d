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
    memset(S, 0, sizeof(*S));
    int m = P->m, n = P->n, nz = P->nz;
    if (log) fprintf(log, "m = %d,n = %d,nz = %d \n", m, n, nz);

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

void orc_std_free(orc_std *p)
{
    free(p->colptr); free(p->rowind); free(p->val); free(p->b); free(p->c); free(p->lo);
    memset(p, 0, sizeof(*p));
}
