/*
 * orc.h -- CPU ORACLE for the ipo interior-point hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * build, load or run it, and only as the checker / the timed CPU baseline.
 *
 * This is a clean-room single-threaded C restatement of the reference's
 * algorithms (romz-pl/linear-programming-Vanderbei, read as text only; the
 * reference itself could not be compiled here -- see SURVEY.md 8(c)):
 *
 *   orc_mps.c      fixed-column MPS reader        src/common/iolp.c:145-838
 *   orc_stdform.c  solvelp() normalisation        src/common/solve.c:28-258
 *   orc_kkt.c      tiered min-degree ordering +   src/ipo/ldlt.c:124-1349
 *                  left-looking LDL^T of the
 *                  quasi-definite KKT matrix +
 *                  refined solves
 *   orc_ipm.c      HSD predictor-corrector        src/ipo/hsd.c:27-311
 *                  path-following                 src/ipo/intpt.c:33-261
 *                  vector helpers                 src/common/linalg.c:17-116
 *
 * Parity pin: the oracle's stdout is compared line-for-line with the
 * reference's captured traces evaluate/v1-cf4d5ba/netlib/ipo/<name>.mps.sol
 * (copied as data to tests/golden/netlib/).  Every floating-point
 * expression keeps the reference's evaluation order so the trace can be
 * reproduced exactly; build with -ffp-contract=off.
 */
#ifndef ORC_H
#define ORC_H

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------- problem as read from an MPS file (iolp.c:806-837) ---------- */
typedef struct {
    int m, n, nz;          /* rows (objective/N rows removed), cols, nonzeros */
    int *colptr;           /* [n+1] CSC column starts                        */
    int *rowind;           /* [nz]                                           */
    double *val;           /* [nz]                                           */
    double *rhs;           /* [m]  b                                          */
    double *obj;           /* [n]  c                                          */
    double *range;         /* [m]  r  (HUGE_VAL = no range)                   */
    double *lo, *hi;       /* [n]  bounds                                     */
    double fixed;          /* f                                               */
    int sense;             /* 1 = MIN (default), -1 = MAX                     */
    char name[256];
    char **rowlab, **collab; /* [m], [n] field text (iolp.c:387, :422)        */
    int qnz;               /* QUADS (iolp.c:583-645, symmetrised :733-793):   */
    int *kQ, *iQ;          /* n x n full symmetric CSC, rows sorted; kQ NULL  */
    double *Q;             /* when the file has no QUADS section              */
} orc_mps;

/* ---------- problem as handed to solver(): max c'x, Ax<=b, x>=0 ---------- */
typedef struct {
    int m, n, nz;
    int *colptr, *rowind;  /* CSC, row indices ascending in each column     */
    double *val;
    double *b, *c;
    double f;
    int sense;
    /* bookkeeping to undo the transform (solve.c:242-255) */
    int m0, n0;
    double *lo;
} orc_std;

/* Returns 0 on success, nonzero on fatal parse error (message on log). */
int  orc_mps_read(const char *path, orc_mps *out, FILE *log);
void orc_mps_free(orc_mps *p);
/* QUADS of an MPS file: kQ == NULL queries n and qnz (-1: no section). */
int  orc_mps_quads(const char *path, int *n, int *qnz, int *kQ, int *iQ, double *Q);

/* solve.c:28-205.  Returns 0, or 3 when a free variable is present
 * ("dual unbounded", solve.c:79-87).  Prints "m = ..,n = ..,nz = .. " to log. */
int  orc_stdform(const orc_mps *in, orc_std *out, FILE *log);
int  orc_stdform_quiet(const orc_mps *in, orc_std *out, FILE *log);   /* without the dims line */
/* Free-variable extension (not in the reference): an equivalent problem
 * with finite lower bounds only (split / reflected columns); see
 * orc_stdform.c.  Q shares the label / name fields of P. */
int  orc_split_free(const orc_mps *P, orc_mps *Q, int **colmap, double **shift);
void orc_split_free_release(orc_mps *Q, int *colmap, double *shift);
void orc_std_free(orc_std *p);

/* ---------- KKT LDL^T (ldlt.c) ----------
 * Factors  K = [ -max(E,eps)   A'  ;  A  max(D,eps) ]  in the reference's
 * symbolic ordering, where the node set is {solver rows (y)} u {solver cols (x)}
 * and A is the solver's m x n constraint matrix.  (The reference's ldltfac
 * is called with the roles of A and A' swapped, hsd.c:218.) */
typedef struct orc_kkt orc_kkt;

orc_kkt *orc_kkt_create(int m, int n, const int *kA, const int *iA, const double *A,
                        const int *kAt, const int *iAt, const double *At);
/* the same K with the Q block of ldlt.c on the y-nodes (ldlt.c's first node
 * class, whose diagonal is -max(E, eps)): K_yy = -max(E, eps) - qmax Q, Q an
 * m x m full symmetric CSC (both triangles, rows sorted, as iolp.c:733-793
 * leaves it), qmax = lp->max (-1 max, 1 min); kQ == NULL: no Q */
orc_kkt *orc_kkt_create_q(int m, int n, const int *kA, const int *iA, const double *A,
                          const int *kAt, const int *iAt, const double *At,
                          const int *kQ, const int *iQ, const double *Q, int qmax);
void orc_kkt_destroy(orc_kkt *k);
/* ldltfac / inv_num: numeric factorisation with row scaling E (m) and column scaling D (n) */
void orc_kkt_factor(orc_kkt *k, const double *E, const double *D);
/* forwardbackward / solve: in-place refined solve of
 *   -E dy + A dx = fy ,  A' dy + D dx = fx     (fy: m, fx: n) */
int  orc_kkt_solve(orc_kkt *k, const double *E, const double *D, double *fy, double *fx);
/* one unrefined L D L' solve on a permuted vector (rawsolve) */
int  orc_kkt_rawsolve(orc_kkt *k, double *zperm);

/* symbolic results, for tests and for pinning the product's ordering */
int  orc_kkt_dim(const orc_kkt *k);
long orc_kkt_lnz(const orc_kkt *k);
double orc_kkt_narth(const orc_kkt *k);
int  orc_kkt_denwin(const orc_kkt *k);
int  orc_kkt_pdf(const orc_kkt *k);            /* 1 = primal, 2 = dual */
void orc_kkt_perm(const orc_kkt *k, int *perm);  /* perm[new] = old (y: 0..m-1, x: m..m+n-1) */
void orc_kkt_colptr(const orc_kkt *k, int *colptr); /* [N+1] strict-lower L column starts */
void orc_kkt_rowind(const orc_kkt *k, int *rowind); /* [lnz] (new indices, sorted) */
void orc_kkt_lvals(const orc_kkt *k, double *lvals);/* [lnz] numeric L after factor */
void orc_kkt_diag(const orc_kkt *k, double *d);     /* [N]   numeric D after factor */
double orc_kkt_epsdiag(const orc_kkt *k);
void   orc_kkt_set_epsdiag(orc_kkt *k, double e);   /* tests: start from a captured state */
int  orc_kkt_ndep(const orc_kkt *k);
double orc_kkt_last_resid(const orc_kkt *k);  /* last refined solve's max residual / (max|rhs| + 1) */
void orc_kkt_live(const orc_kkt *k, int *live);      /* [N] "mark" (new order) after factor */
/* stability probe: lltnum's contributions summed in the reference's order
 * (0), reversed (1) or by increasing source column (2); ORC_PERTURB env */
void orc_set_perturb(int p);
int  orc_kkt_last_passes(const orc_kkt *k);

/* ---------- solver() restatements (identical ABI to solve.c:24-26) ---------- */
typedef struct {
    FILE *trace;        /* where the banner + per-iteration lines go (NULL = silent) */
    int  max_iter;      /* 200 in the reference                                      */
    int  iters;         /* out: iterations printed                                   */
    double t_setup;     /* out: seconds in first (symbolic) factorisation call       */
    double t_total;     /* out: seconds inside the solver                            */
    double final_mu, final_pobj, final_dobj, final_pinf, final_dinf; /* out: last line */
} orc_run;

int orc_hsd(int m, int n, int nz, const int *iA, const int *kA, const double *A,
            const double *b, const double *c, double f,
            double *x, double *y, double *w, double *z, orc_run *run);
int orc_intpt(int m, int n, int nz, const int *iA, const int *kA, const double *A,
              const double *b, const double *c, double f,
              double *x, double *y, double *w, double *z, orc_run *run);

/* Whole ipo pipeline (main.c:16-58 minus writesol): banner, read, normalise,
 * solve, status line.  method: 0 = hsd, 1 = intpt.  Returns status. */
int orc_hsdls(int m, int n, int nz, const int *iA, const int *kA, const double *A,
              const double *b, const double *c, double f,
              double *x, double *y, double *w, double *z, orc_run *run);
double orc_linesearch(double xj, double zj, double dxj, double dzj, double beta, double delta, double mu);
/* method: 0 hsd, 1 intpt, 2 hsdls */
int orc_ipo_run(const char *mps_path, int method, FILE *out, orc_run *run);

/* writesol (iolp.c:976-1045) for the problem P as read, from solver()'s
 * x, y, z of its normalisation S (solve.c:237-255 undone here).  z is the
 * solver's (the reference frees it, hsd.c:290-291, then reads it). */
int orc_writesol(const char *path, const orc_mps *P, const orc_std *S, const double *x, const double *y,
                 const double *z);

int orc_writesol_mps(const char *mps, const double *x, const double *y, const double *z, const char *solfile);

/* linalg.c helpers */
double orc_dot(const double *x, const double *y, int n);
void   orc_spmv(int m, int n, const double *a, const int *ka, const int *ia,
                const double *x, double *y);
void   orc_transpose(int m, int n, const int *ka, const int *ia, const double *a,
                     int *kat, int *iat, double *at);
double orc_maxabs(const double *x, int n);

#ifdef __cplusplus
}
#endif
#endif
