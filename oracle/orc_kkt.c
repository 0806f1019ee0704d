/*
 * orc_kkt.c -- ORACLE (test infrastructure only, see orc.h).
 *
 * Restatement of src/ipo/ldlt.c for the way ipo uses it (every column
 * "bounded below", every row "infinite" -- ldlt.c:140-160; Q empty, or with
 * orc_kkt_create_q the Q block of ldlt.c's first node class: separability
 * test ldlt.c:675-682, Q neighbours in the adjacency ldlt.c:729-745,
 * -max Q scattered into K ldlt.c:253-256, max Q dy in the refinement
 * residual ldlt.c:391-394):
 *
 *   node numbering    y-nodes (solver rows) 0..m-1, x-nodes m..m+n-1
 *                     (ldlt.c's "n" first, then its "m": hsd.c:218 swaps)
 *   ordering          inv_sym ldlt.c:638-858 + lltsym ldlt.c:860-1262:
 *                     primal/dual fill estimates pick which node class is
 *                     tier 0; tier-0 nodes of degree > dense(=3) are moved
 *                     to tier 1; min-degree with key = degree + tier*N,
 *                     binary heap (hfall/hrise ldlt.c:1305-1349), nodes
 *                     indistinguishable from the pivot eliminated with it
 *   numeric           inv_num ldlt.c:164-309 (diag floor eps_diag, scatter
 *                     into the permuted lower pattern, eps_diag *= 10 when
 *                     min |d| < 1e-14) and lltnum ldlt.c:517-636 (left-
 *                     looking, George & Liu linked lists, dependent-pivot
 *                     rule ldlt.c:600-614)
 *   solve             solve ldlt.c:327-425 (iterative refinement on the full
 *                     KKT residual) and rawsolve ldlt.c:433-505
 * Evaluation order of every floating-point update follows the reference so
 * the oracle reproduces its traces bit-for-bit.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include "orc.h"

/* summation-order probe of numeric_ldlt (ORC_PERTURB, below); -1 = read the
 * environment on first use; orc_set_perturb: 0 plain, 1 reverse, 2 sorted */
static int g_perturb = -1;
void orc_set_perturb(int p) { g_perturb = p; }

#define EPS_PIVOT   1.0e-8   /* ldlt.c:27  */
#define EPS_SOLVE   1.0e-6   /* ldlt.c:28  */
#define EPS_NUM     0.0      /* ldlt.c:29  */
#define EPS_DIAG0   1.0e-14  /* ldlt.c:31  */
#define DENSE_THRESHOLD_FACTOR 3.0f  /* ldlt.c:816 */

struct orc_kkt {
    int m, n, T;                 /* solver rows, cols, T = m+n */
    const int *kA, *iA, *kAt, *iAt;
    const double *A, *At;
    const int *kQ, *iQ;          /* Q block on the y-nodes (m x m, full symmetric CSC) or NULL */
    const double *Q;
    int qmax;                    /* lp->max of ldlt.c:185: -1 max, 1 min  */
    int *perm, *iperm;           /* perm[new] = old                       */
    int *Lp, *Li;                /* strict lower L, CSC, new indices      */
    double *Lx, *d;
    int *live;                   /* "mark" in ldlt.c                      */
    int ndep, denwin, pdf;
    long lnz;
    double narth, epsdiag;
    /* work */
    double *acc; int *first, *link, *pos;
    double *zr, *dy, *dx, *ry, *rx, *qy;
    int passes;
    double rs, bc;               /* last refined solve: final residual, its bound scale (diagnostics) */
};

static inline double dmax(double a, double b) { return a > b ? a : b; }   /* macros.h MAX */
static inline double dabs(double a) { return a > 0 ? a : -a; }            /* macros.h ABS */

/* ---------------- binary heap on keys, 1-based (ldlt.c:1305-1349) ---------------- */
static void swapi(int *v, int a, int b) { int t = v[a]; v[a] = v[b]; v[b] = t; }

static void heap_down(int cnt, const int *key, int *where, int *h, int cur)
{
    for (int ch = 2 * cur; ch <= cnt; ch = 2 * cur) {
        if (ch < cnt && key[h[ch + 1]] < key[h[ch]]) ch++;
        if (!(key[h[cur]] > key[h[ch]])) break;
        swapi(h, cur, ch);
        swapi(where, h[cur], h[ch]);
        cur = ch;
    }
}
static void heap_up(const int *key, int *where, int *h, int cur)
{
    for (int par = cur / 2; par > 0; par = cur / 2) {
        if (!(key[h[par]] > key[h[cur]])) break;
        swapi(h, cur, par);
        swapi(where, h[cur], h[par]);
        cur = par;
    }
}

static int cmp_int(const void *a, const void *b) { int x = *(const int *)a, y = *(const int *)b; return (x > y) - (x < y); }

static void adj_push(int **adj, int *deg, int *cap, int v, int w)
{
    if (deg[v] >= cap[v]) { cap[v] = cap[v] > 0 ? 2 * cap[v] : 4; adj[v] = realloc(adj[v], sizeof(int) * (size_t)cap[v]); }
    adj[v][deg[v]++] = w;
}

/* tiered minimum degree with indistinguishable-node merging (lltsym) */
static void order_md(orc_kkt *K, int T, int *deg, int **adj, int *cap, int *tier, int dense)
{
    int penalty = T;             /* stablty(1.0) * T, ldlt.c:889 */
    int *perm = malloc(sizeof(int) * (size_t)T), *iperm = malloc(sizeof(int) * (size_t)T);
    int *grp = malloc(sizeof(int) * (size_t)T), *key = malloc(sizeof(int) * (size_t)T);
    int *h = malloc(sizeof(int) * (size_t)(T + 1)), *where = malloc(sizeof(int) * (size_t)T);
    int *stamp = calloc((size_t)T, sizeof(int));

    long cap_l = 0;
    for (int v = 0; v < T; v++) cap_l += deg[v];
    cap_l /= 2;
    if (cap_l < 1) cap_l = 1;
    int *Lp = malloc(sizeof(int) * (size_t)(T + 1));
    int *Li = malloc(sizeof(int) * (size_t)cap_l);

    for (int v = 0; v < T; v++) { perm[v] = -1; iperm[v] = -1; }
    for (int v = 0; v < T; v++) key[v] = deg[v];
    for (int v = 0; v < T; v++) {
        if (deg[v] > dense && tier[v] == 0) tier[v] = 1;
        key[v] += tier[v] * penalty;
    }
    int hn = T;
    for (int v = T - 1; v >= 0; v--) { where[v] = v + 1; h[v + 1] = v; heap_down(hn, key, where, h, v + 1); }

    int tag = 0, i = 0, denwin = T;
    long nz = 0;
    Lp[0] = 0;
    while (i < T) {
        int piv = h[1], dg = deg[piv];
        int *pn = adj[piv];
        if (dg >= T - 1 - i) denwin = i;
        perm[i] = piv; iperm[piv] = i;

        int ng = 0, i2 = i + 1;
        for (int k = 0; k < dg; k++) iperm[pn[k]] = i;
        for (int k = 0; k < dg; k++) {
            int w = pn[k];
            int twin = 0;
            if (deg[w] == dg && tier[w] == tier[piv]) {
                int kk;
                for (kk = 0; kk < dg; kk++) if (iperm[adj[w][kk]] < i) break;
                twin = (kk == dg);
            }
            if (twin) { perm[i2] = w; iperm[w] = i2; i2++; }
            else grp[ng++] = w;
        }
        int ni = i2 - i;
        long need = nz + ((long)dg * (dg + 1) - (long)(dg - ni) * (dg - ni + 1)) / 2;
        if (need > cap_l) { cap_l = need > 2 * cap_l ? need : 2 * cap_l; Li = realloc(Li, sizeof(int) * (size_t)cap_l); }

        int cdeg = dg;
        for (int ii = i; ii < i2; ii++) {
            int v = perm[ii];
            Lp[ii + 1] = Lp[ii] + cdeg;
            for (int k = 0; k < deg[v]; k++) {
                int w = adj[v][k], r = iperm[w];
                if (r > ii || (r == i && w != perm[i])) Li[nz++] = w;
            }
            cdeg--;
        }

        /* remove the pivot from its distinguishable neighbours' lists */
        for (int k = 0; k < ng; k++) {
            int w = grp[k];
            int *wl = adj[w];
            deg[w]--;
            int kk = 0;
            while (wl[kk] != piv) kk++;
            for (; kk < deg[w]; kk++) wl[kk] = wl[kk + 1];
        }
        if (i2 > i + 1) {  /* ... and the twins eliminated with it */
            for (int k = 0; k < ng; k++) {
                int w = grp[k], gone = 0;
                int *wl = adj[w];
                for (int kk = 0; kk < deg[w]; kk++) {
                    if (iperm[wl[kk]] > i) gone++;
                    else wl[kk - gone] = wl[kk];
                }
                deg[w] -= gone;
            }
        }
        for (int ii = i; ii < i2; ii++) {
            int v = perm[ii];
            int cur = where[v];
            int okey = key[h[cur]];
            h[cur] = h[hn];
            where[h[cur]] = cur;
            hn--;
            if (okey < key[h[cur]]) heap_down(hn, key, where, h, cur);
            else heap_up(key, where, h, cur);
        }
        /* fill: make the remaining neighbourhood a clique */
        for (int k = 0; k < ng; k++) {
            int w = grp[k];
            tag++;
            for (int kk = 0; kk < deg[w]; kk++) stamp[adj[w][kk]] = tag;
            for (int kk = k + 1; kk < ng; kk++) {
                int w2 = grp[kk];
                if (stamp[w2] != tag) {
                    adj_push(adj, deg, cap, w, w2);
                    adj_push(adj, deg, cap, w2, w);
                }
            }
        }
        for (int k = 0; k < ng; k++) {
            int w = grp[k];
            key[w] = deg[w];
            if (tier[w] != 0) key[w] += tier[w] * penalty;
            heap_up(key, where, h, where[w]);
            heap_down(hn, key, where, h, where[w]);
        }
        for (int ii = i; ii < i2; ii++) { free(adj[perm[ii]]); adj[perm[ii]] = NULL; }
        i = i2;
    }

    for (long k = 0; k < Lp[T]; k++) Li[k] = iperm[Li[k]];
    for (int v = 0; v < T; v++) qsort(Li + Lp[v], (size_t)(Lp[v + 1] - Lp[v]), sizeof(int), cmp_int);

    double na = 0.0;
    for (int v = 0; v < T; v++) { int c = Lp[v + 1] - Lp[v]; na += (double)c * c; }
    na = na + 3 * Lp[T] + T;

    K->perm = perm; K->iperm = iperm; K->Lp = Lp; K->Li = Li;
    K->lnz = Lp[T]; K->narth = na; K->denwin = denwin;
    free(grp); free(key); free(h); free(where); free(stamp);
}

/* inv_sym (ldlt.c:638-858) seen from the solver's side */
static void symbolic(orc_kkt *K)
{
    int m = K->m, n = K->n, T = m + n;
    /* fill estimates: "primal" = eliminate y-nodes first */
    double frac = 1.0;
    for (int j = 0; j < m; j++) { double dn = (double)(K->kAt[j + 1] - K->kAt[j]) / (n + 1); frac = frac * (1.0 - dn * dn); }
    double pfill = 0.5 * n * n * (1.0 - frac);
    frac = 1.0;
    for (int i = 0; i < n; i++) { double dn = (double)(K->kA[i + 1] - K->kA[i]) / (m + 1); frac = frac * (1.0 - dn * dn); }
    double dfill = 0.5 * m * m * (1.0 - frac);
    /* a Q with off-diagonal entries makes the problem non-separable, which
     * forces the dual priority (ldlt.c:675-682, 710) */
    int separable = 1;
    if (K->kQ)
        for (int j = 0; j < m && separable; j++)
            for (int k = K->kQ[j]; k < K->kQ[j + 1]; k++)
                if (K->iQ[k] != j) { separable = 0; break; }
    K->pdf = (3 * pfill <= dfill && separable) ? 1 : 2;

    int *deg = malloc(sizeof(int) * (size_t)T), *cap = malloc(sizeof(int) * (size_t)T);
    int **adj = malloc(sizeof(int *) * (size_t)T);
    int *tier = malloc(sizeof(int) * (size_t)T);
    for (int j = 0; j < m; j++) {
        int c = K->kAt[j + 1] - K->kAt[j];
        int cq = K->kQ ? K->kQ[j + 1] - K->kQ[j] : 0;
        adj[j] = malloc(sizeof(int) * (size_t)(c + cq > 0 ? c + cq : 1)); cap[j] = c + cq; deg[j] = c;
        for (int k = 0; k < c; k++) adj[j][k] = m + K->iAt[K->kAt[j] + k];
        for (int k = 0; k < cq; k++)          /* then the Q neighbours, ldlt.c:737-742 */
            if (K->iQ[K->kQ[j] + k] != j) adj[j][deg[j]++] = K->iQ[K->kQ[j] + k];
        tier[j] = K->pdf == 1 ? 0 : 1;
    }
    for (int i = 0; i < n; i++) {
        int c = K->kA[i + 1] - K->kA[i];
        adj[m + i] = malloc(sizeof(int) * (size_t)(c > 0 ? c : 1)); cap[m + i] = c; deg[m + i] = c;
        for (int k = 0; k < c; k++) adj[m + i][k] = K->iA[K->kA[i] + k];
        tier[m + i] = K->pdf == 1 ? 1 : 0;
    }
    /* dense threshold: histogram walk with n1 = 0 stops at degree 0 -> 3*1 (ldlt.c:814-846) */
    int dense;
    {
        int *histo = calloc((size_t)T + 1, sizeof(int));
        for (int v = 0; v < T; v++) if (tier[v] == 0) histo[deg[v]]++;
        int tot = 0, d;
        for (d = 0; d <= T; d++) { tot += histo[d]; if (tot >= 0) break; }
        d++;
        dense = (int)(DENSE_THRESHOLD_FACTOR * d);
        free(histo);
    }
    order_md(K, T, deg, adj, cap, tier, dense);
    free(deg); free(cap); free(adj); free(tier);
}

orc_kkt *orc_kkt_create(int m, int n, const int *kA, const int *iA, const double *A,
                        const int *kAt, const int *iAt, const double *At)
{
    return orc_kkt_create_q(m, n, kA, iA, A, kAt, iAt, At, NULL, NULL, NULL, 1);
}

orc_kkt *orc_kkt_create_q(int m, int n, const int *kA, const int *iA, const double *A,
                          const int *kAt, const int *iAt, const double *At,
                          const int *kQ, const int *iQ, const double *Q, int qmax)
{
    orc_kkt *K = calloc(1, sizeof(*K));
    K->m = m; K->n = n; K->T = m + n;
    K->kA = kA; K->iA = iA; K->A = A; K->kAt = kAt; K->iAt = iAt; K->At = At;
    K->kQ = kQ; K->iQ = iQ; K->Q = Q; K->qmax = qmax;
    K->epsdiag = EPS_DIAG0;
    symbolic(K);
    int T = K->T;
    K->Lx = malloc(sizeof(double) * (size_t)(K->lnz > 0 ? K->lnz : 1));
    K->d = malloc(sizeof(double) * (size_t)T);
    K->live = malloc(sizeof(int) * (size_t)T);
    K->acc = malloc(sizeof(double) * (size_t)T);
    K->first = malloc(sizeof(int) * (size_t)T);
    K->link = malloc(sizeof(int) * (size_t)T);
    K->pos = malloc(sizeof(int) * (size_t)T);
    K->zr = malloc(sizeof(double) * (size_t)T);
    K->dy = malloc(sizeof(double) * (size_t)(m ? m : 1));
    K->ry = malloc(sizeof(double) * (size_t)(m ? m : 1));
    K->qy = malloc(sizeof(double) * (size_t)(m ? m : 1));
    K->dx = malloc(sizeof(double) * (size_t)(n ? n : 1));
    K->rx = malloc(sizeof(double) * (size_t)(n ? n : 1));
    return K;
}

void orc_kkt_destroy(orc_kkt *K)
{
    if (!K) return;
    free(K->perm); free(K->iperm); free(K->Lp); free(K->Li); free(K->Lx); free(K->d);
    free(K->live); free(K->acc); free(K->first); free(K->link); free(K->pos);
    free(K->zr); free(K->dy); free(K->ry); free(K->dx); free(K->rx); free(K->qy);
    free(K);
}

/* left-looking LDL^T (lltnum, ldlt.c:517-636) */
static int g_depblk = -2;   /* ORC_DEBUG_DEPBLK (diagnostics) */

static void numeric_ldlt(orc_kkt *K)
{
    int T = K->T, m = K->m;
    int *Lp = K->Lp, *Li = K->Li, *first = K->first, *link = K->link, *live = K->live;
    double *Lx = K->Lx, *d = K->d, *acc = K->acc;
    memset(acc, 0, sizeof(double) * (size_t)T);
    for (int v = 0; v < T; v++) link[v] = -1;
    double dmaxabs = 0.0;
    for (int v = 0; v < T; v++) if (dabs(d[v]) > dmaxabs) dmaxabs = dabs(d[v]);
    K->ndep = 0;

    /* Stability probe (test infrastructure, tools/rounding_stability.py):
     * ORC_PERTURB=reverse / sorted applies the contributions of the columns
     * j to column col in the reverse of the reference's linked-list order /
     * in increasing j -- the same algorithm and operations, another
     * summation order (like any other implementation's).  The list itself
     * is maintained exactly as lltnum does. */
    if (g_perturb < 0) {
        const char *e = getenv("ORC_PERTURB");
        g_perturb = !e ? 0 : !strcmp(e, "reverse") ? 1 : !strcmp(e, "sorted") ? 2 : 0;
    }
    const int perturb = g_perturb;
    if (g_depblk == -2) {
        const char *e = getenv("ORC_DEBUG_DEPBLK");   /* first column of the GPU's dense tail */
        g_depblk = e ? atoi(e) : -1;
    }
    int *js = perturb ? malloc(sizeof(int) * (size_t)(T ? T : 1)) : NULL;
    int *ks = perturb ? malloc(sizeof(int) * (size_t)(T ? T : 1)) : NULL;

    for (int col = 0; col < T; col++) {
        double piv = d[col];
        int sgn = K->perm[col] < m ? -1 : 1;
        int nj = 0;
        for (int j = link[col], nxt; j != -1; j = nxt) {
            nxt = link[j];
            int k = first[j];
            if (perturb) { js[nj] = j; ks[nj] = k; nj++; }
            else {
            double lij = Lx[k];
            double lijdj = lij * d[j];
            piv -= lij * lijdj;
            }
            int kb = k + 1, ke = Lp[j + 1];
            if (kb < ke) {
                first[j] = kb;
                int r = Li[kb];
                link[j] = link[r];
                link[r] = j;
                if (perturb) continue;
                double lijdj = Lx[k] * d[j];
                if (j < K->denwin) {
                    for (int kk = kb; kk < ke; kk++) acc[Li[kk]] += lijdj * Lx[kk];
                } else {
                    double *p = &acc[r];
                    for (int kk = kb; kk < ke; kk++) { *p += lijdj * Lx[kk]; p++; }
                }
            }
        }
        if (perturb && nj > 0) {
            if (perturb == 2) {     /* increasing j (insertion sort on the pairs) */
                for (int a = 1; a < nj; a++) {
                    int jj = js[a], kk0 = ks[a], b = a - 1;
                    while (b >= 0 && js[b] > jj) { js[b + 1] = js[b]; ks[b + 1] = ks[b]; b--; }
                    js[b + 1] = jj; ks[b + 1] = kk0;
                }
            }
            for (int q = 0; q < nj; q++) {
                int idx = perturb == 1 ? nj - 1 - q : q;
                int j = js[idx], k = ks[idx];
                double lij = Lx[k];
                double lijdj = lij * d[j];
                piv -= lij * lijdj;
                for (int kk = k + 1; kk < Lp[j + 1]; kk++) acc[Li[kk]] += lijdj * Lx[kk];
            }
        }
        int kb = Lp[col], ke = Lp[col + 1];
        for (int kk = kb; kk < ke; kk++) Lx[kk] -= acc[Li[kk]];
        if (fabs(piv) <= EPS_NUM * dmaxabs || !live[col]) {
            K->ndep++;
            double off = 0.0;
            for (int kk = kb; kk < ke; kk++) off = dmax(off, dabs(Lx[kk]));
            if (g_depblk >= 0 && col >= g_depblk) {   /* diagnostics: the off-diagonal max inside col's 64-block */
                double ob = 0.0;
                for (int kk = kb; kk < ke; kk++)
                    if ((Li[kk] - g_depblk) / 64 == (col - g_depblk) / 64) ob = dmax(ob, dabs(Lx[kk]));
                fprintf(stderr, "dep col %d block %d: off_block %.3e off_all %.3e -> %s\n", col, (col - g_depblk) / 64,
                        ob, off, off < 1.0e+6 * EPS_PIVOT ? "drop" : "keep");
            }
            if (off < 1.0e+6 * EPS_PIVOT) live[col] = 0;
            else piv = sgn * EPS_PIVOT;
        }
        d[col] = piv;
        if (kb < ke) {
            first[col] = kb;
            int r = Li[kb];
            link[col] = link[r];
            link[r] = col;
            for (int kk = kb; kk < ke; kk++) {
                if (live[col]) Lx[kk] /= piv;
                else Lx[kk] = 0.0;
                acc[Li[kk]] = 0.0;
            }
        }
    }
    free(js);
    free(ks);
}

void orc_kkt_factor(orc_kkt *K, const double *E, const double *D)
{
    static int fcount = 0;
    if (getenv("ORC_DUMP_ED")) {   /* debug: capture (E, D) of factorisations #N1,N2,... */
        int hit = 0;
        for (const char *q = getenv("ORC_DUMP_ED"); *q;) {
            char *e;
            long v = strtol(q, &e, 10);
            if (e == q) break;
            if (v == fcount) hit = 1;
            q = *e == ',' ? e + 1 : e;
        }
        if (hit) {
            char fn[64];
            snprintf(fn, sizeof fn, "/tmp/orc_ed_%d.bin", fcount);
            FILE *f = fopen(fn, "wb");
            fwrite(&K->m, sizeof(int), 1, f); fwrite(&K->n, sizeof(int), 1, f);
            fwrite(E, sizeof(double), (size_t)K->m, f); fwrite(D, sizeof(double), (size_t)K->n, f);
            fwrite(&K->epsdiag, sizeof(double), 1, f);
            fclose(f);
        }
        fcount++;
    }
    int m = K->m, n = K->n, T = K->T;
    int *iperm = K->iperm, *Lp = K->Lp, *Li = K->Li, *pos = K->pos;
    double *Lx = K->Lx, *d = K->d;
    for (int j = 0; j < m; j++) d[iperm[j]] = -dmax(E[j], K->epsdiag);
    for (int i = 0; i < n; i++) d[iperm[m + i]] = dmax(D[i], K->epsdiag);

    for (int j = 0; j < m; j++) {           /* y-node columns: entries A(j, :) */
        int col = iperm[j];
        for (int k = Lp[col]; k < Lp[col + 1]; k++) { pos[Li[k]] = k; Lx[k] = 0.0; }
        for (int k = K->kAt[j]; k < K->kAt[j + 1]; k++) {
            int r = iperm[m + K->iAt[k]];
            if (r > col) Lx[pos[r]] = K->At[k];
        }
        if (K->kQ)                          /* -max Q (ldlt.c:253-256) */
            for (int k = K->kQ[j]; k < K->kQ[j + 1]; k++) {
                int r = iperm[K->iQ[k]];
                if (r > col) Lx[pos[r]] = -K->qmax * K->Q[k];
                else if (r == col) d[r] -= K->qmax * K->Q[k];
            }
    }
    for (int i = 0; i < n; i++) {           /* x-node columns: entries A(:, i) */
        int col = iperm[m + i];
        for (int k = Lp[col]; k < Lp[col + 1]; k++) { pos[Li[k]] = k; Lx[k] = 0.0; }
        for (int k = K->kA[i]; k < K->kA[i + 1]; k++) {
            int r = iperm[K->iA[k]];
            if (r > col) Lx[pos[r]] = K->A[k];
        }
    }
    for (int v = 0; v < T; v++) K->live[v] = 1;
    numeric_ldlt(K);

    double mind = HUGE_VAL;
    for (int v = 0; v < T; v++) if (dabs(d[v]) < mind) mind = dabs(d[v]);
    if (mind < 1.0e-14) K->epsdiag *= 10;
    {   /* diagnostics (ORC_EPSDIAG_MAX): cap the growth, to test what a stall owes to it */
        static double cap = -1.0;
        if (cap < 0) cap = getenv("ORC_EPSDIAG_MAX") ? atof(getenv("ORC_EPSDIAG_MAX")) : 0.0;
        if (cap > 0 && K->epsdiag > cap) K->epsdiag = cap;
    }
    if (getenv("ORC_DEBUG_NDEP")) {
        int dropped = 0;
        for (int v = 0; v < T; v++) dropped += !K->live[v];
        fprintf(stderr, "factor: ndep=%d dropped=%d mind=%.3e epsdiag=%.1e\n", K->ndep, dropped, mind, K->epsdiag);
    }
}

/* forward / diagonal / backward substitution (rawsolve, ldlt.c:433-505) */
int orc_kkt_rawsolve(orc_kkt *K, double *z)
{
    int T = K->T, ok = 1;
    int *Lp = K->Lp, *Li = K->Li, *live = K->live;
    double *Lx = K->Lx, *d = K->d;
    double eps = 0.0;
    if (K->ndep) eps = EPS_SOLVE * orc_maxabs(z, K->n);

    for (int v = 0; v < T; v++) {
        if (live[v]) {
            double beta = z[v];
            for (int k = Lp[v]; k < Lp[v + 1]; k++) z[Li[k]] -= Lx[k] * beta;
        } else if (fabs(z[v]) > eps) ok = 0;
        else z[v] = 0.0;
    }
    for (int v = T - 1; v >= 0; v--) {
        if (live[v]) z[v] = z[v] / d[v];
        else if (fabs(z[v]) > eps) ok = 0;
        else z[v] = 0.0;
    }
    for (int v = T - 1; v >= 0; v--) {
        if (live[v]) {
            double beta = z[v];
            for (int k = Lp[v]; k < Lp[v + 1]; k++) beta -= Lx[k] * z[Li[k]];
            z[v] = beta;
        } else if (fabs(z[v]) > eps) ok = 0;
        else z[v] = 0.0;
    }
    return ok;
}

/* refined solve (solve, ldlt.c:327-425) */
int orc_kkt_solve(orc_kkt *K, const double *E, const double *D, double *fy, double *fx)
{
    int m = K->m, n = K->n;
    int *iperm = K->iperm;
    double *z = K->zr, *dy = K->dy, *dx = K->dx, *ry = K->ry, *rx = K->rx;
    int pass = 0, ok = 1;
    double bc = dmax(orc_maxabs(fx, n), orc_maxabs(fy, m)) + 1;
    double rs = HUGE_VAL, rs_old;
    do {
        if (pass == 0) {
            for (int j = 0; j < m; j++) z[iperm[j]] = fy[j];
            for (int i = 0; i < n; i++) z[iperm[m + i]] = fx[i];
        } else {
            for (int j = 0; j < m; j++) z[iperm[j]] = ry[j];
            for (int i = 0; i < n; i++) z[iperm[m + i]] = rx[i];
        }
        ok = orc_kkt_rawsolve(K, z);
        if (pass == 0) {
            for (int j = 0; j < m; j++) dy[j] = z[iperm[j]];
            for (int i = 0; i < n; i++) dx[i] = z[iperm[m + i]];
        } else {
            for (int j = 0; j < m; j++) dy[j] = dy[j] + z[iperm[j]];
            for (int i = 0; i < n; i++) dx[i] = dx[i] + z[iperm[m + i]];
        }
        /* rx = A' dy (row-major walk), ry = A dx (column walk) */
        orc_spmv(n, m, K->At, K->kAt, K->iAt, dy, rx);
        orc_spmv(m, n, K->A, K->kA, K->iA, dx, ry);
        if (K->kQ) {                        /* ldlt.c:391-394 */
            orc_spmv(m, m, K->Q, K->kQ, K->iQ, dy, K->qy);
            for (int j = 0; j < m; j++) ry[j] = fy[j] - ((ry[j] - E[j] * dy[j]) - K->qmax * K->qy[j]);
        } else
        for (int j = 0; j < m; j++) ry[j] = fy[j] - (ry[j] - E[j] * dy[j]);
        for (int i = 0; i < n; i++) rx[i] = fx[i] - (rx[i] + D[i] * dx[i]);
        rs_old = rs;
        rs = dmax(orc_maxabs(rx, n), orc_maxabs(ry, m));
        pass++;
    } while (rs > 1.0e-10 * bc && rs < rs_old / 2);

    if (rs > rs_old && pass > 1) {
        for (int j = 0; j < m; j++) dy[j] = dy[j] - z[iperm[j]];
        for (int i = 0; i < n; i++) dx[i] = dx[i] - z[iperm[m + i]];
    }
    for (int j = 0; j < m; j++) fy[j] = dy[j];
    for (int i = 0; i < n; i++) fx[i] = dx[i];
    K->passes = pass;
    K->rs = rs;
    K->bc = bc;
    return ok;
}

int  orc_kkt_dim(const orc_kkt *K) { return K->T; }
long orc_kkt_lnz(const orc_kkt *K) { return K->lnz; }
double orc_kkt_narth(const orc_kkt *K) { return K->narth; }
int  orc_kkt_denwin(const orc_kkt *K) { return K->denwin; }
int  orc_kkt_pdf(const orc_kkt *K) { return K->pdf; }
void orc_kkt_perm(const orc_kkt *K, int *p) { memcpy(p, K->perm, sizeof(int) * (size_t)K->T); }
void orc_kkt_colptr(const orc_kkt *K, int *p) { memcpy(p, K->Lp, sizeof(int) * (size_t)(K->T + 1)); }
void orc_kkt_rowind(const orc_kkt *K, int *p) { memcpy(p, K->Li, sizeof(int) * (size_t)K->lnz); }
void orc_kkt_lvals(const orc_kkt *K, double *p) { memcpy(p, K->Lx, sizeof(double) * (size_t)K->lnz); }
void orc_kkt_diag(const orc_kkt *K, double *p) { memcpy(p, K->d, sizeof(double) * (size_t)K->T); }
double orc_kkt_epsdiag(const orc_kkt *K) { return K->epsdiag; }
void orc_kkt_set_epsdiag(orc_kkt *K, double e) { K->epsdiag = e; }
int  orc_kkt_ndep(const orc_kkt *K) { return K->ndep; }
void orc_kkt_live(const orc_kkt *K, int *p) { memcpy(p, K->live, sizeof(int) * (size_t)K->T); }
int  orc_kkt_last_passes(const orc_kkt *K) { return K->passes; }
double orc_kkt_last_resid(const orc_kkt *K) { return K->rs / K->bc; }
