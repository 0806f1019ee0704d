/*
 * orc_mps.c -- ORACLE (test infrastructure only, see orc.h).
 *
 * Fixed-column MPS reader restating src/common/iolp.c:145-838:
 *  - a 240-byte line buffer; the last character read (normally '\n') and
 *    everything up to column 78 is blanked, then (outside the header)
 *    fields are cut at columns 3,12,22,36,47,61,79      (iolp.c:252-261)
 *  - header keywords MAX/MIN/OBJ/RHS/RANGES/BOUNDS/...   (iolp.c:264-353)
 *  - ROWS: L/E/G/N; r = +inf for L,G and 0 for E          (iolp.c:359-398)
 *  - COLUMNS with 'MARKER' toggling, zero values skipped  (iolp.c:401-472)
 *  - RHS / RANGES: second field pair handled first        (iolp.c:474-534)
 *  - BOUNDS LO/UP/FX/FR/PL/MI/BV/LI/UI/SC                 (iolp.c:536-581)
 *  - QUADS: kept as iolp.c:583-645 reads it (strict lower triangle by
 *    columns, diagonal apart) and symmetrised as iolp.c:733-793; solve.c
 *    never passes Q to solver(), ldlt.c takes it (ldlt.c:253-256)
 *  - objective extraction, N rows dropped, L rows negated (iolp.c:670-727)
 * Label lookups overwrite on re-install like hash.c:99-119.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "orc.h"

/* ---------------- tiny string -> int map (overwrite semantics) ---------------- */
typedef struct lblnode { char *key; int val; struct lblnode *next; } lblnode;
typedef struct { lblnode **slot; unsigned nslot; } lblmap;

static unsigned lbl_hash(const char *s, unsigned nslot)
{
    unsigned h = 2166136261u;
    while (*s) { h ^= (unsigned char)*s++; h *= 16777619u; }
    return h % nslot;
}
static void lbl_init(lblmap *t, unsigned n) { t->nslot = n < 64 ? 64 : n; t->slot = calloc(t->nslot, sizeof(*t->slot)); }
static int lbl_get(const lblmap *t, const char *s)
{
    for (lblnode *p = t->slot[lbl_hash(s, t->nslot)]; p; p = p->next)
        if (strcmp(p->key, s) == 0) return p->val;
    return -1;
}
static void lbl_put(lblmap *t, const char *s, int v)
{
    unsigned h = lbl_hash(s, t->nslot);
    for (lblnode *p = t->slot[h]; p; p = p->next)
        if (strcmp(p->key, s) == 0) { p->val = v; return; }
    lblnode *p = malloc(sizeof(*p));
    p->key = strdup(s); p->val = v; p->next = t->slot[h]; t->slot[h] = p;
}
static void lbl_free(lblmap *t)
{
    for (unsigned i = 0; i < t->nslot; i++) {
        lblnode *p = t->slot[i];
        while (p) { lblnode *q = p->next; free(p->key); free(p); p = q; }
    }
    free(t->slot);
}
/* key = label followed by a one-character namespace tag ('R','C','P') */
static const char *tagged(char *buf, const char *label, char tag)
{
    size_t l = strlen(label);
    memcpy(buf, label, l); buf[l] = tag; buf[l + 1] = '\0';
    return buf;
}

/* non-empty t occurs inside s (iolp.c:1133-1145) */
static int contains(const char *s, const char *t)
{
    if (!*t) return 0;
    return strstr(s, t) != NULL;
}

/* growable arrays */
#define GROW(ptr, cap, need, T) do { if ((need) >= (cap)) { (cap) = 2 * (cap) + 16; (ptr) = (T *)realloc((ptr), (size_t)(cap) * sizeof(T)); } } while (0)

enum { S_HEAD, S_NAME, S_ROWS, S_COLS, S_RHS, S_RNG, S_BND, S_QUAD, S_END, S_BAD };

static int section_of(const char *three)
{
    if (!strcmp(three, "RHS")) return S_RHS;
    if (!strcmp(three, "RAN")) return S_RNG;
    if (!strcmp(three, "BOU")) return S_BND;
    if (!strcmp(three, "QUA")) return S_QUAD;
    if (!strcmp(three, "END")) return S_END;
    return S_BAD;
}

int orc_mps_read(const char *path, orc_mps *P, FILE *log)
{
    memset(P, 0, sizeof(*P));
    FILE *fp = fopen(path, "r");
    if (!fp) { if (log) fprintf(log, "ERROR(2): cannot open file %s\n\n", path); return 2; }

    lblmap rows, cols; lbl_init(&rows, 1 << 14); lbl_init(&cols, 1 << 15);
    char key[300];

    int sense = 1;                 /* MIN unless MAX keyword */
    char nm[256] = "", objnm[256] = "", rhsnm[256] = "", rngnm[256] = "", bndnm[256] = "";

    int m = 0, mcap = 0, n = 0, ncap = 0, nz = 0, nzcap = 0;
    int *kind = NULL;              /* 0 = E/G, 1 = L, 2 = N */
    double *rng = NULL;
    int *colstart = NULL; double *up = NULL;
    int *ia = NULL; double *av = NULL;
    double *b = NULL, *c = NULL, *lo = NULL;
    char **collab = NULL, **rowlab = NULL;

    int quads = 0, qprev = -1, qn = 0, qcap = 0, *qk = NULL, *qi = NULL, qkcap = 0, qkn = 0;
    double *qv = NULL, *qdiag = NULL;
    char line[240], w0[256] = "", w1[256] = "";
    line[79] = '\0';
    char *ty = line + 1, *l0 = line + 4, *l1 = line + 14, *v1 = line + 24, *l2 = line + 39, *v2 = line + 49;
    int st = S_HEAD, len = 0, rc = 0;

    while (fgets(line, 240, fp)) {
        if (line[0] == '*') continue;
        len = (int)strlen(line);
        for (int j = len - 1; j < 79; j++) line[j] = ' ';
        if (st != S_HEAD) {
            line[3] = line[12] = line[22] = line[36] = line[47] = line[61] = line[79] = '\0';
        }
        switch (st) {
        case S_HEAD:
            /* like iolp.c:265 the two words are NOT cleared between lines */
            sscanf(line, "%255s%255s", w0, w1);
            if (!strncmp(w0, "NAME", 4)) { strncpy(nm, w1, 255); st = S_NAME; break; }
            if (!strcmp(w0, "MAX")) sense = -1;
            else if (!strcmp(w0, "MIN")) sense = 1;
            else if (!strcmp(w0, "OBJ")) strncpy(objnm, w1, 255);
            else if (!strcmp(w0, "RHS")) strncpy(rhsnm, w1, 255);
            else if (!strcmp(w0, "RANGES")) strncpy(rngnm, w1, 255);
            else if (!strcmp(w0, "BOUNDS")) strncpy(bndnm, w1, 255);
            break;
        case S_NAME:
            if (!strcmp(line, "ROW")) st = S_ROWS;
            else if (log) fprintf(log, "expected ROWS after NAME instead of %s\n", line);
            break;
        case S_ROWS:
            if (line[0] != ' ') {
                if (!strcmp(line, "COL")) { st = S_COLS; b = calloc((size_t)(m > 0 ? m : 1), sizeof(double)); }
                else if (log) fprintf(log, "expected L, E, G, N, or COLUMNS instead of %s\n", ty);
                break;
            }
            GROW(kind, mcap, m, int);
            rng = realloc(rng, (size_t)mcap * sizeof(double));
            rowlab = realloc(rowlab, (size_t)mcap * sizeof(char *));
            rowlab[m] = strdup(l0);
            {
                char t = ty[0] == ' ' ? ty[1] : ty[0];
                if (t == 'L')      { rng[m] = HUGE_VAL; kind[m] = 1; }
                else if (t == 'E') { rng[m] = 0.0;      kind[m] = 0; }
                else if (t == 'N') {
                    if (!objnm[0]) strncpy(objnm, l0, 255);
                    if (contains(l0, objnm)) strncpy(objnm, l0, 255);
                    kind[m] = 2; rng[m] = HUGE_VAL;
                } else             { rng[m] = HUGE_VAL; kind[m] = 0; } /* 'G' (others undefined upstream) */
            }
            lbl_put(&rows, tagged(key, l0, 'R'), m);
            m++;
            break;
        case S_COLS:
            if (line[0] != ' ') {
                c  = calloc((size_t)(n > 0 ? n : 1), sizeof(double));
                lo = calloc((size_t)(n > 0 ? n : 1), sizeof(double));
                st = section_of(line);
                if (st == S_BAD) { if (log) fprintf(log, "ERROR(26): unrecognized section label: \n   %s \n\n", line); rc = 26; goto done; }
                break;
            }
            if (lbl_get(&cols, tagged(key, l0, 'C')) != -1) {
                if (strcmp(collab[n - 1], l0) != 0) {
                    if (log) fprintf(log, "ERROR(35): column %s out of order in COLUMNS section\n\n", l0);
                    rc = 35; goto done;
                }
            } else if (strcmp(l1, "'MARKER'") != 0) {
                GROW(colstart, ncap, n, int);
                up = realloc(up, (size_t)ncap * sizeof(double));
                collab = realloc(collab, (size_t)ncap * sizeof(char *));
                colstart[n] = nz; collab[n] = strdup(l0); up[n] = HUGE_VAL;
                lbl_put(&cols, key, n);
                n++;
            }
            for (int fld = 0; fld < 2; fld++) {
                if (len < (fld ? 50 : 25)) continue;
                double v = atof(fld ? v2 : v1);
                if (v == 0.0) continue;
                int r = lbl_get(&rows, tagged(key, fld ? l2 : l1, 'R'));
                if (r == -1) { if (log) fprintf(log, "row label %s from COLUMNS section missing in ROWS section\n", fld ? l2 : l1); continue; }
                GROW(ia, nzcap, nz, int);
                av = realloc(av, (size_t)nzcap * sizeof(double));
                ia[nz] = r; av[nz] = v; nz++;
            }
            break;
        case S_RHS:
        case S_RNG: {
            if (line[0] != ' ') { st = section_of(line); if (st == S_BAD) { if (log) fprintf(log, "ERROR(26): unrecognized section label: \n   %s \n\n", line); rc = 26; goto done; } break; }
            char *setnm = st == S_RHS ? rhsnm : rngnm;
            double *dst = st == S_RHS ? b : rng;
            if (!setnm[0]) strncpy(setnm, l0, 255);
            if (!contains(l0, setnm)) break;
            /* second pair first, then first pair (iolp.c:481-500, 512-531) */
            if (len >= 50) {
                double v = atof(v2);
                if (v != 0.0) {
                    int r = lbl_get(&rows, tagged(key, l2, 'R'));
                    if (r != -1) dst[r] = v;
                    else if (log) fprintf(log, "row label %s from %s section missing in ROWS section\n", l2, st == S_RHS ? "RHS" : "RANGES");
                }
            }
            {
                double v = atof(v1);
                if (v != 0.0) {
                    int r = lbl_get(&rows, tagged(key, l1, 'R'));
                    if (r != -1) dst[r] = v;
                    else if (log) fprintf(log, "row label %s from %s section missing in ROWS section\n", l1, st == S_RHS ? "RHS" : "RANGES");
                }
            }
            break;
        }
        case S_BND: {
            if (line[0] != ' ') { st = section_of(line); if (st == S_BAD) { if (log) fprintf(log, "ERROR(26): unrecognized section label: \n   %s \n\n", line); rc = 26; goto done; } break; }
            if (!bndnm[0]) strncpy(bndnm, l0, 255);
            if (!contains(l0, bndnm)) break;
            double v = atof(v1);
            int j = lbl_get(&cols, tagged(key, l1, 'C'));
            if (j == -1) { if (log) fprintf(log, "col label %s from BOUNDS section missing in COLUMNS section\n", l1); break; }
            if      (!strcmp(ty, "LO")) lo[j] = v;
            else if (!strcmp(ty, "UP")) up[j] = v;
            else if (!strcmp(ty, "FX")) { lo[j] = v; up[j] = v; }
            else if (!strcmp(ty, "FR")) { lo[j] = -HUGE_VAL; up[j] = HUGE_VAL; }
            else if (!strcmp(ty, "PL")) up[j] = HUGE_VAL;
            else if (!strcmp(ty, "MI")) { up[j] = lo[j]; lo[j] = -HUGE_VAL; }
            else if (!strcmp(ty, "BV")) { lo[j] = 0.0; up[j] = 1.0; }
            else if (!strcmp(ty, "LI")) lo[j] = v;
            else if (!strcmp(ty, "UI")) up[j] = v;
            else if (!strcmp(ty, "SC")) { lo[j] = 0.0; up[j] = v; }
            else if (log) fprintf(log, "unrecognized bound type %s \n", ty);
            break;
        }
        case S_QUAD: {
            if (line[0] != ' ') { st = section_of(line); if (st == S_BAD) { if (log) fprintf(log, "ERROR(26): unrecognized section label: \n   %s \n\n", line); rc = 26; goto done; } break; }
            if (!quads) { quads = 1; qdiag = calloc((size_t)(n > 0 ? n : 1), sizeof(double)); }
            int j = lbl_get(&cols, tagged(key, l0, 'C'));
            if (j == -1) { if (log) fprintf(log, "column label %s missing (34)\n", l0); break; }
            if (j > qprev) {
                for (int jj = qprev + 1; jj <= j; jj++) { GROW(qk, qkcap, qkn, int); qk[qkn++] = qn; }
                qprev = j;
            } else if (j < qprev) {
                if (log) fprintf(log, "ERROR(36): QUADS columns out of order\n\n");
                rc = 36; goto done;
            }
            for (int fld = 0; fld < 2; fld++) {
                if (len < (fld ? 50 : 25)) continue;
                double v = atof(fld ? v2 : v1);
                if (v == 0.0) continue;
                int i = lbl_get(&cols, tagged(key, fld ? l2 : l1, 'C'));
                if (i == -1) { if (log) fprintf(log, "column label %s missing (34)\n", fld ? l2 : l1); continue; }
                if (i > j) {
                    GROW(qi, qcap, qn, int);
                    qv = realloc(qv, (size_t)qcap * sizeof(double));
                    qi[qn] = i; qv[qn] = v; qn++;
                } else if (i == j) qdiag[j] = v;
                else if (log) fprintf(log, "QUADS entry above the diagonal ignored (35)\n");
            }
            break;
        }
        default:
            break;
        }
    }
    if (!nm[0]) { if (log) fprintf(log, "ERROR(11): NAME not found\n\n"); rc = 11; goto done; }
    if (st != S_END && log) fprintf(log, "ENDATA not found \n");

    if (!c)  c  = calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    if (!lo) lo = calloc((size_t)(n > 0 ? n : 1), sizeof(double));
    if (!b)  b  = calloc((size_t)(m > 0 ? m : 1), sizeof(double));
    GROW(colstart, ncap, n, int);
    colstart[n] = nz;

    /* objective extraction and row compaction (iolp.c:670-727) */
    {
        int ic = lbl_get(&rows, tagged(key, objnm, 'R'));
        if ((ic == -1 || kind[ic] != 2) && log) fprintf(log, "objective function %s not found \n", objnm);
        int knew = 0;
        for (int j = 0; j < n; j++) {
            int k0 = colstart[j], k1 = colstart[j + 1];
            colstart[j] = knew;
            for (int k = k0; k < k1; k++) {
                int i = ia[k];
                if (i == ic) c[j] = av[k];
                else if (kind[i] == 2) { /* other N rows vanish */ }
                else { av[knew] = kind[i] == 1 ? -av[k] : av[k]; ia[knew] = i; knew++; }
            }
        }
        colstart[n] = knew; nz = knew;
        int *newrow = malloc((size_t)(m > 0 ? m : 1) * sizeof(int));
        int mnew = 0;
        for (int i = 0; i < m; i++) {
            if (i == ic || kind[i] == 2) { free(rowlab[i]); rowlab[i] = NULL; continue; }
            newrow[i] = mnew;
            b[mnew] = kind[i] == 1 ? -b[i] : b[i];
            rng[mnew] = rng[i];
            char *keep = rowlab[i];
            rowlab[i] = NULL;
            rowlab[mnew] = keep;   /* i >= mnew: slot i was read before it is reused */
            mnew++;
        }
        for (int i = mnew; i < m; i++) { free(rowlab[i]); rowlab[i] = NULL; }
        for (int k = 0; k < nz; k++) ia[k] = newrow[ia[k]];
        free(newrow);
        m = mnew;
    }

    P->m = m; P->n = n; P->nz = nz;
    P->colptr = colstart; P->rowind = ia; P->val = av;
    P->rhs = b; P->obj = c; P->range = rng; P->lo = lo; P->hi = up;
    P->fixed = 0.0; P->sense = sense;
    strncpy(P->name, nm, 255);
    P->rowlab = rowlab; P->collab = collab;
    colstart = NULL; ia = NULL; av = NULL; b = c = rng = lo = up = NULL;
    rowlab = collab = NULL;
    P->kQ = NULL; P->iQ = NULL; P->Q = NULL; P->qnz = 0;
    if (quads) {   /* symmetrise (iolp.c:733-793) */
        for (int jj = qprev + 1; jj <= n; jj++) { GROW(qk, qkcap, qkn, int); qk[qkn++] = qn; }
        int cnt = 0;
        for (int j = 0; j < n; j++) if (qdiag[j] != 0.0) cnt++;
        int tot = 2 * qn + cnt;
        int *kq = malloc(sizeof(int) * (size_t)(n + 1)), *iq = malloc(sizeof(int) * (size_t)(tot > 0 ? tot : 1));
        double *q = malloc(sizeof(double) * (size_t)(tot > 0 ? tot : 1));
        int *w = calloc((size_t)(n + 1), sizeof(int));
        for (int k = 0; k < qn; k++) w[qi[k]]++;
        for (int j = 0; j < n; j++) if (qdiag[j] != 0.0) w[j]++;
        kq[0] = 0;
        for (int j = 0; j < n; j++) kq[j + 1] = kq[j] + qk[j + 1] - qk[j] + w[j];
        for (int j = 0; j < n; j++) {
            w[j] = kq[j];
            for (int k = qk[j]; k < qk[j + 1]; k++) { q[w[j]] = qv[k]; iq[w[j]] = qi[k]; w[j]++; }
        }
        for (int j = 0; j < n; j++) {
            if (qdiag[j] != 0.0) { iq[w[j]] = j; q[w[j]] = qdiag[j]; w[j]++; }
            for (int k = qk[j]; k < qk[j + 1]; k++) { int r = qi[k]; iq[w[r]] = j; q[w[r]] = qv[k]; w[r]++; }
        }
        for (int j = 0; j < n; j++)          /* insertion sort by row (qksort) */
            for (int a = kq[j] + 1; a < kq[j + 1]; a++) {
                int ri = iq[a]; double rv = q[a]; int b2 = a - 1;
                while (b2 >= kq[j] && iq[b2] > ri) { iq[b2 + 1] = iq[b2]; q[b2 + 1] = q[b2]; b2--; }
                iq[b2 + 1] = ri; q[b2 + 1] = rv;
            }
        free(w);
        P->kQ = kq; P->iQ = iq; P->Q = q; P->qnz = kq[n];
    }

done:
    fclose(fp);
    lbl_free(&rows); lbl_free(&cols);
    if (collab) { for (int j = 0; j < n; j++) free(collab[j]); free(collab); }
    if (rowlab) { for (int i = 0; i < m; i++) free(rowlab[i]); free(rowlab); }
    free(kind); free(qk); free(qi); free(qv); free(qdiag);
    if (rc) { free(rng); free(colstart); free(up); free(ia); free(av); free(b); free(c); free(lo); }
    return rc;
}

void orc_mps_free(orc_mps *p)
{
    if (p->rowlab) { for (int i = 0; i < p->m; i++) free(p->rowlab[i]); free(p->rowlab); }
    if (p->collab) { for (int j = 0; j < p->n; j++) free(p->collab[j]); free(p->collab); }
    free(p->colptr); free(p->rowind); free(p->val); free(p->rhs); free(p->obj);
    free(p->range); free(p->lo); free(p->hi);
    free(p->kQ); free(p->iQ); free(p->Q);
    memset(p, 0, sizeof(*p));
}

int orc_mps_quads(const char *path, int *n, int *qnz, int *kQ, int *iQ, double *Q)
{
    orc_mps p;
    memset(&p, 0, sizeof(p));
    int rc = orc_mps_read(path, &p, NULL);
    if (rc) return rc;
    if (n) *n = p.n;
    if (qnz) *qnz = p.kQ ? p.qnz : -1;
    if (kQ && p.kQ) memcpy(kQ, p.kQ, sizeof(int) * (size_t)(p.n + 1));
    if (iQ && p.qnz) memcpy(iQ, p.iQ, sizeof(int) * (size_t)p.qnz);
    if (Q && p.qnz) memcpy(Q, p.Q, sizeof(double) * (size_t)p.qnz);
    orc_mps_free(&p);
    return 0;
}
