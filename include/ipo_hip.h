/*
 * ipo_hip.h -- C ABI of libipo_hip.so, the MI355X interior-point core.
 *
 * Drop-in boundary: the symbols below are exactly the plug-in points the
 * reference ipo binary links (src/ipo/makefile:49,56-63: $(METHOD) $(LU)).
 * Linking libipo_hip.so in place of hsd.o/intpt.o (and ldlt.o) leaves the
 * MPS/AMPL front end (src/common, src/amplsolver) unchanged.  All pointers
 * are host pointers with the reference's meaning; nothing here exposes
 * device or torch types.
 */
#ifndef IPO_HIP_H
#define IPO_HIP_H

#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- METHOD plug-in ------------------------------------------------------
 * Replaces solver() of src/ipo/hsd.c:27-29 (default, like makefile:57),
 * src/ipo/intpt.c:33-35 (set IPO_HIP_METHOD=intpt) and src/ipo/hsdls.c:38-40
 * (IPO_HIP_METHOD=hsdls); prototype from
 * src/common/solve.c:24-26.  Solves  max c'x + f  s.t.  Ax <= b, x >= 0,
 * A m x n CSC (kA[n+1], iA[nz], A[nz]), 0-based.  x, z: n; y, w: m (the
 * caller may allocate more, as solve.c:194-197 does).  Prints the banner
 * and one trace line per iteration to stdout in the reference format.
 * Returns 0 optimal, 2 primal infeasible, 4 dual infeasible, 5 iteration
 * limit, 7 on a device error (the reference would exit(1)).
 * Unlike hsd.c:290-291 it does NOT free w and z (they belong to the caller). */
int solver(int m, int n, int nz, int *iA, int *kA, double *A, double *b, double *c, double f,
           double *x, double *y, double *w, double *z);

/* ---- LU plug-in ------------------------------------------------------------
 * Replaces src/ipo/ldlt.h:1-20 (ldlt.c:124-162 and ldlt.c:311-319) with the
 * reference's argument convention: ldltfac(m, n, kA, iA, A, dn, dm, kAt,
 * iAt, At, verbose) factors  [ -diag(dn)  A' ; A  diag(dm) ]  where A is
 * m x n (CSC kA/iA/A, transpose kAt/iAt/At), dn has n entries, dm has m.
 * The first call performs the symbolic analysis and keeps it for the rest
 * of the process (one pattern per process, like ldlt.c:108-120).
 * forwardbackward(Dn, Dm, dx, dy) solves in place with iterative refinement
 * (dx: n entries, dy: m entries), ldlt.c:327-425. */
void ldltfac(int m, int n, int *kA, int *iA, double *A, double *dn, double *dm,
             int *kAt, int *iAt, double *At, int verbose);
void forwardbackward(double *Dn, double *Dm, double *dx, double *dy);
/* releases the LU plug-in state (ldlt.c:507-513), and a Q block set below */
void inv_clo(void);
/* The Q block of the reference's K (ldlt.c:178-185, 253-256, 391-394), for a
 * caller of the LU plug-in that has one (the reference's inv_num reads it
 * from lp->Q / kQ / iQ / max; ipo's own solvers never set it, ldlt.c:142-144):
 * call before the first ldltfac (or after inv_clo).  Q is ldltfac's n x n,
 * full symmetric CSC (both triangles and the diagonal, rows sorted in each
 * column, as iolp.c:733-793 stores QUADS); it joins the block of dn:
 * K = [ -(dn + max Q)  A' ; A  dm ], and the refinement residual carries
 * max Q dx.  max = lp->max (-1 maximise, 1 minimise).  kQ == NULL removes it.
 * Returns 0, or -1 after ldltfac (ipo_hip_last_error). */
int ipo_hip_ldlt_set_q(int n, const int *kQ, const int *iQ, const double *Q, int max);

/* ---- extended interface (not in the reference) ---------------------------- */
typedef struct {
    int    iters;            /* trace lines printed                           */
    int    status;
    double t_setup_s;        /* host symbolic analysis + uploads              */
    double t_solve_s;        /* iteration loop wall time                      */
    double factor_ms;        /* device time in factorisations (if timing)     */
    double solve_ms;         /* device time in refined solves (if timing)     */
    long   factors, solves, rawsolves, refine_passes;
    double final_mu, final_pobj, final_dobj, final_pinf, final_dinf;
    long   lnz;              /* nnz of L (reference pattern)                  */
    double narth;            /* reference op count, ldlt.c:1243-1248          */
    int    nsup, nlevels;
    double flops_factor;     /* flops of one numeric factorisation            */
    double lx_bytes;         /* bytes of the supernodal factor storage        */
    double update_ms;        /* device time of the left-looking gather kernel (timing) */
    double panel_ms;         /* device time of the panel LDL'+trsm kernel (timing)     */
    double sweep_ms;         /* device time of triangular substitution sweeps (timing) */
    long   update_launches, panel_launches;
    double flops_update;     /* algorithmic flops of the gather kernel per factorisation */
    double bytes_update;     /* algorithmic bytes of the gather kernel per factorisation */
    /* per phase (timing mode): 0 gather (k_update*), 1 sparse panels (k_panel_w /
     * k_panel_s, or k_diag), 2 panel solve (k_trsm), 3 dense-tail trailing update
     * of the per-phase path (k_tail_syrk), 4 forward sweep, 5 backward sweep,
     * 6 dense-tail factor of the look-ahead path (k_tail_pr with its visits, and
     * the repair launches k_tail_col / k_tail_dep), 7 unused */
    double phase_ms[8];      /* device time (HIP events on the solver's stream)      */
    long   phase_launches[8];/* kernel launches                                       */
    long   phase_count[8];   /* occurrences: factorisations (each counted once, its
                              * dense-tail repairs included) / substitution sweeps    */
    double phase_flops[8];   /* algorithmic flops of one occurrence                   */
    double phase_bytes[8];   /* algorithmic bytes of one occurrence                   */
    long   tail_repairs;     /* dense-tail block columns redone after a bail-out      */
    long   tail_dep_rounds;  /* k_tail_dep launches of those repairs                  */
    long   tail_chain_aborts;/* dense-tail chain launches aborted (a contradicted
                              * dropped column): factorisation redone per step     */
} ipo_hip_stats;

/* method: 0 = hsd, 1 = intpt, 2 = hsdls.  trace may be NULL (silent).  timing != 0
 * records per-phase HIP-event times. */
int ipo_hip_solve(int method, int m, int n, int nz, const int *iA, const int *kA, const double *A,
                  const double *b, const double *c, double f, double *x, double *y, double *w, double *z,
                  FILE *trace, int max_iter, int timing, ipo_hip_stats *stats);

/* Persistent context: uploads the problem to HBM and runs the symbolic
 * analysis once (setup); ipo_hip_ctx_run then iterates from the reference's
 * start point with everything device-resident (used by bench.py). */
typedef struct ipo_hip_ctx ipo_hip_ctx;
ipo_hip_ctx *ipo_hip_ctx_create(int m, int n, const int *kA, const int *iA, const double *A,
                                const double *b, const double *c, double f);
int  ipo_hip_ctx_run(ipo_hip_ctx *ctx, int method, int max_iter, FILE *trace, int timing, ipo_hip_stats *stats);
void ipo_hip_ctx_download(ipo_hip_ctx *ctx, double *x, double *y, double *w, double *z);
void ipo_hip_ctx_destroy(ipo_hip_ctx *ctx);
double ipo_hip_ctx_setup_seconds(const ipo_hip_ctx *ctx);

/* ---- block-angular sharding (not in the reference) --------
 * One process per GPU.  Rank k passes its LOCAL problem: the rows and
 * columns of its diagonal blocks plus a replica of the nlink linking rows,
 * which must be its last nlink rows (ipo_amd.shard_block_angular builds it);
 * m_global, n_global, nz_global describe the whole LP (mu's denominator and
 * the trace).  The linking rows form the dense tail of every shard's KKT
 * factor and are the only place the shards meet: one allreduce of the
 * nlink x nlink tail per factorisation, nlink-vectors per substitution sweep
 * and refinement pass, a few scalars per iteration.  Transport: RCCL
 * (rccl_id = the 128-byte ncclUniqueId rank 0 got from
 * ipo_hip_rccl_unique_id, distributed by the caller; select the device
 * with ipo_hip_set_device first) or, with rccl_id == NULL, the host
 * callback fn (device data staged through pinned host memory; op 0 = sum,
 * 1 = max, 2 = min; returns 0 on success).  nranks == 1: one process, the
 * linking rows in the tail, no exchange.  Run with ipo_hip_ctx_run /
 * _download / _destroy; all ranks call them together (collectives).
 * Returns NULL on error (ipo_hip_last_error). */
typedef int (*ipo_hip_allreduce_fn)(void *user, double *buf, long n, int op);
int ipo_hip_set_device(int device);
int ipo_hip_rccl_unique_id(void *out128);
ipo_hip_ctx *ipo_hip_ctx_create_shard(int m, int n, const int *kA, const int *iA, const double *A,
                                      const double *b, const double *c, double f, int nlink,
                                      int m_global, int n_global, long nz_global, int nranks, int rank,
                                      const void *rccl_id, ipo_hip_allreduce_fn fn, void *user);

/* Read an MPS file, normalise it like solvelp() (src/common/solve.c:28-205)
 * and solve it; prints exactly what `ipo file.mps` prints (main.c:16-58)
 * minus the .out file.  Returns the status (3 = free variable). */
int ipo_hip_run_mps(const char *path, int method, FILE *out, int timing, ipo_hip_stats *stats);

/* ipo_hip_run_mps with options.  flags: IPO_HIP_SPLIT_FREE -- the
 * free-variable extension (not in the reference, which returns 3 "dual
 * unbounded" at solve.c:79-87): free columns are split (x = x+ - x-) or
 * reflected (x = u - x') before the normalisation (lp_io.h
 * split_free_columns).  solfile != NULL: the reference's writesol report
 * (iolp.c:976-1045, main.c:54-56 writes it to <NAME>.out) for the original
 * problem, z as solver() returned it (the reference reads it after freeing
 * it, hsd.c:290-291). */
#define IPO_HIP_SPLIT_FREE 1
int ipo_hip_run_mps_ex(const char *path, int method, int flags, const char *solfile, FILE *out, int timing,
                       ipo_hip_stats *stats);

/* Dimensions of an MPS file after normalisation (for tests/harnesses).
 * Returns 0, 3 (free variable) or the reader's error number. */
int ipo_hip_mps_dims(const char *path, int *m0, int *n0, int *nz0, int *m, int *n, int *nz);

/* Normalised problem export: caller passes NULL to query sizes first. */
int ipo_hip_mps_load(const char *path, int *m, int *n, int *nz, int *kA, int *iA, double *A,
                     double *b, double *c, double *f);

/* The writesol report (iolp.c:976-1045) of an MPS file from solver()-form
 * vectors x (n + m), y (n + m), z (n) of its normalisation (host code, no
 * device; ipo_hip_run_mps_ex calls the same writer).  0 on success. */
int ipo_hip_write_sol(const char *path, int flags, const double *x, const double *y, const double *z,
                      const char *solfile);

/* The QUADS section of an MPS file as the reference's reader keeps it
 * (iolp.c:583-645, symmetrised iolp.c:733-793): n x n over the file's
 * columns, both triangles and the nonzero diagonal, rows sorted in each
 * column.  Pass kQ = NULL to query n and qnz (-1: no QUADS section).
 * Returns 0 or the reader's error number (36: QUADS columns out of order). */
int ipo_hip_mps_quads(const char *path, int *n, int *qnz, int *kQ, int *iQ, double *Q);

/* ipo_hip_mps_load with the flags of ipo_hip_run_mps_ex. */
int ipo_hip_mps_load_ex(const char *path, int flags, int *m, int *n, int *nz, int *kA, int *iA, double *A,
                        double *b, double *c, double *f);

/* KKT factor handle: symbolic + device numeric LDL' of K(E, D) for tests. */
typedef struct ipo_hip_kkt ipo_hip_kkt;
ipo_hip_kkt *ipo_hip_kkt_create(int m, int n, const int *kA, const int *iA, const double *A);
/* the same with a Q block on the y-nodes (K_yy = -max(E, eps) - qmax Q, the
 * first block of ldlt.c's K; Q m x m full symmetric CSC), NULL kQ: none */
ipo_hip_kkt *ipo_hip_kkt_create_q(int m, int n, const int *kA, const int *iA, const double *A, const int *kQ,
                                  const int *iQ, const double *Q, int qmax);
void   ipo_hip_kkt_destroy(ipo_hip_kkt *k);
int    ipo_hip_kkt_factor(ipo_hip_kkt *k, const double *E, const double *D);
int    ipo_hip_kkt_solve(ipo_hip_kkt *k, const double *E, const double *D, double *fy, double *fx);
int    ipo_hip_kkt_info(const ipo_hip_kkt *k, long *lnz, double *narth, int *nsup, int *nlevels, int *denwin,
                        int *pdf, double *epsdiag, int *ndep, int *passes);
int    ipo_hip_kkt_perm(const ipo_hip_kkt *k, int *perm);
/* the last factor's pivots D (diag of ldlt.c's lltnum, new order) and live
 * marks (0 = dependent pivot, ldlt.c:600-614), T = m + n entries each */
int    ipo_hip_kkt_pivots(const ipo_hip_kkt *k, double *d, int *live);
/* start from a captured state: the reference's eps_diag floor (ldlt.c:31,301-305) */
void   ipo_hip_kkt_set_epsdiag(ipo_hip_kkt *k, double epsdiag);

/* Host-only symbolic analysis (no GPU needed): reference ordering stats. */
int ipo_hip_symbolic(int m, int n, const int *kA, const int *iA, int *perm, long *lnz, double *narth,
                     int *denwin, int *pdf, int *nsup, int *nlevels);
/* ipo_hip_symbolic with a Q block on the y-nodes (ipo_hip_kkt_create_q's
 * convention; kQ == NULL: none): the reference ordering of ldlt.c's K with
 * Q (Q neighbours in the adjacency ldlt.c:729-745, separability ldlt.c:675-682). */
int ipo_hip_symbolic_q(int m, int n, const int *kA, const int *iA, const int *kQ, const int *iQ, int *perm,
                       long *lnz, double *narth, int *denwin, int *pdf, int *nsup, int *nlevels);
/* Same with the last nforced rows (linking rows) forced to the end of the
 * order and forming the dense tail (block-angular sharding); colcount[T]
 * = strict-lower nonzeros per column of L in the new order. */
int ipo_hip_symbolic_forced(int m, int n, const int *kA, const int *iA, int nforced, int *perm, int *colcount,
                            long *lnz, int *tail_c0, int *nsup, int *nlevels);

/* Synthetic LPs in solver() form (BASELINE configs[3] and configs[4],
 * SURVEY.md §8(d); not part of the reference): feasible and bounded by
 * construction from an interior point x*, y*, w*, z* in U[0.5,1.5]
 * (b = A x* + w*, c = A' y* - z*).  Pass kA = NULL to query sizes only;
 * otherwise kA[n+1], iA[nz], A[nz], b[m], c[n] are filled, and xs/zs (n),
 * ys/ws (m) when non-NULL.  band = 0: uniform rows; band > 0: rows from a
 * window of that width around floor(j m / n).  Returns 0, or -1 on bad
 * sizes (ipo_hip_last_error). */
/* The HBM-bound per-iteration kernels of the HSD loop (A x / A'y with the
 * residual and right-hand-side vectors, directions + ratio test, step;
 * hsd.c:182-274) timed alone on device-resident inputs for the LP (m, n, A
 * CSC): ms3[k] = average ms per launch over `reps`, bytes3[k] = algorithmic
 * HBM bytes per launch.  Measurement entry of bench.py (no reference
 * counterpart).  Returns 0, or -1 (ipo_hip_last_error). */
int ipo_hip_vector_bench(int m, int n, const int *kA, const int *iA, const double *A, int reps, double *ms3,
                         double *bytes3);

/* sum_i a[i] b[i] over host vectors, by the solver's ordered reduction
 * (linalg.c:17-25 dotprod's order for n < 2^19, dev_common.hip
 * k_reduce_ordered).  Test entry (no reference counterpart: dotprod is
 * internal to the reference).  Returns 0, or -1 (ipo_hip_last_error). */
int ipo_hip_dot_ordered(const double *a, const double *b, int n, double *out);

int ipo_hip_synth_random(int m, int n, int per_col, int band, unsigned long long seed, int *nz, int *kA, int *iA,
                         double *A, double *b, double *c, double *xs, double *ys, double *ws, double *zs);
/* nblocks diagonal blocks (mb x nb, banded random per block) + nlink linking
 * rows with link_nz nonzeros each; block k owns rows [k mb, (k+1) mb) and
 * columns [k nb, (k+1) nb), linking rows come last. */
int ipo_hip_synth_block_angular(int nblocks, int mb, int nb, int per_col, int band, int nlink, int link_nz,
                                unsigned long long seed, int *m, int *n, int *nz, int *kA, int *iA, double *A,
                                double *b, double *c, double *xs, double *ys, double *ws, double *zs);

/* The persistent dense tail's work-item schedule (host-only; test entry, no
 * reference counterpart): kind 0 k_tail_run's (kkt_dense.hip
 * tail_run_schedule), 1 k_tail_chain_run's, for a tail of nt columns, visit
 * chunks of K blocks, latest chunk L, at most cap workgroups per launch.
 * items[2 i], items[2 i + 1] = item i's (x, y) words, ptr[t] = first item of
 * launch t (ntb + 1 entries, ntb = ceil(nt / 64)); either may be NULL.
 * Returns the item count (items are written up to max_items), or -1
 * (ipo_hip_last_error). */
int ipo_hip_tail_schedule(int kind, int nt, int K, int L, int cap, unsigned *items, int max_items, int *ptr);

int ipo_hip_device_count(void);
/* hipDeviceSynchronize on the calling thread's device (bench.py brackets its
 * timed region with it); 0 on success. */
int ipo_hip_device_synchronize(void);
const char *ipo_hip_last_error(void);
const char *ipo_hip_version(void);

#ifdef __cplusplus
}
#endif
#endif /* IPO_HIP_H */
