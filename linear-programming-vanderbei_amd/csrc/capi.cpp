// capi.cpp -- the C ABI of libipo_hip.so (include/ipo_hip.h).
#include "../../include/ipo_hip.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ipm.h"
#include "kkt_device.h"
#include "lp_io.h"
#include "synth.h"

namespace ipo {
// kkt_dense.hip (declared in kkt_kernels.h, which holds device code)
std::vector<uint2> tail_run_schedule(int ntb, int nt, int K, int L, int cap, std::vector<int>& ptr);
std::vector<uint2> tail_chain_schedule(int ntb, int nt, int K, int L, int cap, std::vector<int>& ptr);
}  // namespace ipo

namespace {

thread_local std::string g_err;

void set_err(const std::string& s) { g_err = s; }

const char* kStatusText[] = {"optimal solution", "primal unbounded", "primal infeasible", "dual unbounded",
                             "dual infeasible",  "iteration limit",  "infinite lower bounds - not implemented",
                             "suboptimal solution"};

ipo::Method method_from_env() {
    const char* e = std::getenv("IPO_HIP_METHOD");
    if (e && !std::strcmp(e, "intpt")) return ipo::Method::Intpt;
    if (e && !std::strcmp(e, "hsdls")) return ipo::Method::Hsdls;
    return ipo::Method::Hsd;
}

ipo::Method method_from_int(int m) {
    return m == 1 ? ipo::Method::Intpt : m == 2 ? ipo::Method::Hsdls : ipo::Method::Hsd;
}

// MAX_ITER of each method: hsd.c:25, intpt.c:31, hsdls.c:25
int default_max_iter(ipo::Method m) { return m == ipo::Method::Hsdls ? 600 : 200; }

// hsd.c:70-92 / intpt.c:70-92: tiny problems are echoed before the banner
void print_small(FILE* tr, int m, int n, const int* kA, const int* iA, const double* A, const double* b,
                 const double* c) {
    if (!tr || !(m < 20 && n < 20)) return;
    double AA[20][20];
    for (int j = 0; j < n; j++) for (int i = 0; i < m; i++) AA[i][j] = 0;
    for (int j = 0; j < n; j++) for (int k = kA[j]; k < kA[j + 1]; k++) AA[iA[k]][j] = A[k];
    std::fprintf(tr, "A <= b: \n");
    for (int i = 0; i < m; i++) {
        for (int j = 0; j < n; j++) std::fprintf(tr, " %5.1f", AA[i][j]);
        std::fprintf(tr, "<= %5.1f \n", b[i]);
    }
    std::fprintf(tr, "\n");
    std::fprintf(tr, "c: \n");
    for (int j = 0; j < n; j++) std::fprintf(tr, " %5.1f", c[j]);
    std::fprintf(tr, "\n");
}

void fill_stats(ipo_hip_stats* st, const ipo::IpmResult& r, const ipo::KktDevice* K) {
    const ipo::KktPlan* P = K ? &K->plan() : nullptr;
    if (!st) return;
    std::memset(st, 0, sizeof(*st));
    st->iters = r.iters;
    st->status = r.status;
    st->t_setup_s = r.t_setup_s;
    st->t_solve_s = r.t_solve_s;
    st->factor_ms = r.kkt.factor_ms;
    st->solve_ms = r.kkt.solve_ms;
    st->factors = r.kkt.factors;
    st->solves = r.kkt.solves;
    st->rawsolves = r.kkt.rawsolves;
    st->refine_passes = r.refine_passes;
    st->final_mu = r.final_mu;
    st->final_pobj = r.final_pobj;
    st->final_dobj = r.final_dobj;
    st->final_pinf = r.final_pinf;
    st->final_dinf = r.final_dinf;
    st->update_ms = r.kkt.phase_ms[ipo::kPhGather];
    st->panel_ms = r.kkt.phase_ms[ipo::kPhDiag] + r.kkt.phase_ms[ipo::kPhTrsm] + r.kkt.phase_ms[ipo::kPhSyrk];
    st->sweep_ms = r.kkt.sweep_ms;
    st->update_launches = r.kkt.phase_launches[ipo::kPhGather];
    st->panel_launches = r.kkt.phase_launches[ipo::kPhDiag] + r.kkt.phase_launches[ipo::kPhTrsm] +
                         r.kkt.phase_launches[ipo::kPhSyrk];
    st->tail_repairs = r.kkt.tail_repairs;
    st->tail_dep_rounds = r.kkt.tail_dep_rounds;
    st->tail_chain_aborts = r.kkt.tail_chain_aborts;
    static_assert(ipo::kNumPhases <= 8, "ipo_hip_stats holds 8 phases");
    for (int ph = 0; ph < ipo::kNumPhases; ph++) {
        st->phase_ms[ph] = r.kkt.phase_ms[ph];
        st->phase_launches[ph] = r.kkt.phase_launches[ph];
        st->phase_count[ph] = r.kkt.phase_count[ph];
        if (K) {
            st->phase_flops[ph] = K->work_flops[ph];
            st->phase_bytes[ph] = K->work_bytes[ph];
        }
    }
    if (P) {
        st->flops_update = P->flops_update;
        st->bytes_update = P->bytes_update;
        st->lnz = P->lnz;
        st->narth = P->narth;
        st->nsup = P->nsup;
        st->nlevels = P->nlevels;
        st->flops_factor = P->flops_factor;
        st->lx_bytes = 8.0 * static_cast<double>(P->lx_size);
    }
}

int solve_impl(ipo::Method method, int m, int n, int nz, const int* iA, const int* kA, const double* A,
               const double* b, const double* c, double f, double* x, double* y, double* w, double* z, FILE* trace,
               int max_iter, int timing, ipo_hip_stats* stats, bool* dev_err = nullptr) {
    if (dev_err) *dev_err = false;
    try {
        if (method != ipo::Method::Hsdls) print_small(trace, m, n, kA, iA, A, b, c);   // hsdls.c has no echo
        ipo::IpmSolver S(m, n, kA, iA, A, b, c, f);
        ipo::IpmOptions opt;
        opt.method = method;
        opt.trace = trace;
        opt.max_iter = max_iter > 0 ? max_iter : default_max_iter(method);
        opt.timing = timing != 0;
        ipo::IpmResult res;
        (void)nz;
        const int status = S.run(opt, &res);
        S.download(x, y, w, z);
        fill_stats(stats, res, &S.kkt());
        return status;
    } catch (const std::exception& e) {
        set_err(e.what());
        if (trace) std::fprintf(trace, "ipo_hip: %s\n", e.what());
        if (dev_err) *dev_err = true;
        return 7;
    }
}

// --- LU plug-in state: one pattern per process, like ldlt.c:108-120
struct LuState {
    std::unique_ptr<ipo::KktDevice> kkt;
    hipStream_t stream = nullptr;
    int ms = 0, ns = 0;                 // solver-side dimensions
    ipo::DevBuf<double> E, D, fy, fx;
};
LuState* g_lu = nullptr;
// the Q block attached to the LU plug-in before its first ldltfac
// (ipo_hip_ldlt_set_q): what a caller of the reference's inv_num puts in
// lp->Q / kQ / iQ / max (ldlt.c:178-185)
struct LuQ {
    std::vector<int> kQ, iQ;
    std::vector<double> Q;
    int qmax = 1;
};
std::unique_ptr<LuQ> g_lu_q;

// What the header promises of a caller's Q (ipo_hip.h): kQ[0] = 0 and
// nondecreasing, rows 0 <= iQ < n strictly ascending in every column (so no
// duplicate entries: ldlt.c:253-256 subtracts each entry once), and Q
// symmetric in pattern and value (iolp.c:733-793 leaves QUADS that way).
// Anything else indexes the ordering's arrays out of range on the host or
// factors another matrix than the reference would: refused.
void validate_q(int n, const int* kQ, const int* iQ, const double* Q) {
    if (n < 0) throw std::invalid_argument("Q: negative dimension");
    if (kQ[0] != 0) throw std::invalid_argument("Q: kQ[0] != 0");
    for (int j = 0; j < n; j++) {
        if (kQ[j + 1] < kQ[j]) throw std::invalid_argument("Q: kQ decreasing at column " + std::to_string(j));
        for (int k = kQ[j]; k < kQ[j + 1]; k++) {
            if (iQ[k] < 0 || iQ[k] >= n) throw std::invalid_argument("Q: row index out of range in column " + std::to_string(j));
            if (k > kQ[j] && iQ[k] <= iQ[k - 1])
                throw std::invalid_argument("Q: rows not strictly ascending in column " + std::to_string(j));
        }
    }
    for (int j = 0; j < n; j++)
        for (int k = kQ[j]; k < kQ[j + 1]; k++) {
            const int i = iQ[k];
            const int* b = iQ + kQ[i];
            const int* e = iQ + kQ[i + 1];
            const int* f = std::lower_bound(b, e, j);
            if (f == e || *f != j || Q[f - iQ] != Q[k])
                throw std::invalid_argument("Q: not symmetric at (" + std::to_string(i) + ", " + std::to_string(j) + ")");
        }
}

}  // namespace

struct ipo_hip_ctx {
    std::unique_ptr<ipo::Exchange> xch;          // sharded contexts; outlives the solver (declared first)
    std::unique_ptr<ipo::IpmSolver> solver;
};

struct ipo_hip_kkt {
    std::unique_ptr<ipo::KktDevice> kkt;
    hipStream_t stream = nullptr;
    int m = 0, n = 0;
    ipo::DevBuf<double> E, D, fy, fx;
};

namespace ipo {
double dot_ordered_host(const double* a, const double* b, int n);   // dev_common.hip
}

extern "C" {

int solver(int m, int n, int nz, int* iA, int* kA, double* A, double* b, double* c, double f, double* x, double* y,
           double* w, double* z) {
    return solve_impl(method_from_env(), m, n, nz, iA, kA, A, b, c, f, x, y, w, z, stdout, 0, 0, nullptr);
}

int ipo_hip_solve(int method, int m, int n, int nz, const int* iA, const int* kA, const double* A, const double* b,
                  const double* c, double f, double* x, double* y, double* w, double* z, FILE* trace, int max_iter,
                  int timing, ipo_hip_stats* stats) {
    return solve_impl(method_from_int(method), m, n, nz, iA, kA, A, b, c, f, x, y, w, z,
                      trace, max_iter, timing, stats);
}

ipo_hip_ctx* ipo_hip_ctx_create(int m, int n, const int* kA, const int* iA, const double* A, const double* b,
                                const double* c, double f) {
    try {
        auto* ctx = new ipo_hip_ctx();
        ctx->solver = std::make_unique<ipo::IpmSolver>(m, n, kA, iA, A, b, c, f);
        return ctx;
    } catch (const std::exception& e) {
        set_err(e.what());
        return nullptr;
    }
}

int ipo_hip_ctx_run(ipo_hip_ctx* ctx, int method, int max_iter, FILE* trace, int timing, ipo_hip_stats* stats) {
    try {
        ipo::IpmOptions opt;
        opt.method = method_from_int(method);
        opt.trace = trace;
        opt.max_iter = max_iter > 0 ? max_iter : default_max_iter(opt.method);
        opt.timing = timing != 0;
        ipo::IpmResult res;
        const int st = ctx->solver->run(opt, &res);
        fill_stats(stats, res, &ctx->solver->kkt());
        return st;
    } catch (const std::exception& e) {
        set_err(e.what());
        return 7;
    }
}

void ipo_hip_ctx_download(ipo_hip_ctx* ctx, double* x, double* y, double* w, double* z) {
    ctx->solver->download(x, y, w, z);
}

void ipo_hip_ctx_destroy(ipo_hip_ctx* ctx) { delete ctx; }

double ipo_hip_ctx_setup_seconds(const ipo_hip_ctx* ctx) { return ctx->solver->setup_seconds(); }

int ipo_hip_set_device(int device) {
    const hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        set_err(std::string("hipSetDevice: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int ipo_hip_rccl_unique_id(void* out128) {
    try {
        ipo::rccl_unique_id(out128);
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

ipo_hip_ctx* ipo_hip_ctx_create_shard(int m, int n, const int* kA, const int* iA, const double* A, const double* b,
                                      const double* c, double f, int nlink, int m_global, int n_global,
                                      long nz_global, int nranks, int rank, const void* rccl_id,
                                      ipo_hip_allreduce_fn fn, void* user) {
    try {
        if (nlink < 0 || nlink > m) throw std::invalid_argument("shard: nlink out of range");
        if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("shard: bad rank / nranks");
        auto ctx = std::make_unique<ipo_hip_ctx>();
        // IPO_HIP_SHARD_RCCL=1 with one rank and no transport given: a
        // one-rank RCCL communicator, so the RCCL path runs on a single GPU
        const bool rccl1 = nranks == 1 && !rccl_id && !fn && std::getenv("IPO_HIP_SHARD_RCCL");
        if (rccl1) {
            char id[128];
            ipo::rccl_unique_id(id);
            ctx->xch.reset(ipo::make_rccl_exchange(id, 1, 0));
        } else if (rccl_id) {
            ctx->xch.reset(ipo::make_rccl_exchange(rccl_id, nranks, rank));
        } else if (fn) {
            ctx->xch.reset(ipo::make_host_exchange(nranks, rank, fn, user));
        } else if (nranks > 1) {
            throw std::invalid_argument("shard: nranks > 1 needs an RCCL id or a host allreduce callback");
        }
        ipo::ShardSpec sp;
        sp.nforced = nlink;
        sp.xch = ctx->xch.get();
        sp.m_global = m_global;
        sp.n_global = n_global;
        sp.nz_global = nz_global;
        ctx->solver = std::make_unique<ipo::IpmSolver>(m, n, kA, iA, A, b, c, f, nullptr, &sp);
        return ctx.release();
    } catch (const std::exception& e) {
        set_err(e.what());
        return nullptr;
    }
}

int ipo_hip_run_mps(const char* path, int method, FILE* out, int timing, ipo_hip_stats* stats) {
    return ipo_hip_run_mps_ex(path, method, 0, nullptr, out, timing, stats);
}

namespace {
// read + (optionally) split free columns + normalise; returns the
// to_solver_form status (3: a free variable and no split requested)
int load_form(const char* path, int flags, ipo::MpsProblem& p, ipo::MpsProblem& q, ipo::FreeMap& fm,
              ipo::SolverForm& s, std::string& err, FILE* out) {
    const int rc = ipo::read_mps(path, p, &err);
    if (rc) return -rc;
    if (out) std::fprintf(out, "m = %d,n = %d,nz = %d \n", p.m, p.n, p.kA.empty() ? 0 : p.kA[p.n]);
    if (flags & IPO_HIP_SPLIT_FREE) {
        ipo::split_free_columns(p, q, fm);
        return ipo::to_solver_form(q, s);
    }
    return ipo::to_solver_form(p, s);
}
}  // namespace

int ipo_hip_run_mps_ex(const char* path, int method, int flags, const char* solfile, FILE* out, int timing,
                       ipo_hip_stats* stats) {
    if (out) {
        std::fprintf(out, "%s\n%s\n%s%5s%s\n%s\n%s\n", "\t+-------------------------------------------------+",
                     "\t                                                   ", "\t   ", "./ipo",
                     ":   Version 1.00 : (Copyright) 1995        ",
                     "\t                                                   ",
                     "\t+-------------------------------------------------+");
        std::fflush(out);
    }
    ipo::MpsProblem p, q;
    ipo::FreeMap fm;
    ipo::SolverForm s;
    std::string err;
    int status = load_form(path, flags, p, q, fm, s, err, out);
    if (status < 0) {
        set_err(err);
        if (out) std::fprintf(out, "ERROR(%d): %s\n\n", -status, err.c_str());
        return status;
    }
    bool dev_err = false;
    if (stats) std::memset(stats, 0, sizeof(*stats));
    std::vector<double> x(s.n + s.m, 0.0), y(s.n + s.m, 0.0), w(s.m > 0 ? s.m : 1, 0.0), z(s.n > 0 ? s.n : 1, 0.0);
    if (status == 0) {
        if (out && s.m < 7 && s.n < 7) {   // solve.c:210-222
            std::fprintf(out, "A: \n");
            for (int j = 0; j < s.n; j++) {
                for (int k = s.kA[j]; k < s.kA[j + 1]; k++) std::fprintf(out, "%5d %10.5f \n", s.iA[k], s.A[k]);
                std::fprintf(out, "\n");
            }
            std::fprintf(out, "\n");
            std::fprintf(out, "b: \n");
            for (int i = 0; i < s.m; i++) std::fprintf(out, "%10.5f \n", s.b[i]);
            std::fprintf(out, "\n");
            std::fprintf(out, "c: \n");
            for (int j = 0; j < s.n; j++) std::fprintf(out, "%10.5f \n", s.c[j]);
            std::fprintf(out, "\n");
        }
        status = solve_impl(method_from_int(method), s.m, s.n, s.nz, s.iA.data(),
                            s.kA.data(), s.A.data(), s.b.data(), s.c.data(), s.f, x.data(), y.data(), w.data(),
                            z.data(), out, 0, timing, stats, &dev_err);   // 0: the method's MAX_ITER
    }
    // a device / host exception is not a numerical outcome: no status text for it
    if (out) {
        if (dev_err) std::fprintf(out, "device error: %s\n", g_err.c_str());
        else std::fprintf(out, "%s \n", kStatusText[status]);
        std::fflush(out);
    }
    if (solfile && !dev_err) {
        const ipo::MpsProblem& src = (flags & IPO_HIP_SPLIT_FREE) ? q : p;
        ipo::SolutionOut so = ipo::untransform(src, s, x.data(), y.data(), z.data());
        if (flags & IPO_HIP_SPLIT_FREE) ipo::merge_split(p, fm, so);
        if (ipo::write_sol(solfile, p, so, &err)) set_err(err);
    }
    return status;
}

int ipo_hip_mps_dims(const char* path, int* m0, int* n0, int* nz0, int* m, int* n, int* nz) {
    ipo::MpsProblem p;
    std::string err;
    const int rc = ipo::read_mps(path, p, &err);
    if (rc) { set_err(err); return rc; }
    ipo::SolverForm s;
    const int st = ipo::to_solver_form(p, s);
    if (m0) *m0 = p.m;
    if (n0) *n0 = p.n;
    if (nz0) *nz0 = p.kA.empty() ? 0 : p.kA[p.n];
    if (m) *m = s.m;
    if (n) *n = s.n;
    if (nz) *nz = s.nz;
    return st;
}

int ipo_hip_mps_quads(const char* path, int* n, int* qnz, int* kQ, int* iQ, double* Q) {
    ipo::MpsProblem p;
    std::string err;
    const int rc = ipo::read_mps(path, p, &err);
    if (rc) { set_err(err); return rc; }
    const int nq = p.kQ.empty() ? 0 : p.kQ.back();
    if (n) *n = p.n;
    if (qnz) *qnz = p.kQ.empty() ? -1 : nq;
    if (kQ && !p.kQ.empty()) std::memcpy(kQ, p.kQ.data(), sizeof(int) * (p.n + 1));
    if (iQ && nq) std::memcpy(iQ, p.iQ.data(), sizeof(int) * nq);
    if (Q && nq) std::memcpy(Q, p.Q.data(), sizeof(double) * nq);
    return 0;
}

int ipo_hip_write_sol(const char* path, int flags, const double* x, const double* y, const double* z,
                      const char* solfile) {
    ipo::MpsProblem p, q;
    ipo::FreeMap fm;
    ipo::SolverForm s;
    std::string err;
    const int st = load_form(path, flags, p, q, fm, s, err, nullptr);
    if (st < 0) { set_err(err); return -st; }
    if (st) return st;
    ipo::SolutionOut so = ipo::untransform((flags & IPO_HIP_SPLIT_FREE) ? q : p, s, x, y, z);
    if (flags & IPO_HIP_SPLIT_FREE) ipo::merge_split(p, fm, so);
    if (ipo::write_sol(solfile, p, so, &err)) { set_err(err); return 2; }
    return 0;
}

int ipo_hip_mps_load(const char* path, int* m, int* n, int* nz, int* kA, int* iA, double* A, double* b, double* c,
                     double* f) {
    return ipo_hip_mps_load_ex(path, 0, m, n, nz, kA, iA, A, b, c, f);
}

int ipo_hip_mps_load_ex(const char* path, int flags, int* m, int* n, int* nz, int* kA, int* iA, double* A, double* b,
                        double* c, double* f) {
    ipo::MpsProblem p, q;
    ipo::FreeMap fm;
    ipo::SolverForm s;
    std::string err;
    const int st = load_form(path, flags, p, q, fm, s, err, nullptr);
    if (st < 0) { set_err(err); return -st; }
    if (st) return st;
    if (m) *m = s.m;
    if (n) *n = s.n;
    if (nz) *nz = s.nz;
    if (kA) std::memcpy(kA, s.kA.data(), sizeof(int) * (s.n + 1));
    if (iA) std::memcpy(iA, s.iA.data(), sizeof(int) * s.nz);
    if (A) std::memcpy(A, s.A.data(), sizeof(double) * s.nz);
    if (b) std::memcpy(b, s.b.data(), sizeof(double) * s.m);
    if (c) std::memcpy(c, s.c.data(), sizeof(double) * s.n);
    if (f) *f = s.f;
    return 0;
}

// ---- LU plug-in (ldlt.h).  In the reference's own naming the matrix is
// A_l (m x n) with its transpose; solver-side this is A_s = A_l' with
// E = dn (n entries) and D = dm (m entries), so KktDevice gets kAt/iAt/At.
void ldltfac(int m, int n, int* kA, int* iA, double* A, double* dn, double* dm, int* kAt, int* iAt, double* At,
             int verbose) {
    (void)kA; (void)iA; (void)A; (void)verbose;
    try {
        if (!g_lu) {
            g_lu = new LuState();
            IPO_HIP_CHECK(hipStreamCreateWithFlags(&g_lu->stream, hipStreamNonBlocking));
            g_lu->ms = n;
            g_lu->ns = m;
            ipo::QBlock qb;
            if (g_lu_q) {
                if (static_cast<int>(g_lu_q->kQ.size()) != n + 1)
                    throw std::invalid_argument("ldltfac: the Q block's order is not ldltfac's n");
                qb.kQ = g_lu_q->kQ.data();
                qb.iQ = g_lu_q->iQ.data();
                qb.Q = g_lu_q->Q.data();
                qb.qmax = g_lu_q->qmax;
            }
            g_lu->kkt = std::make_unique<ipo::KktDevice>(n, m, kAt, iAt, At, g_lu->stream, 0, g_lu_q ? &qb : nullptr);
            g_lu->E.alloc(n > 0 ? n : 1);
            g_lu->fy.alloc(n > 0 ? n : 1);
            g_lu->D.alloc(m > 0 ? m : 1);
            g_lu->fx.alloc(m > 0 ? m : 1);
        }
        g_lu->E.upload(dn, g_lu->ms, g_lu->stream);
        g_lu->D.upload(dm, g_lu->ns, g_lu->stream);
        g_lu->kkt->factor(g_lu->E.get(), g_lu->D.get());
    } catch (const std::exception& e) {
        set_err(e.what());
        std::fprintf(stderr, "ipo_hip ldltfac: %s\n", e.what());
        std::exit(1);   // the reference exits on allocation failure (myalloc.h:16-44)
    }
}

void forwardbackward(double* Dn, double* Dm, double* dx, double* dy) {
    try {
        if (!g_lu) throw std::runtime_error("forwardbackward before ldltfac");
        LuState& L = *g_lu;
        L.E.upload(Dn, L.ms, L.stream);
        L.D.upload(Dm, L.ns, L.stream);
        L.fy.upload(dx, L.ms, L.stream);
        L.fx.upload(dy, L.ns, L.stream);
        L.kkt->solve(L.E.get(), L.D.get(), L.fy.get(), L.fx.get());
        L.fy.download(dx, L.ms, L.stream);
        L.fx.download(dy, L.ns, L.stream);
        IPO_HIP_CHECK(hipStreamSynchronize(L.stream));
    } catch (const std::exception& e) {
        set_err(e.what());
        std::fprintf(stderr, "ipo_hip forwardbackward: %s\n", e.what());
        std::exit(1);
    }
}

int ipo_hip_ldlt_set_q(int n, const int* kQ, const int* iQ, const double* Q, int max) {
    if (g_lu) { set_err("ipo_hip_ldlt_set_q after ldltfac (call inv_clo first)"); return -1; }
    if (!kQ || n < 0) { g_lu_q.reset(); return 0; }
    try {
        validate_q(n, kQ, iQ, Q);
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
    auto q = std::make_unique<LuQ>();
    q->kQ.assign(kQ, kQ + n + 1);
    q->iQ.assign(iQ, iQ + kQ[n]);
    q->Q.assign(Q, Q + kQ[n]);
    q->qmax = max;
    g_lu_q = std::move(q);
    return 0;
}

void inv_clo(void) {
    g_lu_q.reset();
    if (!g_lu) return;
    g_lu->kkt.reset();
    if (g_lu->stream) (void)hipStreamDestroy(g_lu->stream);
    delete g_lu;
    g_lu = nullptr;
}

// ---- KKT handle for tests
ipo_hip_kkt* ipo_hip_kkt_create(int m, int n, const int* kA, const int* iA, const double* A) {
    return ipo_hip_kkt_create_q(m, n, kA, iA, A, nullptr, nullptr, nullptr, 1);
}

ipo_hip_kkt* ipo_hip_kkt_create_q(int m, int n, const int* kA, const int* iA, const double* A, const int* kQ,
                                  const int* iQ, const double* Q, int qmax) {
    try {
        if (kQ) validate_q(m, kQ, iQ, Q);
        auto* k = new ipo_hip_kkt();
        IPO_HIP_CHECK(hipStreamCreateWithFlags(&k->stream, hipStreamNonBlocking));
        k->m = m;
        k->n = n;
        ipo::QBlock qb;
        qb.kQ = kQ; qb.iQ = iQ; qb.Q = Q; qb.qmax = qmax;
        k->kkt = std::make_unique<ipo::KktDevice>(m, n, kA, iA, A, k->stream, 0, kQ ? &qb : nullptr);
        k->E.alloc(m > 0 ? m : 1);
        k->fy.alloc(m > 0 ? m : 1);
        k->D.alloc(n > 0 ? n : 1);
        k->fx.alloc(n > 0 ? n : 1);
        return k;
    } catch (const std::exception& e) {
        set_err(e.what());
        return nullptr;
    }
}

void ipo_hip_kkt_destroy(ipo_hip_kkt* k) {
    if (!k) return;
    k->kkt.reset();
    if (k->stream) (void)hipStreamDestroy(k->stream);
    delete k;
}

int ipo_hip_kkt_factor(ipo_hip_kkt* k, const double* E, const double* D) {
    try {
        k->E.upload(E, k->m, k->stream);
        k->D.upload(D, k->n, k->stream);
        k->kkt->factor(k->E.get(), k->D.get());
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_kkt_solve(ipo_hip_kkt* k, const double* E, const double* D, double* fy, double* fx) {
    try {
        k->E.upload(E, k->m, k->stream);
        k->D.upload(D, k->n, k->stream);
        k->fy.upload(fy, k->m, k->stream);
        k->fx.upload(fx, k->n, k->stream);
        const int ok = k->kkt->solve(k->E.get(), k->D.get(), k->fy.get(), k->fx.get());
        k->fy.download(fy, k->m, k->stream);
        k->fx.download(fx, k->n, k->stream);
        IPO_HIP_CHECK(hipStreamSynchronize(k->stream));
        return ok;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_kkt_info(const ipo_hip_kkt* k, long* lnz, double* narth, int* nsup, int* nlevels, int* denwin, int* pdf,
                     double* epsdiag, int* ndep, int* passes) {
    const ipo::KktPlan& P = k->kkt->plan();
    if (lnz) *lnz = P.lnz;
    if (narth) *narth = P.narth;
    if (nsup) *nsup = P.nsup;
    if (nlevels) *nlevels = P.nlevels;
    if (denwin) *denwin = P.denwin;
    if (pdf) *pdf = P.pdf;
    if (epsdiag) *epsdiag = k->kkt->epsdiag();
    if (ndep) *ndep = k->kkt->ndep();
    if (passes) *passes = k->kkt->last_passes();
    return 0;
}

int ipo_hip_kkt_perm(const ipo_hip_kkt* k, int* perm) {
    const ipo::KktPlan& P = k->kkt->plan();
    std::memcpy(perm, P.perm.data(), sizeof(int) * P.T);
    return 0;
}

void ipo_hip_kkt_set_epsdiag(ipo_hip_kkt* k, double e) { k->kkt->set_epsdiag(e); }

int ipo_hip_kkt_pivots(const ipo_hip_kkt* k, double* d, int* live) {
    try {
        k->kkt->download_factor(nullptr, d, live);
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "ipo_hip_kkt_pivots: %s\n", e.what());
        return -1;
    }
}

int ipo_hip_symbolic(int m, int n, const int* kA, const int* iA, int* perm, long* lnz, double* narth, int* denwin,
                     int* pdf, int* nsup, int* nlevels) {
    return ipo_hip_symbolic_q(m, n, kA, iA, nullptr, nullptr, perm, lnz, narth, denwin, pdf, nsup, nlevels);
}

int ipo_hip_symbolic_q(int m, int n, const int* kA, const int* iA, const int* kQ, const int* iQ, int* perm, long* lnz,
                       double* narth, int* denwin, int* pdf, int* nsup, int* nlevels) {
    try {
        std::vector<int> kat, iat;
        std::vector<double> at, a(kA[n], 1.0);
        ipo::csc_transpose(m, n, kA, iA, a.data(), kat, iat, at);
        ipo::QPattern qp;
        qp.kQ = kQ;
        qp.iQ = iQ;
        ipo::KktPlan P = ipo::build_kkt_plan(m, n, kA, iA, kat.data(), iat.data(), 0, 1.0, kQ ? &qp : nullptr);
        if (perm) std::memcpy(perm, P.perm.data(), sizeof(int) * P.T);
        if (lnz) *lnz = P.lnz;
        if (narth) *narth = P.narth;
        if (denwin) *denwin = P.denwin;
        if (pdf) *pdf = P.pdf;
        if (nsup) *nsup = P.nsup;
        if (nlevels) *nlevels = P.nlevels;
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_symbolic_forced(int m, int n, const int* kA, const int* iA, int nforced, int* perm, int* colcount,
                            long* lnz, int* tail_c0, int* nsup, int* nlevels) {
    try {
        if (nforced < 0 || nforced > m) throw std::invalid_argument("nforced out of range");
        std::vector<int> kat, iat;
        std::vector<double> at, a(kA[n], 1.0);
        ipo::csc_transpose(m, n, kA, iA, a.data(), kat, iat, at);
        ipo::KktPlan P = ipo::build_kkt_plan(m, n, kA, iA, kat.data(), iat.data(), nforced);
        if (perm) std::memcpy(perm, P.perm.data(), sizeof(int) * P.T);
        if (colcount) {
            for (int s = 0; s < P.nsup; s++)
                for (int j = P.col0[s]; j < P.col0[s + 1]; j++)
                    colcount[j] = (P.col0[s + 1] - 1 - j) + (P.rowptr[s + 1] - P.rowptr[s]);
            for (int j = P.tail_c0; j < P.T; j++) colcount[j] = P.T - 1 - j;
        }
        if (lnz) *lnz = P.lnz;
        if (tail_c0) *tail_c0 = P.tail_c0;
        if (nsup) *nsup = P.nsup;
        if (nlevels) *nlevels = P.nlevels;
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ipo_hip_device_synchronize(void) {
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        set_err(std::string("hipDeviceSynchronize: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}

const char* ipo_hip_last_error(void) { return g_err.c_str(); }
const char* ipo_hip_version(void) { return "ipo-hip 0.1 (gfx950)"; }

}  // extern "C"

namespace {
void synth_out(const ipo::SynthLP& o, int* kA, int* iA, double* A, double* b, double* c, double* xs, double* ys,
               double* ws, double* zs) {
    std::copy(o.kA.begin(), o.kA.end(), kA);
    std::copy(o.iA.begin(), o.iA.end(), iA);
    std::copy(o.A.begin(), o.A.end(), A);
    std::copy(o.b.begin(), o.b.end(), b);
    std::copy(o.c.begin(), o.c.end(), c);
    if (xs) std::copy(o.xs.begin(), o.xs.end(), xs);
    if (ys) std::copy(o.ys.begin(), o.ys.end(), ys);
    if (ws) std::copy(o.ws.begin(), o.ws.end(), ws);
    if (zs) std::copy(o.zs.begin(), o.zs.end(), zs);
}
}  // namespace

extern "C" {

int ipo_hip_vector_bench(int m, int n, const int* kA, const int* iA, const double* A, int reps, double* ms3,
                         double* bytes3) {
    try {
        ipo::vector_bench(m, n, kA, iA, A, reps, ms3, bytes3);
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_tail_schedule(int kind, int nt, int K, int L, int cap, unsigned* items, int max_items, int* ptr) {
    try {
        if (nt <= 0 || K <= 0 || L <= 0 || cap <= 1 || (kind != 0 && kind != 1))
            throw std::invalid_argument("tail_schedule: bad arguments");
        const int ntb = (nt + ipo::kPanelCols - 1) / ipo::kPanelCols;
        std::vector<int> pv;
        const std::vector<uint2> v = kind == 0 ? ipo::tail_run_schedule(ntb, nt, K, L, cap, pv)
                                               : ipo::tail_chain_schedule(ntb, nt, K, L, cap, pv);
        const int n = static_cast<int>(v.size());
        if (items)
            for (int i = 0; i < std::min(n, max_items); i++) {
                items[2 * i] = v[i].x;
                items[2 * i + 1] = v[i].y;
            }
        if (ptr) std::copy(pv.begin(), pv.end(), ptr);
        return n;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_dot_ordered(const double* a, const double* b, int n, double* out) {
    try {
        if (n < 0 || (n > 0 && (!a || !b)) || !out) throw std::invalid_argument("dot_ordered: bad arguments");
        *out = ipo::dot_ordered_host(a, b, n);
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_synth_random(int m, int n, int per_col, int band, unsigned long long seed, int* nz, int* kA, int* iA,
                         double* A, double* b, double* c, double* xs, double* ys, double* ws, double* zs) {
    try {
        if (nz) *nz = static_cast<int>(static_cast<long long>(n) * per_col);
        if (!kA) return 0;
        ipo::SynthLP o;
        ipo::synth_random(m, n, per_col, band, seed, o);
        synth_out(o, kA, iA, A, b, c, xs, ys, ws, zs);
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

int ipo_hip_synth_block_angular(int nblocks, int mb, int nb, int per_col, int band, int nlink, int link_nz,
                                unsigned long long seed, int* m, int* n, int* nz, int* kA, int* iA, double* A,
                                double* b, double* c, double* xs, double* ys, double* ws, double* zs) {
    try {
        if (m) *m = nblocks * mb + nlink;
        if (n) *n = nblocks * nb;
        if (nz) *nz = static_cast<int>(static_cast<long long>(nblocks) * nb * per_col +
                                       static_cast<long long>(nlink) * link_nz);
        if (!kA) return 0;
        ipo::SynthLP o;
        ipo::synth_block_angular(nblocks, mb, nb, per_col, band, nlink, link_nz, seed, o);
        synth_out(o, kA, iA, A, b, c, xs, ys, ws, zs);
        return 0;
    } catch (const std::exception& e) {
        set_err(e.what());
        return -1;
    }
}

}  // extern "C"
