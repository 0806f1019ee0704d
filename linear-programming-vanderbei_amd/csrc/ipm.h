// ipm.h -- device-resident interior-point drivers behind solver().
//
//   Method::Hsd    homogeneous self-dual predictor-corrector, src/ipo/hsd.c:27-311
//   Method::Intpt  primal-dual path following,               src/ipo/intpt.c:33-261
//   Method::Hsdls  homogeneous self-dual long step,          src/ipo/hsdls.c:38-296
//
// The host keeps the handful of scalars the reference keeps (phi, psi, mu,
// theta, ...) and prints the reference's per-iteration trace; every O(m+n)
// vector, both SpMVs and the KKT factor/solve live on the GPU.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdio>
#include <memory>

#include "exchange.h"
#include "hip_util.h"
#include "kkt_device.h"
#include "row_ax.h"

namespace ipo {

enum class Method { Hsd = 0, Intpt = 1, Hsdls = 2 };

struct IpmOptions {
    Method method = Method::Hsd;
    int max_iter = 200;          // MAX_ITER, hsd.c:25 / intpt.c:31 (hsdls.c:25: 600)
    FILE* trace = nullptr;       // banner + one line per iteration, reference format
    bool timing = false;         // per-phase HIP-event timing
};

struct IpmResult {
    int status = 5;
    int iters = 0;
    double t_setup_s = 0.0;      // symbolic analysis + uploads (first ldltfac in the reference)
    double t_solve_s = 0.0;      // iteration loop, wall clock
    double final_mu = 0.0, final_pobj = 0.0, final_dobj = 0.0, final_pinf = 0.0, final_dinf = 0.0;
    double phi = 1.0, psi = 1.0;
    KktTimers kkt;
    long refine_passes = 0;
};

// One shard of a block-angular LP (not in the reference).
// The local problem holds this shard's diagonal blocks (rows, columns) and a
// replica of the nforced linking rows, numbered last.  Column quantities
// (x, z) are disjoint between shards, block-row quantities (y, w) too, and
// the linking-row values are replicated bitwise: every shard computes them
// from the same allreduced inputs.  Sums count linking rows on rank 0 only.
// nforced > 0 without an Exchange: one process, linking rows in the tail.
struct ShardSpec {
    int nforced = 0;              // linking rows = the last nforced local rows
    Exchange* xch = nullptr;      // not owned
    int m_global = 0, n_global = 0;
    long nz_global = 0;
};

// Problem uploaded to HBM once; run() iterates from the reference's start
// point and can be called repeatedly (the bench times run()).
// bench.py's HBM-roofline leg: the HBM-bound HSD vector kernels timed alone
// (ipm_device.hip); out[3] ms per launch, bytes[3] algorithmic bytes per launch
void vector_bench(int m, int n, const int* kA, const int* iA, const double* A, int reps, double* out, double* bytes);

class IpmSolver {
  public:
    IpmSolver(int m, int n, const int* kA, const int* iA, const double* A, const double* b, const double* c,
              double f, hipStream_t stream = nullptr, const ShardSpec* shard = nullptr);
    ~IpmSolver();
    int run(const IpmOptions& opt, IpmResult* res);
    // copy x (n), y (m), w (m), z (n) of the last run to the host
    void download(double* x, double* y, double* w, double* z) const;
    KktDevice& kkt() { return *kkt_; }
    double setup_seconds() const { return t_setup_; }

  private:
    int run_hsd(const IpmOptions& opt, IpmResult* res);
    int run_intpt(const IpmOptions& opt, IpmResult* res);
    int run_hsdls(const IpmOptions& opt, IpmResult* res);
    void reduce(const struct RedJobs& j, int nout);
    // sharded solve: linking-row products A_link x summed over the shards
    // into lax_ (no-op unsharded), and the cross-shard reduction of scalars
    void link_ax(const double* x);
    void xsum(double* d, size_t n, RedOp op) { if (xch_) xch_->allreduce(d, n, op, stream_); }
    // rows >= mrow() take A x from lax(): the summed linking rows of a shard,
    // or every row when A x is formed column-blocked (row_ax) beforehand
    const double* lax() const { return xch_ ? lax_.get() : axsliced_ ? ax_.get() : nullptr; }
    int mrow() const { return xch_ ? m_ - nforced_ : axsliced_ ? 0 : m_; }   // rows below are shard-local
    // A x of every row in column blocks whose x-slice fits one XCD's L2
    // (RowAxPlan, row_ax.h; bitwise the residual kernels' own sums), when x is
    // larger than a slice and the solver is not sharded
    void row_ax(const double* x, hipStream_t st);
    int axblocks_ = 1;
    bool axsliced_ = false;   // A x by RowAxPlan (x over one L2 slice, or IPO_HIP_AX_JDS=1)
    DevBuf<double> ax_;
    RowAxPlan axplan_;
    void print_dims(FILE* tr) const;

    int m_, n_;
    double f_;
    hipStream_t stream_;
    bool own_stream_ = false;
    double t_setup_ = 0.0;
    int nforced_ = 0;
    Exchange* xch_ = nullptr;
    int mcnt_ = 0;               // rows this shard counts in sums (linking rows on rank 0 only)
    int mg_ = 0, ng_ = 0;        // global sizes (mu's denominator, the trace)
    int dot_segmin_ = 0;         // RedJobs::segmin of the solver's dots (dev_common.h)
    long nzg_ = 0;
    std::unique_ptr<KktDevice> kkt_;
    DevBuf<double> b_, c_, x_, y_, w_, z_;
    DevBuf<double> rho_, sig_, D_, E_, fx_, fy_, gx_, gy_, dx_, dy_, dz_, dw_;
    DevBuf<double> part_, part2_, scal_, lax_;
    hipStream_t side_ = nullptr;            // mu / residuals beside the factorisation (run_hsd)
    hipEvent_t ev_step_ = nullptr, ev_side_ = nullptr;
    double* hs_ = nullptr;       // pinned scalars
    bool full_trace_ = false;    // IPO_HIP_TRACE_FULL: full-precision scalars per iteration on stderr
};

// Whole-pipeline convenience used by the C ABI: host arrays in, host out.
int ipm_solve_host(int m, int n, int nz, const int* iA, const int* kA, const double* A, const double* b,
                   const double* c, double f, double* x, double* y, double* w, double* z, const IpmOptions& opt,
                   IpmResult* res);

}  // namespace ipo
