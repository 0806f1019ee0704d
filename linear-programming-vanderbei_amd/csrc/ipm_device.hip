// ipm_device.hip -- HSD and path-following iterations on gfx950.
//
// Fused O(m+n) kernels (HBM-bound; coalesced CSR/CSC gathers, one pass per
// phase) + the KKT factor/solve of kkt_device.hip.  Per iteration the host
// reads back only the scalars the reference prints or branches on.
//
// Sharded (block-angular, ipm.h ShardSpec): the same kernels run on the
// shard's local problem; rows >= mrow (the replicated linking rows) take
// their A x from lax (A_link x summed over the shards), rows >= mcnt are
// left out of the shard's partial sums, and every scalar the host reads is
// allreduced before it is read.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <stdexcept>
#include <vector>

#include "dev_common.h"
#include "hip_util.h"
#include "ipm.h"

namespace ipo {

namespace {

constexpr int NT = 256;

__global__ void __launch_bounds__(NT) k_fill(int n, double v, double* __restrict__ a) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i < n) a[i] = v;
}

// ---------------------------------------------------------------- HSD
// rows i < m (hsd.c:182-189, 216, 221, 226):
//   r1 = (A x)_i - b_i phi + w_i ;  ||r1||^2 partial
//   rho = -(1-delta) r1 + w - delta mu / y ;  E = w / y ;  fy = rho ;  gy = -b
// cols j < n (hsd.c:191-198, 215, 220, 225):
//   s1 = -(A'y)_j + c_j phi + z_j ;  ||s1||^2 partial
//   sigma = -(1-delta) s1 + z - delta mu / x ;  D = z / x ;  fx = -sigma ;  gx = -c
__global__ void __launch_bounds__(kResThreads)
k_hsd_residuals(int m, int n, const int* __restrict__ kAt, const int* __restrict__ iAt, const double* __restrict__ At,
                const int* __restrict__ kA, const int* __restrict__ iA, const double* __restrict__ A,
                const double* __restrict__ b, const double* __restrict__ c, const double* __restrict__ x,
                const double* __restrict__ y, const double* __restrict__ w, const double* __restrict__ z, double phi_h,
                double delta, double mu_h, double* __restrict__ E, double* __restrict__ D, double* __restrict__ fy,
                double* __restrict__ fx, double* __restrict__ gy, double* __restrict__ gx, double* __restrict__ part,
                int mrow, int mcnt, const double* __restrict__ lax, const double* __restrict__ phimu) {
    __shared__ double sh[kResThreads / 64];
    // phimu: {phi, mu} computed on the device (the overlapped HSD iteration;
    // E and D are then written by k_hsd_scaling ahead of the factorisation)
    const double phi = phimu ? phimu[0] : phi_h;
    const double mu = phimu ? phimu[1] : mu_h;
    const bool wde = phimu == nullptr;
    double sr = 0.0, ss = 0.0;
    for (int i = blockIdx.x * kResThreads + threadIdx.x; i < m + n; i += kRedBlocks * kResThreads) {
        if (i < m) {
            double ax = 0.0;
            if (i >= mrow) ax = lax[i - mrow];      // linking row of a shard: summed over the shards
            else
                ax = sparse_dot(kAt[i], kAt[i + 1], At, iAt, x);
            const double r1 = ax - b[i] * phi + w[i];
            if (i < mcnt) sr += r1 * r1;
            const double rho = -(1 - delta) * r1 + w[i] - delta * mu / y[i];
            if (wde) E[i] = w[i] / y[i];
            fy[i] = rho;
            gy[i] = -b[i];
        } else {
            const int j = i - m;
            double aty = 0.0;
            aty = sparse_dot(kA[j], kA[j + 1], A, iA, y);
            const double s1 = -aty + c[j] * phi + z[j];
            ss += s1 * s1;
            const double sg = -(1 - delta) * s1 + z[j] - delta * mu / x[j];
            if (wde) D[j] = z[j] / x[j];
            fx[j] = -sg;
            gx[j] = -c[j];
        }
    }
    sr = block_sum_w<kResThreads / 64>(sr, sh);
    ss = block_sum_w<kResThreads / 64>(ss, sh);
    if (threadIdx.x == 0) { part[blockIdx.x] = sr; part[kRedBlocks + blockIdx.x] = ss; }
}

// directions + ratio test (hsd.c:233-237, 249-256)
__global__ void __launch_bounds__(NT)
k_hsd_directions(int m, int n, const double* __restrict__ dphip, double delta, double mu, const double* __restrict__ fx,
                 const double* __restrict__ gx, const double* __restrict__ fy, const double* __restrict__ gy,
                 const double* __restrict__ x, const double* __restrict__ z, const double* __restrict__ y,
                 const double* __restrict__ w, const double* __restrict__ D, const double* __restrict__ E,
                 double* __restrict__ dx, double* __restrict__ dz, double* __restrict__ dy, double* __restrict__ dw,
                 double* __restrict__ part) {
    __shared__ double sh[4];
    const double dphi = *dphip;
    double th = 0.0;
    for (int i = blockIdx.x * NT + threadIdx.x; i < m + n; i += kRedBlocks * NT) {
        if (i < n) {
            const double ddx = fx[i] - gx[i] * dphi;
            const double ddz = delta * mu / x[i] - z[i] - D[i] * ddx;
            dx[i] = ddx; dz[i] = ddz;
            th = fmax(th, -ddx / x[i]);
            th = fmax(th, -ddz / z[i]);
        } else {
            const int j = i - n;
            const double ddy = fy[j] - gy[j] * dphi;
            const double ddw = delta * mu / y[j] - w[j] - E[j] * ddy;
            dy[j] = ddy; dw[j] = ddw;
            th = fmax(th, -ddy / y[j]);
            th = fmax(th, -ddw / w[j]);
        }
    }
    th = block_max(th, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = th;
}

__global__ void __launch_bounds__(NT)
k_step(int m, int n, double theta_h, const double* __restrict__ thetap, double* __restrict__ x,
       const double* __restrict__ dx, double* __restrict__ z, const double* __restrict__ dz, double* __restrict__ y,
       const double* __restrict__ dy, double* __restrict__ w, const double* __restrict__ dw) {
    const double theta = thetap ? *thetap : theta_h;     // device-computed step (hsd) or the host's
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i < n) { x[i] = x[i] + theta * dx[i]; z[i] = z[i] + theta * dz[i]; }
    else if (i < n + m) { const int j = i - n; y[j] = y[j] + theta * dy[j]; w[j] = w[j] + theta * dw[j]; }
}

// E = w / y, D = z / x (hsd.c:188-189; the same divisions as k_hsd_residuals)
__global__ void __launch_bounds__(NT)
k_hsd_scaling(int m, int n, const double* __restrict__ x, const double* __restrict__ y, const double* __restrict__ w,
              const double* __restrict__ z, double* __restrict__ E, double* __restrict__ D) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i < m) E[i] = w[i] / y[i];
    else if (i < m + n) { const int j = i - m; D[j] = z[j] / x[j]; }
}

// mu of hsd.c:168 on the device, the host's expression: sc[0..3] = z'x,
// w'y, c'x, b'y; phi / psi from sc[14..15] (dev != 0) or the arguments;
// out: sc[6] = phi, sc[7] = mu (the residual kernel's phimu)
__global__ void k_hsd_mu(double* sc, double denom, double phi_h, double psi_h, int dev) {
    const double phi = dev ? sc[14] : phi_h, psi = dev ? sc[15] : psi_h;
    sc[6] = phi;
    sc[7] = (sc[0] + sc[1] + phi * psi) / denom;
}

// hsd.c:226-231 on the device (same operations and order as the host code
// it replaces): sc[0..3] = c'fx, b'fy, c'gx, b'gy -> sc[12] = dphi, sc[13] = dpsi
__global__ void k_hsd_dphi(double* sc, double gamma, double delta, double mu, double phi, double psi) {
    const double dphi = (sc[0] - sc[1] + gamma) / (sc[2] - sc[3] - psi / phi);
    const double dpsi = delta * mu / phi - psi - (psi / phi) * dphi;
    sc[12] = dphi;
    sc[13] = dpsi;
}

// hsd.c:249-266: step length from the largest ratio sc[0] and dphi / dpsi;
// sc[11] = theta, sc[14] / sc[15] = the next phi / psi (read by the host at
// the next iteration's synchronisation)
__global__ void k_hsd_theta(double* sc, double phi, double psi) {
    const double dphi = sc[12], dpsi = sc[13];
    double theta = sc[0];
    if (theta < -dphi / phi) theta = -dphi / phi;
    if (theta < -dpsi / psi) theta = -dpsi / psi;
    theta = (0.95 / theta > 1.0) ? 1.0 : 0.95 / theta;
    sc[11] = theta;
    sc[14] = phi + theta * dphi;
    sc[15] = psi + theta * dpsi;
}

__global__ void __launch_bounds__(NT)
k_unscale(int m, int n, double phi, double* __restrict__ x, double* __restrict__ z, double* __restrict__ y,
          double* __restrict__ w) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i < n) { x[i] /= phi; z[i] /= phi; }
    else if (i < n + m) { const int j = i - n; y[j] /= phi; w[j] /= phi; }
}

// ---------------------------------------------------------------- hsdls
// hsdls.c:298-336: largest step keeping x z >= (1-beta) mu along the direction
__device__ __forceinline__ double ls_step(double xj, double zj, double dxj, double dzj, double beta, double delta,
                                          double mu) {
    const double a = dxj * dzj;
    const double b = zj * dxj + xj * dzj + (1 - beta) * (1 - delta) * mu;
    const double c = xj * zj - (1 - beta) * mu;
    const double d = b * b - 4 * a * c;
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

// directions (hsdls.c:209-215) + the linesearch minimum (hsdls.c:221-230),
// returned as a max of -step so the common max finisher applies
__global__ void __launch_bounds__(NT)
k_hsdls_directions(int m, int n, double dphi, double beta, double delta, double mu, const double* __restrict__ fx,
                   const double* __restrict__ gx, const double* __restrict__ fy, const double* __restrict__ gy,
                   const double* __restrict__ x, const double* __restrict__ z, const double* __restrict__ y,
                   const double* __restrict__ w, const double* __restrict__ D, const double* __restrict__ E,
                   double* __restrict__ dx, double* __restrict__ dz, double* __restrict__ dy, double* __restrict__ dw,
                   double* __restrict__ part) {
    __shared__ double sh[4];
    double th = -HUGE_VAL;
    for (int i = blockIdx.x * NT + threadIdx.x; i < m + n; i += kRedBlocks * NT) {
        if (i < n) {
            const double ddx = fx[i] - gx[i] * dphi;
            const double ddz = delta * mu / x[i] - z[i] - D[i] * ddx;
            dx[i] = ddx; dz[i] = ddz;
            th = fmax(th, -ls_step(x[i], z[i], ddx, ddz, beta, delta, mu));
        } else {
            const int j = i - n;
            const double ddy = fy[j] - gy[j] * dphi;
            const double ddw = delta * mu / y[j] - w[j] - E[j] * ddy;
            dy[j] = ddy; dw[j] = ddw;
            th = fmax(th, -ls_step(y[j], w[j], ddy, ddw, beta, delta, mu));
        }
    }
    th = block_max(th, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = th;
}

// ---------------------------------------------------------------- intpt
// rho = b - A x - w, sigma = c - A'y + z and their squared norms (intpt.c:139-149)
__global__ void __launch_bounds__(kResThreads)
k_pf_residuals(int m, int n, const int* __restrict__ kAt, const int* __restrict__ iAt, const double* __restrict__ At,
               const int* __restrict__ kA, const int* __restrict__ iA, const double* __restrict__ A,
               const double* __restrict__ b, const double* __restrict__ c, const double* __restrict__ x,
               const double* __restrict__ y, const double* __restrict__ w, const double* __restrict__ z,
               double* __restrict__ rho, double* __restrict__ sig, double* __restrict__ part, int mrow, int mcnt,
               const double* __restrict__ lax) {
    __shared__ double sh[kResThreads / 64];
    double sr = 0.0, ss = 0.0;
    for (int i = blockIdx.x * kResThreads + threadIdx.x; i < m + n; i += kRedBlocks * kResThreads) {
        if (i < m) {
            double ax = 0.0;
            if (i >= mrow) ax = lax[i - mrow];      // linking row of a shard: summed over the shards
            else
                ax = sparse_dot(kAt[i], kAt[i + 1], At, iAt, x);
            const double r = b[i] - ax - w[i];
            rho[i] = r;
            if (i < mcnt) sr += r * r;
        } else {
            const int j = i - m;
            double aty = 0.0;
            aty = sparse_dot(kA[j], kA[j + 1], A, iA, y);
            const double s = c[j] - aty + z[j];
            sig[j] = s;
            ss += s * s;
        }
    }
    sr = block_sum_w<kResThreads / 64>(sr, sh);
    ss = block_sum_w<kResThreads / 64>(ss, sh);
    if (threadIdx.x == 0) { part[blockIdx.x] = sr; part[kRedBlocks + blockIdx.x] = ss; }
}

// D, E and the right-hand side (intpt.c:194-200)
__global__ void __launch_bounds__(NT)
k_pf_rhs(int m, int n, double mu, const double* __restrict__ x, const double* __restrict__ z,
         const double* __restrict__ y, const double* __restrict__ w, const double* __restrict__ rho,
         const double* __restrict__ sig, double* __restrict__ D, double* __restrict__ E, double* __restrict__ dx,
         double* __restrict__ dy) {
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i < n) { D[i] = z[i] / x[i]; dx[i] = sig[i] - z[i] + mu / x[i]; }
    else if (i < n + m) { const int j = i - n; E[j] = w[j] / y[j]; dy[j] = rho[j] + w[j] - mu / y[j]; }
}

// dz, dw and the ratio test (intpt.c:204-219)
__global__ void __launch_bounds__(NT)
k_pf_directions(int m, int n, double mu, const double* __restrict__ x, const double* __restrict__ z,
                const double* __restrict__ y, const double* __restrict__ w, const double* __restrict__ D,
                const double* __restrict__ E, const double* __restrict__ dx, const double* __restrict__ dy,
                double* __restrict__ dz, double* __restrict__ dw, double* __restrict__ part) {
    __shared__ double sh[4];
    double th = 0.0;
    for (int i = blockIdx.x * NT + threadIdx.x; i < m + n; i += kRedBlocks * NT) {
        if (i < n) {
            const double v = mu / x[i] - z[i] - D[i] * dx[i];
            dz[i] = v;
            th = fmax(th, -dx[i] / x[i]);
            th = fmax(th, -v / z[i]);
        } else {
            const int j = i - n;
            const double v = mu / y[j] - w[j] - E[j] * dy[j];
            dw[j] = v;
            th = fmax(th, -dy[j] / y[j]);
            th = fmax(th, -v / w[j]);
        }
    }
    th = block_max(th, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = th;
}

// host copy of ls_step for the (phi, psi) pair (hsdls.c:229)
double ls_step_host(double xj, double zj, double dxj, double dzj, double beta, double delta, double mu) {
    const double a = dxj * dzj;
    const double b = zj * dxj + xj * dzj + (1 - beta) * (1 - delta) * mu;
    const double c = xj * zj - (1 - beta) * mu;
    const double d = b * b - 4 * a * c;
    if (a == 0.0) return -c / b;
    if (a > 0) return (b < 0 && d >= 0) ? 2 * c / (-b + std::sqrt(d)) : HUGE_VAL;
    if (b < 0) return 2 * c / (-b + std::sqrt(d));
    return (-b - std::sqrt(d)) / (2 * a);
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

const char* kHsdHeader =
    "--------------------------------------------------------------------------\n"
    "         |           Primal          |            Dual           |       |\n"
    "  Iter   |  Obj Value       Infeas   |  Obj Value       Infeas   |  mu   |\n"
    "- - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - \n";
const char* kIntptHeader =
    "------------------------------------------------------------------\n"
    "         |           Primal          |            Dual           |\n"
    "  Iter   |  Obj Value       Infeas   |  Obj Value       Infeas   |\n"
    "- - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - - \n";

}  // namespace

IpmSolver::IpmSolver(int m, int n, const int* kA, const int* iA, const double* A, const double* b, const double* c,
                     double f, hipStream_t stream, const ShardSpec* shard)
    : m_(m), n_(n), f_(f), stream_(stream) {
    const double t0 = now_s();
    mg_ = m;
    ng_ = n;
    nzg_ = kA[n];
    mcnt_ = m;
    if (shard) {
        if (shard->nforced < 0 || shard->nforced > m) throw std::invalid_argument("shard: nforced out of range");
        nforced_ = shard->nforced;
        xch_ = shard->xch;
        if (xch_) {
            mg_ = shard->m_global;
            ng_ = shard->n_global;
            nzg_ = shard->nz_global;
            if (xch_->rank() != 0) mcnt_ = m - nforced_;   // linking rows are counted on rank 0
        }
    }
    // LPs with a vector of kOrderedMaxLen entries (none in netlib) take every
    // dot of theirs in the segmented order; IPO_HIP_DOT_SEGMIN overrides
    dot_segmin_ = std::max(mg_, ng_) >= kOrderedMaxLen ? kSegDotLen : 0;
    if (const char* e = std::getenv("IPO_HIP_DOT_SEGMIN")) dot_segmin_ = std::max(0, std::atoi(e));
    if (!stream_) {
        IPO_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        own_stream_ = true;
    }
    kkt_ = std::make_unique<KktDevice>(m, n, kA, iA, A, stream_, nforced_);
    kkt_->set_exchange(xch_);
    if (dot_segmin_ > 0 && !xch_) {
        // trailing rows of at least kLongRow entries (the linking rows of a
        // block-angular LP): their serial row products held up the whole
        // refinement residual (1.5 ms a launch on configs[4])
        constexpr int kLongRow = 256;
        std::vector<int> cnt(m > 0 ? m : 1, 0);
        for (int k = 0; k < kA[n]; k++) cnt[iA[k]]++;
        int r0 = m;
        while (r0 > 0 && cnt[r0 - 1] >= kLongRow) r0--;
        if (r0 < m) kkt_->set_long_rows(r0);
    }
    const size_t mm = m > 0 ? m : 1, nn = n > 0 ? n : 1;
    b_.upload(b, m, stream_);
    c_.upload(c, n, stream_);
    for (DevBuf<double>* v : {&x_, &z_, &sig_, &D_, &fx_, &gx_, &dx_, &dz_}) v->alloc(nn);
    for (DevBuf<double>* v : {&y_, &w_, &rho_, &E_, &fy_, &gy_, &dy_, &dw_}) v->alloc(mm);
    if (m == 0) b_.alloc(1);
    if (n == 0) c_.alloc(1);
    part_.alloc(8 * kRedBlocks);
    part2_.alloc(8 * kRedBlocks);
    scal_.alloc(16);
    IPO_HIP_CHECK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    IPO_HIP_CHECK(hipEventCreateWithFlags(&ev_step_, hipEventDisableTiming));
    IPO_HIP_CHECK(hipEventCreateWithFlags(&ev_side_, hipEventDisableTiming));
    lax_.alloc(nforced_ > 0 ? nforced_ : 1);
    axblocks_ = rows_ax_blocks(n_);
    axsliced_ = rows_ax_sliced(n_) && !xch_;
    if (axsliced_) {
        ax_.alloc(m_ > 0 ? m_ : 1);
        axplan_.build(m, n, kA, iA, A, axblocks_, stream_);
    }
    IPO_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&hs_), 16 * sizeof(double), hipHostMallocDefault));
    IPO_HIP_CHECK(hipStreamSynchronize(stream_));
    t_setup_ = now_s() - t0;
}

IpmSolver::~IpmSolver() {
    if (side_) (void)hipStreamSynchronize(side_);
    if (hs_) (void)hipHostFree(hs_);
    if (ev_step_) (void)hipEventDestroy(ev_step_);
    if (ev_side_) (void)hipEventDestroy(ev_side_);
    if (side_) (void)hipStreamDestroy(side_);
    kkt_.reset();
    if (own_stream_) (void)hipStreamDestroy(stream_);
}

void IpmSolver::reduce(const RedJobs& j, int nout) {
    launch_reduce(j, part_.get(), scal_.get(), stream_);
    xsum(scal_.get(), nout, RedOp::Sum);
    IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), nout * sizeof(double), hipMemcpyDeviceToHost, stream_));
    IPO_HIP_CHECK(hipStreamSynchronize(stream_));
}

void IpmSolver::row_ax(const double* x, hipStream_t st) {
    if (!axsliced_) return;
    axplan_.launch(x, ax_.get(), st);
}

void IpmSolver::link_ax(const double* x) {
    row_ax(x, stream_);
    if (!xch_ || nforced_ == 0) return;
    launch_link_ax(m_ - nforced_, m_, kkt_->kAt(), kkt_->iAt(), kkt_->At(), x, lax_.get(), stream_);
    xsum(lax_.get(), nforced_, RedOp::Sum);
}

void IpmSolver::print_dims(FILE* tr) const { std::fprintf(tr, "m = %d,n = %d,nz = %ld\n", mg_, ng_, nzg_); }

void IpmSolver::download(double* x, double* y, double* w, double* z) const {
    if (x) x_.download(x, n_, stream_);
    if (y) y_.download(y, m_, stream_);
    if (w) w_.download(w, m_, stream_);
    if (z) z_.download(z, n_, stream_);
    IPO_HIP_CHECK(hipStreamSynchronize(stream_));
}

int IpmSolver::run(const IpmOptions& opt, IpmResult* res) {
    IpmResult local;
    if (!res) res = &local;
    *res = IpmResult();
    res->t_setup_s = t_setup_;
    kkt_->enable_timing(opt.timing);
    kkt_->reset_timers();         // the counters and phase times of this solve only
    kkt_->set_epsdiag(1.0e-14);   // ldlt.c:31: every solve starts from the reference's eps_diag
    const double t0 = now_s();
    const int st = opt.method == Method::Intpt   ? run_intpt(opt, res)
                   : opt.method == Method::Hsdls ? run_hsdls(opt, res)
                                                 : run_hsd(opt, res);
    res->t_solve_s = now_s() - t0;
    res->status = st;
    res->kkt = kkt_->timers();
    return st;
}

int IpmSolver::run_hsd(const IpmOptions& opt, IpmResult* res) {
    full_trace_ = std::getenv("IPO_HIP_TRACE_FULL") != nullptr;
    // mu, residuals and right-hand sides on a side stream beside the
    // factorisation (one GPU, no exchange); IPO_HIP_OVERLAP=0 turns it off
    bool overlap = xch_ == nullptr;
    if (const char* e = std::getenv("IPO_HIP_OVERLAP")) overlap = overlap && std::atoi(e) != 0;
    const int m = m_, n = n_;
    hipStream_t s = stream_;
    const int gv = ceil_div(m + n, NT);
    FILE* tr = opt.trace;
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(n, NT)), dim3(NT), 0, s, n, 1.0, x_.get());
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(n, NT)), dim3(NT), 0, s, n, 1.0, z_.get());
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(m, NT)), dim3(NT), 0, s, m, 1.0, w_.get());
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(m, NT)), dim3(NT), 0, s, m, 1.0, y_.get());
    double phi = 1.0, psi = 1.0;
    if (tr) {
        print_dims(tr);
        std::fputs(kHsdHeader, tr);
        std::fflush(tr);
    }
    KktDevice& K = *kkt_;
    int status = 5, iter;
    // one host synchronisation per iteration outside the KKT solver: the
    // dots of mu (with phi / psi of the device step, hsd.c:264-265); the
    // residual norms are only printed (read back without a wait), dphi /
    // dpsi / theta / phi / psi are computed on the device (k_hsd_dphi,
    // k_hsd_theta: the host's operations in the host's order)
    for (iter = 0; iter < opt.max_iter; iter++) {
        RedJobs j{};
        j.nj = 4;
        j.segmin = dot_segmin_;
        j.a[0] = z_.get(); j.b[0] = x_.get(); j.len[0] = n; j.op[0] = 0;
        j.a[1] = w_.get(); j.b[1] = y_.get(); j.len[1] = mcnt_; j.op[1] = 0;
        j.a[2] = c_.get(); j.b[2] = x_.get(); j.len[2] = n; j.op[2] = 0;
        j.a[3] = b_.get(); j.b[3] = y_.get(); j.len[3] = mcnt_; j.op[3] = 0;
        const double delta = (iter % 2 == 0) ? 0.0 : 1.0;
        KktDevice::HostState spec{};
        std::exception_ptr spec_err;
        if (overlap) {
            // side stream: the dots of mu, mu, the residuals and their norms
            // (device phi / mu) beside the factorisation on the main stream
            IPO_HIP_CHECK(hipEventRecord(ev_step_, s));
            IPO_HIP_CHECK(hipStreamWaitEvent(side_, ev_step_, 0));
            launch_reduce(j, part2_.get(), scal_.get(), side_);
            hipLaunchKernelGGL(k_hsd_mu, dim3(1), dim3(1), 0, side_, scal_.get(), static_cast<double>(ng_ + mg_ + 1), phi,
                               psi, iter > 0 ? 1 : 0);
            row_ax(x_.get(), side_);
            hipLaunchKernelGGL(k_hsd_residuals, dim3(kRedBlocks), dim3(kResThreads), 0, side_, m, n, K.kAt(), K.iAt(),
                               K.At(), K.kA(), K.iA(), K.A(), b_.get(), c_.get(), x_.get(), y_.get(), w_.get(), z_.get(),
                               phi, delta, 0.0, E_.get(), D_.get(), fy_.get(), fx_.get(), gy_.get(), gx_.get(),
                               part2_.get(), mrow(), mcnt_, lax(), static_cast<const double*>(scal_.get() + 6));
            hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, side_, part2_.get(), 2, 0u, scal_.get() + 8);
            IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), 16 * sizeof(double), hipMemcpyDeviceToHost, side_));
            IPO_HIP_CHECK(hipEventRecord(ev_side_, side_));
            hipLaunchKernelGGL(k_hsd_scaling, dim3(gv), dim3(NT), 0, s, m, n, x_.get(), y_.get(), w_.get(), z_.get(),
                               E_.get(), D_.get());
            // speculative: the host learns mu (and so whether hsd.c:155 stops
            // here, where the reference does not factor) only after it; its
            // host-side effects are undone and an error it raised is held
            // back unless the iteration goes on to use the factor
            spec = K.host_state();
            try {
                K.factor(E_.get(), D_.get());
            } catch (...) {
                spec_err = std::current_exception();
            }
            IPO_HIP_CHECK(hipEventSynchronize(ev_side_));
            if (iter > 0) { phi = hs_[14]; psi = hs_[15]; }
        } else {
            launch_reduce(j, part_.get(), scal_.get(), s);
            xsum(scal_.get(), 4, RedOp::Sum);
            IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), 4 * sizeof(double), hipMemcpyDeviceToHost, s));
            if (iter > 0)
                IPO_HIP_CHECK(hipMemcpyAsync(hs_ + 14, scal_.get() + 14, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
            IPO_HIP_CHECK(hipStreamSynchronize(s));
            if (iter > 0) { phi = hs_[14]; psi = hs_[15]; }
        }
        const double mu = (hs_[0] + hs_[1] + phi * psi) / (ng_ + mg_ + 1);
        // the device's mu / phi must be the host's bit for bit (NaNs included:
        // a diverging solve then takes the sequential path's status route)
        if (overlap && (std::memcmp(&mu, &hs_[7], sizeof mu) != 0 || std::memcmp(&phi, &hs_[6], sizeof phi) != 0))
            throw std::runtime_error("hsd: device mu / phi differ from the host's");
        const double pobj = hs_[2], dobj = hs_[3];
        if (mu < 1.0e-12) {
            if (overlap) K.restore_host_state(spec);     // the speculative factorisation is not used
            if (phi > psi) status = 0;
            else if (dobj < 0.0) status = 2;
            else if (pobj > 0.0) status = 4;
            else { if (tr) std::fprintf(tr, "Trouble in river city \n"); status = 4; }
            break;
        }
        if (!overlap) {
            link_ax(x_.get());
            hipLaunchKernelGGL(k_hsd_residuals, dim3(kRedBlocks), dim3(kResThreads), 0, s, m, n, K.kAt(), K.iAt(), K.At(),
                               K.kA(), K.iA(), K.A(), b_.get(), c_.get(), x_.get(), y_.get(), w_.get(), z_.get(), phi,
                               delta, mu, E_.get(), D_.get(), fy_.get(), fx_.get(), gy_.get(), gx_.get(), part_.get(),
                               mrow(), mcnt_, lax(), static_cast<const double*>(nullptr));
            hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, part_.get(), 2, 0u, scal_.get());
            xsum(scal_.get(), 2, RedOp::Sum);
            IPO_HIP_CHECK(hipMemcpyAsync(hs_ + 8, scal_.get(), 2 * sizeof(double), hipMemcpyDeviceToHost, s));
            K.factor(E_.get(), D_.get());    // synchronises the stream: hs_[8..9] have landed
        } else {
            if (spec_err) std::rethrow_exception(spec_err);
            IPO_HIP_CHECK(hipStreamWaitEvent(s, ev_side_, 0));   // fy fx gy gx before the solves
        }
        const double gamma = -(1 - delta) * (dobj - pobj + psi) + psi - delta * mu / phi;

        const double normr = std::sqrt(hs_[8]) / phi;
        const double norms = std::sqrt(hs_[9]) / phi;
        if (tr) {
            std::fprintf(tr, "%8d   %14.7e  %8.1e    %14.7e  %8.1e  %8.1e \n", iter, pobj / phi + f_, normr,
                         dobj / phi + f_, norms, mu);
            std::fflush(tr);
        }
        res->final_mu = mu; res->final_pobj = pobj / phi + f_; res->final_dobj = dobj / phi + f_;
        res->final_pinf = normr; res->final_dinf = norms;
        if (full_trace_) {
            std::fprintf(stderr, "FT %d %.17g %.17g %.17g %.17g %.17g %.17g\n", iter, pobj, dobj, mu, phi, psi, normr);
            std::fprintf(stderr, "FT   ndep=%d eps=%.1e\n", K.ndep(), K.epsdiag());
        }
        // the two forwardbackward calls of hsd.c:218-224 / hsdls.c:194-203,
        // independent systems with one factor: sweeps batched
        K.solve2(E_.get(), D_.get(), fy_.get(), fx_.get(), gy_.get(), gx_.get());
        res->refine_passes += K.last_passes();

        RedJobs q{};
        q.nj = 4;
        q.segmin = dot_segmin_;
        q.a[0] = c_.get(); q.b[0] = fx_.get(); q.len[0] = n; q.op[0] = 0;
        q.a[1] = b_.get(); q.b[1] = fy_.get(); q.len[1] = mcnt_; q.op[1] = 0;
        q.a[2] = c_.get(); q.b[2] = gx_.get(); q.len[2] = n; q.op[2] = 0;
        q.a[3] = b_.get(); q.b[3] = gy_.get(); q.len[3] = mcnt_; q.op[3] = 0;
        launch_reduce(q, part_.get(), scal_.get(), s);
        xsum(scal_.get(), 4, RedOp::Sum);
        hipLaunchKernelGGL(k_hsd_dphi, dim3(1), dim3(1), 0, s, scal_.get(), gamma, delta, mu, phi, psi);
        hipLaunchKernelGGL(k_hsd_directions, dim3(kRedBlocks), dim3(NT), 0, s, m, n, scal_.get() + 12, delta, mu,
                           fx_.get(), gx_.get(), fy_.get(), gy_.get(), x_.get(), z_.get(), y_.get(), w_.get(), D_.get(),
                           E_.get(), dx_.get(), dz_.get(), dy_.get(), dw_.get(), part_.get());
        hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, part_.get(), 1, 1u, scal_.get());
        xsum(scal_.get(), 1, RedOp::Max);
        hipLaunchKernelGGL(k_hsd_theta, dim3(1), dim3(1), 0, s, scal_.get(), phi, psi);
        hipLaunchKernelGGL(k_step, dim3(gv), dim3(NT), 0, s, m, n, 0.0, scal_.get() + 11, x_.get(), dx_.get(),
                           z_.get(), dz_.get(), y_.get(), dy_.get(), w_.get(), dw_.get());
    }
    hipLaunchKernelGGL(k_unscale, dim3(gv), dim3(NT), 0, s, m, n, phi, x_.get(), z_.get(), y_.get(), w_.get());
    IPO_HIP_CHECK(hipGetLastError());
    IPO_HIP_CHECK(hipStreamSynchronize(s));
    res->iters = iter;
    res->phi = phi;
    res->psi = psi;
    return status;
}

// hsdls.c:38-296 -- same residuals and solves as HSD with a fixed centring
// delta = 2 (1 - beta), beta = 0.8, and a quadratic linesearch for theta
int IpmSolver::run_hsdls(const IpmOptions& opt, IpmResult* res) {
    const int m = m_, n = n_;
    hipStream_t s = stream_;
    const int gv = ceil_div(m + n, NT);
    FILE* tr = opt.trace;
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(n, NT)), dim3(NT), 0, s, n, 1.0, x_.get());
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(n, NT)), dim3(NT), 0, s, n, 1.0, z_.get());
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(m, NT)), dim3(NT), 0, s, m, 1.0, w_.get());
    hipLaunchKernelGGL(k_fill, dim3(ceil_div(m, NT)), dim3(NT), 0, s, m, 1.0, y_.get());
    double phi = 1.0, psi = 1.0;
    if (tr) {
        print_dims(tr);
        std::fputs(kHsdHeader, tr);
        std::fflush(tr);
    }
    const double beta = 0.80, delta = 2 * (1 - beta);
    KktDevice& K = *kkt_;
    int status = 5, iter;
    for (iter = 0; iter < opt.max_iter; iter++) {
        RedJobs j{};
        j.nj = 4;
        j.segmin = dot_segmin_;
        j.a[0] = z_.get(); j.b[0] = x_.get(); j.len[0] = n; j.op[0] = 0;
        j.a[1] = w_.get(); j.b[1] = y_.get(); j.len[1] = mcnt_; j.op[1] = 0;
        j.a[2] = c_.get(); j.b[2] = x_.get(); j.len[2] = n; j.op[2] = 0;
        j.a[3] = b_.get(); j.b[3] = y_.get(); j.len[3] = mcnt_; j.op[3] = 0;
        reduce(j, 4);
        const double mu = (hs_[0] + hs_[1] + phi * psi) / (ng_ + mg_ + 1);
        const double pobj = hs_[2], dobj = hs_[3];
        if (mu < 1.0e-12) {                                   // hsdls.c:131-153
            if (phi > 1.0e-12) status = 0;
            else if (dobj < 0.0) status = 2;
            else if (pobj > 0.0) status = 4;
            else status = 7;
            break;
        }
        link_ax(x_.get());
        hipLaunchKernelGGL(k_hsd_residuals, dim3(kRedBlocks), dim3(kResThreads), 0, s, m, n, K.kAt(), K.iAt(), K.At(), K.kA(),
                           K.iA(), K.A(), b_.get(), c_.get(), x_.get(), y_.get(), w_.get(), z_.get(), phi, delta, mu,
                           E_.get(), D_.get(), fy_.get(), fx_.get(), gy_.get(), gx_.get(), part_.get(), mrow(), mcnt_,
                           lax(), static_cast<const double*>(nullptr));
        hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, part_.get(), 2, 0u, scal_.get());
        xsum(scal_.get(), 2, RedOp::Sum);
        IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), 2 * sizeof(double), hipMemcpyDeviceToHost, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        const double normr = std::sqrt(hs_[0]) / phi;
        const double norms = std::sqrt(hs_[1]) / phi;
        const double gamma = -(1 - delta) * (dobj - pobj + psi) + psi - delta * mu / phi;
        if (tr) {
            std::fprintf(tr, "%8d   %14.7e  %8.1e    %14.7e  %8.1e  %8.1e \n", iter, pobj / phi + f_, normr,
                         dobj / phi + f_, norms, mu);
            std::fflush(tr);
        }
        res->final_mu = mu; res->final_pobj = pobj / phi + f_; res->final_dobj = dobj / phi + f_;
        res->final_pinf = normr; res->final_dinf = norms;

        K.factor(E_.get(), D_.get());
        // the two forwardbackward calls of hsd.c:218-224 / hsdls.c:194-203,
        // independent systems with one factor: sweeps batched
        K.solve2(E_.get(), D_.get(), fy_.get(), fx_.get(), gy_.get(), gx_.get());
        res->refine_passes += K.last_passes();

        RedJobs q{};
        q.nj = 4;
        q.segmin = dot_segmin_;
        q.a[0] = c_.get(); q.b[0] = fx_.get(); q.len[0] = n; q.op[0] = 0;
        q.a[1] = b_.get(); q.b[1] = fy_.get(); q.len[1] = mcnt_; q.op[1] = 0;
        q.a[2] = c_.get(); q.b[2] = gx_.get(); q.len[2] = n; q.op[2] = 0;
        q.a[3] = b_.get(); q.b[3] = gy_.get(); q.len[3] = mcnt_; q.op[3] = 0;
        reduce(q, 4);
        const double dphi = (hs_[0] - hs_[1] + gamma) / (hs_[2] - hs_[3] - psi / phi);
        const double dpsi = delta * mu / phi - psi - (psi / phi) * dphi;

        hipLaunchKernelGGL(k_hsdls_directions, dim3(kRedBlocks), dim3(NT), 0, s, m, n, dphi, beta, delta, mu, fx_.get(),
                           gx_.get(), fy_.get(), gy_.get(), x_.get(), z_.get(), y_.get(), w_.get(), D_.get(), E_.get(),
                           dx_.get(), dz_.get(), dy_.get(), dw_.get(), part_.get());
        hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, part_.get(), 1, 1u, scal_.get());
        xsum(scal_.get(), 1, RedOp::Max);
        IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), sizeof(double), hipMemcpyDeviceToHost, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        double theta = 1.0;
        const double tv = -hs_[0];                            // min over the vector entries
        theta = theta < tv ? theta : tv;
        const double tp = ls_step_host(phi, psi, dphi, dpsi, beta, delta, mu);
        theta = theta < tp ? theta : tp;
        if (theta < 1.0) theta *= 0.9999;

        hipLaunchKernelGGL(k_step, dim3(gv), dim3(NT), 0, s, m, n, theta, static_cast<const double*>(nullptr), x_.get(), dx_.get(), z_.get(), dz_.get(),
                           y_.get(), dy_.get(), w_.get(), dw_.get());
        phi = phi + theta * dphi;
        psi = psi + theta * dpsi;
    }
    hipLaunchKernelGGL(k_unscale, dim3(gv), dim3(NT), 0, s, m, n, phi, x_.get(), z_.get(), y_.get(), w_.get());
    IPO_HIP_CHECK(hipGetLastError());
    IPO_HIP_CHECK(hipStreamSynchronize(s));
    res->iters = iter;
    res->phi = phi;
    res->psi = psi;
    return status;
}

int IpmSolver::run_intpt(const IpmOptions& opt, IpmResult* res) {
    const int m = m_, n = n_;
    hipStream_t s = stream_;
    const int gv = ceil_div(m + n, NT);
    FILE* tr = opt.trace;
    for (DevBuf<double>* v : {&x_, &z_}) hipLaunchKernelGGL(k_fill, dim3(ceil_div(n, NT)), dim3(NT), 0, s, n, 1000.0, v->get());
    for (DevBuf<double>* v : {&y_, &w_}) hipLaunchKernelGGL(k_fill, dim3(ceil_div(m, NT)), dim3(NT), 0, s, m, 1000.0, v->get());
    const double delta = 0.02, r = 0.9;
    double normr0 = HUGE_VAL, norms0 = HUGE_VAL;
    if (tr) {
        print_dims(tr);
        std::fputs(kIntptHeader, tr);
        std::fflush(tr);
    }
    KktDevice& K = *kkt_;
    int status = 5, iter;
    for (iter = 0; iter < opt.max_iter; iter++) {
        link_ax(x_.get());
        hipLaunchKernelGGL(k_pf_residuals, dim3(kRedBlocks), dim3(kResThreads), 0, s, m, n, K.kAt(), K.iAt(), K.At(), K.kA(),
                           K.iA(), K.A(), b_.get(), c_.get(), x_.get(), y_.get(), w_.get(), z_.get(), rho_.get(),
                           sig_.get(), part_.get(), mrow(), mcnt_, lax());
        hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, part_.get(), 2, 0u, scal_.get() + 8);
        RedJobs j{};
        j.nj = 4;
        j.segmin = dot_segmin_;
        j.a[0] = z_.get(); j.b[0] = x_.get(); j.len[0] = n; j.op[0] = 0;
        j.a[1] = y_.get(); j.b[1] = w_.get(); j.len[1] = mcnt_; j.op[1] = 0;
        j.a[2] = c_.get(); j.b[2] = x_.get(); j.len[2] = n; j.op[2] = 0;
        j.a[3] = b_.get(); j.b[3] = y_.get(); j.len[3] = mcnt_; j.op[3] = 0;
        launch_reduce(j, part_.get(), scal_.get(), s);
        xsum(scal_.get(), 4, RedOp::Sum);
        xsum(scal_.get() + 8, 2, RedOp::Sum);
        IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), 10 * sizeof(double), hipMemcpyDeviceToHost, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        // intpt.c:47 keeps the printed quantities in single precision
        const float normr = static_cast<float>(std::sqrt(hs_[8]));
        const float norms = static_cast<float>(std::sqrt(hs_[9]));
        const double gamma = hs_[0] + hs_[1];
        const float pobj = static_cast<float>(hs_[2] + f_);
        const float dobj = static_cast<float>(hs_[3] + f_);
        if (tr) {
            std::fprintf(tr, "%8d   %14.7e  %8.1e    %14.7e  %8.1e \n", iter, pobj, normr, dobj, norms);
            std::fflush(tr);
        }
        res->final_mu = gamma; res->final_pobj = pobj; res->final_dobj = dobj;
        res->final_pinf = normr; res->final_dinf = norms;
        if (normr < 1.0e-6 && norms < 1.0e-6 && gamma < 1.0e-6) { status = 0; break; }
        if (normr > 10 * normr0) { status = 2; break; }
        if (norms > 10 * norms0) { status = 4; break; }
        const double mu = delta * gamma / (ng_ + mg_);
        hipLaunchKernelGGL(k_pf_rhs, dim3(gv), dim3(NT), 0, s, m, n, mu, x_.get(), z_.get(), y_.get(), w_.get(),
                           rho_.get(), sig_.get(), D_.get(), E_.get(), dx_.get(), dy_.get());
        K.factor(E_.get(), D_.get());
        K.solve(E_.get(), D_.get(), dy_.get(), dx_.get());
        res->refine_passes += K.last_passes();
        hipLaunchKernelGGL(k_pf_directions, dim3(kRedBlocks), dim3(NT), 0, s, m, n, mu, x_.get(), z_.get(), y_.get(),
                           w_.get(), D_.get(), E_.get(), dx_.get(), dy_.get(), dz_.get(), dw_.get(), part_.get());
        hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, s, part_.get(), 1, 1u, scal_.get());
        xsum(scal_.get(), 1, RedOp::Max);
        IPO_HIP_CHECK(hipMemcpyAsync(hs_, scal_.get(), sizeof(double), hipMemcpyDeviceToHost, s));
        IPO_HIP_CHECK(hipStreamSynchronize(s));
        double theta = hs_[0];
        theta = (r / theta > 1.0) ? 1.0 : r / theta;
        hipLaunchKernelGGL(k_step, dim3(gv), dim3(NT), 0, s, m, n, theta, static_cast<const double*>(nullptr), x_.get(), dx_.get(), z_.get(), dz_.get(),
                           y_.get(), dy_.get(), w_.get(), dw_.get());
        normr0 = normr;
        norms0 = norms;
    }
    IPO_HIP_CHECK(hipGetLastError());
    IPO_HIP_CHECK(hipStreamSynchronize(s));
    res->iters = iter;
    return status;
}

// The HBM-bound per-iteration kernels of the HSD loop timed on their own
// (bench.py's hbm_roofline leg, BASELINE configs[3] uniform): A x / A' y
// with the residual and right-hand-side vectors (k_hsd_residuals), the
// directions + ratio test (k_hsd_directions) and the step (k_step), each
// with the launch geometry of run_hsd, on device-resident inputs, `reps`
// launches timed with HIP events on one stream.  out[3] = average ms per
// launch; bytes[3] = algorithmic HBM bytes per launch (every array element
// read or written once).
void vector_bench(int m, int n, const int* kA, const int* iA, const double* A, int reps, double* out, double* bytes) {
    const long nz = kA[n];
    // CSR of A (the reference's atnum, hsd.c:111)
    std::vector<int> kAt(m + 1, 0), iAt(nz);
    std::vector<double> At(nz);
    for (long k = 0; k < nz; k++) kAt[iA[k] + 1]++;
    for (int i = 0; i < m; i++) kAt[i + 1] += kAt[i];
    {
        std::vector<int> pos(kAt.begin(), kAt.end() - 1);
        for (int j = 0; j < n; j++)
            for (int k = kA[j]; k < kA[j + 1]; k++) { iAt[pos[iA[k]]] = j; At[pos[iA[k]]++] = A[k]; }
    }
    hipStream_t s;
    IPO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    DevBuf<int> dkA, diA, dkAt, diAt;
    DevBuf<double> dA, dAt, vec;
    dkA.upload(kA, n + 1, s);
    diA.upload(iA, nz, s);
    dA.upload(A, nz, s);
    dkAt.upload(kAt, s);
    diAt.upload(iAt, s);
    dAt.upload(At, s);
    const size_t N = static_cast<size_t>(m) + n;
    vec.alloc(24 * N + 2 * kRedBlocks);
    {
        std::vector<double> v(24 * N, 1.0);
        for (size_t i = 0; i < v.size(); i++) v[i] = 0.5 + (i % 997) * 1e-3;
        vec.upload(v, s);
    }
    double* V = vec.get();
    auto col = [&](int q) { return V + q * N; };      // n-vectors at col(q), m-vectors at col(q) + n
    double* part = V + 24 * N;
    DevBuf<double> dphi03;
    dphi03.upload(std::vector<double>{0.3}, s);
    hipEvent_t e0, e1;
    IPO_HIP_CHECK(hipEventCreate(&e0));
    IPO_HIP_CHECK(hipEventCreate(&e1));
    const int gv = static_cast<int>((N + NT - 1) / NT);
    // the residuals as run_hsd forms them: A x column-blocked first when x
    // exceeds one L2 slice (IpmSolver::row_ax), timed together
    const int axb = rows_ax_blocks(n);
    const bool sliced = rows_ax_sliced(n);
    DevBuf<double> axv;
    RowAxPlan axplan;
    if (sliced) { axv.alloc(m > 0 ? m : 1); axplan.build(m, n, kA, iA, A, axb, s); }
    for (int kq = 0; kq < 3; kq++) {
        for (int r = -2; r < reps; r++) {                 // two untimed launches first
            if (r == 0) IPO_HIP_CHECK(hipEventRecord(e0, s));
            if (kq == 0) {
                if (sliced) axplan.launch(col(2), axv.get(), s);
                hipLaunchKernelGGL(k_hsd_residuals, dim3(kRedBlocks), dim3(kResThreads), 0, s, m, n, dkAt.get(), diAt.get(),
                                   dAt.get(), dkA.get(), diA.get(), dA.get(), col(0) + n, col(1), col(2), col(3) + n,
                                   col(4) + n, col(5), 1.0, 0.5, 0.1, col(6) + n, col(7), col(8) + n, col(9),
                                   col(10) + n, col(11), part, sliced ? 0 : m, m,
                                   sliced ? static_cast<const double*>(axv.get()) : static_cast<const double*>(nullptr),
                                   static_cast<const double*>(nullptr));
            }
            else if (kq == 1)
                hipLaunchKernelGGL(k_hsd_directions, dim3(kRedBlocks), dim3(NT), 0, s, m, n, dphi03.get(), 0.5, 0.1, col(9),
                                   col(11), col(8) + n, col(10) + n, col(2), col(5), col(3) + n, col(4) + n, col(7),
                                   col(6) + n, col(12), col(13), col(14) + n, col(15) + n, part);
            else
                hipLaunchKernelGGL(k_step, dim3(gv), dim3(NT), 0, s, m, n, 1e-9, static_cast<const double*>(nullptr), col(16), col(12), col(17), col(13),
                                   col(18) + n, col(14) + n, col(19) + n, col(15) + n);
        }
        IPO_HIP_CHECK(hipEventRecord(e1, s));
        IPO_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0;
        IPO_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        out[kq] = ms / reps;
    }
    IPO_HIP_CHECK(hipGetLastError());
    // algorithmic bytes (N = m + n): residuals -- CSR + CSC of A (12 B per
    // entry each, 4 B per pointer), b w y / c z x read once (x, y also the
    // gathered operands), E fy gy / D fx gx written: 24 nz + 4 N + 48 N;
    // directions -- 5 vectors read per row / column, 2 written: 56 N;
    // step -- 4 read, 2 written: 48 N
    bytes[0] = 24.0 * nz + 52.0 * N;
    bytes[1] = 56.0 * N;
    bytes[2] = 48.0 * N;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    IPO_HIP_CHECK(hipStreamSynchronize(s));
    (void)hipStreamDestroy(s);
}

int ipm_solve_host(int m, int n, int nz, const int* iA, const int* kA, const double* A, const double* b,
                   const double* c, double f, double* x, double* y, double* w, double* z, const IpmOptions& opt,
                   IpmResult* res) {
    (void)nz;
    IpmSolver S(m, n, kA, iA, A, b, c, f);
    const int st = S.run(opt, res);
    S.download(x, y, w, z);
    return st;
}

}  // namespace ipo
