// dev_common.h -- device helpers: deterministic block reductions (fixed
// grid, fixed tree) for dots and max-norms, shared by the KKT and IPM code.
#pragma once
#include <hip/hip_runtime.h>

#include "row_ax.h"

namespace ipo {

constexpr int kRedBlocks = 256;    // fixed partial count -> reproducible sums
constexpr int kRedThreads = 256;

// the reference's MAX(x,y) = (x > y ? x : y) (macros.h); NaN in x loses
__device__ __forceinline__ double ref_max(double x, double y) { return x > y ? x : y; }
__device__ __forceinline__ double ref_abs(double x) { return x > 0 ? x : -x; }

// Lane l reads lane l + N of its 16-lane row (DPP row_shl:N, a VALU
// modifier instead of an LDS-crossbar ds_bpermute); lanes whose source
// leaves the row keep their own value.
template <int N>
__device__ __forceinline__ double dpp_row_down(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = (int)b, hi = (int)(b >> 32);
    const int lo2 = __builtin_amdgcn_update_dpp(lo, lo, 0x100 + N, 0xf, 0xf, false);
    const int hi2 = __builtin_amdgcn_update_dpp(hi, hi, 0x100 + N, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi2 << 32) | (unsigned int)lo2);
}

// Tree v[l] (+)= v[l + o], o = 32, 16, 8, 4, 2, 1; result valid in lane 0.
// The two cross-row steps go through ds_bpermute, the four in-row steps
// through DPP; lane 0 sees exactly the adds of the all-shuffle tree.
__device__ __forceinline__ double wave_sum(double v) {
    v += __shfl_down(v, 32, 64);
    v += __shfl_down(v, 16, 64);
    v += dpp_row_down<8>(v);
    v += dpp_row_down<4>(v);
    v += dpp_row_down<2>(v);
    v += dpp_row_down<1>(v);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, __shfl_down(v, 32, 64));
    v = fmax(v, __shfl_down(v, 16, 64));
    v = fmax(v, dpp_row_down<8>(v));
    v = fmax(v, dpp_row_down<4>(v));
    v = fmax(v, dpp_row_down<2>(v));
    v = fmax(v, dpp_row_down<1>(v));
    return v;
}

// Sparse row (or column) product sum_k v[k] x[idx[k]] for k in [kb, ke),
// accumulated in k order (the reference's smx order, linalg.c:62-70) with
// sixteen index and value loads in flight: a long row costs a few memory
// round trips instead of one per entry.
__device__ __forceinline__ double sparse_dot(int kb, int ke, const double* __restrict__ v, const int* __restrict__ idx,
                                             const double* __restrict__ x) {
    double s = 0.0;
    int k = kb;
    for (; k + 16 <= ke; k += 16) {
        int ix[16];
        double a[16], b[16];
#pragma unroll
        for (int u = 0; u < 16; u++) { ix[u] = idx[k + u]; a[u] = v[k + u]; }
#pragma unroll
        for (int u = 0; u < 16; u++) b[u] = x[ix[u]];
#pragma unroll
        for (int u = 0; u < 16; u++) s += a[u] * b[u];
    }
    // the rest (< 16 entries: every column of a typical LP) the same way,
    // masked, so its loads are in flight together too (one dependent pair
    // of loads per entry made short rows latency-bound)
    const int rem = ke - k;
    if (rem > 0) {
        int ix[16];
        double a[16], b[16];
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (u < rem) { ix[u] = idx[k + u]; a[u] = v[k + u]; }
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (u < rem) b[u] = x[ix[u]];
#pragma unroll
        for (int u = 0; u < 16; u++)
            if (u < rem) s += a[u] * b[u];
    }
    return s;
}

// Sum / max over a block of NW waves in a fixed order; result in thread 0.
template <int NW>
__device__ __forceinline__ double block_sum_w(double v, double* sh /* >= NW */) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        r = sh[0];
#pragma unroll
        for (int q = 1; q < NW; q++) r += sh[q];
    }
    __syncthreads();
    return r;
}
template <int NW>
__device__ __forceinline__ double block_max_w(double v, double* sh) {
    v = wave_max(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        r = sh[0];
#pragma unroll
        for (int q = 1; q < NW; q++) r = fmax(r, sh[q]);
    }
    __syncthreads();
    return r;
}
// Threads per block of the SpMV residual kernels (k_hsd_residuals,
// k_pf_residuals, k_kkt_residual): kRedBlocks blocks of kResThreads, so a
// large LP keeps 16 waves per CU of independent rows in flight; their
// partials (printed norms, order-free maxima) stay kRedBlocks per quantity.
constexpr int kResThreads = 1024;

// Sum over a 256-thread block; result valid in thread 0.
__device__ __forceinline__ double block_sum(double v, double* sh /* >= 4 */) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    return r;
}
__device__ __forceinline__ double block_max(double v, double* sh) {
    v = wave_max(v);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) r = fmax(fmax(sh[0], sh[1]), fmax(sh[2], sh[3]));
    __syncthreads();
    return r;
}

// partials laid out part[q * kRedBlocks + block]; bit q of maxmask selects
// max instead of sum.  One 256-thread block finishes nq quantities.
__global__ void __launch_bounds__(kRedThreads)
k_finish_reduce(const double* __restrict__ part, int nq, unsigned maxmask, double* __restrict__ out);
__global__ void __launch_bounds__(kRedThreads)
k_finish_reduce_pack(const double* __restrict__ part, int nq, unsigned maxmask, double* __restrict__ out,
                     const int* __restrict__ f, int nf, double* __restrict__ outi);

// Multi-job dot / max-abs partials: job j reduces a[j][i]*b[j][i] (dot) or
// |a[j][i]| (maxabs, b == nullptr) over i < len[j].
struct RedJobs {
    const double* a[8];
    const double* b[8];
    int len[8];
    int op[8];    // 0 = dot, 1 = maxabs, 2 = max(-a/b) (ratio test)
    int nj;
    int segmin;   // dots of at least this many entries in the segmented order (0: kOrderedMaxLen)
};
__global__ void __launch_bounds__(kRedThreads)
k_reduce_jobs(RedJobs jobs, double* __restrict__ part);

// Host helper: run jobs, finish into out[0..nj) (device), async on stream.
// With g_ordered_reductions (default) dot jobs are summed in index order like
// the reference's dotprod(); otherwise by a fixed-shape tree.
// dots of at least kOrderedMaxLen entries (RedJobs::segmin when set) use a
// fixed segmented order instead, and maxima of at least kSegMaxLen entries
// are taken over the same segments (order-free: bitwise the one-block form)
// (dev_common.hip, k_dot_segments / k_dot_finish; part: kRedBlocks per job).
// No netlib problem has a vector of kOrderedMaxLen entries; problems that do
// (the synthetic configs) set segmin = kSegDotLen for every dot of theirs
// (IpmSolver, dot_segmin), whose serial chains took ~1 ms each at m = 2e5.
constexpr int kOrderedMaxLen = 1 << 19;
constexpr int kSegDotLen = 1 << 12;
constexpr int kSegMaxLen = 1 << 16;
__host__ __device__ inline int dot_segmin(const RedJobs& j) { return j.segmin > 0 ? j.segmin : kOrderedMaxLen; }
__host__ __device__ inline bool job_segmented(const RedJobs& j, int q) {
    return j.len[q] >= (j.op[q] == 0 ? dot_segmin(j) : kSegMaxLen);
}
extern bool g_ordered_reductions;
void launch_reduce(const RedJobs& jobs, double* part, double* out, hipStream_t st);
// the ordered dot of two host vectors (tests: ipo_hip_dot_ordered)
double dot_ordered_host(const double* a, const double* b, int n);

// Linking-row products of the sharded solve (exchange.h): out[i - mrow] =
// sum_k At[k] x[iAt[k]] for rows mrow <= i < m (CSR of A), one wave per row.
void launch_link_ax(int mrow, int m, const int* kAt, const int* iAt, const double* At, const double* x, double* out,
                    hipStream_t st);

}  // namespace ipo
