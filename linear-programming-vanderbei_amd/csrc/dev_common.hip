// dev_common.hip -- deterministic multi-job reductions (see dev_common.h).
#include "dev_common.h"
#include "hip_util.h"

namespace ipo {

__global__ void __launch_bounds__(kRedThreads)
k_reduce_jobs(RedJobs jobs, double* __restrict__ part) {
    __shared__ double sh[4];
    for (int j = 0; j < jobs.nj; j++) {
        const double* a = jobs.a[j];
        const double* b = jobs.b[j];
        const int len = jobs.len[j];
        const int op = jobs.op[j];
        double acc = op == 0 ? 0.0 : (op == 2 ? 0.0 : 0.0);
        for (int i = blockIdx.x * kRedThreads + threadIdx.x; i < len; i += kRedBlocks * kRedThreads) {
            if (op == 0) acc += a[i] * b[i];
            else if (op == 1) acc = fmax(acc, ref_abs(a[i]));
            else acc = fmax(acc, -a[i] / b[i]);      // NaN ratios are ignored like hsd.c:249-258
        }
        const double r = op == 0 ? block_sum(acc, sh) : block_max(acc, sh);
        if (threadIdx.x == 0) part[j * kRedBlocks + blockIdx.x] = r;
    }
}

__global__ void __launch_bounds__(kRedThreads)
k_finish_reduce(const double* __restrict__ part, int nq, unsigned maxmask, double* __restrict__ out) {
    __shared__ double sh[4];
    for (int q = 0; q < nq; q++) {
        const bool mx = (maxmask >> q) & 1u;
        double v = part[q * kRedBlocks + threadIdx.x];   // kRedBlocks == kRedThreads
        const double r = mx ? block_max(v, sh) : block_sum(v, sh);
        if (threadIdx.x == 0) out[q] = r;
    }
}

// dotprod() of linalg.c:17-25 in its own order: one running sum, i = 0..n-1.
// One block per job; the products are independent (prefetched), only the
// adds form the sequential chain.  Max-type jobs are order-free.
__global__ void __launch_bounds__(64)
k_reduce_ordered(RedJobs jobs, double* __restrict__ out) {
    const int j = blockIdx.x;
    const double* a = jobs.a[j];
    const double* b = jobs.b[j];
    const int len = jobs.len[j];
    const int op = jobs.op[j];
    if (op != 0) {
        __shared__ double sh[1];
        double acc = 0.0;
        for (int i = threadIdx.x; i < len; i += 64) {
            if (op == 1) acc = fmax(acc, ref_abs(a[i]));
            else acc = fmax(acc, -a[i] / b[i]);
        }
        acc = wave_max(acc);
        if (threadIdx.x == 0) { sh[0] = acc; out[j] = acc; }
        return;
    }
    // products in parallel into LDS, then one lane adds them in index order
    constexpr int CH = 4096;
    __shared__ double prod[CH];
    double s = 0.0e0;
    for (int base = 0; base < len; base += CH) {
        const int cnt = min(CH, len - base);
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += 64) prod[i] = a[base + i] * b[base + i];
        __syncthreads();
        if (threadIdx.x == 0) {
            int i = 0;
            for (; i + 8 <= cnt; i += 8) {
                const double p0 = prod[i], p1 = prod[i + 1], p2 = prod[i + 2], p3 = prod[i + 3];
                const double p4 = prod[i + 4], p5 = prod[i + 5], p6 = prod[i + 6], p7 = prod[i + 7];
                s += p0; s += p1; s += p2; s += p3; s += p4; s += p5; s += p6; s += p7;
            }
            for (; i < cnt; i++) s += prod[i];
        }
    }
    if (threadIdx.x == 0) out[j] = s;
}

__global__ void __launch_bounds__(256)
k_link_ax(int mrow, int m, const int* __restrict__ kAt, const int* __restrict__ iAt, const double* __restrict__ At,
          const double* __restrict__ x, double* __restrict__ out) {
    const int i = mrow + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= m) return;
    double s = 0.0;
    for (int k = kAt[i] + lane; k < kAt[i + 1]; k += 64) s += At[k] * x[iAt[k]];
    s = wave_sum(s);
    if (lane == 0) out[i - mrow] = s;
}

void launch_link_ax(int mrow, int m, const int* kAt, const int* iAt, const double* At, const double* x, double* out,
                    hipStream_t st) {
    if (m <= mrow) return;
    hipLaunchKernelGGL(k_link_ax, dim3((m - mrow + 3) / 4), dim3(256), 0, st, mrow, m, kAt, iAt, At, x, out);
    IPO_HIP_CHECK(hipGetLastError());
}

bool g_ordered_reductions = true;

void launch_reduce(const RedJobs& jobs, double* part, double* out, hipStream_t st) {
    if (g_ordered_reductions) {
        hipLaunchKernelGGL(k_reduce_ordered, dim3(jobs.nj), dim3(64), 0, st, jobs, out);
        IPO_HIP_CHECK(hipGetLastError());
        return;
    }
    unsigned mask = 0;
    for (int j = 0; j < jobs.nj; j++) if (jobs.op[j] != 0) mask |= 1u << j;
    hipLaunchKernelGGL(k_reduce_jobs, dim3(kRedBlocks), dim3(kRedThreads), 0, st, jobs, part);
    hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, st, part, jobs.nj, mask, out);
    IPO_HIP_CHECK(hipGetLastError());
}

}  // namespace ipo
