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

void launch_reduce(const RedJobs& jobs, double* part, double* out, hipStream_t st) {
    unsigned mask = 0;
    for (int j = 0; j < jobs.nj; j++) if (jobs.op[j] != 0) mask |= 1u << j;
    hipLaunchKernelGGL(k_reduce_jobs, dim3(kRedBlocks), dim3(kRedThreads), 0, st, jobs, part);
    hipLaunchKernelGGL(k_finish_reduce, dim3(1), dim3(kRedThreads), 0, st, part, jobs.nj, mask, out);
    IPO_HIP_CHECK(hipGetLastError());
}

}  // namespace ipo
