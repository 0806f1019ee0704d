// f64 VALU issue-rate probe (developer tool): cycles per v_mul_f64 + v_add_f64
// pair on 16 independent register chains, one or two waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(512) k_probe(double* out, long long* cyc, int iters, double l0) {
    double a[16], c[16];
    const int t = threadIdx.x;
    for (int q = 0; q < 16; q++) { a[q] = t + q; c[q] = 1e-9 * (q + 1); }
    double l = l0 + t * 1e-12;
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int q = 0; q < 16; q++) a[q] = a[q] - l * c[q];
        l = l * 0.999999;
    }
    const long long t1 = clock64();
    double s = 0;
    for (int q = 0; q < 16; q++) s += a[q];
    out[blockIdx.x * blockDim.x + t] = s;
    if ((t & 63) == 0) cyc[blockIdx.x * 8 + (t >> 6)] = t1 - t0;
}

__global__ void __launch_bounds__(512) k_probe_fma(double* out, long long* cyc, int iters, double l0) {
    double a[16], c[16];
    const int t = threadIdx.x;
    for (int q = 0; q < 16; q++) { a[q] = t + q; c[q] = 1e-9 * (q + 1); }
    double l = l0 + t * 1e-12;
    __syncthreads();
    const long long t0 = clock64();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int q = 0; q < 16; q++) a[q] = __builtin_fma(-l, c[q], a[q]);
        l = l * 0.999999;
    }
    const long long t1 = clock64();
    double s = 0;
    for (int q = 0; q < 16; q++) s += a[q];
    out[blockIdx.x * blockDim.x + t] = s;
    if ((t & 63) == 0) cyc[blockIdx.x * 8 + (t >> 6)] = t1 - t0;
}

int main() {
    double* out; long long* cyc;
    hipMalloc(&out, 1 << 20); hipMalloc(&cyc, 8 * 1024);
    const int iters = 4096;
    for (int which = 0; which < 2; which++)
        for (int nt : {64, 256, 512}) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (which == 0) hipLaunchKernelGGL(k_probe, dim3(1), dim3(nt), 0, 0, out, cyc, iters, 0.5);
            else hipLaunchKernelGGL(k_probe_fma, dim3(1), dim3(nt), 0, 0, out, cyc, iters, 0.5);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long h[8]; hipMemcpy(h, cyc, 64, hipMemcpyDeviceToHost);
            const double ops = (which == 0 ? 2.0 : 1.0) * 16 * iters;
            std::printf("%s threads %d: wave0 %lld cycles, %.2f cycles per f64 instr per wave; kernel %.1f us -> %.2f GHz\n",
                        which ? "fma    " : "mul+add", nt, h[0], h[0] / ops, ms * 1e3, h[0] / (ms * 1e3) / 1e3);
        }
    return 0;
}
