// Throughput of v_mfma_f64_16x16x4_f64 (developer tool): G workgroups of W
// waves, each wave issuing N MFMAs over C independent accumulator chains,
// operands in registers (no memory).  Reports the MFMA rate per SIMD in
// cycles per instruction (at the clock the host passes, GHz).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_mfma.hip -o tools/ubench_mfma
//   tools/ubench_mfma [ghz]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double double4_t __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <int C>
__global__ void k_mfma(double* out, int n, double seed) {
    double4_t acc[C];
#pragma unroll
    for (int c = 0; c < C; c++) acc[c] = (double4_t){0.0, 0.0, 0.0, 0.0};
    double a = seed + threadIdx.x, b = seed * 0.5 + threadIdx.x;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int c = 0; c < C; c++) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < C; c++) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int C>
void run(int G, int W, double ghz, double* d) {
    const int n = 2048 / C;
    hipLaunchKernelGGL(k_mfma<C>, dim3(G), dim3(64 * W), 0, 0, d, n, 1.0);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_mfma<C>, dim3(G), dim3(64 * W), 0, 0, d, n, 1.0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    // waves per SIMD: W / 4 per workgroup (workgroups spread one per CU up to 256)
    const double per_simd = (double)n * C * (W / 4.0) * ((G + 255) / 256);
    std::printf("  G %4d W %2d chains %d: %.1f us, %.1f cycles per MFMA per SIMD, %.1f TFLOP/s\n", G, W, C, ms * 1e3,
                ms * 1e-3 * ghz * 1e9 / per_simd, (double)G * W * n * C * 2048 / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
    const double ghz = argc > 1 ? std::atof(argv[1]) : 2.4;
    double* d;
    CK(hipMalloc(&d, 1 << 24));
    for (int W : {4, 8, 16}) {
        run<1>(256, W, ghz, d);
        run<2>(256, W, ghz, d);
        run<4>(256, W, ghz, d);
    }
    run<4>(1024, 8, ghz, d);
    return 0;
}
