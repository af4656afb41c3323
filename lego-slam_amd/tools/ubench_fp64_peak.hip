// Micro-benchmark (diagnostic, not product): chip-wide FP64 throughput on this MI355X, VALU
// v_fma_f64 and MFMA v_mfma_f64_16x16x4_f64, to pin the roofline peak used by bench.py.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_valu(double* out, int iters) {
    double a0 = threadIdx.x * 1e-9, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const double m = 0.999999, c = 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
            a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) {
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const double a = 1.0 + threadIdx.x * 1e-6, b = 0.5;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

int main() {
    const int blocks = 256 * 8, iters = 2000;
    double* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int which = 0; which < 2; ++which) {
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            if (which == 0) hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, iters);
            else hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
            const double flops = which == 0 ? 2.0 * blocks * 256.0 * iters * 64 : 2.0 * 1024 * (blocks * 4.0) * iters * 32;
            if (rep == 2) printf("%s: %.1f TFLOP/s (%.3f ms)\n", which == 0 ? "v_fma_f64 (VALU)" : "v_mfma_f64_16x16x4", flops / ms / 1e9, ms);
        }
    }
    return 0;
}
