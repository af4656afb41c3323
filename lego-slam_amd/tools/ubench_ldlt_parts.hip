// Micro-benchmark (diagnostic, not product): the pieces of lds_ldlt_solve timed one at a time
// with s_memtime in one wave (the critical wave's view): the 8x8 block factor, the diagonal
// tile (T + update), a full tile row, and a readlane / f64 FMA latency probe.
#include "../csrc/lh_kernels.hip"
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(64) void k_parts(const double* __restrict__ img, unsigned long long* __restrict__ cyc,
                                              double* __restrict__ sink, int reps) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ __attribute__((aligned(16))) LdltBlockLds F;
    const int lane = threadIdx.x;
    for (int i = lane; i < (NP + 1) * AS; i += 64) A[i] = img[i];
    for (int i = lane; i < 64; i += 64) { F.ND[1][i] = 1e-3 * (i & 7); F.N[0][i] = 1e-3 * (i >> 3); }
    wave_sync();
    unsigned long long t0, acc[6] = {0, 0, 0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        const int k0 = 8 * (r & 7);
        t0 = __builtin_amdgcn_s_memtime();
        factor_block8(A, F.N[1], F.ND[0], k0, lane);
        wave_sync();
        acc[0] += __builtin_amdgcn_s_memtime() - t0;
        t0 = __builtin_amdgcn_s_memtime();
        ldlt_tile_row(A, F.N[0], F.ND[1], 0, 16, 16, 32, -1, false, lane);
        wave_sync();
        acc[1] += __builtin_amdgcn_s_memtime() - t0;
        t0 = __builtin_amdgcn_s_memtime();
        ldlt_tile_row(A, F.N[0], F.ND[1], 0, 112, 16, 128, -1, true, lane);
        wave_sync();
        acc[2] += __builtin_amdgcn_s_memtime() - t0;
        t0 = __builtin_amdgcn_s_memtime();
        ldlt_tile_row(A, F.N[0], F.ND[1], 0, 112, 16, 32, -1, true, lane);
        wave_sync();
        acc[3] += __builtin_amdgcn_s_memtime() - t0;
    }
    // dependent readlane chain: v -> readlane -> fma -> readlane ...
    double v = img[lane];
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; ++i) v = fma(readlane_d(v, i & 63), 0.5, v);
    __builtin_amdgcn_s_waitcnt(0);
    acc[4] = (__builtin_amdgcn_s_memtime() - t0) * reps / 256;
    double u = img[lane + 1];
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; ++i) u = fma(u, 0.999, 1e-3);
    __builtin_amdgcn_s_waitcnt(0);
    acc[5] = (__builtin_amdgcn_s_memtime() - t0) * reps / 256;
    if (lane == 0)
        for (int i = 0; i < 6; ++i) cyc[i] = acc[i] / reps;
    sink[lane] = v + u + A[lane];
}

int main() {
    std::vector<double> img((NP + 1) * AS, 0.0);
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j <= i; ++j) img[i * AS + j] = (i == j) ? 100.0 + i : 1.0 / (1.0 + i + j);
    double *d_img, *d_sink;
    unsigned long long* d_c;
    (void)hipMalloc(&d_img, img.size() * 8);
    (void)hipMalloc(&d_sink, 64 * 8);
    (void)hipMalloc(&d_c, 64);
    (void)hipMemcpy(d_img, img.data(), img.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_parts, dim3(1), dim3(64), 0, 0, d_img, d_c, d_sink, 4);
    hipLaunchKernelGGL(k_parts, dim3(1), dim3(64), 0, 0, d_img, d_c, d_sink, 64);
    unsigned long long c[6];
    (void)hipMemcpy(c, d_c, sizeof(c), hipMemcpyDeviceToHost);
    printf("factor_block8 (+N, ND)         %6llu ticks\n", c[0]);
    printf("diag tile (L, T, 1 tile)      %6llu ticks\n", c[1]);
    printf("tile row, L + rhs + 7 tiles   %6llu ticks\n", c[2]);
    printf("tile row, L + rhs + 1 tile    %6llu ticks\n", c[3]);
    printf("readlane+fma dependent step   %6.1f ticks\n", c[4] / 1.0);
    printf("f64 fma dependent step        %6.1f ticks\n", c[5] / 1.0);
    return 0;
}
