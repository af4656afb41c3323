// Micro-benchmark (diagnostic, not product): lds_ldlt_solve (k_ctrl phases 3-4) timed in
// isolation with s_memtime, one 512-thread workgroup, on a synthetic SPD system.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_ldlt.hip -o lib/ubench_ldlt [-DKFILE='"..."']
#ifndef KFILE
#define KFILE "../csrc/lh_kernels.hip"
#endif
#include KFILE
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(CT) void k_ldlt_bench(const double* __restrict__ img, int n, int reps, double* __restrict__ x,
                                                   unsigned long long* __restrict__ cyc) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ __attribute__((aligned(16))) double xsol[NP];
    const int tid = threadIdx.x, NE = (n + 15) & ~15;
    unsigned long long acc = 0;
    for (int r = 0; r < reps; ++r) {
        for (int i = tid; i < (NP + 1) * AS; i += CT) A[i] = img[i];
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        #ifdef OLD_API
        __shared__ double Xp[NP * XS];
        lds_ldlt_solve(A, Xp, xsol, n, NE, tid);
#else
        lds_ldlt_solve(A, xsol, n, NE, tid);
#endif
        __syncthreads();
        acc += __builtin_amdgcn_s_memtime() - t0;
    }
    if (tid < n) x[tid] = xsol[tid];
    if (tid == 0) cyc[0] = acc / reps;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 120;
    const int reps = 200;
    const int NE = (n + 15) & ~15;
    srand(7);
    std::vector<double> M((size_t)n * n), S((size_t)n * n, 0.0), b(n);
    for (auto& v : M) v = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int k = 0; k < n; ++k) s += M[(size_t)i * n + k] * M[(size_t)j * n + k];
            S[(size_t)i * n + j] = s + (i == j ? 1.0 + 1e3 * pow(0.9, i) : 0.0);
        }
    for (auto& v : b) v = (double)rand() / RAND_MAX - 0.5;
    std::vector<double> img((size_t)(NP + 1) * AS, 0.0);
    for (int i = 0; i < NE; ++i)
        for (int j = 0; j <= i; ++j) img[(size_t)i * AS + j] = (i < n) ? S[(size_t)i * n + j] : (i == j ? 1.0 : 0.0);
    for (int j = 0; j < n; ++j) img[(size_t)NP * AS + j] = b[j];

    // reference: dense Cholesky solve
    std::vector<double> Lc(S);
    for (int j = 0; j < n; ++j) {
        double d = Lc[(size_t)j * n + j];
        for (int k = 0; k < j; ++k) d -= Lc[(size_t)j * n + k] * Lc[(size_t)j * n + k];
        d = sqrt(d);
        Lc[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = Lc[(size_t)i * n + j];
            for (int k = 0; k < j; ++k) s -= Lc[(size_t)i * n + k] * Lc[(size_t)j * n + k];
            Lc[(size_t)i * n + j] = s / d;
        }
    }
    std::vector<double> y(b), xr(n);
    for (int i = 0; i < n; ++i) {
        for (int k = 0; k < i; ++k) y[i] -= Lc[(size_t)i * n + k] * y[k];
        y[i] /= Lc[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < n; ++k) s -= Lc[(size_t)k * n + i] * xr[k];
        xr[i] = s / Lc[(size_t)i * n + i];
    }

    double *d_img, *d_x;
    unsigned long long* d_c;
    (void)hipMalloc(&d_img, img.size() * 8);
    (void)hipMalloc(&d_x, NP * 8);
    (void)hipMalloc(&d_c, 64);
    (void)hipMemcpy(d_img, img.data(), img.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_ldlt_bench, dim3(1), dim3(CT), 0, 0, d_img, n, 2, d_x, d_c);
#ifdef LH_STAMPS
    unsigned long long zs[64] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(lh_stamps), zs, sizeof(zs));
#endif
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_ldlt_bench, dim3(1), dim3(CT), 0, 0, d_img, n, reps, d_x, d_c);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("kernel %.2f us per rep (solve + LDS reload)\n", 1e3 * ms / reps);
#ifdef LH_STAMPS
    (void)hipMemcpyFromSymbol(zs, HIP_SYMBOL(lh_stamps), sizeof(zs));
    const char* nm[24] = {};
    nm[18] = "block0"; nm[15] = "panel"; nm[22] = "tiles w0"; nm[23] = "tiles w1-7"; nm[12] = "factor w0";
    nm[16] = "update barrier"; nm[13] = "back-subst";
    for (int i = 10; i < 24; ++i)
        if (zs[i]) printf("  %-16s %10.1f ticks/solve (summed over waves)\n", nm[i] ? nm[i] : "?", (double)zs[i] / reps);
#endif
    std::vector<double> xg(NP);
    unsigned long long cyc = 0;
    (void)hipMemcpy(xg.data(), d_x, NP * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&cyc, d_c, 8, hipMemcpyDeviceToHost);
    double err = 0.0, nx = 0.0;
    for (int i = 0; i < n; ++i) { err = fmax(err, fabs(xg[i] - xr[i])); nx = fmax(nx, fabs(xr[i])); }
    printf("n=%d lds_ldlt_solve: %llu s_memtime ticks/solve, max|x-x_ref|/max|x| = %.3e\n", n, cyc, err / nx);
    return 0;
}
