// Micro-benchmark (diagnostic, not product): k_ctrl building blocks timed in isolation
// with s_memtime, one workgroup, on synthetic SPD data.
#include "../csrc/lh_kernels.hip"
#include <cstdio>
#include <vector>

__global__ void k_factor_bench(const double* src, double* out, unsigned long long* cyc, int reps, int waves_busy) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ double blk[48];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < (NP + 1) * AS; i += blockDim.x) A[i] = src[i % (NP * AS)];
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave == 0) {
        for (int r = 0; r < reps; ++r) {
            factor_block8(A, 8 * (r & 7), lane);
            wave_sync();
        }
    } else if (wave < waves_busy) {
        // keep other waves busy with f64 MFMA like the trailing update
        v4d acc = {0, 0, 0, 0};
        for (int r = 0; r < reps * 8; ++r) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[lane], A[lane + 64], acc, 0, 0, 0);
        if (acc[0] == 12345.0) out[1] = acc[1];
    }
    __builtin_amdgcn_s_waitcnt(0);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[0] = (t1 - t0) / reps;
    if (tid == 0) out[0] = blk[3];
}

__global__ void k_mfma_lat(unsigned long long* cyc) {
    const int lane = threadIdx.x;
    v4d acc = {0, 0, 0, 0};
    double a = 1.0 + lane * 1e-3;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 256; ++r) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, acc, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    double s = acc[0] + acc[1];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) { cyc[1] = (t1 - t0) / 256; cyc[2] = (unsigned long long)s; }
}

int main() {
    std::vector<double> h(NP * AS);
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j < AS; ++j) h[i * AS + j] = (i == j) ? 100.0 + i : 1.0 / (1.0 + i + j);
    double *src, *out; unsigned long long* cyc;
    (void)hipMalloc(&src, h.size() * 8); (void)hipMalloc(&out, 64); (void)hipMalloc(&cyc, 64);
    (void)hipMemcpy(src, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    unsigned long long c[4];
    for (int busy : {1, 8}) {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_factor_bench, dim3(1), dim3(512), 0, 0, src, out, cyc, 64, busy);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(c, cyc, 32, hipMemcpyDeviceToHost);
        printf("factor_block8: %llu cycles per call (waves busy with MFMA: %d)\n", c[0], busy - 1);
    }
    hipLaunchKernelGGL(k_mfma_lat, dim3(1), dim3(64), 0, 0, cyc);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(c, cyc, 32, hipMemcpyDeviceToHost);
    printf("mfma_f64_16x16x4 dependent: %llu cycles\n", c[1]);
    return 0;
}
