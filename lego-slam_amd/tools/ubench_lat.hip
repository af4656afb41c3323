// Micro-benchmark (diagnostic, not product): dependent-latency of the f64 operations
// that make up k_ctrl's pivot chain, LDS round trips and workgroup barriers on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 256
__global__ void k_lat(double* out, unsigned long long* cyc, double seed) {
    __shared__ double lds[1024];
    const int tid = threadIdx.x;
    double x = seed + tid * 1e-9, y = 1.0000001;
    lds[tid] = x;
    __syncthreads();
    unsigned long long t0, t1;
    // 1. dependent v_fma_f64
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) x = fma(x, y, 1e-7);
    __builtin_amdgcn_s_waitcnt(0);
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[0] = t1 - t0;
    // 2. dependent v_rcp_f64
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) x = __builtin_amdgcn_rcp(x) + 1e-300;
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[1] = t1 - t0;
    // 3. dependent IEEE division
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < N; ++i) x = 1.0 / x + 1e-300;
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[2] = t1 - t0;
    // 4. dependent LDS load chain (address from data)
    int idx = tid;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) idx = ((int)lds[idx & 1023] + idx + 1) & 1023;
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[3] = t1 - t0;
    // 5. __syncthreads cost (all waves arrive together)
    __syncthreads();
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) __syncthreads();
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[4] = t1 - t0;
    // 6. LDS write -> barrier -> LDS read round trip (producer wave 0, consumer wave 1)
    t0 = __builtin_amdgcn_s_memtime();
    double z = 0.0;
    for (int i = 0; i < N; ++i) {
        if (tid == 0) lds[512 + (i & 7)] = z + 1.0;
        __syncthreads();
        z = lds[512 + (i & 7)];
        __syncthreads();
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[5] = t1 - t0;
    // 7. readlane broadcast chain
    t0 = __builtin_amdgcn_s_memtime();
    double q = x;
    for (int i = 0; i < N; ++i) {
        long long b = __double_as_longlong(q);
        int lo = __builtin_amdgcn_readlane((int)b, i & 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), i & 63);
        q = __longlong_as_double(((long long)hi << 32) | (unsigned)lo) * 1.0000001 + (double)tid * 1e-20;
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[6] = t1 - t0;
    // 8. s_memrealtime pair -> clock estimate
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), m0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
    for (int i = 0; i < 4096; ++i) x = fma(x, y, 1e-7);
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), m1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) { cyc[7] = m1 - m0; cyc[8] = r1 - r0; }
    out[tid] = x + z + q + idx;
}

int main() {
    double* out; unsigned long long* cyc;
    hipMalloc(&out, 1024 * 8); hipMalloc(&cyc, 64 * 8);
    for (int threads : {64, 512}) {
        for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k_lat, dim3(1), dim3(threads), 0, 0, out, cyc, 1.5);
        hipDeviceSynchronize();
        unsigned long long h[16];
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        printf("threads=%d  per-op cycles: fma_f64 %.1f  rcp_f64 %.1f  div_f64 %.1f  lds_dep %.1f  syncthreads %.1f  lds_bar_roundtrip %.1f  readlane_chain %.1f  clock %.2f GHz\n",
               threads, h[0] / (double)N, h[1] / (double)N, h[2] / (double)N, h[3] / (double)N, h[4] / (double)N,
               h[5] / (double)N, h[6] / (double)N, (double)h[7] / (double)h[8] * 0.1);
    }
    return 0;
}
