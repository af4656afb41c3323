// Micro-benchmark (diagnostic, not product): variants of the 8x8 LDL^T block factor.
#include "../csrc/lh_kernels.hip"
#include <cstdio>
#include <vector>

template <int NEWTON, bool STORE, bool LOAD>
__device__ __forceinline__ void fb8_variant(double* A, double* blk, int k0, int lane, double seed) {
    double B[8][8], Wb[8][8], dv[8], inv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) B[r][c] = LOAD ? A[(k0 + r) * AS + k0 + c] : (r == c ? 100.0 + seed * r : seed / (1 + r + c));
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        dv[c] = B[c][c];
        const bool valid = fabs(dv[c]) > 0.0;
        double r = __builtin_amdgcn_rcp(dv[c]);
        if (NEWTON >= 1) r = fma(r, fma(-dv[c], r, 1.0), r);
        if (NEWTON >= 2) r = fma(r, fma(-dv[c], r, 1.0), r);
        inv[c] = valid ? r : 1.0;
#pragma unroll
        for (int rr = c + 1; rr < 8; ++rr) Wb[rr][c] = B[rr][c];
#pragma unroll
        for (int rr = c + 1; rr < 8; ++rr) {
            const double l = Wb[rr][c] * inv[c];
            B[rr][c] = l;
#pragma unroll
            for (int r2 = c + 1; r2 <= rr; ++r2) B[rr][r2] -= l * Wb[r2][c];
        }
    }
    if (STORE) {
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < 8; ++c) { blk[c] = dv[c]; blk[8 + c] = inv[c]; }
#pragma unroll
            for (int r = 1; r < 8; ++r)
#pragma unroll
                for (int c = 0; c < r; ++c) blk[16 + TRI8(r, c)] = Wb[r][c];
        } else if (lane == 32) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
#pragma unroll
                for (int c = 0; c < r; ++c) A[(k0 + r) * AS + k0 + c] = B[r][c];
                A[(k0 + r) * AS + k0 + r] = dv[r];
            }
        }
    } else {
        double s = 0;
#pragma unroll
        for (int r = 0; r < 8; ++r) { s += dv[r] + inv[r]; for (int c = 0; c < r; ++c) s += B[r][c] * Wb[r][c]; }
        if (s == 1.2345) blk[0] = s;
    }
}

// distributed variant: lane r < 8 holds row r of the block; pivots broadcast with readlane
__device__ __forceinline__ void fb8_lanes(double* A, double* blk, int k0, int lane) {
    const int r = lane & 7;
    double a[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) a[c] = A[(k0 + r) * AS + k0 + c];
    double dvr = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const double d = readlane_d(a[c], c);
        const bool valid = fabs(d) > 0.0;
        const double inv = valid ? fast_rcp(d) : 1.0;
        const double w = a[c];
        if (r == c) dvr = d;
        const double l = (r > c) ? w * inv : a[c];
#pragma unroll
        for (int c2 = c + 1; c2 < 8; ++c2) {
            const double wc2 = readlane_d(w, c2);
            if (r >= c2) a[c2] -= l * wc2;
        }
        if (r > c) a[c] = l;
        if (lane == c) blk[8 + c] = inv;
        if (lane > c && lane < 8) blk[16 + TRI8(r, c)] = w;
    }
    if (lane < 8) {
#pragma unroll
        for (int c = 0; c < 8; ++c) if (c < r) A[(k0 + r) * AS + k0 + c] = a[c];
        A[(k0 + r) * AS + k0 + r] = dvr;
    }
}

template <int V>
__global__ __launch_bounds__(512) void k_bench(const double* src, double* out, unsigned long long* cyc, int reps) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ double blk[48];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < (NP + 1) * AS; i += blockDim.x) A[i] = src[i % (NP * AS)];
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        const int k0 = 8 * (r & 7);
        if (V == 0) factor_block8(A, k0, lane);
        if (V == 1) fb8_variant<1, true, true>(A, blk, k0, lane, 0);
        if (V == 2) fb8_variant<2, false, true>(A, blk, k0, lane, 0);
        if (V == 3) fb8_variant<2, true, false>(A, blk, k0, lane, 0.5 + r);
        if (V == 4) fb8_variant<2, false, false>(A, blk, k0, lane, 0.5 + r);
        if (V == 5) fb8_lanes(A, blk, k0, lane);
        wave_sync();
    }
    __builtin_amdgcn_s_waitcnt(0);
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (tid == 0) cyc[V] = (t1 - t0) / reps;
    if (tid == 0) out[V] = blk[9] + A[5 * AS + 3];
}

int main() {
    std::vector<double> h(NP * AS);
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j < AS; ++j) h[i * AS + j] = (i == j) ? 100.0 + i : 1.0 / (1.0 + i + j);
    double *src, *out; unsigned long long* cyc;
    (void)hipMalloc(&src, h.size() * 8); (void)hipMalloc(&out, 64 * 8); (void)hipMalloc(&cyc, 64 * 8);
    (void)hipMemcpy(src, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, src, out, cyc, 64);
        hipLaunchKernelGGL(k_bench<1>, dim3(1), dim3(64), 0, 0, src, out, cyc, 64);
        hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(64), 0, 0, src, out, cyc, 64);
        hipLaunchKernelGGL(k_bench<3>, dim3(1), dim3(64), 0, 0, src, out, cyc, 64);
        hipLaunchKernelGGL(k_bench<4>, dim3(1), dim3(64), 0, 0, src, out, cyc, 64);
        hipLaunchKernelGGL(k_bench<5>, dim3(1), dim3(64), 0, 0, src, out, cyc, 64);
    }
    (void)hipDeviceSynchronize();
    unsigned long long c[8];
    (void)hipMemcpy(c, cyc, 64, hipMemcpyDeviceToHost);
    printf("factor_block8 (product)        %llu cycles\n", c[0]);
    printf("1 Newton, store, load          %llu\n", c[1]);
    printf("2 Newton, no store, load       %llu\n", c[2]);
    printf("2 Newton, store, no load       %llu\n", c[3]);
    printf("2 Newton, no store, no load    %llu\n", c[4]);
    printf("lane-distributed (readlane)    %llu\n", c[5]);
    return 0;
}
