// Micro-benchmark (diagnostic, not product): the pieces of the LDL^T step's critical chain (wave 0 of
// k_ctrl / k_ctrl_b) timed one at a time with s_memtime, one wave alone in the workgroup:
//   [0] factor_block8 (the kernel's factor column, 64-bit DPP broadcasts)
//   [1] the round-3 factor column (32-bit DPP halves)
//   [2] diag_tile (the specialised diagonal tile)
//   [3] ldlt_tile_row on the diagonal tile (the generic path wave 0 took before)
//   [4] a dependent f64 FMA chain, per FMA x 100
//   [5] a dependent v_rcp_f64 -> FMA chain, per pair x 100
//   [6] a dependent 64-bit DPP row_newbcast -> FMA chain, per pair x 100
#include "../csrc/lh_kernels.hip"
#include <cstdio>
#include <vector>

template <int L>
__device__ __forceinline__ double bcast16_32(double v) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)x, 0x150 + L, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), 0x150 + L, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int Q>
__device__ __forceinline__ void factor_column_r3(double (&R)[8], double (&dl)[8]) {
    const double d = bcast16_32<Q>(R[Q]);
    dl[Q] = fabs(d) > 0.0 ? d : 1.0;
    const double inv = fast_rcp(dl[Q]);
    const double coef = R[Q] * inv;
    double u[8];
    if (Q < 1) u[1] = bcast16_32<1>(R[Q]);
    if (Q < 2) u[2] = bcast16_32<2>(R[Q]);
    if (Q < 3) u[3] = bcast16_32<3>(R[Q]);
    if (Q < 4) u[4] = bcast16_32<4>(R[Q]);
    if (Q < 5) u[5] = bcast16_32<5>(R[Q]);
    if (Q < 6) u[6] = bcast16_32<6>(R[Q]);
    if (Q < 7) u[7] = bcast16_32<7>(R[Q]);
#pragma unroll
    for (int j = Q + 1; j < 8; ++j) R[j] -= coef * u[j];
    R[Q] = coef;
}

__device__ __forceinline__ void factor_block8_r3(double* A, double* No, double* NDo, int k0, int lane) {
    const int p = lane & 15, r = p & 7;
    const bool ident = p >= 8;
    double R[8], dl[8], v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = A[(k0 + r) * AS + k0 + q];
#pragma unroll
    for (int q = 0; q < 8; ++q) R[q] = ident ? (q == r ? 1.0 : 0.0) : v[q];
    factor_column_r3<0>(R, dl); factor_column_r3<1>(R, dl); factor_column_r3<2>(R, dl); factor_column_r3<3>(R, dl);
    factor_column_r3<4>(R, dl); factor_column_r3<5>(R, dl); factor_column_r3<6>(R, dl); factor_column_r3<7>(R, dl);
    if (lane < 8) {
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q <= r) A[(k0 + q) * AS + k0 + r] = (q == r) ? dl[q] : R[q];
    } else if (lane < 16) {
#pragma unroll
        for (int q = 0; q < 8; ++q) { No[8 * r + q] = R[q]; NDo[8 * r + q] = R[q] * dl[q]; }
    }
}

__global__ __launch_bounds__(64) void k_chain(const double* __restrict__ img, unsigned long long* __restrict__ cyc,
                                              double* __restrict__ sink, int reps) {
    __shared__ double A[(NP + 1) * AS];
    __shared__ __attribute__((aligned(16))) double N[2][64], ND[2][64];
    const int lane = threadIdx.x;
    const LdsSys SY{A};
    unsigned long long t0, acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        for (int i = lane; i < (NP + 1) * AS; i += 64) A[i] = img[i];
        for (int i = lane; i < 64; i += 64) { ND[1][i] = 1e-3 * (i & 7); N[0][i] = 1e-3 * (i >> 3); }
        wave_sync();
        const int k0 = 8 * (r & 7);
        t0 = __builtin_amdgcn_s_memtime();
        factor_block8(SY, N[1], ND[0], k0, lane);
        wave_sync();
        acc[0] += __builtin_amdgcn_s_memtime() - t0;
        t0 = __builtin_amdgcn_s_memtime();
        factor_block8_r3(A, N[1], ND[0], k0 + 64, lane);
        wave_sync();
        acc[1] += __builtin_amdgcn_s_memtime() - t0;
        t0 = __builtin_amdgcn_s_memtime();
        diag_tile(SY, N[0], ND[1], 8, 16, lane);
        wave_sync();
        acc[2] += __builtin_amdgcn_s_memtime() - t0;
        t0 = __builtin_amdgcn_s_memtime();
        ldlt_tile_row(SY, N[0], ND[1], 8, 16, 16, 32, -1, false, lane);
        wave_sync();
        acc[3] += __builtin_amdgcn_s_memtime() - t0;
    }
    double u = img[lane + 1];
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; ++i) u = fma(u, 0.999, 1e-3);
    sink[64 + lane] = u;
    __builtin_amdgcn_s_waitcnt(0);
    acc[4] = (__builtin_amdgcn_s_memtime() - t0) * 100 * reps / 256;
    double w = img[lane + 2] + 2.0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; ++i) w = fma(__builtin_amdgcn_rcp(w), 0.5, 2.0);
    sink[128 + lane] = w;
    __builtin_amdgcn_s_waitcnt(0);
    acc[5] = (__builtin_amdgcn_s_memtime() - t0) * 100 * reps / 256;
    double x = img[lane + 3];
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 256; ++i) x = fma(bcast16<3>(x), 0.5, 1.0);
    sink[192 + lane] = x;
    __builtin_amdgcn_s_waitcnt(0);
    acc[6] = (__builtin_amdgcn_s_memtime() - t0) * 100 * reps / 256;
    if (lane == 0)
        for (int i = 0; i < 8; ++i) cyc[i] = acc[i] / reps;
    sink[lane] = A[lane] + N[1][lane & 63] + ND[0][lane & 63];
}

int main() {
    std::vector<double> img((NP + 1) * AS, 0.0);
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j <= i; ++j) img[i * AS + j] = (i == j) ? 100.0 + i : 1.0 / (1.0 + i + j);
    double *d_img, *d_sink;
    unsigned long long* d_c;
    if (hipMalloc(&d_img, img.size() * 8) != hipSuccess || hipMalloc(&d_sink, 256 * 8) != hipSuccess ||
        hipMalloc(&d_c, 64) != hipSuccess)
        return 1;
    (void)hipMemcpy(d_img, img.data(), img.size() * 8, hipMemcpyHostToDevice);
    const char* names[7] = {"factor_block8 (kernel)", "factor r3 (two Newton)", "diag_tile", "ldlt_tile_row diag",
                            "f64 FMA dep x100", "rcp->FMA dep x100", "dpp bcast->FMA dep x100"};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, d_img, d_c, d_sink, 200);
        unsigned long long c[8];
        if (hipMemcpy(c, d_c, 64, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        for (int i = 0; i < 7; ++i) printf("%-28s %8llu cycles\n", names[i], c[i]);
        printf("--\n");
    }
    return 0;
}
