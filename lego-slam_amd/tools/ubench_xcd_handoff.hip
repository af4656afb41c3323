// Probe: does a one-workgroup kernel read a 74 KB buffer faster when the previous kernel wrote it from
// the reader's own XCD?  (k_ctrl's prologue reads the staged system k_reduce wrote from blocks on all
// eight XCDs, and its L2 counters show misses)
// Writer: 8 (or 8 k) blocks, dispatched round robin over the XCDs (block b on XCD b % 8, checked by the
// XCC_ID hardware register); only the chosen blocks store, the same bytes every time but new values.
// Reader: one 1024-thread block (block 0: XCD 0) loads the buffer k_ctrl's way (coalesced rounds of
// 1024 doubles, all in flight), sums it and stores the sum; its start-to-end time is taken from the
// constant 100 MHz clock by thread 0 around the loads and the barrier that follows them.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int NDBL = 9472;   // 74 KB of doubles
constexpr int RT = 1024;
constexpr int NR = (NDBL + RT - 1) / RT;

__global__ __launch_bounds__(256) void k_write(double* buf, int* xcc, int mode, int it) {
    // mode 0..7: only the block on XCD `mode` writes; mode 8: the eight blocks write one eighth each
    const int b = blockIdx.x;
    if (threadIdx.x == 0) xcc[b] = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15;
    const bool all = mode == 8;
    if (!all && b != mode) return;
    const int lo = all ? (NDBL * b) / 8 : 0, hi = all ? (NDBL * (b + 1)) / 8 : NDBL;
    for (int i = lo + threadIdx.x; i < hi; i += 256) buf[i] = (double)(i + it);
}

__global__ __launch_bounds__(RT) void k_read(const double* buf, double* out, unsigned long long* t, int it) {
    __shared__ double red[RT / 64];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double v[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int i = u * RT + threadIdx.x;
        v[u] = i < NDBL ? buf[i] : 0.0;
    }
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < NR; ++u) s += v[u];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        double a = 0.0;
        for (int w = 0; w < RT / 64; ++w) a += red[w];
        out[it] = a;
        t[it] = t1 - t0;
    }
}

int main() {
    const int iters = 200;
    double *buf, *out;
    unsigned long long* t;
    int* xcc;
    if (hipMalloc(&buf, NDBL * 8) || hipMalloc(&out, iters * 8) || hipMalloc(&t, iters * 8) || hipMalloc(&xcc, 64 * 4))
        return 1;
    hipMemset(buf, 0, NDBL * 8);
    const char* names[10] = {"XCD0 (reader's)", "XCD1", "XCD2", "XCD3", "XCD4", "XCD5", "XCD6", "XCD7",
                             "all 8 XCDs", "no writer"};
    for (int mode = 0; mode < 10; ++mode) {
        for (int it = 0; it < iters; ++it) {
            if (mode < 9) hipLaunchKernelGGL(k_write, dim3(8), dim3(256), 0, 0, buf, xcc, mode, it);
            hipLaunchKernelGGL(k_read, dim3(1), dim3(RT), 0, 0, buf, out, t, it);
        }
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        std::vector<unsigned long long> th(iters);
        std::vector<double> oh(iters);
        std::vector<int> xh(8);
        hipMemcpy(th.data(), t, iters * 8, hipMemcpyDeviceToHost);
        hipMemcpy(oh.data(), out, iters * 8, hipMemcpyDeviceToHost);
        hipMemcpy(xh.data(), xcc, 8 * 4, hipMemcpyDeviceToHost);
        bool ok = true;   // every read saw its own iteration's values (or, with no writer, the last ones)
        for (int it = 10; it < iters && mode < 9; ++it) {
            const double want = (double)NDBL * (NDBL - 1) / 2.0 + (double)NDBL * it;
            ok = ok && oh[it] == want;
        }
        std::sort(th.begin() + 10, th.end());
        const double med = th[10 + (iters - 10) / 2] * 0.01, p10 = th[10 + (iters - 10) / 10] * 0.01;
        printf("writer %-16s reader 74 KB: median %6.2f us  p10 %6.2f us  sums %s  xcc of blocks 0-7: %d %d %d %d %d %d %d %d\n",
               names[mode], med, p10, ok ? "ok" : "WRONG", xh[0], xh[1], xh[2], xh[3], xh[4], xh[5], xh[6], xh[7]);
    }
    return 0;
}
