// Probe: the order in which one ds_add_f64 instruction applies the lanes that hit the same LDS address.
// Each lane adds a value whose rounding depends on the order; the result is compared with the
// sequential sums in ascending and descending lane order, over many launches.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_add(const double* v, const int* slot, double* out, int reps) {
    __shared__ double cell[64];
    const int lane = threadIdx.x;
    for (int r = 0; r < reps; ++r) {
        cell[lane] = 1.0;
        __syncthreads();
        atomicAdd(&cell[slot[lane]], v[r * 64 + lane]);
        __syncthreads();
        out[r * 64 + lane] = cell[lane];
        __syncthreads();
    }
}

int main() {
    const int reps = 2000;
    std::vector<double> v(reps * 64);
    std::vector<int> slot(64);
    srand(7);
    for (int i = 0; i < reps * 64; ++i) v[i] = ((rand() % 2) ? 1e16 : 1.0) * ((rand() % 1000) + 1) * 1.0000001;
    for (int l = 0; l < 64; ++l) slot[l] = (l * 5 + 3) % 8;   // 8 lanes per address, interleaved
    double *dv, *dout; int* ds;
    if (hipMalloc(&dv, v.size() * 8) || hipMalloc(&dout, v.size() * 8) || hipMalloc(&ds, 64 * 4)) return 1;
    hipMemcpy(dv, v.data(), v.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(ds, slot.data(), 64 * 4, hipMemcpyHostToDevice);
    std::vector<double> out(v.size());
    int asc = 0, desc = 0, other = 0, runs = 0, diffrun = 0;
    std::vector<double> first;
    for (int launch = 0; launch < 20; ++launch) {
        hipLaunchKernelGGL(k_add, dim3(1), dim3(64), 0, 0, dv, ds, dout, reps);
        hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
        if (launch == 0) first = out; else diffrun += (out != first);
        for (int r = 0; r < reps; ++r)
            for (int c = 0; c < 8; ++c) {
                double a = 1.0, d = 1.0;
                for (int l = 0; l < 64; ++l) if (slot[l] == c) a += v[r * 64 + l];
                for (int l = 63; l >= 0; --l) if (slot[l] == c) d += v[r * 64 + l];
                const double g = out[r * 64 + c];
                ++runs;
                if (g == a) ++asc; else if (g == d) ++desc; else ++other;
            }
    }
    printf("cells %d: ascending-lane order %d, descending %d, other %d; launches differing from the first: %d\n",
           runs, asc, desc, other, diffrun);
    return 0;
}
