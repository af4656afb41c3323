// Probe: accuracy of the raw v_rcp_f64 / v_rsq_f64 and of one Newton step, against 1/x and 1/sqrt(x)
// computed on the host in long double (rounded once to double).  Max and mean error in ulps.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_probe(const double* x, double* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = x[i];
    const double r = __builtin_amdgcn_rcp(d);
    const double r1 = fma(r, fma(-d, r, 1.0), r);
    const double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    const double y1 = y * fma(-h * y, y, 1.5);
    out[4 * i + 0] = r;
    out[4 * i + 1] = r1;
    out[4 * i + 2] = y;
    out[4 * i + 3] = y1;
}

static double ulp_err(double got, long double ref) {
    const double rd = (double)ref;
    const double u = std::nextafter(rd, INFINITY) - rd;
    return (double)std::fabs((long double)got - ref) / u;
}

int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), out(4 * (size_t)n);
    srand(11);
    for (int i = 0; i < n; ++i) {
        const double m = 1.0 + (double)rand() / RAND_MAX;
        const int e = (rand() % 121) - 60;   // 2^-60 .. 2^60
        x[i] = std::ldexp(m, e);
    }
    double *dx, *dout;
    if (hipMalloc(&dx, n * 8) || hipMalloc(&dout, 4 * (size_t)n * 8)) return 1;
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dout, n);
    hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost);
    double mx[4] = {0}, mean[4] = {0};
    for (int i = 0; i < n; ++i) {
        const long double rr = 1.0L / (long double)x[i], ry = 1.0L / std::sqrt((long double)x[i]);
        const long double ref[4] = {rr, rr, ry, ry};
        for (int k = 0; k < 4; ++k) {
            const double e = ulp_err(out[4 * (size_t)i + k], ref[k]);
            mx[k] = std::fmax(mx[k], e);
            mean[k] += e / n;
        }
    }
    printf("rcp raw: max %.3f mean %.3f ulp | rcp+1 Newton: max %.3f mean %.3f | rsq raw: max %.3f mean %.3f | rsq+1 Newton: max %.3f mean %.3f\n",
           mx[0], mean[0], mx[1], mean[1], mx[2], mean[2], mx[3], mean[3]);
    return 0;
}
