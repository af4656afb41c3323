// lh_lk.hip — CDNA4 (gfx950) kernels of the reference's Gauss-Newton pyramidal LK optical flow
// (src/algorithm.cpp:11-206, include/legoslam/algorithm.h:40-66):
//   k_lk_pyr    one pyramid level of one image, cv::resize(INTER_LINEAR, scale 0.5) as
//               oracle/lk_oracle.c restates it (2x exact: rounded 2x2 mean; otherwise the fixed-
//               point bilinear path), one thread per output pixel;
//   k_lk_track  LKOpticalFlow4Layer / LKOpticalFlow1Layer: one wave per keypoint runs every level
//               coarse to fine.  Lane p < 49 owns patch pixel (x, y) = (p / 7 - 3, p % 7 - 3), the
//               reference's loop order (x outer, y inner).  Per Gauss-Newton iteration each lane
//               evaluates its error and Jacobian (GetPixelValue in float, as written); the six
//               double sums (b, cost, H) are then formed sequentially in that pixel order by every
//               lane from LDS, so every decision of the loop (NaN step, cost increase, |dx| < 1e-2)
//               is taken on bitwise the reference's values and control flow stays wave-uniform.
// The arithmetic is a bitwise mirror of the oracle with contraction off.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "lh_lk.h"

#pragma clang fp contract(off)

namespace {

struct Img {
    const uint8_t* data;
    int32_t cols, rows;
    int64_t step;
};

__device__ __forceinline__ int lk_byte(const Img& im, int64_t i) {
    return (i >= 0 && i < (int64_t)im.rows * im.step) ? (int)im.data[i] : 0;
}

// GetPixelValue (algorithm.h:40-57), float arithmetic in the reference's order
__device__ __forceinline__ float lk_pixel(const Img& im, float x, float y) {
    if (x < 0) x = 0;
    if (y < 0) y = 0;
    if (x >= im.cols) x = im.cols - 1;
    if (y >= im.rows) y = im.rows - 1;
    const int64_t o = (int64_t)(int)y * im.step + (int)x;
    const float xx = x - floorf(x);
    const float yy = y - floorf(y);
    return (float)((1 - xx) * (1 - yy) * lk_byte(im, o) + xx * (1 - yy) * lk_byte(im, o + 1) +
                   (1 - xx) * yy * lk_byte(im, o + im.step) + xx * yy * lk_byte(im, o + im.step + 1));
}

// The same sample with its four bytes read from an LDS copy of the image when the taps fall inside it.
// The window holds win[r][c] = lk_byte(im, (wy0 + r) * step + wx0 + c): bytes by linear index, so
// tap o + 1 is column c + 1 even where it wraps into the next image row (as the reference's does)
// and out-of-buffer taps are the same zeros.  Taps outside it read global memory.
#define LK_WW 32
#define LK_WH 24
__device__ __forceinline__ float lk_pixel_w(const Img& im, const uint8_t* win, int wx0, int wy0, float x, float y) {
    if (x < 0) x = 0;
    if (y < 0) y = 0;
    if (x >= im.cols) x = im.cols - 1;
    if (y >= im.rows) y = im.rows - 1;
    const int xi = (int)x, yi = (int)y;
    const float xx = x - floorf(x);
    const float yy = y - floorf(y);
    const int c = xi - wx0, r = yi - wy0;
    int b00, b01, b10, b11;
    if ((unsigned)c < LK_WW - 1 && (unsigned)r < LK_WH - 1) {
        const uint8_t* q = win + r * LK_WW + c;
        b00 = q[0];
        b01 = q[1];
        b10 = q[LK_WW];
        b11 = q[LK_WW + 1];
    } else {
        const int64_t o = (int64_t)yi * im.step + xi;
        b00 = lk_byte(im, o);
        b01 = lk_byte(im, o + 1);
        b10 = lk_byte(im, o + im.step);
        b11 = lk_byte(im, o + im.step + 1);
    }
    return (float)((1 - xx) * (1 - yy) * b00 + xx * (1 - yy) * b01 + (1 - xx) * yy * b10 + xx * yy * b11);
}

// Eigen Matrix2d::ldlt().solve(b): the oracle's ldlt_solve (Eigen ldlt_inplace with diagonal
// pivoting + LDLT::_solve_impl) for n = 2, operation for operation
__device__ __forceinline__ void ldlt2_solve(const double H[4], const double b[2], double x[2]) {
    double A[4] = {H[0], H[1], H[2], H[3]};   // row-major; the lower triangle is used
    int tr[2] = {0, 1};
    bool all_zero = false;
    (void)all_zero;
    // k = 0: pivot on the larger |diagonal|
    {
        int idx = 0;
        double big = fabs(A[0]);
        if (fabs(A[3]) > big) { big = fabs(A[3]); idx = 1; }
        tr[0] = idx;
        if (idx != 0) { const double t = A[0]; A[0] = A[3]; A[3] = t; }
        const double akk = A[0];
        const bool valid = fabs(akk) > 0.0;
        if (!valid) {
            tr[0] = 0;
            tr[1] = 1;
            all_zero = true;
        } else {
            A[2] /= akk;
            // k = 1
            tr[1] = 1;
            const double temp0 = A[0] * A[2];
            const double s = 0.0 + A[2] * temp0;   // the oracle's dot product, from 0.0
            A[3] -= s;
        }
    }
    x[0] = b[0];
    x[1] = b[1];
    if (tr[0] != 0) { const double t = x[0]; x[0] = x[1]; x[1] = t; }
    // L solve (Eigen triangular_solve_vector semantics, oracle/lego_oracle.c ldlt_solve)
    if (x[0] != 0.0) x[1] -= A[2] * x[0];
    const double tol = 2.2250738585072014e-308;
    x[0] = fabs(A[0]) > tol ? x[0] / A[0] : 0.0;
    x[1] = fabs(A[3]) > tol ? x[1] / A[3] : 0.0;
    x[0] -= A[2] * x[1];
    if (tr[0] != 0) { const double t = x[0]; x[0] = x[1]; x[1] = t; }
}

}  // namespace

// ---- one pyramid level of one image ----
__global__ __launch_bounds__(256) void k_lk_pyr(const uint8_t* __restrict__ src, int sw, int sh, int64_t sstep,
                                                uint8_t* __restrict__ dst, int dw, int dh) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)dw * dh) return;
    const int y = (int)(i / dw), x = (int)(i - (int64_t)y * dw);
    if (sw == 2 * dw && sh == 2 * dh) {   // INTER_AREA fast path
        const uint8_t* s = src + (int64_t)(2 * y) * sstep + 2 * x;
        dst[i] = (uint8_t)((s[0] + s[1] + s[sstep] + s[sstep + 1] + 2) >> 2);
        return;
    }
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    float fx = (float)((x + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx + 1 >= sw) { fx = 0; sx = sw - 1; }
    float fy = (float)((y + 0.5) * scale_y - 0.5);
    int sy = (int)floorf(fy);
    fy -= sy;
    if (sy < 0) { fy = 0; sy = 0; }
    if (sy + 1 >= sh) { fy = 0; sy = sh - 1; }
    const int a0 = (int)rintf((1.f - fx) * 2048.f), a1 = (int)rintf(fx * 2048.f);
    const int b0 = (int)rintf((1.f - fy) * 2048.f), b1 = (int)rintf(fy * 2048.f);
    const int x1 = sx + 1 < sw ? sx + 1 : sx, y1 = sy + 1 < sh ? sy + 1 : sy;
    const int h0 = src[(int64_t)sy * sstep + sx] * a0 + src[(int64_t)sy * sstep + x1] * a1;
    const int h1 = src[(int64_t)y1 * sstep + sx] * a0 + src[(int64_t)y1 * sstep + x1] * a1;
    const int v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
    dst[i] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// ---- LKOpticalFlow{4,1}Layer, one wave per keypoint ----
#define LKW 4   // keypoints (waves) per workgroup
#define LK_TROW 66

__device__ __forceinline__ double lk_readlane(double v, int l) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__global__ __launch_bounds__(64 * LKW) void k_lk_track(lh_lk_levels L1, lh_lk_levels L2, int levels, int n,
                                                       const float* __restrict__ kp1, const float* __restrict__ kp2_in,
                                                       float* __restrict__ kp2_out, uint8_t* __restrict__ success,
                                                       int inverse, int has_initial) {
    // row stride 66 doubles: 16-byte aligned rows, and the six summing lanes (one row each) hit
    // banks 4 apart
    __shared__ double terms[LKW][6][LK_TROW];
    __shared__ uint8_t window[LKW][LK_WH * LK_WW];   // the second image around this level's guess
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = blockIdx.x * LKW + w;
    if (i >= n) return;   // wave-uniform: no barrier below spans waves
    const int px = lane / 7 - 3, py = lane - 7 * (lane / 7) - 3;
    const bool act = lane < 49;
    double (*T)[LK_TROW] = terms[w];
    uint8_t* win = window[w];

    const double scale_top = levels == 4 ? 0.125 : 1.0;
    float k1x = (float)(kp1[2 * i] * scale_top), k1y = (float)(kp1[2 * i + 1] * scale_top);
    float k2x = (float)(kp2_in[2 * i] * scale_top), k2y = (float)(kp2_in[2 * i + 1] * scale_top);
    int succ = 1;
    for (int level = levels - 1; level >= 0; --level) {
        const Img i1 = {L1.data[level], L1.cols[level], L1.rows[level], L1.step[level]};
        const Img i2 = {L2.data[level], L2.cols[level], L2.rows[level], L2.step[level]};
        const int hi = (level == levels - 1) ? has_initial : 1;
        // ---- calcLKOpticalFlow (algorithm.cpp:37-126) ----
        double dx = 0, dy = 0;
        if (hi) {
            dx = k2x - k1x;
            dy = k2y - k1y;
        }
        double cost = 0, lastCost = 0;
        succ = 1;
        double H[4] = {0, 0, 0, 0};
        double Jlast0 = 0, Jlast1 = 0;   // inverse mode: the J variable after iteration 0 (last pixel's)
        const float ax = k1x + px, ay = k1y + py;
        const float v1 = act ? lk_pixel(i1, ax, ay) : 0.f;   // the template sample is loop-invariant
        // stage i2 around the initial guess: the iterations' taps stay inside while |dx - dx0| <= 11
        // and |dy - dy0| <= 7 pixels (placement only decides which taps come from LDS, not values)
        const int wx0 = (int)floorf(fminf(fmaxf((float)(k1x + dx), -1e6f), 1e6f)) - 15;
        const int wy0 = (int)floorf(fminf(fmaxf((float)(k1y + dy), -1e6f), 1e6f)) - 11;
#pragma unroll
        for (int k = 0; k < LK_WH * LK_WW / 64; ++k) {
            const int idx = k * 64 + lane;
            win[idx] = (uint8_t)lk_byte(i2, (int64_t)(wy0 + idx / LK_WW) * i2.step + wx0 + idx % LK_WW);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int iter = 0; iter < 10; ++iter) {
            double e = 0, J0 = 0, J1 = 0;
            if (act) {
                e = v1 - lk_pixel_w(i2, win, wx0, wy0, (float)(ax + dx), (float)(ay + dy));
                if (!inverse) {
                    const double gx = 0.5 * (lk_pixel_w(i2, win, wx0, wy0, (float)(ax + dx + 1), (float)(ay + dy)) -
                                             lk_pixel_w(i2, win, wx0, wy0, (float)(ax + dx - 1), (float)(ay + dy)));
                    const double gy = 0.5 * (lk_pixel_w(i2, win, wx0, wy0, (float)(ax + dx), (float)(ay + dy + 1)) -
                                             lk_pixel_w(i2, win, wx0, wy0, (float)(ax + dx), (float)(ay + dy - 1)));
                    J0 = -1.0 * gx;
                    J1 = -1.0 * gy;
                } else if (iter == 0) {
                    const double gx = 0.5 * (lk_pixel(i1, ax + 1, ay) - lk_pixel(i1, ax - 1, ay));
                    const double gy = 0.5 * (lk_pixel(i1, ax, ay + 1) - lk_pixel(i1, ax, ay - 1));
                    J0 = -1.0 * gx;
                    J1 = -1.0 * gy;
                } else {
                    J0 = Jlast0;
                    J1 = Jlast1;
                }
            }
            const bool hterm = !inverse || iter == 0;
            T[0][lane] = -e * J0;
            T[1][lane] = -e * J1;
            T[2][lane] = e * e;
            T[3][lane] = J0 * J0;
            T[4][lane] = J0 * J1;
            T[5][lane] = J1 * J1;
            if (inverse && iter == 0) {   // the last pixel's J stays in the reference's variable
                Jlast0 = __shfl(J0, 48);
                Jlast1 = __shfl(J1, 48);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // the patch loop's sums, in pixel order: lane k < 6 runs sum k sequentially from 0.0
            // (b0, b1, cost, H00, H01, H11).  H starts at 0.0 in each level, so inverse mode's
            // "H += ..." at iteration 0 is this same sum, and later iterations keep H.
            double acc = 0.0;
            if (lane < 6) {
                const double* row = T[lane];
#pragma unroll
                for (int p = 0; p < 49; ++p) acc += row[p];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double b0 = lk_readlane(acc, 0), b1 = lk_readlane(acc, 1);
            cost = lk_readlane(acc, 2);
            if (hterm) {
                const double h00 = lk_readlane(acc, 3), h01 = lk_readlane(acc, 4), h11 = lk_readlane(acc, 5);
                H[0] = h00; H[1] = h01; H[2] = h01; H[3] = h11;   // J1 * J0 == J0 * J1 bitwise
            }
            const double bb[2] = {b0, b1};
            double u[2];
            ldlt2_solve(H, bb, u);
            if (isnan(u[0]) || isnan(u[1]) || isinf(u[0]) || isinf(u[1])) {
                succ = 0;
                break;
            }
            if (iter > 0 && cost > lastCost) break;
            dx += u[0];
            dy += u[1];
            lastCost = cost;
            succ = 1;
            if (sqrt(u[0] * u[0] + u[1] * u[1]) < 1e-2) break;
        }
        k2x = k1x + (float)dx;
        k2y = k1y + (float)dy;
        {
            const double qx = k2x, qy = k2y;   // IsPtInImg (algorithm.h:60-66)
            if (qx < 0 || qy < 0 || qx >= i2.cols || qy >= i2.rows) succ = 0;
        }
        if (level > 0) {   // LKOpticalFlow4Layer: pt /= pyramid_scale
            k1x = (float)(k1x / 0.5);
            k1y = (float)(k1y / 0.5);
            if (succ) {
                k2x = (float)(k2x / 0.5);
                k2y = (float)(k2y / 0.5);
            } else {
                k2x = k1x;
                k2y = k1y;
            }
        }
    }
    if (lane == 0) {
        kp2_out[2 * i] = k2x;
        kp2_out[2 * i + 1] = k2y;
        success[i] = (uint8_t)succ;
    }
}

extern "C" {

hipError_t lh_launch_lk_pyr(hipStream_t st, const uint8_t* src, int sw, int sh, int64_t sstep, uint8_t* dst, int dw,
                            int dh) {
    const int64_t np = (int64_t)dw * dh;
    if (np <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_lk_pyr, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, src, sw, sh, sstep, dst, dw, dh);
    return hipGetLastError();
}

hipError_t lh_launch_lk_track(hipStream_t st, const lh_lk_levels* L1, const lh_lk_levels* L2, int levels, int n,
                              const float* kp1, const float* kp2_in, float* kp2_out, uint8_t* success, int inverse,
                              int has_initial) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_lk_track, dim3((unsigned)((n + LKW - 1) / LKW)), dim3(64 * LKW), 0, st, *L1, *L2, levels, n,
                       kp1, kp2_in, kp2_out, success, inverse, has_initial);
    return hipGetLastError();
}

}  // extern "C"
