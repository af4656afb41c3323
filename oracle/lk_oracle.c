/*
 * lk_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product): a plain-C restatement
 * of the reference's Gauss-Newton pyramidal LK optical flow, SURVEY.md 8(f) row 4:
 *   GetPixelValue            include/legoslam/algorithm.h:40-57
 *   calcLKOpticalFlow        src/algorithm.cpp:37-126   (one keypoint, one pyramid level)
 *   LKOpticalFlow1Layer      src/algorithm.cpp:11-31
 *   LKOpticalFlow4Layer      src/algorithm.cpp:128-206
 * and of the pyramid it builds with cv::resize(INTER_LINEAR) at scale 0.5 (algorithm.cpp:146-153;
 * OpenCV is absent here and its version is unpinned, imgproc/resize.cpp):
 *   - a level whose source has even width and height is exactly 2x smaller; cv::resize then
 *     switches INTER_LINEAR to the fast INTER_AREA path, whose 8-bit result is the rounded 2x2
 *     mean (a + b + c + d + 2) >> 2 (its scalar and SIMD paths agree);
 *   - otherwise it runs the generic fixed-point bilinear path: 11-bit coefficients from the
 *     float source offsets, int horizontal pass, vertical pass (v + (1 << 21)) >> 22.  This is the
 *     scalar formula; OpenCV's SSE2 vertical pass truncates differently and may differ by one gray
 *     level on such levels (parity there is unpinned).
 * Arithmetic follows the C++ types exactly (compile with -ffp-contract=off): GetPixelValue is
 * float, `kp.pt.x + x` is float and `+ dx` (double) promotes, error = float - float, J = 0.5 *
 * (float difference) in double, the 7x7 sums accumulate in double in the loop order (x outer, y
 * inner), and the 2x2 solve is Eigen's pivoted LDLT (orc_ldlt_solve).
 * Two reference behaviours are kept as written:
 *   - inverse mode: J is one variable, computed only at iteration 0 (algorithm.cpp:73-78), so from
 *     iteration 1 on every pixel of the patch uses the last pixel's J;
 *   - GetPixelValue reads data[1] / data[step] next to the clamped pixel (one past the row end, and
 *     past the image on its last row).  Such reads carry weight 0 except for x in (cols-1, cols):
 *     here they read the next byte of the image in memory order, and 0 past its end (the reference
 *     reads outside the buffer there).
 * The NaN/Inf message (algorithm.cpp:98) is not printed.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

void orc_ldlt_solve(const double *A, int n, const double *b, double *x);

typedef struct {
    const uint8_t *data;
    int32_t cols, rows;
    int64_t step;
} lk_img;

static inline int lk_byte(const lk_img *im, int64_t i) {
    return (i >= 0 && i < (int64_t)im->rows * im->step) ? im->data[i] : 0;
}

/* GetPixelValue (algorithm.h:40-57) */
static float lk_pixel(const lk_img *im, float x, float y) {
    if (x < 0) x = 0;
    if (y < 0) y = 0;
    if (x >= im->cols) x = im->cols - 1;
    if (y >= im->rows) y = im->rows - 1;
    const int64_t o = (int64_t)(int)y * im->step + (int)x;
    const float xx = x - floorf(x);
    const float yy = y - floorf(y);
    return (float)((1 - xx) * (1 - yy) * lk_byte(im, o) + xx * (1 - yy) * lk_byte(im, o + 1) +
                   (1 - xx) * yy * lk_byte(im, o + im->step) + xx * yy * lk_byte(im, o + im->step + 1));
}

/* cv::resize(src, dst, Size(cols * 0.5, rows * 0.5)), INTER_LINEAR, CV_8UC1 (see header) */
void orc_lk_pyr_down(const uint8_t *src, int32_t sw, int32_t sh, int64_t sstep, uint8_t *dst, int32_t dw, int32_t dh) {
    if (sw == 2 * dw && sh == 2 * dh) {
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x) {
                const uint8_t *s = src + (int64_t)(2 * y) * sstep + 2 * x;
                dst[(int64_t)y * dw + x] = (uint8_t)((s[0] + s[1] + s[sstep] + s[sstep + 1] + 2) >> 2);
            }
        return;
    }
    /* hal::resize: inv_scale = dsize / ssize, scale = 1 / inv_scale (not ssize / dsize) */
    const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
    int *xofs = (int *)malloc(sizeof(int) * (size_t)dw), *yofs = (int *)malloc(sizeof(int) * (size_t)dh);
    short *ax = (short *)malloc(sizeof(short) * 2 * (size_t)dw), *by = (short *)malloc(sizeof(short) * 2 * (size_t)dh);
    for (int d = 0; d < dw; ++d) {
        float f = (float)((d + 0.5) * scale_x - 0.5);
        int s = (int)floorf(f);
        f -= s;
        if (s < 0) { f = 0; s = 0; }
        if (s + 1 >= sw) { f = 0; s = sw - 1; }
        xofs[d] = s;
        ax[2 * d] = (short)lrintf((1.f - f) * 2048.f);
        ax[2 * d + 1] = (short)lrintf(f * 2048.f);
    }
    for (int d = 0; d < dh; ++d) {
        float f = (float)((d + 0.5) * scale_y - 0.5);
        int s = (int)floorf(f);
        f -= s;
        if (s < 0) { f = 0; s = 0; }
        if (s + 1 >= sh) { f = 0; s = sh - 1; }
        yofs[d] = s;
        by[2 * d] = (short)lrintf((1.f - f) * 2048.f);
        by[2 * d + 1] = (short)lrintf(f * 2048.f);
    }
    for (int y = 0; y < dh; ++y) {
        const int y0 = yofs[y], y1 = y0 + 1 < sh ? y0 + 1 : y0;
        for (int x = 0; x < dw; ++x) {
            const int x0 = xofs[x], x1 = x0 + 1 < sw ? x0 + 1 : x0;
            const int h0 = src[(int64_t)y0 * sstep + x0] * ax[2 * x] + src[(int64_t)y0 * sstep + x1] * ax[2 * x + 1];
            const int h1 = src[(int64_t)y1 * sstep + x0] * ax[2 * x] + src[(int64_t)y1 * sstep + x1] * ax[2 * x + 1];
            int v = (h0 * by[2 * y] + h1 * by[2 * y + 1] + (1 << 21)) >> 22;
            dst[(int64_t)y * dw + x] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
    free(xofs); free(yofs); free(ax); free(by);
}

/* LKOpticalFlowTracker::calcLKOpticalFlow for keypoint i (algorithm.cpp:37-126); kp2 holds the
   initial guess on entry (has_initial) and the result on exit */
static void lk_track_point(const lk_img *i1, const lk_img *i2, const float *kp1, float *kp2, uint8_t *success,
                           int inverse, int has_initial) {
    const int half_patch_size = 3, half_grad_step = 1, iterations = 10;
    const float kx = kp1[0], ky = kp1[1];
    double dx = 0, dy = 0;
    if (has_initial) {
        dx = kp2[0] - kx;
        dy = kp2[1] - ky;
    }
    double cost = 0, lastCost = 0;
    int succ = 1;
    double H[4] = {0, 0, 0, 0}, b[2] = {0, 0}, J[2] = {0, 0};
    for (int iter = 0; iter < iterations; ++iter) {
        if (!inverse) H[0] = H[1] = H[2] = H[3] = 0;
        b[0] = b[1] = 0;
        cost = 0;
        for (int x = -half_patch_size; x <= half_patch_size; ++x) {
            for (int y = -half_patch_size; y <= half_patch_size; ++y) {
                const float ax = kx + x, ay = ky + y;
                const double error = lk_pixel(i1, ax, ay) - lk_pixel(i2, (float)(ax + dx), (float)(ay + dy));
                if (!inverse) {
                    const double gx = 0.5 * (lk_pixel(i2, (float)(ax + dx + half_grad_step), (float)(ay + dy)) -
                                             lk_pixel(i2, (float)(ax + dx - half_grad_step), (float)(ay + dy)));
                    const double gy = 0.5 * (lk_pixel(i2, (float)(ax + dx), (float)(ay + dy + half_grad_step)) -
                                             lk_pixel(i2, (float)(ax + dx), (float)(ay + dy - half_grad_step)));
                    J[0] = -1.0 * gx;
                    J[1] = -1.0 * gy;
                } else if (iter == 0) {
                    const double gx = 0.5 * (lk_pixel(i1, ax + half_grad_step, ay) - lk_pixel(i1, ax - half_grad_step, ay));
                    const double gy = 0.5 * (lk_pixel(i1, ax, ay + half_grad_step) - lk_pixel(i1, ax, ay - half_grad_step));
                    J[0] = -1.0 * gx;
                    J[1] = -1.0 * gy;
                }
                b[0] += -error * J[0];
                b[1] += -error * J[1];
                cost += error * error;
                if (!inverse || iter == 0) {
                    H[0] += J[0] * J[0];
                    H[1] += J[0] * J[1];
                    H[2] += J[1] * J[0];
                    H[3] += J[1] * J[1];
                }
            }
        }
        double update[2];
        orc_ldlt_solve(H, 2, b, update);   /* H.ldlt().solve(b) */
        if (isnan(update[0]) || isnan(update[1]) || isinf(update[0]) || isinf(update[1])) {
            succ = 0;
            break;
        }
        if (iter > 0 && cost > lastCost) break;
        dx += update[0];
        dy += update[1];
        lastCost = cost;
        succ = 1;
        if (sqrt(update[0] * update[0] + update[1] * update[1]) < 1e-2) break;
    }
    *success = (uint8_t)succ;
    kp2[0] = kx + (float)dx;   /* kp.pt + cv::Point2f(dx, dy) */
    kp2[1] = ky + (float)dy;
    const double px = kp2[0], py = kp2[1];   /* IsPtInImg (algorithm.h:60-66) */
    if (px < 0 || py < 0 || px >= i2->cols || py >= i2->rows) *success = 0;
}

/* LKOpticalFlow4Layer (levels = 4, algorithm.cpp:128-206) or LKOpticalFlow1Layer (levels = 1).
   kp2: [n][2], the initial guess on entry when has_initial, the tracked points on exit. */
int orc_lk_track(const uint8_t *img1, const uint8_t *img2, int32_t cols, int32_t rows, int64_t step, int32_t n,
                 const float *kp1, float *kp2, uint8_t *success, int32_t inverse, int32_t has_initial, int32_t levels) {
    if (levels != 1 && levels != 4) return 2;
    if (cols < 1 || rows < 1 || step < cols || n < 0) return 2;
    enum { NL = 4 };
    lk_img p1[NL], p2[NL];
    uint8_t *own[2 * NL] = {0};
    p1[0] = (lk_img){img1, cols, rows, step};
    p2[0] = (lk_img){img2, cols, rows, step};
    for (int l = 1; l < levels; ++l) {
        const int w = (int)(p1[l - 1].cols * 0.5), h = (int)(p1[l - 1].rows * 0.5);
        if (w < 1 || h < 1) { for (int k = 0; k < 2 * NL; ++k) free(own[k]); return 2; }
        own[2 * l] = (uint8_t *)malloc((size_t)w * h);
        own[2 * l + 1] = (uint8_t *)malloc((size_t)w * h);
        orc_lk_pyr_down(p1[l - 1].data, p1[l - 1].cols, p1[l - 1].rows, p1[l - 1].step, own[2 * l], w, h);
        orc_lk_pyr_down(p2[l - 1].data, p2[l - 1].cols, p2[l - 1].rows, p2[l - 1].step, own[2 * l + 1], w, h);
        p1[l] = (lk_img){own[2 * l], w, h, w};
        p2[l] = (lk_img){own[2 * l + 1], w, h, w};
    }
    float *k1 = (float *)malloc(sizeof(float) * 2 * (size_t)(n > 0 ? n : 1));
    const double scale_top = levels == 4 ? 0.125 : 1.0;
    for (int i = 0; i < n; ++i) {   /* kp.pt *= scales[pyramids - 1]: saturate_cast<float>(x * s) */
        k1[2 * i] = (float)(kp1[2 * i] * scale_top);
        k1[2 * i + 1] = (float)(kp1[2 * i + 1] * scale_top);
        kp2[2 * i] = (float)(kp2[2 * i] * scale_top);
        kp2[2 * i + 1] = (float)(kp2[2 * i + 1] * scale_top);
    }
    for (int level = levels - 1; level >= 0; --level) {
        const int hi = (level == levels - 1) ? has_initial : 1;
        for (int i = 0; i < n; ++i) lk_track_point(&p1[level], &p2[level], k1 + 2 * i, kp2 + 2 * i, success + i, inverse, hi);
        if (level > 0) {
            for (int i = 0; i < n; ++i) {   /* pt /= pyramid_scale: saturate_cast<float>(x / 0.5) */
                k1[2 * i] = (float)(k1[2 * i] / 0.5);
                k1[2 * i + 1] = (float)(k1[2 * i + 1] / 0.5);
                if (success[i]) {
                    kp2[2 * i] = (float)(kp2[2 * i] / 0.5);
                    kp2[2 * i + 1] = (float)(kp2[2 * i + 1] / 0.5);
                } else {
                    kp2[2 * i] = k1[2 * i];
                    kp2[2 * i + 1] = k1[2 * i + 1];
                }
            }
        }
    }
    free(k1);
    for (int k = 0; k < 2 * NL; ++k) free(own[k]);
    return 0;
}
