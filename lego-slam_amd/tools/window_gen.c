/*
 * window_gen.c — synthetic LEGO-SLAM BA windows (see lh_window.h).
 *
 * Geometry: a stereo rig moving step_m per keyframe along
 * +z with a small random yaw per keyframe; landmarks 8–60 m in front of the
 * keyframe in the middle of their observation run; pinhole projection
 * u = fx*X/Z + cx, v = fy*Y/Z + cy (Camera::camera2pixel, src/camera.cpp:17-20);
 * N(0, noise_px^2) noise, float32 rounding and a fraction of gross outliers
 * uniform in the image (they exercise the Huber kernel, cost_function.cpp:5-17).
 */
#include "lh_window.h"

#include <math.h>
#include <string.h>

/* exported C symbols: the generator is loaded by Python through ctypes */

/* ---- counter-based RNG: splitmix64 over (seed, stream, counter) ---------- */
typedef struct { uint64_t s; } rng_t;

static uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static rng_t rng_stream(uint64_t seed, uint64_t stream) {
    rng_t r;
    r.s = mix64(seed * 0xD1B54A32D192ED03ull + mix64(stream + 0x632BE59BD9B4E019ull));
    return r;
}
static uint64_t rng_next(rng_t *r) { r->s += 0x9E3779B97F4A7C15ull; return mix64(r->s); }
static double rng_uniform(rng_t *r) { return (double)(rng_next(r) >> 11) * 0x1.0p-53; }
static double rng_normal(rng_t *r) {
    double u1 = 1.0 - rng_uniform(r); /* (0, 1] */
    double u2 = rng_uniform(r);
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}
static int32_t rng_int(rng_t *r, int32_t lo, int32_t hi) { /* inclusive */
    uint64_t span = (uint64_t)(hi - lo + 1);
    return lo + (int32_t)(rng_next(r) % span);
}

#define STREAM_POSES 0xFFFFFFFF00000001ull

/* ---- small rigid-body helpers ------------------------------------------- */
static void rot_exp(const double w[3], double R[9]) { /* Rodrigues */
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double th = sqrt(th2);
    double a, b;
    if (th < 1e-12) { a = 1.0; b = 0.5; }
    else { a = sin(th) / th; b = (1.0 - cos(th)) / th2; }
    double K[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double K2[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0;
            for (int m = 0; m < 3; ++m) s += K[3 * i + m] * K[3 * m + j];
            K2[3 * i + j] = s;
        }
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * K[i] + b * K2[i];
}
static void mat3_mul(const double A[9], const double B[9], double C[9]) {
    double T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
    memcpy(C, T, sizeof(T));
}
static void apply(const double T[12], const double X[3], double Y[3]) {
    for (int i = 0; i < 3; ++i)
        Y[i] = T[4 * i] * X[0] + T[4 * i + 1] * X[1] + T[4 * i + 2] * X[2] + T[4 * i + 3];
}

void lhw_default_params(lhw_params *p) {
    memset(p, 0, sizeof(*p));
    p->n_poses = 20;
    p->n_landmarks = 50000;
    p->k_min = p->k_max = 8;
    p->pose_mode = 0;
    p->seed = 0;
    p->noise_px = 1.0;
    p->outlier_frac = 0.02;
    p->right_frac = 0.0;
    p->baseline = 0.537;
    p->step_m = 1.0;
    p->yaw_sigma = 0.02;
    p->depth_min = 8.0;
    p->depth_max = 60.0;
    p->pose_rot_sigma = 0.01;
    p->pose_trans_sigma = 0.05;
    p->lm_sigma = 0.1;
    p->K[0] = 517.3; p->K[1] = 516.5; p->K[2] = 325.1; p->K[3] = 249.7; /* config/kitti_00.yaml:10-13 */
    p->width = 640.0;
    p->height = 480.0;
}

/* True T_cw of keyframe i: centre (0, 0, i*step), yaw psi_i about +y. */
static void true_pose(const lhw_params *p, int32_t i, double T[12]) {
    rng_t r = rng_stream(p->seed, STREAM_POSES + 2ull * (uint64_t)i);
    double psi = p->yaw_sigma * rng_normal(&r);
    double pitch = 0.25 * p->yaw_sigma * rng_normal(&r);
    double w[3] = {pitch, psi, 0.0};
    double Rwc[9];
    rot_exp(w, Rwc);
    double c[3] = {0.0, 0.0, (double)i * p->step_m};
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) T[4 * a + b] = Rwc[3 * b + a]; /* R_cw = R_wc^T */
        T[4 * a + 3] = -(Rwc[a] * c[0] + Rwc[3 + a] * c[1] + Rwc[6 + a] * c[2]);
    }
}

void lhw_poses(const lhw_params *p, double *pose_true, double *pose_init) {
    for (int32_t i = 0; i < p->n_poses; ++i) {
        double T[12];
        true_pose(p, i, T);
        if (pose_true) memcpy(pose_true + 12 * i, T, sizeof(T));
        if (pose_init) {
            rng_t r = rng_stream(p->seed, STREAM_POSES + 2ull * (uint64_t)i + 1ull);
            double w[3], dt[3], dR[9], R[9];
            for (int a = 0; a < 3; ++a) w[a] = p->pose_rot_sigma * rng_normal(&r);
            for (int a = 0; a < 3; ++a) dt[a] = p->pose_trans_sigma * rng_normal(&r);
            rot_exp(w, dR);
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) R[3 * a + b] = T[4 * a + b];
            mat3_mul(dR, R, R); /* left-multiplicative perturbation, as VertexPose::add */
            double t[3] = {T[3], T[7], T[11]};
            double *o = pose_init + 12 * i;
            for (int a = 0; a < 3; ++a) {
                for (int b = 0; b < 3; ++b) o[4 * a + b] = R[3 * a + b];
                o[4 * a + 3] = dR[3 * a] * t[0] + dR[3 * a + 1] * t[1] + dR[3 * a + 2] * t[2] + dt[a];
            }
        }
    }
}

void lhw_cameras(const lhw_params *p, double *cam_ext) {
    memset(cam_ext, 0, 24 * sizeof(double));
    for (int c = 0; c < 2; ++c) {
        cam_ext[12 * c + 0] = cam_ext[12 * c + 5] = cam_ext[12 * c + 10] = 1.0;
    }
    cam_ext[12 + 3] = -p->baseline;
}

static int32_t lm_k(const lhw_params *p, int32_t l) {
    if (p->k_max <= p->k_min) return p->k_min;
    rng_t r = rng_stream(p->seed, 3ull * (uint64_t)l + 7ull);
    return rng_int(&r, p->k_min, p->k_max);
}

int64_t lhw_count_obs(const lhw_params *p, int32_t lm_begin, int32_t lm_end) {
    int64_t n = 0;
    for (int32_t l = lm_begin; l < lm_end; ++l) {
        int32_t k = lm_k(p, l);
        if (k > p->n_poses) k = p->n_poses;
        n += k;
    }
    return n;
}

int64_t lhw_landmarks(const lhw_params *p, int32_t lm_begin, int32_t lm_end,
                      double *lm_true, double *lm_init,
                      uint32_t *obs_pose, uint32_t *obs_lm, uint8_t *obs_cam,
                      double *obs_uv) {
    const int32_t P = p->n_poses;
    double Tall[12 * 256];
    double *T = Tall;
    if (P > 256) return -1;
    for (int32_t i = 0; i < P; ++i) true_pose(p, i, T + 12 * i);
    double ext1[12] = {1, 0, 0, -p->baseline, 0, 1, 0, 0, 0, 0, 1, 0};

    int64_t o = 0;
    int32_t poses[256];
    for (int32_t l = lm_begin; l < lm_end; ++l) {
        int32_t k = lm_k(p, l);
        if (k > P) k = P;
        rng_t r = rng_stream(p->seed, 3ull * (uint64_t)l + 8ull);
        /* pose set, ascending */
        if (p->pose_mode == 0) {
            int32_t s = rng_int(&r, 0, P - k);
            for (int32_t j = 0; j < k; ++j) poses[j] = s + j;
        } else {
            /* random k-subset by partial Fisher-Yates, then sort */
            int32_t all[256];
            for (int32_t j = 0; j < P; ++j) all[j] = j;
            for (int32_t j = 0; j < k; ++j) {
                int32_t q = rng_int(&r, j, P - 1);
                int32_t t = all[j]; all[j] = all[q]; all[q] = t;
            }
            for (int32_t j = 0; j < k; ++j) poses[j] = all[j];
            for (int32_t a = 1; a < k; ++a) {
                int32_t v = poses[a], b = a - 1;
                while (b >= 0 && poses[b] > v) { poses[b + 1] = poses[b]; --b; }
                poses[b + 1] = v;
            }
        }
        /* position: pixel + depth in the middle keyframe of the run, retried
           until it projects inside the image with depth > 1 m in every KF */
        const double *Tm = T + 12 * poses[k / 2];
        double Xw[3] = {0, 0, 0};
        for (int attempt = 0; attempt < 64; ++attempt) {
            double u = rng_uniform(&r) * p->width, v = rng_uniform(&r) * p->height;
            double d = p->depth_min + (p->depth_max - p->depth_min) * rng_uniform(&r);
            double pc[3] = {(u - p->K[2]) * d / p->K[0], (v - p->K[3]) * d / p->K[1], d};
            /* X_w = R^T (pc - t) */
            double q[3] = {pc[0] - Tm[3], pc[1] - Tm[7], pc[2] - Tm[11]};
            for (int a = 0; a < 3; ++a) Xw[a] = Tm[a] * q[0] + Tm[4 + a] * q[1] + Tm[8 + a] * q[2];
            int ok = 1;
            for (int32_t j = 0; j < k && ok; ++j) {
                double y[3];
                apply(T + 12 * poses[j], Xw, y);
                if (y[2] < 1.0) { ok = 0; break; }
                double uu = p->K[0] * y[0] / y[2] + p->K[2], vv = p->K[1] * y[1] / y[2] + p->K[3];
                if (uu < 0 || uu >= p->width || vv < 0 || vv >= p->height) ok = 0;
            }
            if (ok) break;
        }
        int32_t li = l - lm_begin;
        if (lm_true) for (int a = 0; a < 3; ++a) lm_true[3 * li + a] = Xw[a];
        if (lm_init) for (int a = 0; a < 3; ++a) lm_init[3 * li + a] = Xw[a] + p->lm_sigma * rng_normal(&r);
        for (int32_t j = 0; j < k; ++j) {
            int cam = (p->right_frac > 0 && rng_uniform(&r) < p->right_frac) ? 1 : 0;
            double y[3];
            apply(T + 12 * poses[j], Xw, y);
            if (cam == 1) apply(ext1, y, y);
            double uu = p->K[0] * y[0] / y[2] + p->K[2] + p->noise_px * rng_normal(&r);
            double vv = p->K[1] * y[1] / y[2] + p->K[3] + p->noise_px * rng_normal(&r);
            if (rng_uniform(&r) < p->outlier_frac) {
                uu = rng_uniform(&r) * p->width;
                vv = rng_uniform(&r) * p->height;
            }
            if (obs_pose) obs_pose[o] = (uint32_t)poses[j];
            if (obs_lm) obs_lm[o] = (uint32_t)li;
            if (obs_cam) obs_cam[o] = (uint8_t)cam;
            if (obs_uv) {
                obs_uv[2 * o] = (double)(float)uu; /* cv::KeyPoint is float (feature.h:32) */
                obs_uv[2 * o + 1] = (double)(float)vv;
            }
            ++o;
        }
    }
    return o;
}
