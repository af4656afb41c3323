/*
 * lh_window.h — deterministic synthetic sliding-window generator for the
 * LEGO-SLAM bundle-adjustment backend (SURVEY.md §8(d) "Synthetic windows").
 *
 * The reference has no fixtures for Backend::Optimize, so every
 * window used by tests and bench.py comes from this generator.  It is
 * counter-based: every landmark draws from its own random stream, so any
 * landmark range [lm_begin, lm_end) of a window can be generated on its own
 * (that is how bench.py shards a window across ranks without materialising it).
 *
 * Conventions follow the reference:
 *   - poses are T_cw (world -> camera), stored row-major [R | t] (12 doubles),
 *     as Frame::pose_ is (include/legoslam/frame.h:49-56);
 *   - camera c maps a camera-0 point p to ext_c * p, ext_0 = identity and
 *     ext_1 = (I, (-baseline, 0, 0)) as Dataset::Init builds them
 *     (src/dataset.cpp:36-42);
 *   - pixels are float32 values widened to double, as toVec2 does
 *     (include/legoslam/algorithm.h:37).
 */
#ifndef LH_WINDOW_H
#define LH_WINDOW_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lhw_params {
    int32_t n_poses;          /* P keyframes                                  */
    int32_t n_landmarks;      /* L landmarks in the whole window              */
    int32_t k_min, k_max;     /* observations per landmark, uniform in range  */
    int32_t pose_mode;        /* 0: contiguous run of KFs, 1: random subset   */
    uint64_t seed;
    double noise_px;          /* measurement noise sigma (px)                 */
    double outlier_frac;      /* gross outliers, uniform in the image         */
    double right_frac;        /* fraction of obs on camera 1 (right image)    */
    double baseline;          /* camera-1 baseline (m)                        */
    double step_m;            /* forward motion per keyframe (m, +z)          */
    double yaw_sigma;         /* per-KF yaw (rad)                             */
    double depth_min, depth_max;
    double pose_rot_sigma;    /* initial-guess perturbation of poses (rad)    */
    double pose_trans_sigma;  /* (m)                                          */
    double lm_sigma;          /* initial-guess perturbation of landmarks (m)  */
    double K[4];              /* fx, fy, cx, cy                               */
    double width, height;     /* image size (px)                              */
} lhw_params;

/* Fill `p` with the SURVEY.md §8(d) defaults (C3-shaped: P=20, L=50000, k=8). */
void lhw_default_params(lhw_params *p);

/* Number of observations landmarks [lm_begin, lm_end) produce. */
int64_t lhw_count_obs(const lhw_params *p, int32_t lm_begin, int32_t lm_end);

/* Poses: true and initial-guess T_cw, [n_poses][12] each (either may be NULL). */
void lhw_poses(const lhw_params *p, double *pose_true, double *pose_init);

/* Cameras: [2][12] extrinsics (camera 0 identity, camera 1 right). */
void lhw_cameras(const lhw_params *p, double *cam_ext);

/*
 * Landmarks [lm_begin, lm_end) and their observations, landmark-major, each
 * landmark's observations in ascending pose order.  obs_lm is relative to
 * lm_begin.  Arrays must hold lhw_count_obs(...) observations.
 * Returns the number of observations written.
 */
int64_t lhw_landmarks(const lhw_params *p, int32_t lm_begin, int32_t lm_end,
                      double *lm_true, double *lm_init,
                      uint32_t *obs_pose, uint32_t *obs_lm, uint8_t *obs_cam,
                      double *obs_uv);

#ifdef __cplusplus
}
#endif
#endif
