/*
 * lego_ba.h — C ABI of the MI355X sliding-window bundle-adjustment solver.
 *
 * Drop-in boundary for LEGO-SLAM's backend optimisation.
 * The reference builds a `lego::Problem` inside `Backend::Optimize`
 * (src/backend_lego.cpp:57-158), calls `problem.solve(10)` (:161) and then reads
 * each edge's robust chi2 and the vertex estimates back (:163-217).  This ABI
 * replaces exactly that block with one call:
 *
 *     reference                                   this ABI
 *     ---------------------------------------     ----------------------------
 *     lego::Problem problem(SLAM)  problem.h:53   lh_create
 *     addVertex / addEdge          problem.h:65,69 lh_window (flat arrays)
 *     setInitialLambda             problem.h:99   lh_options.lambda_init
 *     setVerbose                   problem.h:104  lh_options.verbose
 *     setStrategyType              problem.h:62   lh_options.strategy
 *     solve(iterations)            problem.cpp:156 lh_solve
 *     edge->getRobustChi2()        base_edge.cpp:33 lh_result.edge_robust_chi2
 *     vertex->getEstimate()        base_vertex.h:34 lh_result.pose_Tcw / lm_xyz
 *     outlier threshold loop       backend_lego.cpp:163-194 lh_result.is_outlier (on the device, ABI 5)
 *                                                                  or lh_classify_outliers (host, on edge_robust_chi2)
 *     Frontend::EstimateCurrentPose frontend_lego.cpp:157-250 lh_estimate_pose (batched)
 *     LKOpticalFlow4Layer / 1Layer  algorithm.cpp:11-206      lh_lk_track
 *     ~Problem                     problem.cpp:32 lh_destroy
 *
 * Plain C types only (no torch, Eigen or Sophus in any signature).  No C++
 * exception crosses the ABI; every entry point returns an lh_status.
 * A handle is single-threaded; use one handle per calling thread (the
 * reference runs one Problem on the backend thread and one on the frontend
 * thread).  Handles share no global state (the reference's global_vertex_id /
 * global_edge_id counters, base_vertex.cpp:5 / base_edge.cpp:6, have no analogue).
 */
#ifndef LEGO_BA_H
#define LEGO_BA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LH_ABI_VERSION 5   /* lh_create accepts 4 and 5; the lh_result fields marked ABI 5 are read only at 5 */

typedef enum lh_status {
    LH_OK = 0,
    LH_E_EMPTY = 1,       /* no vertices or no edges: Problem::solve returns false (problem.cpp:157-161) */
    LH_E_BADARG = 2,      /* null pointer, index out of range, bad option                              */
    LH_E_HIP = 3,         /* HIP runtime error (device missing, OOM, launch failure)                    */
    LH_E_RCCL = 4,        /* RCCL communicator / collective error                                       */
    LH_E_UNSUPPORTED = 5, /* window outside the supported envelope (see DESIGN.md "Limits")            */
    LH_E_STATE = 6        /* call out of order (e.g. lh_solve_resident before lh_upload)               */
} lh_status;

/* Problem::StrategyType (problem.h:45-50) */
typedef enum lh_strategy { LH_STRATEGY_DEFAULT = 0, LH_STRATEGY_1 = 1 } lh_strategy;

/* Reduced pose-system solver: the reference uses Eigen LDLT (problem.cpp:420);
   PCG is the reference's Jacobi-PCG (Problem::PCGSolver, :584-614), which it left commented out
   (:422), with its first-step bug fixed (:595-596 never add alpha*p to x). */
typedef enum lh_linear_solver { LH_SOLVER_LDLT = 0, LH_SOLVER_PCG = 1 } lh_linear_solver;

/* Arithmetic of the per-edge path.  FP64: double throughout, the residual a bitwise
   mirror of the reference's (lego_types.h:200-216).  FP32_RESID: BASELINE config 3's "fp32 residuals
   + fp64 accumulate" as far as it can be taken without changing the LM decisions: each edge's
   Jacobians (the projection derivative and its chain through the extrinsic and the pose rotation,
   lego_types.h:218-254) in float, widened to double before any product that is summed; the camera
   point, the residual, the Huber weight, rho0, chi2, b's residual factor and the gain ratio stay the
   fp64 mirror, and every sum over edges (H blocks, b, chi2, the Schur complement) is double.  Parity
   to tolerance, not to the bit. */
typedef enum lh_precision { LH_PREC_FP64 = 0, LH_PREC_FP32_RESID = 1 } lh_precision;

/* The per-trial exchange of a landmark-sharded solve (world_size > 1): RCCL on the handle's stream
   (one process per GPU), or a caller-supplied all-reduce over host buffers (any transport: MPI, gloo,
   sockets), called once per LM trial from inside lh_solve on the calling thread, or (LH_COMM_P2P) a one-shot
   exchange on the device: every rank writes its partial reduced system into every rank's IPC-mapped buffer
   (xGMI between GPUs) and sums the ranks' slots in rank order; the caller's all-reduce (as LH_COMM_HOST) then
   only carries the upload-time agreement and the IPC handles.  At most 16 ranks; every rank's device must be
   able to map the others' memory. */
typedef enum lh_comm_mode { LH_COMM_RCCL = 0, LH_COMM_HOST = 1, LH_COMM_P2P = 2 } lh_comm_mode;
/* in-place all-reduce of count doubles over the ranks; op 0 = sum, 1 = max; returns 0 on success */
typedef int (*lh_allreduce_fn)(void *user, double *buf, int64_t count, int32_t op);

typedef struct lh_options {
    int32_t abi_version;      /* LH_ABI_VERSION (4 is still accepted: no ABI-5 lh_result fields)   */
    int32_t max_iters;        /* outer LM iterations, solve(10)          backend_lego.cpp:161 */
    int32_t max_trials;       /* false_cnt_threshold = 10                problem.cpp:178      */
    int32_t strategy;         /* lh_strategy                             problem.h:45         */
    double huber_delta;       /* HuberCost(5.991); <= 0: no robust kernel backend_lego.cpp:92-94 */
    double stop_dchi2;        /* diffChiThreshold_ = 1e-5 (absolute)     problem.h:165        */
    double tau;               /* 1e-5                                    problem.cpp:495      */
    double lambda_cap;        /* 5e10                                    problem.cpp:494      */
    double lambda_init;       /* < 0: computed; >= 0: setInitialLambda   problem.h:99-102     */
    int32_t linear_solver;    /* lh_linear_solver                                             */
    int32_t verbose;          /* print the reference's per-iteration line problem.cpp:180-184 */
    int32_t device;           /* HIP device ordinal, -1 = current device                      */
    int32_t world_size;       /* landmark shards (one process per GPU); 1 = single GPU.  Every rank
                                 must pass the same solver options (iteration caps, strategy, Huber
                                 delta, tolerances, solver, gate, depth): lh_create compares them
                                 across the ranks with one MAX all-reduce and returns LH_E_BADARG on
                                 every rank when they differ (the collective count per solve is a
                                 function of them)                                               */
    int32_t rank;             /* this process's shard                                         */
    int32_t degenerate_guard; /* 0: reference semantics: a landmark with one edge (rank-2 H_ll) or a
                                 non-positive-definite H_ll poisons the step, as the LU inverse's
                                 inf does (problem.cpp:396-400; the solve then rejects every trial);
                                 1: such landmarks are held fixed (no Schur term, no update)   */
    int32_t trials_per_sync;  /* LM trials kept enqueued past the last one the device has decided (0: auto = 2; one while the next completed iteration reaches max_iters) */
    int32_t profile;          /* 1: time every kernel with HIP events (lh_kernel_stats)       */
    int32_t pcg_max_iters;    /* PCG: iteration cap; <= 0: 2 * rows (problem.cpp:422)          */
    double pcg_tol;           /* PCG: stop when ||r|| <= pcg_tol * ||b|| (1e-6, problem.cpp:597) */
    uint8_t comm_id[128];     /* ncclUniqueId from lh_comm_unique_id on rank 0 (world_size>1) */
    /* ---- ABI 3 ---- */
    int32_t gate_mode;        /* 0: the reference's Huber gate rho1 + 2 rho2 e2 > 0 (base_edge.cpp:55);
                                 1: diagnostic, its analytically-zero residue on outlier edges taken
                                 as 0 (the oracle's gate_mode 1; parity tests only)            */
    int32_t chunk_landmarks;  /* landmarks per k_lin chunk; 0 = auto (~2 workgroups per CU)     */
    int32_t comm_mode;        /* lh_comm_mode (world_size > 1)                                  */
    int32_t host_threads;     /* window-preprocessing threads; 0 = auto (the CPUs this process may
                                 use: affinity mask capped by the cgroup CPU quota, <= 8)        */
    lh_allreduce_fn allreduce;  /* LH_COMM_HOST: the exchange                                    */
    void *allreduce_user;       /* its first argument                                            */
    /* ---- ABI 4 ---- */
    int32_t precision;        /* lh_precision (default LH_PREC_FP64)                             */
} lh_options;

/*
 * One sliding window.  Caller-owned, read-only during the call.
 * Order contract: poses in ascending keyframe id and landmarks in ascending
 * landmark id, i.e. the reference's ordering (Problem::setOrdering,
 * problem.cpp:234-255: std::map by vertex id, poses first).  Observation order
 * is free (the reference's is unordered_map hash order).
 */
typedef struct lh_window {
    int32_t n_poses;
    const double *pose_Tcw;    /* [n_poses][12] row-major [R | t], T_cw (VertexPose estimate, lego_types.h:37,57) */
    const uint8_t *pose_fixed; /* [n_poses] or NULL; nonzero = BaseVertex::setFixed (base_vertex.h:50)              */
    int32_t n_landmarks;
    const double *lm_xyz;      /* [n_landmarks][3] world position (VertexXYZ, lego_types.h:97-115) */
    int64_t n_obs;
    const uint32_t *obs_pose;  /* [n_obs] pose index                                                */
    const uint32_t *obs_lm;    /* [n_obs] landmark index                                            */
    const uint8_t *obs_cam;    /* [n_obs] camera index or NULL (all camera 0)                       */
    const double *obs_uv;      /* [n_obs][2] pixel measurement: toVec2 of cv::KeyPoint::pt (algorithm.h:37),
                                  i.e. float values widened; a value no float holds exactly (or a NaN) is
                                  LH_E_BADARG (the device keeps the pixels as floats)                 */
    double K[4];               /* fx, fy, cx, cy (Camera::K, camera.h:36-41)                         */
    int32_t n_cams;            /* number of extrinsics in cam_ext (0 with cam_ext NULL = identity)   */
    const double *cam_ext;     /* [n_cams][12] row-major [R | t] camera extrinsic (Camera::pose_)    */
} lh_window;

typedef struct lh_result {
    /* caller-owned outputs; any pointer may be NULL */
    double *pose_Tcw;          /* [n_poses][12]                                                   */
    double *lm_xyz;            /* [n_landmarks][3]                                                */
    double *edge_robust_chi2;  /* [n_obs] rho0 of the residuals as last evaluated, window order
                                  (stale after an all-rejected exit, as backend_lego.cpp:171 sees) */
    double *trace_chi2;        /* [trace_cap] currentChi_ at the top of each outer iteration       */
    double *trace_lambda;      /* [trace_cap] currentLambda_ at the same point                     */
    int32_t trace_cap;
    /* scalar outputs */
    int32_t trace_len;
    int32_t iterations;        /* outer LM iterations completed (problem.cpp:207)                  */
    int32_t trials;            /* solveLinearEquation calls                                        */
    int32_t accepted;          /* accepted trials                                                  */
    double chi2_initial;       /* 0.5 * sum rho0 at the input state (problem.cpp:475-479)          */
    double chi2_final;         /* currentChi_ at exit                                              */
    double lambda_final;
    double time_ms;            /* wall time of the LM solve on the device (excludes upload); host
                                  clock from the first launch to the stop when no array is requested */
    int32_t pcg_iterations;    /* PCG iterations summed over all trials (0 with LH_SOLVER_LDLT)    */
    int32_t degenerate;        /* landmarks with a rank-deficient H_ll at the initial linearisation */
    double time_prep_ms;       /* lh_solve / lh_upload: host preprocessing of the window           */
    double time_upload_ms;     /* lh_solve / lh_upload: preprocessing + host-to-device copies      */
    double time_download_ms;   /* device-to-host copies of the requested outputs                   */
    /* ---- ABI 5 (read only when lh_options.abi_version >= 5) ---- */
    uint8_t *is_outlier;       /* [n_obs] window order, or NULL.  Backend::Optimize's outlier pass
                                  (backend_lego.cpp:163-194) on the device over rho0 as last evaluated:
                                  starting from outlier_chi2_th, the threshold doubles (at most 5 times)
                                  while the inlier ratio is <= 0.5, then is_outlier = rho0 > threshold.
                                  Only the flags cross the link (edge_robust_chi2 may stay NULL); the
                                  same result as lh_classify_outliers on edge_robust_chi2          */
    double outlier_chi2_th;    /* in: the pass's starting threshold (the reference's 5.991, :92)  */
    double outlier_th;         /* out: the threshold after the doubling loop                       */
    int64_t n_inlier;          /* out: the loop's last counts (the reference's LOG line, :196)     */
    int64_t n_outlier;
} lh_result;

typedef struct lh_kernel_stats {
    int64_t launches[8];       /* per kernel class, see lh_kernel_name                             */
    double total_ms[8];
} lh_kernel_stats;

typedef struct lh_handle lh_handle;

const char *lh_strerror(int status);
/* The defaults for a caller built against ABI `abi` (its LH_ABI_VERSION at compile time): abi_version = abi, so the
   library reads exactly the lh_result fields that caller's struct has.  Callers write lh_default_options(&opt),
   which this header maps to lh_default_options_v(&opt, LH_ABI_VERSION).  The plain symbol lh_default_options,
   which binaries built against the ABI-4 header call, fills abi_version = 4 (no ABI-5 fields read). */
void lh_default_options_v(lh_options *opt, int abi);
void lh_default_options(lh_options *opt);
#define lh_default_options(opt) lh_default_options_v((opt), LH_ABI_VERSION)
const char *lh_kernel_name(int kernel_class);

/* RCCL: rank 0 creates the id and ships it to the other ranks (any transport). */
int lh_comm_unique_id(uint8_t out[128]);

int lh_create(lh_handle **h, const lh_options *opt);
void lh_destroy(lh_handle *h);

/* Host-buffer path: upload, solve, download.  The drop-in for problem.solve(). */
int lh_solve(lh_handle *h, const lh_window *in, lh_result *out);

/* Device-resident path (bench): lh_upload preprocesses and copies the window
   once; every lh_solve_resident restarts from the uploaded initial state.
   A solve that requests no array (pose_Tcw, lm_xyz, edge_robust_chi2 all NULL) returns as soon as
   the device has stopped the LM loop: its scalars and trace come with the stop flag in mapped
   host memory, and the kernels still draining are stream-ordered before any later call on the
   handle (lh_destroy synchronises). */
int lh_upload(lh_handle *h, const lh_window *in);
int lh_solve_resident(lh_handle *h, lh_result *out);

int lh_kernel_stats_get(lh_handle *h, lh_kernel_stats *out);
int lh_set_profiling(lh_handle *h, int on);   /* toggle lh_options.profile on a live handle */
void lh_kernel_stats_reset(lh_handle *h);

/*
 * Backend::Optimize outlier pass (backend_lego.cpp:163-194): starting from
 * chi2_th, double the threshold (at most 5 times) while the inlier ratio is
 * <= 0.5, then flag edges with robust chi2 > threshold.  is_outlier may be NULL.
 */
int lh_classify_outliers(const double *edge_robust_chi2, int64_t n_obs, double chi2_th,
                         uint8_t *is_outlier, double *th_out, int64_t *n_inlier, int64_t *n_outlier);

/*
 * Frontend pose-only LM: Frontend::EstimateCurrentPose
 * (src/frontend_lego.cpp:157-250) for a batch of independent frames.  Per frame:
 * one VertexPose, one EdgeProjectionPoseOnly per observation (lego_types.h:116-180),
 * four rounds of problem.solve(max_iters) each restarting from the frame's pose,
 * the outlier flags refreshed after each round (robust chi2 > 5.991, :205-226;
 * flagged features recomputed at the final estimate first), Huber(huber_delta) on
 * rounds one to three and none on round four (:223-225).  Flags never remove an
 * edge (the reference's setLevel is commented out).  Uses the handle's options
 * (max_iters, max_trials, strategy, huber_delta, stop_dchi2, tau, lambda_cap,
 * lambda_init); one workgroup per frame, the whole batch in one launch.
 */
typedef struct lh_frames {
    int32_t n_frames;
    const int64_t *obs_ptr;     /* [n_frames + 1] CSR: frame f owns observations [obs_ptr[f], obs_ptr[f+1]) */
    const double *pose_Tcw;     /* [n_frames][12] row-major [R | t]: current_frame_->Pose()           */
    const double *pts_w;        /* [n_obs][3] map-point world positions (mp->pos_)                     */
    const double *obs_uv;       /* [n_obs][2] feature pixels (toVec2(feat->position_.pt))              */
    const uint8_t *is_outlier;  /* [n_obs] the features' is_outlier_ on entry, or NULL (all false)     */
    double K[4];                /* fx, fy, cx, cy (camera_left_->K())                                   */
} lh_frames;

typedef struct lh_frames_result {
    double *pose_Tcw;           /* [n_frames][12] SE3(vertex_pose->getEstimate()) after round four     */
    uint8_t *is_outlier;        /* [n_obs] flags after round four, or NULL                             */
    double *edge_chi2;          /* [n_obs] chi2 the last classification compared with 5.991, or NULL  */
    int32_t *n_inliers;         /* [n_frames] EstimateCurrentPose's return value, or NULL               */
    int32_t *iterations;        /* [n_frames] LM iterations summed over the four rounds, or NULL       */
    double time_ms;             /* device time of the batch (upload and download excluded)             */
} lh_frames_result;

int lh_estimate_pose(lh_handle *h, const lh_frames *in, lh_frames_result *out);

/*
 * Gauss-Newton pyramidal LK optical flow, replacing
 *   void LKOpticalFlow4Layer(const cv::Mat &img1, const cv::Mat &img2,
 *                            const std::vector<cv::KeyPoint> &kp1, std::vector<cv::KeyPoint> &kp2,
 *                            std::vector<bool> &success, bool inverse, bool has_initial)
 *                                                                      (src/algorithm.cpp:128-206)
 * (levels = 4) and LKOpticalFlow1Layer (algorithm.cpp:11-31, levels = 1), as the frontend's
 * *LKOpticalFlow4LayerSelf trackers call them (frontend_lego.cpp:466-556).  Images are 8-bit gray
 * (CV_8UC1 layout: rows of `step` bytes); keypoints are cv::KeyPoint::pt.  The pyramid is built as
 * cv::resize(INTER_LINEAR, 0.5) does (exactly for even-sized levels; see oracle/lk_oracle.c).
 * Semantics as written, including inverse mode's single J variable (from iteration 1 on every
 * patch pixel uses the last pixel's J, algorithm.cpp:73-78).  kp2 and success are overwritten;
 * with has_initial, kp2 holds the initial guess on entry.
 */
typedef struct lh_lk_input {
    int32_t cols, rows;         /* level-0 image size                                                */
    int64_t step;               /* bytes per image row (>= cols)                                      */
    const uint8_t *img1;        /* [rows][step] previous / left image                                 */
    const uint8_t *img2;        /* [rows][step] current / right image                                 */
    int32_t n_points;
    const float *kp1;           /* [n_points][2] keypoints in img1                                    */
    int32_t inverse;            /* 0: forward (the frontend's mode), 1: inverse                       */
    int32_t has_initial;        /* kp2 on entry is the initial guess                                  */
    int32_t levels;             /* 4 (LKOpticalFlow4Layer) or 1 (LKOpticalFlow1Layer)                  */
} lh_lk_input;

typedef struct lh_lk_result {
    float *kp2;                 /* [n_points][2] in: initial guess (has_initial); out: tracked points */
    uint8_t *success;           /* [n_points] out                                                     */
    double time_ms;             /* device time: pyramid + tracking (copies excluded)                  */
} lh_lk_result;

int lh_lk_track(lh_handle *h, const lh_lk_input *in, lh_lk_result *out);

/* ---- test hooks (not part of the reference interface) ---- */
/* f64 MFMA accumulator-layout probe: D(16x16) = A(16x4) * B(4x16), device pointers, row-major */
int lh_debug_mfma_probe(const double *A, const double *B, double *D);
/* k_ctrl's reduced-system solve (natural order, blocked LDL^T over a dense envelope, back
   substitution) on a dense symmetric n x n S (row-major), n <= 384: x = S^-1 b.  Device pointers.
   n > 128 runs k_ctrl_g's global-memory solve (Eigen-LDLT pivot order: dense windows of 22..64
   keyframes). */
int lh_debug_ldlt_probe(const double* S, const double* b, int n, double* x);
/* k_ctrl's PCG solve (same LDS layout and pivot order) on a dense symmetric n x n S, n <= 128:
   x ~= S^-1 b to ||r|| <= tol ||b|| within max_iters (<= 0: 2n).  Device pointers; *iters host. */
int lh_debug_pcg_probe(const double* S, const double* b, int n, double tol, int max_iters, double* x, int* iters);
/* mean HIP-event bracket (ms) of an empty kernel on the handle's stream: the launch floor of the
   per-kernel times lh_set_profiling reports (bench.py subtracts it for the roofline) */
int lh_debug_event_floor(lh_handle *h, double *ms);
/* per-phase wave-cycle totals of a -DLH_STAMPS diagnostic build (all zero in the product build) */
int lh_debug_stamps(unsigned long long *out, int n, int reset);
/* k_lin's duration per LM trial, measured after a solve: the trial-mode k_lin launch(es) replayed
   reps times back to back between two HIP events on the handle's stream (ms per replay).  The
   replay rewrites the candidate buffers and the per-edge chi2: read the solve's outputs first. */
int lh_debug_time_lin(lh_handle *h, int reps, double *ms);
/* reduced-system all-reduces (data-path collectives) the last solve issued on this rank */
int lh_debug_comm_count(lh_handle *h, int64_t *n);
/* the controller the uploaded window's trials run: 0 k_ctrl (LDS, <= 21 poses), 1 k_ctrl_g (dense
   LDL^T in global memory), 2 k_ctrl_p (PCG on the block-sparse system), 3 k_ctrl_b (banded LDL^T);
   bit 8: k_ctrl_b's back substitution holds one row per lane (every row's envelope within 56 rows);
   bit 9: some k_ctrl_b step needs more than 11 unit waves, so its stream loaders take units too */
int lh_debug_controller(lh_handle *h, int *which);
/* the LM chains (k_lin, k_reduce, exchange, controller) the last solve decided past the initial
   linearisation: its trials, plus one re-linearisation per evaluate-only trial accepted outside the
   final iteration (a trial after a rejection only evaluates).  Solves that return arrays only. */
int lh_debug_chains(lh_handle *h, int *chains);
/* the lambda ladder: the rungs a factoring controller of the uploaded window builds (1: off),
   and the rejections of the last solve whose step a rung had already solved, so that no controller factored
   for them.  Solves that return arrays only (else skipped = -1). */
int lh_debug_ladder(lh_handle *h, int *rungs, int *skipped);

/* batched evaluation of rejection runs: the most rungs one chain of the uploaded window evaluates
   (1: off -- LH_NO_BATCH=1, or a ladder of one rung), the batches the last solve decided, and (retrials, two ints,
   may be NULL) the acceptances among them: [0] re-run by the next chain as a full trial, [1] re-run and stopping
   the loop.  Solves that return arrays only (else -1). */
int lh_debug_batch(lh_handle *h, int *batch_max, int *batches, int *retrials);

#ifdef __cplusplus
}
#endif
#endif
