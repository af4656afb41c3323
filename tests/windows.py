"""Window families used by the parity tests (see DESIGN.md "Parity").

The reference LM (problem.cpp:156-230) is not reproducible under a change of
summation order on every window: the Huber second-order gate
(base_edge.cpp:55) tests the sign of a rounding residue, and the absolute
stop rule (problem.cpp:210) and the accept test sit on knife edges of
not-yet-converged, gauge-free problems.  Two builds of the oracle that differ
only in summation order (thread count) disagree on final chi2 by 1e-6..1e-3 on
such windows.  Parity at 1e-6 is therefore asserted on window families whose
oracle trajectory is itself reproducible ("stable"), and the rest are checked
against the oracle's own spread ("envelope").
"""
import numpy as np

import lego_ba

# stereo edges + first keyframe fixed (removes the 6-DoF gauge), landmarks 8-30 m,
# small initial perturbation: oracle self-spread ~1e-15 (no outliers) / <=1e-6 (2 % outliers)
STABLE = dict(right_frac=0.5, depth_max=30.0, pose_rot_sigma=0.0005, pose_trans_sigma=0.005, lm_sigma=0.02)


def _family_params(family, fix_first, kw):
    params = {}
    if family in ("stable", "stable_noout"):
        params.update(STABLE)
        if family == "stable_noout":
            params["outlier_frac"] = 0.0
        if fix_first is None:
            fix_first = True
    params.update(kw)
    return params, fix_first


def _fix(w, fix_first):
    if fix_first:
        f = np.zeros(w["n_poses"], np.uint8)
        f[0] = 1
        w["pose_fixed"] = f
    return w


def window(cfg, seed=0, family="default", fix_first=None, **kw):
    params, fix_first = _family_params(family, fix_first, kw)
    return _fix(lego_ba.config_window(cfg, seed=seed, **params), fix_first)


def window_shard(cfg, l0, l1, seed=0, family="default", fix_first=None, **kw):
    """Landmarks [l0, l1) of window(cfg, seed, family) and their observations, generated directly (the
    generator draws each landmark from its own counter stream, so this equals slicing the whole
    window, with shard-local landmark indices): one rank's unit in the landmark-sharded path."""
    params, fix_first = _family_params(family, fix_first, kw)
    c = dict(lego_ba.CONFIGS[cfg])
    c.update(params)
    return _fix(lego_ba.generate_window(seed=seed, lm_begin=l0, lm_end=l1, **c), fix_first)


def _rot(axis, angle):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(angle) * K + (1 - np.cos(angle)) * K @ K


# extra camera rigs for the multi-camera windows: (rotation axis, angle, translation); camera 0 is the
# generator's identity (KITTI left, dataset.cpp:36-42) and camera 1 its stereo baseline
EXTRA_CAMS = [((0.0, 1.0, 0.0), 0.05, (0.20, -0.10, 0.05)),
              ((1.0, 1.0, 0.3), 0.08, (-0.30, 0.05, 0.10))]


def multi_camera(w, n_cams, seed=0, noise_px=1.0):
    """Window `w` re-observed through a rig of n_cams (3 or 4) cameras: cameras 2, 3 have non-identity
    extrinsic rotations (Camera::pose_, the ext of EdgeProjection's K * (ext * (T * X)),
    lego_types.h:211-215).  Each observation is assigned a random camera and re-measured from the true
    pose and landmark (float32 pixels + N(0, noise_px^2)), so the window stays consistent."""
    rng = np.random.default_rng(1000 + seed)
    ext = np.zeros((n_cams, 12))
    ext[:2] = w["cam_ext"][:2]
    for c in range(2, n_cams):
        axis, ang, t = EXTRA_CAMS[c - 2]
        ext[c, [0, 1, 2, 4, 5, 6, 8, 9, 10]] = _rot(axis, ang).reshape(9)
        ext[c, [3, 7, 11]] = t
    O = len(w["obs_pose"])
    cam = rng.integers(0, n_cams, O).astype(np.uint8)
    T = w["pose_true"][w["obs_pose"]].reshape(O, 3, 4)
    X = w["lm_true"][w["obs_lm"]]
    Pb = np.einsum("oij,oj->oi", T[:, :, :3], X) + T[:, :, 3]
    E = ext[cam].reshape(O, 3, 4)
    Pc = np.einsum("oij,oj->oi", E[:, :, :3], Pb) + E[:, :, 3]
    fx, fy, cx, cy = w["K"]
    u = (fx * Pc[:, 0] + cx * Pc[:, 2]) / Pc[:, 2] + rng.normal(0, noise_px, O)
    v = (fy * Pc[:, 1] + cy * Pc[:, 2]) / Pc[:, 2] + rng.normal(0, noise_px, O)
    out = dict(w)
    out["cam_ext"] = ext
    out["obs_cam"] = cam
    out["obs_uv"] = np.stack([u, v], 1).astype(np.float32).astype(np.float64)
    return out


# Windows whose LM run rejects and then accepts inside an iteration before the last one, whatever the
# summation order: no robust kernel (or the reproducible gate), large initial errors and a small lambda_init,
# so the first steps overshoot by a wide margin.  Each was picked with the oracle's per-trial log (verbose 2):
# the same accept/reject string at 1, 2, 8 and 16 threads and under 1e-12 relative landmark perturbations,
# every trial's candidate chi2 within `spread` of the others (scripts/relin_windows.py regenerates the table).
# (kind, generator args, solver options, the oracle's decision string, controller)
_RELIN_FAR = dict(right_frac=0.5, depth_max=30.0, outlier_frac=0.0, pose_rot_sigma=0.3, pose_trans_sigma=1.0,
                  lm_sigma=2.0, depth_min=3.0)
_RELIN_NEAR = dict(right_frac=0.5, depth_max=30.0, outlier_frac=0.0, pose_rot_sigma=0.05, pose_trans_sigma=0.3,
                   lm_sigma=2.0, depth_min=4.0)
RELIN_WINDOWS = [
    ("k_ctrl LDLT", dict(P=10, L=500, k=8, seed=3, **_RELIN_FAR), dict(huber_delta=0.0, lambda_init=1e-3),
     "RRRRRRAAA", "k_ctrl"),
    ("k_ctrl LDLT small lambda", dict(P=10, L=500, k=8, seed=3, **_RELIN_FAR), dict(huber_delta=0.0, lambda_init=1e-6),
     "RRRRRRRRAAA", "k_ctrl"),
    ("k_ctrl strategy 1", dict(P=10, L=500, k=8, seed=3, **_RELIN_FAR), dict(huber_delta=0.0, strategy=1),
     "RRAAA", "k_ctrl"),
    ("k_ctrl PCG strategy 1", dict(P=10, L=500, k=8, seed=3, **_RELIN_FAR),
     dict(huber_delta=0.0, strategy=1, linear_solver=lego_ba.LH_SOLVER_PCG), "RRAAA", "k_ctrl"),
    ("k_ctrl_b", dict(P=30, L=300, k=8, seed=1, **_RELIN_NEAR), dict(huber_delta=0.0, lambda_init=1e-3),
     "RRRRRRRAAA", "k_ctrl_b"),
    ("k_ctrl_b strategy 1", dict(P=30, L=300, k=8, seed=1, **_RELIN_NEAR), dict(huber_delta=0.0, strategy=1),
     "RRRAAA", "k_ctrl_b"),
    ("k_ctrl_b second iteration", dict(P=30, L=300, k=8, seed=2, **_RELIN_NEAR), dict(huber_delta=0.0, lambda_init=1e-3),
     "ARRRRRRRRAA", "k_ctrl_b"),
    ("k_ctrl_g", dict(P=24, L=400, k=2, k_max=8, pose_mode=1, seed=4, **_RELIN_NEAR),
     dict(huber_delta=0.0, lambda_init=1e-3), "RRRRRAAA", "k_ctrl_g"),
    ("k_ctrl_p", dict(P=30, L=300, k=8, seed=1, **_RELIN_NEAR),
     dict(huber_delta=0.0, lambda_init=1e-3, linear_solver=lego_ba.LH_SOLVER_PCG), "RRRRRRRAAA", "k_ctrl_p"),
]


def relin_window(gen):
    """A RELIN_WINDOWS window: pose 0 fixed (the gauge), 3 LM iterations."""
    w = lego_ba.generate_window(**gen)
    return _fix(w, True)
