"""Synthetic frames for the frontend pose-only path (Frontend::EstimateCurrentPose,
src/frontend_lego.cpp:157-250).  Test data only.

A frame: the true pose T_cw (camera moving along +z with small yaw, as the
backend windows), map points in front of the camera (depth 8-60 m, the
windows' ranges), their projections with N(0, 1 px) noise rounded to float32
(cv::KeyPoint, toVec2), a fraction of gross outliers uniform in the image, and
the frame's initial pose: the truth perturbed (the constant-velocity guess the
frontend starts from).  Counter-based: frame f of seed s is the same whatever
batch it is generated in.
"""
import numpy as np

K = np.array([517.3, 516.5, 325.1, 249.7])   # config/kitti_00.yaml:10-13


def _rot(axis_angle):
    th = np.linalg.norm(axis_angle)
    if th < 1e-15:
        return np.eye(3)
    k = axis_angle / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def frame(seed, f, n_obs=150, outlier_frac=0.05, rot_sigma=0.01, trans_sigma=0.05):
    rng = np.random.default_rng([seed, f])
    R_true = _rot(np.array([0.0, rng.normal(0, 0.02), 0.0]))
    c = np.array([rng.normal(0, 0.5), 0.0, float(f)])          # camera centre (world)
    t_true = -R_true @ c
    # points in the camera frame, then to the world
    z = rng.uniform(8.0, 60.0, n_obs)
    u = rng.uniform(0, 640, n_obs)
    v = rng.uniform(0, 480, n_obs)
    Xc = np.stack([(u - K[2]) / K[0] * z, (v - K[3]) / K[1] * z, z], axis=1)
    Xw = (Xc - t_true) @ R_true                                  # R^T (Xc - t)
    proj = np.stack([K[0] * Xc[:, 0] / Xc[:, 2] + K[2], K[1] * Xc[:, 1] / Xc[:, 2] + K[3]], axis=1)
    uv = proj + rng.normal(0, 1.0, proj.shape)
    out = rng.random(n_obs) < outlier_frac
    ang = rng.uniform(0, 2 * np.pi, out.sum())
    mag = rng.uniform(10.0, 40.0, out.sum())
    uv[out] += np.stack([mag * np.cos(ang), mag * np.sin(ang)], axis=1)
    uv = uv.astype(np.float32).astype(np.float64)
    dR = _rot(rng.normal(0, rot_sigma, 3))
    R0 = dR @ R_true
    t0 = t_true + rng.normal(0, trans_sigma, 3)
    pose_true = np.hstack([R_true, t_true[:, None]]).reshape(12)
    pose0 = np.hstack([R0, t0[:, None]]).reshape(12)
    return dict(pose_true=pose_true, pose_Tcw=pose0, pts=Xw, obs_uv=uv, outlier=out)


def batch(seed, n_frames, n_obs=150, **kw):
    """n_frames frames as one CSR batch (obs_ptr), the lh_frames layout."""
    fs = [frame(seed, f, n_obs=n_obs if np.isscalar(n_obs) else n_obs[f], **kw) for f in range(n_frames)]
    ptr = np.zeros(n_frames + 1, np.int64)
    ptr[1:] = np.cumsum([len(x["pts"]) for x in fs])
    cat = lambda k, shape: (np.concatenate([x[k] for x in fs]) if fs else np.zeros(shape))
    return dict(n_frames=n_frames, obs_ptr=ptr,
                pose_Tcw=np.stack([x["pose_Tcw"] for x in fs]) if fs else np.zeros((0, 12)),
                pose_true=np.stack([x["pose_true"] for x in fs]) if fs else np.zeros((0, 12)),
                pts=np.ascontiguousarray(cat("pts", (0, 3)), np.float64),
                obs_uv=np.ascontiguousarray(cat("obs_uv", (0, 2)), np.float64),
                gross=cat("outlier", (0,)).astype(bool), K=K.copy())
