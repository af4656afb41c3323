"""Gauge-aware comparison of two solutions of the same window.

The reference fixes no vertex (backend_lego.cpp:67-79): the window's gauge (rotation, translation
and, with left-image edges only, scale) is held only by lambda, so two solves whose summation
orders differ drift apart along it while chi2 agrees to 1e-9.  States are compared after the
similarity transform (Umeyama, least squares over the landmark positions) that maps one solution
onto the other: what remains is the part of the difference the gauge does not explain.
"""
import numpy as np


def umeyama(src, dst):
    """s, R, t minimising sum |dst - (s R src + t)|^2 (src, dst: (N, 3))."""
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    cov = xd.T @ xs / len(src)
    U, D, Vt = np.linalg.svd(cov)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1.0
    R = U @ S @ Vt
    var = (xs ** 2).sum() / len(src)
    s = np.trace(np.diag(D) @ S) / var
    t = mu_d - s * R @ mu_s
    return s, R, t


def aligned_errors(lm_a, lm_b, pose_a=None, pose_b=None):
    """Max landmark and camera-centre distance between solution a mapped onto b by the Sim(3)
    fitted on the landmarks, and the fitted transform's departure from identity."""
    s, R, t = umeyama(np.asarray(lm_a, float), np.asarray(lm_b, float))
    lm_err = np.abs((s * (R @ np.asarray(lm_a).T)).T + t - lm_b).max()
    cam_err = 0.0
    if pose_a is not None:
        def centres(P):
            P = np.asarray(P).reshape(-1, 3, 4)
            return np.einsum("nji,nj->ni", P[:, :, :3], -P[:, :, 3])   # c = -R^T t
        ca, cb = centres(pose_a), centres(pose_b)
        cam_err = np.abs((s * (R @ ca.T)).T + t - cb).max()
    gauge = max(abs(s - 1.0), np.abs(R - np.eye(3)).max(), np.abs(t).max())
    return lm_err, cam_err, gauge


def oracle_state_spread(w, threads=(1, 2, 8), **opt):
    """The oracle re-run with different summation orders (OpenMP thread counts): its first run and
    the largest landmark and pose differences among the runs (what the reference's own rounding
    leaves undetermined on this window)."""
    import oracle_bind as ob
    runs = [ob.solve(w, n_threads=t, **opt) for t in threads]
    lm = max(np.abs(r["lm_xyz"] - runs[0]["lm_xyz"]).max() for r in runs)
    pose = max(np.abs(r["pose_Tcw"] - runs[0]["pose_Tcw"]).max() for r in runs)
    return runs[0], lm, pose
