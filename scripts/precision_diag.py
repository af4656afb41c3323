"""One LM iteration of C3 in FP64 and FP32_RESID: where the states differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
for it in (0, 1):
    r = {p: lego_ba.Solver(precision=p, max_iters=it).solve(w) for p in (0, 1)}
    a, b = r[0], r[1]
    print("max_iters", it, "chi2", a["chi2_final"], b["chi2_final"], "lambda", a["lambda_final"], b["lambda_final"])
    dl = np.linalg.norm(b["lm_xyz"] - a["lm_xyz"], axis=1)
    dp = np.abs(b["pose_Tcw"] - a["pose_Tcw"]).max(axis=1)
    print("  pose diff per pose", np.array2string(dp, precision=2))
    o = np.argsort(dl)[::-1][:8]
    cnt = np.bincount(w["obs_lm"], minlength=len(w["lm_xyz"]))
    print("  worst landmarks", o, dl[o], "obs", cnt[o], "median", np.median(dl))
    for l in o[:3]:
        e = np.flatnonzero(w["obs_lm"] == l)
        print("   lm", l, "poses", w["obs_pose"][e], "cams", w["obs_cam"][e], "xyz", w["lm_xyz"][l], "rho32", b["edge_robust_chi2"][e], "rho64", a["edge_robust_chi2"][e])
