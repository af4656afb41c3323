"""The frontend paths the bench measures, for a rocprofv3 kernel trace: lh_estimate_pose on one frame
(x20) and on a 2048-frame batch (x3), and lh_lk_track on a 1241x376 pair with 2000 keypoints (x5)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import frames       # noqa: E402
import images       # noqa: E402
import lego_ba      # noqa: E402

s = lego_ba.Solver()
one = frames.batch(0, 1, n_obs=150)
for _ in range(20):
    s.estimate_pose(one)
fb = frames.batch(0, 2048, n_obs=150)
for _ in range(3):
    s.estimate_pose(fb)
li1, li2 = images.pair(376, 1241, shift=(3.1, 0.4), seed=11)
lk1 = images.keypoints(376, 1241, 2000, seed=11, border=False)
for _ in range(5):
    r = s.lk_track(li1, li2, lk1, kp2_init=lk1 + np.float32([2.0, 0.0]))
print("tracked", int(r["success"].sum()))
s.close()
