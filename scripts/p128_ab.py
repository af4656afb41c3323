"""128-keyframe window (C3 size) with PCG (k_ctrl_p): ms per resident solve, trials, PCG steps, for the
current build and each LIB in $LIB_OLD."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import lego_ba      # noqa: E402
from test_pcg import _many_pose_window  # noqa: E402

w = _many_pose_window(128, 50000, 3)
for lib in [None] + os.environ.get("LIB_OLD", "").split():
    if lib:
        lego_ba._balib = None
        lego_ba.BA_LIB = lib
    s = lego_ba.Solver(linear_solver=lego_ba.LH_SOLVER_PCG)
    s.upload(w)
    r = s.solve_resident()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = s.solve_resident()
        ts.append((time.perf_counter() - t0) * 1e3)
    print(lib or "current", "ms/solve %.2f" % np.median(ts), "iters", r["iterations"], "trials", r["trials"],
          "pcg steps", r["pcg_iterations"], "chi2 %.12e" % r["chi2_final"], flush=True)
    s.close()
