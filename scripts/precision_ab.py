"""C3 (stable_noout) with precision FP64 and FP32_RESID: ms per resident solve (median of 15), k_lin
replay time, chi2 and state differences."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
res = {}
for prec in (0, 1):
    s = lego_ba.Solver(precision=prec)
    s.upload(w)
    r = s.solve_resident(want_states=True)
    ts = []
    for _ in range(15):
        t0 = time.perf_counter()
        s.solve_resident()
        ts.append((time.perf_counter() - t0) * 1e3)
    kl = s.time_lin_ms(reps=50)
    res[prec] = r
    print("precision", prec, "ms/solve %.3f" % np.median(ts), "k_lin ms %.4f" % kl, "iters", r["iterations"],
          "chi2 %.12e" % r["chi2_final"], flush=True)
    s.close()
a, b = res[0], res[1]
print("chi2 rel %.3e" % (abs(b["chi2_final"] - a["chi2_final"]) / a["chi2_final"]),
      "lm max abs %.3e" % np.abs(b["lm_xyz"] - a["lm_xyz"]).max(), "pose max abs %.3e" % np.abs(b["pose_Tcw"] - a["pose_Tcw"]).max())
