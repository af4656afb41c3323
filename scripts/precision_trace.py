"""Per-iteration chi2 / lambda traces of C1 and C3 solves in FP64 and FP32_RESID."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402
from windows import window  # noqa: E402

np.set_printoptions(linewidth=200, precision=10)
for name, w in (("C1", window("C1", seed=0, family="stable_noout")), ("C3", bench.make_window("C3", "stable_noout", 0, 0, 1))):
    for prec in (0, 1):
        r = lego_ba.Solver(precision=prec).solve(w)
        print(name, "prec", prec, "iters", r["iterations"], "trials", r["trials"], "chi2 %.10e -> %.10e" % (r["chi2_initial"], r["chi2_final"]))
        print("   chi2", r["trace_chi2"])
        print("   lam ", r["trace_lambda"])
