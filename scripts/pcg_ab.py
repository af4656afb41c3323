"""C3 with linear_solver = PCG (k_ctrl<1>, lds_pcg_solve): ms per solve and PCG steps, for the current
build and each LIB in $LIB_OLD (median of 15 resident solves)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
for lib in [None] + os.environ.get("LIB_OLD", "").split():
    if lib:
        lego_ba._balib = None
        lego_ba.BA_LIB = lib
    for solver in (0, 1):
        s = lego_ba.Solver(linear_solver=solver)
        s.upload(w)
        r = s.solve_resident()
        ts = []
        for _ in range(15):
            t0 = time.perf_counter()
            r = s.solve_resident()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(lib or "current", "PCG" if solver else "LDLT", "ms/solve %.3f" % np.median(ts), "iters", r["iterations"],
              "pcg steps", r["pcg_iterations"], "chi2 %.12e" % r["chi2_final"], flush=True)
        s.close()
