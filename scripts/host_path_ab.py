"""Host-buffer lh_solve time on the C3 window (median of 15), for the library LH_LIB points at."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
s = lego_ba.Solver()
s.solve(w)
t, prep = [], []
for _ in range(15):
    t0 = time.perf_counter()
    r = s.solve(w)
    t.append((time.perf_counter() - t0) * 1e3)
    prep.append(r["time_prep_ms"])
print(os.environ.get("LH_LIB", "default"), f"ms_per_solve {np.median(t):.3f} prep {np.median(prep):.3f}", flush=True)
