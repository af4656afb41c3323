"""lh_upload (returns after its copies) against its preprocessing time: the copy tail; and lh_solve's parts."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
lib = os.environ.get("LIB")
if lib:
    lego_ba.BA_LIB = lib
s = lego_ba.Solver()
s.upload(w)
rows = []
for _ in range(15):
    t0 = time.perf_counter()
    s.upload(w)
    t1 = time.perf_counter()
    r = s.solve_resident(want_states=True, want_edges=True)
    t2 = time.perf_counter()
    rows.append(((t1 - t0) * 1e3, r["time_prep_ms"], r["time_upload_ms"], (t2 - t1) * 1e3, r["time_ms"], r["time_download_ms"]))
a = np.median(np.array(rows), axis=0)
print(lib or "current", "upload(sync) wall %.3f prep %.3f upload(enqueue) %.3f | solve_resident wall %.3f device %.3f download %.3f" % tuple(a))
