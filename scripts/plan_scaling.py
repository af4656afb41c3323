"""Planner time (plan_structure, plan_fill) on the C3 window against the thread count (CPU only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import bench      # noqa: E402
import lego_ba    # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
for t in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8, 16]:
    s, f = lego_ba.plan_time_ms(w, threads=t, reps=10)
    print(f"threads {t:2d}: structure {s:.3f} ms, fill {f:.3f} ms", flush=True)
import numpy as np  # noqa: E402
for t in (1, 16):
    st = lego_ba.plan_stages_ms(w, threads=t)
    print(f"threads {t:2d} stage ms:", np.round(np.diff(np.concatenate([[0], st])), 3).tolist(), "total", round(st[-1], 3))
