"""The reference's live configuration (survey-default C3, reference gate): repeated array-free solves, for a
kernel trace of its trial mix (full trials, evaluate-only trials, re-linearisations); then the planner's
stage times on this box's host (lh_plan.cpp stages, 8 threads)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

w = window("C3", seed=0)
s = lego_ba.Solver()
r = s.solve(w)
print("trials", r["trials"], "iterations", r["iterations"], "chains", s.chains(), flush=True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
s.upload(w)
s.solve_resident()
t0 = time.perf_counter()
for _ in range(n):
    r = s.solve_resident()
t = (time.perf_counter() - t0) / n
print(f"live config: {1e3 * t:.3f} ms per solve, {r['iterations'] / t:.0f} it/s", flush=True)
s.close()
st = [lego_ba.plan_stages_ms(w, threads=8, reps=20) for _ in range(5)]
st = np.median(np.array(st), axis=0)
print("planner stages (cumulative ms, median of 5 x 20):", " ".join(f"{x:.3f}" for x in st), flush=True)
print("  chunking stage:", f"{st[4] - st[3]:.3f} ms", flush=True)
