"""k_lin replays on the C3 window (stable_noout, seed 0): the kernel alone, for profilers."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import bench    # noqa: E402
import lego_ba  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 500
w = bench.make_window("C3", "stable_noout", 0, 0, 1)
s = lego_ba.Solver()
s.upload(w)
s.solve_resident()
print("k_lin replay ms", s.time_lin_ms(reps=reps), flush=True)
s.close()
