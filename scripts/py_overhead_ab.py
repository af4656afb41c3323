"""The array-free solve_resident's Python wrapper: the lean path (one reused lh_result) against the general one
(fresh result buffers and a dict per call), alternated on the same resident C3 window; ms per solve."""
import ctypes as C
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

s = lego_ba.Solver()
s.upload(window("C3", seed=0, family="stable_noout"))


def general():
    w = s._win.s
    r, out = s._result(w.n_poses, w.n_landmarks, w.n_obs, 64, False, False)
    lego_ba._check(lego_ba.ba_lib().lh_solve_resident(s.h, C.byref(r)), "lh_solve_resident")
    return s._finish(r, out)


for _ in range(20):
    s.solve_resident()
for rnd in range(4):
    for name, f in (("lean", s.solve_resident), ("general", general)):
        t0 = time.perf_counter()
        for _ in range(300):
            f()
        print(f"round {rnd} {name:8s} {(time.perf_counter() - t0) / 300 * 1e3:.4f} ms per solve", flush=True)
s.close()
