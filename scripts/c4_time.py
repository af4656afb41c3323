"""C4 (500 k landmarks) on one GPU, gate mode 1 (bench.py's c4_1gpu): ms per solve over 3 rounds of 10 array-free
solves after 2 warm-up solves (LH_LIB selects the library)."""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

w = window("C4", seed=0, family="stable_noout")
s = lego_ba.Solver(gate_mode=1)
s.upload(w)
for _ in range(2):
    s.solve_resident()
for rnd in range(3):
    t0 = time.perf_counter()
    for _ in range(10):
        r = s.solve_resident()
    print(f"round {rnd}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per solve ({r['trials']} trials)", flush=True)
s.close()
