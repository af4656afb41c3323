"""k_lin launch time and solve rate on the C3 window against the planner's chunk size
(lh_options.chunk_landmarks; 0 = the planner's default).  GPU only.
usage: python scripts/chunk_sweep.py [chunk ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python"))
import numpy as np
import bench
import lego_ba

chunks = [int(a) for a in sys.argv[1:]] or [0, 64, 96, 128, 160, 192]
w = bench.make_window("C3", "stable_noout", 0, 0, 1)
pl0 = None
for c in chunks:
    pl = lego_ba.plan_window(w, chunk_lm=c, threads=8)
    s = lego_ba.Solver(chunk_landmarks=c)
    s.upload(w)
    s.solve_resident()
    lin = s.time_lin_ms(50)
    t = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = s.solve_resident()
        t.append((time.perf_counter() - t0) * 1e3)
    ck = pl["chunks"]
    nsb = ck["sb_end"].astype(int) - ck["sb_begin"].astype(int)
    per_wave = -(-nsb // 4)
    print(f"chunk_lm={c:4d} n_chunks={len(ck)} sb/chunk mean {nsb.mean():.1f} max {nsb.max()} max sb/wave {per_wave.max()} "
          f"k_lin={lin * 1e3:.2f} us solve={min(t):.3f} ms it={r['iterations']} chi2={r['chi2_final']:.10e}", flush=True)
    s.close()
