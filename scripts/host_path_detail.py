"""Host-buffer path detail on the box: planner stages by thread count, and lh_solve's parts (median of 15)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import bench        # noqa: E402
import lego_ba      # noqa: E402

w = bench.make_window("C3", "stable_noout", 0, 0, 1)
print("host", bench.host_info())
for th in (1, 4, 8, 16):
    st = lego_ba.plan_stages_ms(w, threads=th, reps=5)
    print(f"threads {th:2d} stage ends ms", " ".join(f"{x:.3f}" for x in st),
          "structure/fill ms", " ".join(f"{x:.3f}" for x in lego_ba.plan_time_ms(w, threads=th, reps=10)), flush=True)
for lib in [None] + os.environ.get("LIB_OLD", "").split():
    if lib:
        lego_ba._balib = None
        lego_ba.BA_LIB = lib
    s = lego_ba.Solver()
    prev = s.solve(w)
    for mode in ("fresh outputs", "reused outputs"):
        rows = []
        for _ in range(15):
            t0 = time.perf_counter()
            r = s.solve(w, reuse=prev if mode.startswith("reused") else None)
            rows.append(((time.perf_counter() - t0) * 1e3, r["time_prep_ms"], r["time_upload_ms"], r["time_ms"], r["time_download_ms"]))
        a = np.median(np.array(rows), axis=0)
        print(lib or "current", mode, "total %.3f prep %.3f upload %.3f solve %.3f download %.3f" % tuple(a), flush=True)
    s.close()
# lh_solve by planner thread count (the default is auto_host_threads: the usable CPUs, at most 8)
lego_ba._balib = None
lego_ba.BA_LIB = os.path.join(ROOT, "lego-slam_amd", "lib", "liblego_ba.so")
for th in (4, 8, 12, 16):
    s = lego_ba.Solver(host_threads=th)
    prev = s.solve(w)
    rows = []
    for _ in range(15):
        t0 = time.perf_counter()
        r = s.solve(w, reuse=prev)
        rows.append(((time.perf_counter() - t0) * 1e3, r["time_prep_ms"], r["time_upload_ms"], r["time_ms"], r["time_download_ms"]))
    a = np.median(np.array(rows), axis=0)
    print(f"host_threads {th:2d} total %.3f prep %.3f upload %.3f solve %.3f download %.3f" % tuple(a), flush=True)
    s.close()
