"""Frontend pose-only LM A/B: one frame (host-to-host and device ms, median of 40) and a 2048-frame batch
(device ms, best of 5) for the current library and each LIB given, alternated twice, each in a fresh process.
usage: python3 scripts/frames_ab.py [LIB ...]"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
    import numpy as np
    import lego_ba
    import frames
    s = lego_ba.Solver()
    one = frames.batch(0, 1, n_obs=150)
    s.estimate_pose(one)
    lat, dev = [], []
    for _ in range(40):
        t0 = time.perf_counter()
        r = s.estimate_pose(one)
        lat.append((time.perf_counter() - t0) * 1e3)
        dev.append(r["time_ms"])
    fb = frames.batch(0, 2048, n_obs=150)
    s.estimate_pose(fb)
    tb = [s.estimate_pose(fb)["time_ms"] for _ in range(5)]
    rb = s.estimate_pose(fb)
    print(json.dumps({"single_ms": round(float(np.median(lat)), 4), "single_dev_ms": round(float(np.median(dev)), 4),
                      "batch_ms": round(min(tb), 4), "pose_sum": float(np.sum(rb["pose_Tcw"]))}))
    sys.exit(0)
libs = [os.path.join(ROOT, "lego-slam_amd", "lib", "liblego_ba.so")] + sys.argv[1:]
for rnd in range(2):
    for lib in libs:
        r = subprocess.run([sys.executable, __file__, "--child"], env=dict(os.environ, LH_LIB=lib),
                           capture_output=True, text=True, timeout=300)
        print(rnd, os.path.relpath(lib, ROOT), (r.stdout.strip().splitlines() or [r.stderr[-300:]])[-1], flush=True)
