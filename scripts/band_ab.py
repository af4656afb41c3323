"""k_ctrl_b A/B: the banded LDL^T's time per trial (event-bracketed kernel stats, as bench.py's p*_window_ldlt
lines) at 64 / 128 / 256 keyframes for the current library and each LIB given, alternated twice, each in a
fresh process.  usage: python3 scripts/band_ab.py [LIB ...]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
    import numpy as np
    import lego_ba
    from windows import STABLE
    out = {}
    for P in (64, 128, 256):
        w = lego_ba.generate_window(P=P, L=50000, k=8, seed=3, **dict(STABLE, outlier_frac=0.0))
        f = np.zeros(P, np.uint8)
        f[0] = 1
        w["pose_fixed"] = f
        s = lego_ba.Solver()
        s.upload(w)
        s.solve_resident()
        s.set_profiling(True)
        s.kernel_stats_reset()
        r = None
        for _ in range(3):
            r = s.solve_resident()
        k = s.kernel_stats()
        out[P] = {"controller": s.controller(), "ms_per_trial": round(k["k_ctrl"][1] / max(1, k["k_ctrl"][0]), 4),
                  "trials": r["trials"], "chi2": r["chi2_final"]}
        s.close()
    print(json.dumps(out))
    sys.exit(0)
libs = [os.path.join(ROOT, "lego-slam_amd", "lib", "liblego_ba.so")] + sys.argv[1:]
for rnd in range(2):
    for lib in libs:
        r = subprocess.run([sys.executable, __file__, "--child"], env=dict(os.environ, LH_LIB=lib),
                           capture_output=True, text=True, timeout=300)
        print(rnd, os.path.relpath(lib, ROOT), (r.stdout.strip().splitlines() or [r.stderr[-300:]])[-1], flush=True)
