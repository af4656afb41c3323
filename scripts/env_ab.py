"""Per-kernel ms per trial (event-bracketed kernel stats) of C3 and of 64- / 128-keyframe banded windows, with and
without an environment switch, alternated twice, each in a fresh process.
usage: python3 scripts/env_ab.py VAR=VALUE"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
    import numpy as np
    import lego_ba
    from windows import STABLE, window
    out = {}
    for P in (20, 64, 128):
        if P == 20:
            w = window("C3", seed=0, family="stable_noout")
        else:
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
        for _ in range(5):
            r = s.solve_resident()
        k = s.kernel_stats()
        out[P] = {n: round(v[1] / max(1, v[0]), 5) for n, v in k.items() if n in ("k_reduce", "k_ctrl", "k_lin")}
        out[P]["chi2"] = r["chi2_final"]
        s.close()
    print(json.dumps(out))
    sys.exit(0)
var, val = sys.argv[1].split("=", 1)
for rnd in range(2):
    for on in (False, True):
        env = dict(os.environ)
        if on:
            env[var] = val
        else:
            env.pop(var, None)
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
        print(rnd, f"{var}={val}" if on else "default", (r.stdout.strip().splitlines() or [r.stderr[-300:]])[-1], flush=True)
