"""Banded-LDL^T windows (64 / 128 / 256 keyframes of C3's size) solved in one process, for a rocprofv3 kernel
trace of k_ctrl_b (scripts/gpu.sh py=... under rocprofv3, or directly: rocprofv3 --kernel-trace --stats --
python3 scripts/band_trace.py).  Prints the per-trial controller time from the event-bracketed kernel stats."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import lego_ba  # noqa: E402
from windows import STABLE  # noqa: E402

out = {}
for P in (64, 128, 256):
    w = lego_ba.generate_window(P=P, L=50000, k=8, seed=3, **dict(STABLE, outlier_frac=0.0))
    f = np.zeros(P, np.uint8)
    f[0] = 1
    w["pose_fixed"] = f
    s = lego_ba.Solver()
    s.upload(w)
    for _ in range(5):
        r = s.solve_resident()
    out[P] = {"controller": s.controller(), "trials_per_solve": r["trials"], "chi2": r["chi2_final"]}
    s.close()
print(json.dumps(out))
