"""Diagnostic: lh_estimate_pose outputs on a 2048-frame batch and a single frame, saved to the .npz given
(A/B bit-identity check of two builds: run once per LH_LIB, then compare the files)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "lego-slam_amd", "python")]
import numpy as np  # noqa: E402
import frames       # noqa: E402
import lego_ba      # noqa: E402

s = lego_ba.Solver()
out = {}
for name, fb in (("batch", frames.batch(0, 2048, n_obs=150)), ("one", frames.batch(1, 1, n_obs=150))):
    r = s.estimate_pose(fb)
    for k, v in r.items():
        if isinstance(v, np.ndarray):
            out[f"{name}_{k}"] = v
s.close()
np.savez(sys.argv[1], **out)
print("saved", len(out), "arrays")
