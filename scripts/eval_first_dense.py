"""k_ctrl_g windows (dense reduced system, 22-64 keyframes) that run re-linearisation chains."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import lego_ba  # noqa: E402
from windows import STABLE  # noqa: E402

for P, L in ((24, 2000), (32, 3000), (40, 3000)):
    for seed in range(4):
        for fam, params in (("default", {}), ("stable", STABLE)):
            for kw in ({}, dict(strategy=1)):
                w = lego_ba.generate_window(P=P, L=L, k=8, seed=seed, pose_mode=1, k_min=2, k_max=8, **params)
                s = lego_ba.Solver(**kw)
                r = s.solve(w)
                print(f"P{P} seed {seed} {fam:8s} {kw} {s.controller()} it {r['iterations']} trials {r['trials']} "
                      f"acc {r['accepted']} chains {s.chains()}", flush=True)
                s.close()
