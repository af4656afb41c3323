"""Which windows run re-linearisation chains (an evaluate-only trial accepted outside the final iteration):
trials and chains per candidate window and controller, eval-first on (the default)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import lego_ba  # noqa: E402
from windows import window  # noqa: E402

PCG = dict(linear_solver=lego_ba.LH_SOLVER_PCG)
cands = []
for seed in range(4):
    cands += [(f"C2 default {seed}", lambda s=seed: window("C2", seed=s), {}),
              (f"mini default {seed}", lambda s=seed: window("mini", seed=s), {}),
              (f"C2 default {seed} PCG", lambda s=seed: window("C2", seed=s), PCG),
              (f"P96 {seed}", lambda s=seed: lego_ba.generate_window(P=96, L=6000, k=8, seed=s), {}),
              (f"P96 {seed} PCG", lambda s=seed: lego_ba.generate_window(P=96, L=6000, k=8, seed=s), PCG)]
for seed in range(6):
    cands.append((f"P40 dense {seed}", lambda s=seed: lego_ba.generate_window(P=40, L=3000, k=8, seed=s, pose_mode=1, k_min=2, k_max=8), {}))
for name, mk, kw in cands:
    w = mk()
    s = lego_ba.Solver(**kw)
    r = s.solve(w)
    print(f"{name:22s} {s.controller():9s} it {r['iterations']:2d} trials {r['trials']:3d} acc {r['accepted']:2d} chains {s.chains():3d}",
          flush=True)
    s.close()
