"""Diagnostic: GPU vs oracle LM traces for one window: python scripts/diag_window.py CFG SEED FAMILY"""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import numpy as np
import lego_ba
import oracle_bind as ob
from windows import window
np.set_printoptions(precision=6, linewidth=200)
cfg, seed, fam = sys.argv[1], int(sys.argv[2]), sys.argv[3]
w = window(cfg, seed=seed, family=fam)
o = ob.solve(w)
g = lego_ba.Solver().solve(w)
print(cfg, seed, fam, "oracle", o["iterations"], o["trials"], o["accepted"], "gpu", g["iterations"], g["trials"], g["accepted"])
print(" o chi", np.array(o["trace_chi2"]))
print(" g chi", np.array(g["trace_chi2"]))
print(" o lam", np.array(o["trace_lambda"]))
print(" g lam", np.array(g["trace_lambda"]))
for k in (1, 2, 3, 4):
    g1 = lego_ba.Solver(max_iters=k).solve(w)
    o1 = ob.solve(w, max_iters=k)
    print(f" after {k} its: chi g {g1['chi2_final']:.12e} o {o1['chi2_final']:.12e}  pose diff {np.abs(g1['pose_Tcw'] - o1['pose_Tcw']).max():.3e}"
          f"  lm diff {np.nanmax(np.abs(g1['lm_xyz'] - o1['lm_xyz'])):.3e} nan {np.isnan(g1['lm_xyz']).sum()}")
