"""Diagnostic: GPU vs oracle LM traces for one window (prints both)."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "lego-slam_amd", "python")]
import numpy as np
import lego_ba
import oracle_bind as ob
from windows import window
np.set_printoptions(precision=6, linewidth=200)
for strat, cfg, seed, fam in [(1, "C1", 0, "stable"), (1, "C1", 1, "stable"), (1, "mini", 0, "stable_noout")]:
    w = window(cfg, seed=seed, family=fam)
    o = ob.solve(w, strategy=strat)
    g = lego_ba.Solver(strategy=strat).solve(w)
    print(cfg, seed, fam, "oracle", o["iterations"], o["trials"], o["accepted"], "gpu", g["iterations"], g["trials"], g["accepted"])
    print(" o chi", np.array(o["trace_chi2"]) - o["trace_chi2"][0])
    print(" g chi", np.array(g["trace_chi2"]) - g["trace_chi2"][0])
    print(" o lam", np.array(o["trace_lambda"]))
    print(" g lam", np.array(g["trace_lambda"]))
    g1 = lego_ba.Solver(strategy=strat, max_iters=1, max_trials=1).solve(w)
    o1 = ob.solve(w, strategy=strat, max_iters=1, max_trials=1)
    print(" 1-trial chi", g1["chi2_final"], o1["chi2_final"], abs(g1["chi2_final"] - o1["chi2_final"]) / o1["chi2_final"])
    print(" 1-trial pose diff", np.abs(g1["pose_Tcw"] - o1["pose_Tcw"]).max(), "lm diff", np.abs(g1["lm_xyz"] - o1["lm_xyz"]).max())
