"""
make_golden — generates the committed golden fixtures tests/golden/*.npz.

TEST INFRASTRUCTURE.  Each fixture is data only: one small sliding window
(inputs in the lh_window layout) and the expected outputs of the reference
solve `problem.solve(10)` on it (src/lego/base/problem.cpp:156-230) as the two
independent CPU restatements compute it:
  * oracle/lego_oracle.c      (C, Eigen/Sophus arithmetic restated, dense
                               literal variant 0 and block-sparse variant 1)
  * oracle/lego_oracle_np.py  (NumPy twin, written separately; shares no code)
A fixture is written only when the restatements agree: the two C variants
on one LM trial (1e-11) and, on windows reproducible under summation
reorders, on the whole solve (iterations, trials, final chi2 1e-9); the NumPy
twin, which is not a bitwise mirror, with the C oracle under gate_mode 1 (the
Huber gate's rounding-residue sign, base_edge.cpp:55, taken as 0 on both
sides) on one trial (1e-9) and on the whole solve.  The stored outputs are the
C oracle's in reference mode (gate_mode 0).  The reference
itself cannot be built here (Eigen3/Sophus absent), so parity
stays unpinned by reference output; these vectors freeze the oracle's answers
so the GPU path (and any later change to the oracle) is checked against data
that does not move.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "lego-slam_amd", "python"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]

import lego_oracle_np as onp   # noqa: E402
import oracle_bind as ob       # noqa: E402
from windows import window     # noqa: E402

INPUT_KEYS = ("pose_Tcw", "pose_fixed", "lm_xyz", "obs_pose", "obs_lm", "obs_cam", "obs_uv", "K", "cam_ext")
OUTPUT_KEYS = ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "trace_chi2", "trace_lambda")
SCALAR_KEYS = ("chi2_initial", "chi2_final", "lambda_final", "iterations", "trials")

# (name, config, family, seed, solver options, window overrides)
CASES = [
    ("c1_stable_noout_s0", "C1", "stable_noout", 0, {}, {}),
    ("c1_stable_noout_s3", "C1", "stable_noout", 3, {}, {}),
    ("c1_stable_s1", "C1", "stable", 1, {}, {}),
    ("c1_default_s0", "C1", "default", 0, {}, {}),
    ("c1_strategy1_s2", "C1", "stable_noout", 2, dict(strategy=1), {}),
    ("c1_nohuber_lambda_s4", "C1", "stable_noout", 4, dict(huber_delta=0.0, lambda_init=1e-3), {}),
    ("c1_fixed_first_default_s5", "C1", "default", 5, {}, dict(fix_first=True)),
    ("c1_right_edges_s6", "C1", "stable_noout", 6, {}, dict(right_frac=0.5)),
    ("mini_stable_noout_s0", "mini", "stable_noout", 0, {}, {}),
    ("w24s_stable_noout_s1", "W24s", "stable_noout", 1, {}, {}),
]


def shrink(w):
    """Keep the fields the solver reads, in their ABI dtypes."""
    out = {}
    dts = dict(pose_Tcw=np.float64, pose_fixed=np.uint8, lm_xyz=np.float64, obs_pose=np.uint32, obs_lm=np.uint32,
               obs_cam=np.uint8, obs_uv=np.float64, K=np.float64, cam_ext=np.float64)
    for k in INPUT_KEYS:
        if w.get(k) is not None:
            out[k] = np.ascontiguousarray(w[k], dtype=dts[k])
    return out


def np_kwargs(opt):
    kw = {}
    if "strategy" in opt:
        kw["strategy"] = opt["strategy"]
    if "huber_delta" in opt:
        kw["huber_delta"] = opt["huber_delta"] if opt["huber_delta"] > 0 else None
    if "lambda_init" in opt:
        kw["lambda_init"] = opt["lambda_init"]
    return kw


def make(name, cfg, fam, seed, opt, over):
    fix_first = over.pop("fix_first", None)
    w = shrink(window(cfg, seed=seed, family=fam, fix_first=fix_first, **over))
    c1 = ob.solve(w, variant=1, **opt)
    c0 = ob.solve(w, variant=0, **opt)
    twin_rel = float("nan")
    # reproducible under summation reorders?  (decides the tolerance tier; a window with
    # outliers and a free gauge is chaotic, DESIGN.md §4.2, and only its first trial is compared)
    chis = [ob.solve(w, variant=1, n_threads=t, **opt)["chi2_final"] for t in (1, 2, 8)]
    spread = (max(chis) - min(chis)) / min(chis)
    # one LM trial (solve(1) with one trial) and the initial per-edge rho0 (solve(0)): the
    # per-linearisation arithmetic, comparable on every window, chaotic or not
    t1 = ob.solve(w, variant=1, max_iters=1, max_trials=1, **opt)
    e0 = ob.solve(w, variant=1, max_iters=0, **opt)
    t1d = ob.solve(w, variant=0, max_iters=1, max_trials=1, **opt)
    # the twin is not a bitwise mirror, so it meets the C oracle with the outlier gate's
    # rounding residue taken as 0 (gate_mode 1) - the only sign-of-rounding decision in the path
    t1g = ob.solve(w, variant=1, max_iters=1, max_trials=1, gate_mode=1, **opt)
    t1n = onp.solve(w, max_iters=1, max_trials=1, gate_mode=1, **np_kwargs(opt))
    # (the gauge-free "default" windows amplify summation-order rounding to ~1e-11 in one step)
    for other, ref, tag, tol in ((t1d, t1, "C dense, one trial", 1e-11),
                                 (t1n, t1g, "numpy twin, one trial, gate 1", 1e-9)):
        rel = abs(other["chi2_final"] - ref["chi2_final"]) / ref["chi2_final"]
        assert rel < tol, (name, tag, rel)
        assert np.allclose(other["pose_Tcw"], ref["pose_Tcw"], atol=100 * tol), (name, tag)
    if spread < 1e-12:
        cg = ob.solve(w, variant=1, gate_mode=1, **opt)
        tw = onp.solve(w, gate_mode=1, **np_kwargs(opt))
        for other, ref, tag in ((c0, c1, "C dense"), (tw, cg, "numpy twin, gate 1")):
            assert other["iterations"] == ref["iterations"] and other["trials"] == ref["trials"], (name, tag)
            rel = abs(other["chi2_final"] - ref["chi2_final"]) / ref["chi2_final"]
            assert rel < 1e-9, (name, tag, rel)
        twin_rel = abs(tw["chi2_final"] - cg["chi2_final"]) / cg["chi2_final"]
    data ={"in_" + k: v for k, v in w.items()}
    for k in OUTPUT_KEYS:
        data["out_" + k] = np.asarray(c1[k])
    for k in SCALAR_KEYS:
        data["out_" + k] = np.asarray(c1[k])
    for k in ("pose_Tcw", "lm_xyz", "edge_robust_chi2", "chi2_final", "accepted"):
        data["trial1_" + k] = np.asarray(t1[k])
    data["init_edge_robust_chi2"] = e0["edge_robust_chi2"]
    data["reorder_spread"] = np.asarray(spread)
    data["opt_json"] = np.asarray(repr(sorted(opt.items())))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **data)
    print(f"{name}: P={w['pose_Tcw'].shape[0]} L={w['lm_xyz'].shape[0]} O={w['obs_pose'].shape[0]} "
          f"iters={c1['iterations']} trials={c1['trials']} chi2={c1['chi2_final']:.12g} "
          f"twin_rel(gate 1)={twin_rel:.2e} spread={spread:.1e} "
          f"({os.path.getsize(path)} B)")


if __name__ == "__main__":
    only = set(sys.argv[1:])   # optional: names of the cases to (re)generate
    for case in CASES:
        if not only or case[0] in only:
            make(*case[:4], dict(case[4]), dict(case[5]))
