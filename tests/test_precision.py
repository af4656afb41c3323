"""lh_options.precision = LH_PREC_FP32_RESID (BASELINE config 3's "fp32 residuals + fp64
accumulate"): k_lin<T, TRIAL, true> evaluates each edge's Jacobians in float and widens them before any
product that is summed.  The residual, the Huber weight, rho0, chi2, b's residual factor and the gain
ratio stay the fp64 mirror of the reference's arithmetic: an earlier form that
also took the residual in float (~3e-5 px of rounding per edge) stopped C3 after 2 iterations at chi2
+1.8 % (round-3 VERDICT), because that noise entered b and the LM decision on C3's weakly observed
stereo scale.  The step is now Gauss-Newton on a Jacobian rounded to float: the same fixed point to
second order, so the solve ends within tolerance of the fp64 solve of the same window."""
import numpy as np
import pytest

import lego_ba
from windows import window

pytestmark = pytest.mark.gpu


def rel(a, b):
    return abs(a - b) / abs(b)


@pytest.mark.parametrize("cfg,seed,family", [("C1", 0, "stable_noout"), ("C2", 1, "stable_noout"), ("C3", 0, "default")])
def test_fp32_mode_evaluation_is_the_fp64_mirror(cfg, seed, family):
    """The evaluation (no step) is the fp64 path's: the same chi2 and every edge's robust chi2, bit for bit."""
    w = window(cfg, seed=seed, family=family)
    a = lego_ba.Solver(device=0, max_iters=0).solve(w)
    b = lego_ba.Solver(device=0, max_iters=0, precision=lego_ba.LH_PREC_FP32_RESID).solve(w)
    assert a["chi2_initial"] == b["chi2_initial"]
    assert np.array_equal(a["edge_robust_chi2"], b["edge_robust_chi2"])


@pytest.mark.parametrize("cfg,seed", [("C1", 0), ("mini", 5), ("C2", 1)])
def test_fp32_mode_solve_on_small_windows(cfg, seed):
    """Reproducible windows (no outliers): the fp64 solve's path and final chi2 to 1e-6."""
    w = window(cfg, seed=seed, family="stable_noout")
    a = lego_ba.Solver(device=0).solve(w)
    b = lego_ba.Solver(device=0, precision=lego_ba.LH_PREC_FP32_RESID).solve(w)
    assert b["iterations"] == a["iterations"]
    assert rel(b["chi2_final"], a["chi2_final"]) <= 1e-6, (a["iterations"], b["iterations"])


def test_fp32_mode_on_an_outlier_window_lands_in_the_oracle_envelope():
    """With outliers the reference LM itself is chaotic (the Huber gate's rounding residue,
    base_edge.cpp:55): a Jacobian rounded to float moves the path like a change of summation order
    does (mini seed 3: 9 iterations against fp64's 10).  The solve must end inside the oracle's own
    reorder envelope."""
    import oracle_bind as ob
    w = window("mini", seed=3, family="stable")
    b = lego_ba.Solver(device=0, precision=lego_ba.LH_PREC_FP32_RESID).solve(w)
    chis = [ob.solve(w, n_threads=t)["chi2_final"] for t in range(1, 17)]
    spread = (max(chis) - min(chis)) / min(chis)
    assert min(rel(b["chi2_final"], c) for c in chis) <= max(1e-6, 10 * spread)


def test_fp32_mode_full_solve_on_c3():
    """BASELINE config 3's window (C3, 20 KF / 50 k landmarks / 400 k observations) in the fp32 mode: the
    same LM path as the fp64 solve (iterations, trials) and the final chi2 within 1e-6 (north star)."""
    w = window("C3", seed=0, family="stable_noout")
    a = lego_ba.Solver(device=0).solve(w)
    b = lego_ba.Solver(device=0, precision=lego_ba.LH_PREC_FP32_RESID).solve(w)
    assert (b["iterations"], b["trials"]) == (a["iterations"], a["trials"])
    assert rel(b["chi2_final"], a["chi2_final"]) <= 1e-6
    assert np.allclose(b["pose_Tcw"], a["pose_Tcw"], atol=1e-6)


def test_fp32_mode_is_repeatable_and_a_valid_option():
    w = window("C1", seed=4, family="stable")
    s = lego_ba.Solver(device=0, precision=lego_ba.LH_PREC_FP32_RESID)
    r1, r2 = s.solve(w), s.solve(w)
    assert r1["chi2_final"] == r2["chi2_final"] and np.array_equal(r1["lm_xyz"], r2["lm_xyz"])
    with pytest.raises(lego_ba.LhError) as e:
        lego_ba.Solver(device=0, precision=2)
    assert e.value.status == lego_ba.LH_E_BADARG


def test_config3_as_written_fp32_and_pcg_against_the_oracle_pcg():
    """BASELINE configs[2] as written: C3 (20 KF / 50 k landmarks / 400 k observations), fp32 residual
    path + fp64 accumulation AND Schur + PCG, together, against the oracle's (fixed) PCG
    (problem.cpp:584-614, oracle/lego_oracle.c pcg_solve) on the reproducible C3 window: the same
    iterations and trials, the final chi2 and the poses within 1e-6 (north star), landmarks 1e-6."""
    import oracle_bind as ob
    w = window("C3", seed=0, family="stable_noout")
    s = lego_ba.Solver(device=0, precision=lego_ba.LH_PREC_FP32_RESID, linear_solver=lego_ba.LH_SOLVER_PCG)
    g = s.solve(w)
    assert s.controller() == "k_ctrl"
    assert g["pcg_iterations"] > 0
    o = ob.solve(w, linear_solver=1)
    assert (g["iterations"], g["trials"]) == (o["iterations"], o["trials"])
    assert rel(g["chi2_initial"], o["chi2_initial"]) < 1e-12
    assert rel(g["chi2_final"], o["chi2_final"]) <= 1e-6
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-6)
    assert np.allclose(g["lm_xyz"], o["lm_xyz"], atol=1e-6)
    # and the reference's own solver (LDLT) on the same window lands at the same chi2
    r = ob.solve(w)
    assert rel(g["chi2_final"], r["chi2_final"]) <= 1e-6


def test_fp32_mode_on_the_live_c3_configuration_lands_in_the_oracle_envelope():
    """The reference's live configuration at the headline size (survey-default C3: free gauge, left
    image only, 2 % outliers, reference Huber gate) in the fp32 mode.  No summation order of the
    reference reproduces this window (tests/test_live_config.py: 16 oracle thread counts, 16 outcomes),
    so the fp32 solve must end inside the envelope of those 16 outcomes, its iteration count in their
    range, with the initial chi2 bitwise the fp64 evaluation's."""
    import oracle_bind as ob
    w = window("C3", seed=0)
    g = lego_ba.Solver(device=0, precision=lego_ba.LH_PREC_FP32_RESID).solve(w)
    runs = [ob.solve(w, n_threads=t) for t in range(1, 17)]
    chis = [r["chi2_final"] for r in runs]
    its = [r["iterations"] for r in runs]
    assert rel(g["chi2_initial"], runs[0]["chi2_initial"]) < 1e-12
    assert min(chis) * (1 - 1e-6) <= g["chi2_final"] <= max(chis) * (1 + 1e-6)
    assert min(its) <= g["iterations"] <= max(its)
