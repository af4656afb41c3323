"""Backend::Optimize's outlier pass on the device (lh_result.is_outlier, ABI 5; backend_lego.cpp:163-194).

The reference counts the edges whose robust chi2 exceeds chi2_th, doubles chi2_th (at most five times)
while the inlier ratio is <= 0.5, then flags every edge above the final threshold.  The device pass
counts all five candidate thresholds in one pass and replays the loop on the counts; only the flags
cross the link.  Its flags, threshold and counts must equal the host pass (lh_classify_outliers, the
loop as written) on the per-edge chi2 of the same solve: bitwise, since both read the same rho0.
"""
import numpy as np
import pytest

import lego_ba
from windows import window

pytestmark = pytest.mark.gpu


def _check_same(g, th0):
    flags, th, ni, no = lego_ba.classify_outliers(g["edge_robust_chi2"], th0)
    assert np.array_equal(g["is_outlier"], flags.astype(bool))
    assert g["outlier_th"] == th
    assert (g["n_inlier"], g["n_outlier"]) == (ni, no)
    return th, ni, no


@pytest.mark.parametrize("cfg,seed,family", [("C1", 0, "default"), ("C2", 1, "default"), ("C3", 0, "default"),
                                             ("C2", 0, "stable_noout")])
def test_device_outlier_pass_equals_the_reference_loop(cfg, seed, family):
    w = window(cfg, seed=seed, family=family)
    s = lego_ba.Solver()
    g = s.solve(w, outlier_chi2_th=5.991)
    th, ni, no = _check_same(g, 5.991)
    assert ni + no == len(w["obs_pose"])
    # the flags alone (no per-edge chi2 download) are the same flags
    f = s.solve(w, outlier_chi2_th=5.991, want_edges=False)
    assert f["edge_robust_chi2"] is None
    assert np.array_equal(f["is_outlier"], g["is_outlier"]) and f["outlier_th"] == th
    s.close()


def test_device_outlier_pass_threshold_doubling():
    """A window where most edges are far off (70 % of the pixels moved by 40-80 px): the inlier ratio
    stays <= 0.5 at 5.991 and the loop doubles the threshold; a starting threshold so small that all
    five doublings run (the counts then are those at the fifth threshold, 16 x th0)."""
    w = window("C2", seed=3, family="default")
    rng = np.random.default_rng(7)
    uv = np.array(w["obs_uv"], np.float64)
    bad = rng.random(len(uv)) < 0.7
    uv[bad] += rng.uniform(40.0, 80.0, size=(bad.sum(), 2)).astype(np.float32).astype(np.float64)
    w["obs_uv"] = uv.astype(np.float32).astype(np.float64)
    s = lego_ba.Solver()
    for th0 in (5.991, 1e-6):
        g = s.solve(w, outlier_chi2_th=th0)
        th, ni, no = _check_same(g, th0)
        assert th > th0
    assert th == 1e-6 * 32
    s.close()


def test_device_outlier_pass_resident_and_abi4():
    """The resident path runs the same pass; an ABI-4 handle never reads the ABI-5 fields."""
    w = window("C2", seed=1, family="default")
    s = lego_ba.Solver()
    s.upload(w)
    g = s.solve_resident(want_edges=True, outlier_chi2_th=5.991)
    _check_same(g, 5.991)
    s.close()
    s4 = lego_ba.Solver(abi_version=4)
    g4 = s4.solve(w, outlier_chi2_th=5.991)
    assert not g4["is_outlier"].any() and g4["outlier_th"] == 0.0 and g4["n_outlier"] == 0
    s4.close()
