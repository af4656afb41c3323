"""Frontend pose-only LM: Frontend::EstimateCurrentPose
(src/frontend_lego.cpp:157-250) batched over frames, lh_estimate_pose.

The oracle (oracle/lego_oracle.c orc_estimate_pose) restates the reference
loop: four rounds of problem.solve(10) from the frame's pose on one VertexPose
with EdgeProjectionPoseOnly edges (lego_types.h:116-180), outlier flags after
each round, no robust cost on round four.  Parity is unpinned by reference
output (the reference cannot be built).

Tolerances: the per-edge residual is a bitwise mirror of the oracle; sums over a
frame's edges are in a different (fixed) order, so states agree to rounding.
The pose problem has no gauge freedom (6 DoF, >= 3 points): the final pose is
compared at 1e-8, flags exactly except edges within 1e-6 of the 5.991 threshold,
iteration counts on 90 % of frames (the absolute stop rule, problem.cpp:210, sits
on rounding noise once a round has converged).
"""
import numpy as np
import pytest

import frames
import lego_ba
import oracle_bind as ob


def rot_err(a, b):
    Ra, Rb = a.reshape(3, 4)[:, :3], b.reshape(3, 4)[:, :3]
    return float(np.arccos(np.clip((np.trace(Ra.T @ Rb) - 1) / 2, -1, 1)))


# ------------------------------------------------------------------ CPU: the oracle
def test_oracle_recovers_pose():
    fb = frames.batch(0, 8)
    o = ob.estimate_pose(fb)
    for f in range(8):
        assert rot_err(o["pose_Tcw"][f], fb["pose_true"][f]) < 5e-3
        t = o["pose_Tcw"][f].reshape(3, 4)[:, 3] - fb["pose_true"][f].reshape(3, 4)[:, 3]
        assert np.linalg.norm(t) < 0.2
    # most tracking outliers are flagged (the last round is plain least squares over every edge)
    assert o["is_outlier"][fb["gross"]].mean() > 0.8


def test_oracle_rounds_semantics():
    """Rounds one to three are identical solves (same start, same edges: the flags never remove an
    edge); round four drops the robust cost (frontend_lego.cpp:223-225).  With no outliers and a
    loose start every edge is an inlier, so the flags are all clear and the pose is the plain
    least-squares optimum."""
    fb = frames.batch(3, 4, outlier_frac=0.0)
    o = ob.estimate_pose(fb)
    assert not o["is_outlier"][o["rchi2"] <= 5.991].any()
    assert np.all(o["iterations"] >= 4)
    plain = ob.estimate_pose(fb, huber_delta=0.0)   # no robust cost in any round: same final round
    assert np.allclose(plain["pose_Tcw"], o["pose_Tcw"], atol=1e-9)


def test_oracle_empty_and_tiny_frames():
    fb = frames.batch(1, 3, n_obs=[0, 1, 4])
    o = ob.estimate_pose(fb)
    assert np.array_equal(o["pose_Tcw"][0], fb["pose_Tcw"][0])   # solve() returns false: pose kept
    assert o["iterations"][0] == 0
    assert np.all(np.isfinite(o["pose_Tcw"]))


# ------------------------------------------------------------------ GPU
def _compare(g, o, fb):
    assert np.allclose(g["pose_Tcw"], o["pose_Tcw"], atol=1e-8, rtol=0)
    # the absolute stop rule (last_chi - chi < 1e-5, problem.cpp:210) sits on rounding noise once a
    # round has converged: an extra iteration or two moves the pose by far less than the bar above
    assert np.mean(g["iterations"] == o["iterations"]) >= 0.9
    near = np.abs(o["rchi2"] - 5.991) < 1e-6
    assert np.array_equal(g["is_outlier"][~near], o["is_outlier"][~near])
    assert np.allclose(g["edge_chi2"], o["rchi2"], rtol=1e-7, atol=1e-9)
    ptr = fb["obs_ptr"]
    for f in range(int(fb["n_frames"])):
        assert g["n_inliers"][f] == (ptr[f + 1] - ptr[f]) - int(g["is_outlier"][ptr[f]:ptr[f + 1]].sum())


@pytest.mark.gpu
def test_gpu_estimate_pose_matches_oracle():
    fb = frames.batch(0, 64)
    g = lego_ba.Solver().estimate_pose(fb)
    o = ob.estimate_pose(fb)
    _compare(g, o, fb)


@pytest.mark.gpu
def test_gpu_estimate_pose_ragged_and_flags_in():
    """Ragged frames (0, 1, 3, 300, 1000 edges: more edges than threads per frame) and features
    already flagged on entry (recomputed at the final estimate before classification, :208-210)."""
    sizes = [0, 1, 3, 150, 300, 1000, 7, 64]
    fb = frames.batch(5, len(sizes), n_obs=sizes)
    rng = np.random.default_rng(1)
    fin = rng.random(int(fb["obs_ptr"][-1])) < 0.1
    g = lego_ba.Solver().estimate_pose(fb, is_outlier_in=fin)
    o = ob.estimate_pose(fb, is_outlier_in=fin)
    _compare(g, o, fb)
    assert np.array_equal(g["pose_Tcw"][0], fb["pose_Tcw"][0])


@pytest.mark.gpu
@pytest.mark.parametrize("opt", [dict(strategy=1), dict(huber_delta=0.0), dict(lambda_init=1e-2)])
def test_gpu_estimate_pose_options(opt):
    fb = frames.batch(2, 16)
    g = lego_ba.Solver(**opt).estimate_pose(fb)
    o = ob.estimate_pose(fb, **opt)
    _compare(g, o, fb)


@pytest.mark.gpu
def test_gpu_estimate_pose_deterministic():
    fb = frames.batch(4, 32)
    s = lego_ba.Solver()
    a, b = s.estimate_pose(fb), s.estimate_pose(fb)
    assert np.array_equal(a["pose_Tcw"], b["pose_Tcw"]) and np.array_equal(a["edge_chi2"], b["edge_chi2"])
