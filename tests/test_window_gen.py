"""CPU tests of the synthetic window generator (lego-slam_amd/tools)."""
import numpy as np

import lego_ba


def test_deterministic():
    a = lego_ba.config_window("C1", seed=3)
    b = lego_ba.config_window("C1", seed=3)
    for k in a:
        if isinstance(a[k], np.ndarray):
            assert np.array_equal(a[k], b[k]), k
    c = lego_ba.config_window("C1", seed=4)
    assert not np.array_equal(a["obs_uv"], c["obs_uv"])


def test_shards_compose_the_window():
    full = lego_ba.generate_window(P=10, L=300, k=6, seed=1)
    parts = [lego_ba.generate_window(P=10, L=300, k=6, seed=1, lm_begin=b, lm_end=e) for b, e in [(0, 120), (120, 300)]]
    assert np.array_equal(np.vstack([p["lm_xyz"] for p in parts]), full["lm_xyz"])
    assert np.array_equal(np.concatenate([p["obs_uv"] for p in parts]), full["obs_uv"])
    assert np.array_equal(np.concatenate([parts[0]["obs_lm"], parts[1]["obs_lm"] + 120]), full["obs_lm"])
    assert np.array_equal(parts[1]["pose_Tcw"], full["pose_Tcw"])


def test_shapes_and_layout():
    w = lego_ba.config_window("C2", seed=0)
    assert w["pose_Tcw"].shape == (10, 12) and w["lm_xyz"].shape == (5000, 3)
    assert w["obs_uv"].shape == (40000, 2)
    # landmark-major, ascending pose inside a landmark, contiguous runs of k keyframes
    assert np.all(np.diff(w["obs_lm"].astype(np.int64)) >= 0)
    ol, op = w["obs_lm"].astype(np.int64), w["obs_pose"].astype(np.int64)
    same = ol[1:] == ol[:-1]
    assert np.all(op[1:][same] == op[:-1][same] + 1)
    # pixels are float32 values (toVec2 of a cv::KeyPoint)
    assert np.array_equal(w["obs_uv"].astype(np.float32).astype(np.float64), w["obs_uv"])


def test_measurements_consistent_with_truth():
    w = lego_ba.generate_window(P=10, L=2000, k=8, seed=5, outlier_frac=0.0, noise_px=0.0)
    K = w["K"]
    T = w["pose_true"].reshape(-1, 3, 4)[w["obs_pose"]]
    X = w["lm_true"][w["obs_lm"]]
    Pc = np.einsum("nij,nj->ni", T[:, :, :3], X) + T[:, :, 3]
    uv = np.stack([K[0] * Pc[:, 0] / Pc[:, 2] + K[2], K[1] * Pc[:, 1] / Pc[:, 2] + K[3]], 1)
    assert np.max(np.abs(uv - w["obs_uv"])) < 1e-3   # float32 rounding only
    assert np.all(Pc[:, 2] > 1.0)


def test_right_camera_and_outliers():
    w = lego_ba.generate_window(P=10, L=2000, k=8, seed=6, right_frac=0.5)
    frac = w["obs_cam"].mean()
    assert 0.45 < frac < 0.55
    assert np.allclose(w["cam_ext"][1], [1, 0, 0, -0.537, 0, 1, 0, 0, 0, 0, 1, 0])
