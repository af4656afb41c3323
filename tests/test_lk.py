"""Pyramidal Gauss-Newton LK optical flow: LKOpticalFlow4Layer / 1Layer of
src/algorithm.cpp:11-206 through lh_lk_track (include/lego_ba.h).

Parity is unpinned: the reference ships no fixtures for it and needs OpenCV (absent).  The oracle
(oracle/lk_oracle.c) restates it; CPU tests pin the restatement with known answers (a moved
texture is tracked to its true flow, a flat image leaves points in place) and an independent NumPy
restatement of its pyramid.  GPU tests: the HIP path is a bitwise mirror (kp2 and success equal),
in both modes, 4 and 1 levels, with and without an initial guess, on even and odd image sizes."""
import numpy as np
import pytest

import images
import oracle_bind as ob


def true_flow(k, shift, seed):
    """The flow of images.pair at the tracked points: q = p + d(q), solved by fixed point."""
    p = k.astype(np.float64)
    q = p.copy()
    for _ in range(20):
        dx, dy = images.flow(q[:, 0], q[:, 1], shift, seed)
        q = p + np.stack([dx, dy], 1)
    return q - p


@pytest.mark.parametrize("shift", [(2.3, -1.7), (9.6, 4.2)])
def test_oracle_tracks_a_moved_texture(shift):
    rows, cols = 240, 320
    i1, i2 = images.pair(rows, cols, shift=shift, seed=3)
    k1 = images.keypoints(rows, cols, 300, seed=3, border=False)
    inner = (k1[:, 0] > 20) & (k1[:, 0] < cols - 20) & (k1[:, 1] > 20) & (k1[:, 1] < rows - 20)
    c = images.cornerness(i1, k1)                 # textured points, as a corner detector picks them
    inner &= c >= np.percentile(c[inner], 67)
    r = ob.lk_track(i1, i2, k1, kp2_init=k1)   # the frontend's call: has_initial, forward
    err = np.linalg.norm(r["kp2"] - k1 - true_flow(k1, shift, 3), axis=1)
    good = r["success"] & inner
    assert good.sum() > 0.9 * inner.sum()
    assert np.median(err[good]) < 0.1 and np.percentile(err[good], 90) < 0.25


def test_oracle_flat_image_keeps_points():
    img = np.full((120, 160), 77, np.uint8)
    k1 = images.keypoints(120, 160, 20, seed=1, border=False)
    r = ob.lk_track(img, img, k1, kp2_init=k1)
    assert np.array_equal(r["kp2"], k1) and np.all(r["success"])


def np_pyr_down(src, dw, dh):
    """Independent NumPy restatement of cv::resize(INTER_LINEAR, 0.5) on 8-bit images."""
    sh, sw = src.shape
    s = src.astype(np.int64)
    if sw == 2 * dw and sh == 2 * dh:
        return ((s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2).astype(np.uint8)
    def coefs(dn, sn):
        scale = 1.0 / (dn / sn)
        d = np.arange(dn)
        f = ((d + 0.5) * scale - 0.5).astype(np.float32)
        i = np.floor(f).astype(np.int64)
        f = (f - i.astype(np.float32)).astype(np.float32)
        f[i < 0] = 0
        i[i < 0] = 0
        hi = i + 1 >= sn
        f[hi] = 0
        i[hi] = sn - 1
        a0 = np.rint(((np.float32(1) - f) * np.float32(2048)).astype(np.float32)).astype(np.int64)
        a1 = np.rint((f * np.float32(2048)).astype(np.float32)).astype(np.int64)
        return i, np.minimum(i + 1, sn - 1), a0, a1
    x0, x1, a0, a1 = coefs(dw, sw)
    y0, y1, b0, b1 = coefs(dh, sh)
    h0 = s[y0][:, x0] * a0 + s[y0][:, x1] * a1
    h1 = s[y1][:, x0] * a0 + s[y1][:, x1] * a1
    v = (h0 * b0[:, None] + h1 * b1[:, None] + (1 << 21)) >> 22
    return np.clip(v, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("rows,cols", [(480, 640), (376, 1241), (47, 81), (240, 320)])
def test_oracle_pyramid_matches_numpy(rows, cols):
    rng = np.random.default_rng(rows + cols)
    img = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    for _ in range(3):
        dw, dh = int(img.shape[1] * 0.5), int(img.shape[0] * 0.5)
        a = ob.lk_pyr_down(img, dw, dh)
        assert np.array_equal(a, np_pyr_down(img, dw, dh))
        img = a


def test_lk_symbol_exported():
    import lego_ba
    assert "lh_lk_track" in lego_ba.ABI_SYMBOLS


# ------------------------------------------------------------------------------------- GPU
CASES = [  # rows, cols, shift, inverse, levels, initial
    (480, 640, (2.3, -1.7), False, 4, True),
    (480, 640, (9.6, 4.2), False, 4, False),
    (480, 640, (2.3, -1.7), True, 4, True),
    (376, 1241, (3.1, 0.4), False, 4, True),
    (240, 320, (0.8, 0.6), False, 1, True),
    (121, 163, (1.2, -2.5), True, 1, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("rows,cols,shift,inverse,levels,initial", CASES)
def test_gpu_lk_bitwise_vs_oracle(rows, cols, shift, inverse, levels, initial):
    import lego_ba
    i1, i2 = images.pair(rows, cols, shift=shift, seed=rows)
    k1 = images.keypoints(rows, cols, 500, seed=cols)
    init = (k1 + np.float32(0.5) * np.array(shift, np.float32)) if initial else None
    s = lego_ba.Solver(device=0)
    g = s.lk_track(i1, i2, k1, kp2_init=init, inverse=inverse, levels=levels)
    o = ob.lk_track(i1, i2, k1, kp2_init=init, inverse=inverse, levels=levels)
    s.close()
    assert np.array_equal(g["success"], o["success"])
    assert np.array_equal(g["kp2"], o["kp2"])
    assert g["success"].mean() > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("inverse,levels,init_off", [(False, 1, None), (True, 1, None), (False, 4, (90.0, -70.0))])
def test_gpu_lk_taps_outside_the_staged_window(inverse, levels, init_off):
    """k_lk_track reads the second image from an LDS window placed at each level's initial guess
    (32 x 24 bytes); a large motion tracked on one level, or a far-off initial guess, drives the
    taps out of it onto the global-memory path, which must give the same bits."""
    import lego_ba
    rows, cols, shift = 200, 300, (13.5, -9.2)
    i1, i2 = images.pair(rows, cols, shift=shift, seed=5)
    k1 = images.keypoints(rows, cols, 400, seed=6)
    init = None if init_off is None else k1 + np.float32(init_off)
    s = lego_ba.Solver(device=0)
    g = s.lk_track(i1, i2, k1, kp2_init=init, inverse=inverse, levels=levels)
    o = ob.lk_track(i1, i2, k1, kp2_init=init, inverse=inverse, levels=levels)
    s.close()
    assert np.array_equal(g["success"], o["success"])
    assert np.array_equal(g["kp2"], o["kp2"])
    moved = np.abs(o["kp2"] - (k1 if init is None else init)).max(axis=1)
    assert (moved > 11).any()   # some keypoints did leave the window


@pytest.mark.gpu
def test_gpu_lk_empty_and_errors():
    import lego_ba
    s = lego_ba.Solver(device=0)
    img = np.zeros((32, 48), np.uint8)
    r = s.lk_track(img, img, np.zeros((0, 2), np.float32))
    assert r["kp2"].shape == (0, 2)
    with pytest.raises(lego_ba.LhError) as e:
        s.lk_track(img, img, np.zeros((3, 2), np.float32), levels=3)
    assert e.value.status == lego_ba.LH_E_BADARG
    s.close()
