"""Synthetic image pairs for the LK optical-flow tests (no dataset is available: SURVEY.md 8(f) row 4).

A smooth random texture (sum of Gaussian blobs and a little fine noise, 8-bit) and the same scene
moved by a known sub-pixel flow (a global shift plus a smooth per-pixel field), rendered by bilinear
sampling of a 4x supersampled texture; keypoints are drawn inside the frame, near its borders and
outside it."""
import numpy as np


def _blobs(seed, rows, cols, n):
    rng = np.random.default_rng(seed)
    return (rng.uniform(-30, cols + 30, n), rng.uniform(-30, rows + 30, n), rng.uniform(2.0, 8.0, n),
            rng.uniform(-1, 1, n))


def _render(blobs, X, Y):
    """The analytic texture (a sum of Gaussian blobs) at real-valued positions X, Y, each blob
    evaluated only inside its 4-sigma box."""
    cx, cy, s, a = blobs
    out = np.zeros(X.shape)
    rows, cols = X.shape
    for i in range(len(cx)):
        r = 4.0 * s[i] + 16.0   # + the flow's reach
        x0, x1 = int(max(0, cx[i] - r)), int(min(cols, cx[i] + r + 1))
        y0, y1 = int(max(0, cy[i] - r)), int(min(rows, cy[i] + r + 1))
        if x0 >= x1 or y0 >= y1:
            continue
        dx = X[y0:y1, x0:x1] - cx[i]
        dy = Y[y0:y1, x0:x1] - cy[i]
        out[y0:y1, x0:x1] += a[i] * np.exp(-(dx * dx + dy * dy) / (2.0 * s[i] * s[i]))
    return out


def pair(rows=480, cols=640, shift=(2.3, -1.7), seed=0, noise=1.0):
    """img1, img2 (uint8) of one analytic scene, img2(x) = scene(x - d(x)): the content at x in img1
    moves to about x + d(x), d = shift + a smooth field of +-0.5 px (true_flow)."""
    rng = np.random.default_rng(seed + 1000)
    B = _blobs(seed, rows, cols, max(200, rows * cols // 80))
    yy, xx = np.mgrid[0:rows, 0:cols].astype(np.float64)
    fxd, fyd = flow(xx, yy, shift, seed)
    i1 = _render(B, xx, yy)
    i2 = _render(B, xx - fxd, yy - fyd)
    lo, hi = min(i1.min(), i2.min()), max(i1.max(), i2.max())
    to8 = lambda a: np.clip(np.rint((a - lo) / (hi - lo) * 230 + 12 + rng.normal(0, noise, a.shape)), 0, 255).astype(np.uint8)
    return to8(i1), to8(i2)


def flow(x, y, shift, seed):
    return (shift[0] + 0.5 * np.sin(x / 97.0 + seed) * np.cos(y / 71.0),
            shift[1] + 0.5 * np.cos(x / 83.0) * np.sin(y / 59.0 + seed))


def keypoints(rows, cols, n, seed, border=True):
    rng = np.random.default_rng(seed + 7)
    k = np.stack([rng.uniform(8, cols - 8, n), rng.uniform(8, rows - 8, n)], 1)
    if border:   # near and past the frame edges, fractional and integral
        extra = np.array([[0.0, 0.0], [cols - 1.0, rows - 1.0], [cols - 0.5, 10.5], [3.25, rows - 0.25],
                          [-2.0, 50.0], [cols + 3.0, 40.0], [1.5, 1.5], [cols - 2.0, rows - 2.0]])
        k = np.vstack([k, extra])
    return k.astype(np.float32)


def cornerness(img, k):
    """Smaller eigenvalue of the 7x7 structure tensor at keypoints k (GFTT's score): the points a
    feature detector would hand to the tracker."""
    g = img.astype(np.float64)
    gx = np.zeros_like(g)
    gy = np.zeros_like(g)
    gx[:, 1:-1] = 0.5 * (g[:, 2:] - g[:, :-2])
    gy[1:-1, :] = 0.5 * (g[2:, :] - g[:-2, :])
    out = np.zeros(len(k))
    for i, (x, y) in enumerate(k):
        xi, yi = int(x), int(y)
        if xi < 4 or yi < 4 or xi >= g.shape[1] - 4 or yi >= g.shape[0] - 4:
            continue
        a = gx[yi - 3:yi + 4, xi - 3:xi + 4]
        b = gy[yi - 3:yi + 4, xi - 3:xi + 4]
        sxx, syy, sxy = (a * a).sum(), (b * b).sum(), (a * b).sum()
        out[i] = 0.5 * (sxx + syy - np.sqrt((sxx - syy) ** 2 + 4 * sxy * sxy))
    return out
