"""Synthetic camera sequences for the CMC tests (CPU and GPU): a textured scene seen through a
moving camera (known similarity per frame), rendered as BGR uint8 frames."""
import numpy as np
from scipy import ndimage


def scene(h, w, seed):
    rng = np.random.default_rng(seed)
    base = ndimage.gaussian_filter(rng.normal(0, 1, (h, w)), 6) * 40
    base += ndimage.gaussian_filter(rng.normal(0, 1, (h, w)), 2) * 25
    return np.clip(128 + base, 0, 255)


def similarity(theta_deg, s, tx, ty):
    t = np.deg2rad(theta_deg)
    return np.array([[s * np.cos(t), -s * np.sin(t), tx], [s * np.sin(t), s * np.cos(t), ty]])


def warp(img, M):
    """dst(x) = src(M^-1 x), bilinear, reflected borders."""
    h, w = img.shape[:2]
    Ai = np.linalg.inv(np.vstack([M, [0, 0, 1]]))
    ys, xs = np.mgrid[0:h, 0:w]
    sx = Ai[0, 0] * xs + Ai[0, 1] * ys + Ai[0, 2]
    sy = Ai[1, 0] * xs + Ai[1, 1] * ys + Ai[1, 2]
    return ndimage.map_coordinates(img, [sy, sx], order=1, mode="reflect")


def bgr(gray, seed=0):
    """A BGR frame whose channels differ (so the gray conversion's weights matter)."""
    g = np.clip(np.rint(gray), 0, 255)
    rng = np.random.default_rng(seed)
    off = rng.integers(-20, 21, size=3)
    return np.stack([np.clip(g + o, 0, 255) for o in off], axis=2).astype(np.uint8)


def sequence(h, w, n, seed, step=(0.2, 1.0, 6.0, -4.0)):
    """n frames; frame k = scene warped by the k-th power of a small similarity step
    (theta deg, scale, tx, ty per frame).  Returns (frames, per-frame cumulative 2x3)."""
    g = scene(h, w, seed)
    th, s, tx, ty = step
    frames, Ms = [], []
    for k in range(n):
        M = similarity(th * k, s ** k, tx * k, ty * k)
        frames.append(bgr(warp(g, M), seed))
        Ms.append(M)
    return frames, Ms


def boxes(h, w, n, seed):
    """n random detection boxes (x1 y1 x2 y2) inside / across the frame, some negative."""
    rng = np.random.default_rng(seed)
    x1 = rng.uniform(-40, w - 20, n)
    y1 = rng.uniform(-40, h - 20, n)
    return np.stack([x1, y1, x1 + rng.uniform(20, 200, n), y1 + rng.uniform(20, 300, n)], 1)
