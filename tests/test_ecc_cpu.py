"""CPU: the ECC restatement (oracle/cmc_ecc.py) on its own terms.  cv2 is absent, so parity with
OpenCV's findTransformECC itself is unpinned; these tests pin the restatement's building blocks
(fixed-point warp coordinates, exact bilinear samples, the fixed reduction order, cv::invert) and
its end-to-end behaviour: identical frames, known shifts and rotations recovered, the MOT17-mini
fixture frames, and the reference's identity-on-error path (ecc.py:82-84, prev_img kept)."""
import os

import numpy as np
import pytest
from scipy import ndimage

from oracle import cmc_ecc as ce

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "cmc_mot17.npz")


def smooth_scene(h, w, seed, sigma=12.0):
    rng = np.random.default_rng(seed)
    lo = ndimage.gaussian_filter(rng.normal(0, 1, (h, w)), sigma)
    hi = ndimage.gaussian_filter(rng.normal(0, 1, (h, w)), sigma / 3)
    base = lo / lo.std() * 35 + hi / hi.std() * 8
    return np.clip(128 + base, 0, 255)


def warp_scene(g, M):
    """out(x) = g(A x) for the 2x3 A = M, bilinear, reflected borders."""
    h, w = g.shape
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float64)
    sx = M[0, 0] * xs + M[0, 1] * ys + M[0, 2]
    sy = M[1, 0] * xs + M[1, 1] * ys + M[1, 2]
    return ndimage.map_coordinates(g, [sy, sx], order=1, mode="reflect")


def u8(a):
    return np.clip(np.rint(a), 0, 255).astype(np.uint8)


def test_block_sum_order():
    rng = np.random.default_rng(0)
    for n in (1, 63, 1024, 1500, 20736):
        v = rng.normal(0, 1, n)
        assert abs(ce.block_sum(v) - v.sum()) <= 1e-12 * max(1.0, np.abs(v).sum())
    # the documented order: thread t adds pixels t, t + 1024, ... then halving trees over groups
    # of 16 threads and over the 64 group partials
    v = rng.normal(0, 1, (2, 3000))
    acc = np.zeros((2, 1024))
    for r in range(3):
        blk = np.zeros((2, 1024))
        seg = v[:, r * 1024:(r + 1) * 1024]
        blk[:, :seg.shape[1]] = seg
        acc = acc + blk
    lanes = acc.reshape(2, 64, 16)
    while lanes.shape[-1] > 1:
        lanes = lanes[..., :lanes.shape[-1] // 2] + lanes[..., lanes.shape[-1] // 2:]
    waves = lanes[..., 0]
    while waves.shape[-1] > 1:
        waves = waves[..., :waves.shape[-1] // 2] + waves[..., waves.shape[-1] // 2:]
    assert np.array_equal(ce.block_sum(v), waves[:, 0])
    assert ce.block_sum(np.arange(10.0), n_threads=512) == 45.0


def test_warp_coords_fixed_point():
    sx, sy, al, nx, ny = ce.warp_coords(np.eye(2, 3, dtype=np.float32), 3, 4)
    assert np.array_equal(sx, np.tile(np.arange(4), (3, 1))) and not al.any()
    assert np.array_equal(ny, np.tile(np.arange(3)[:, None], (1, 4)))
    # a quarter-pixel shift lands on table entry 8 (of 32), nearest rounds half up
    M = np.array([[1, 0, 0.25], [0, 1, -0.5]], np.float32)
    sx, sy, al, nx, ny = ce.warp_coords(M, 2, 3)
    assert np.array_equal(sx[0], [0, 1, 2]) and np.all(al % 32 == 8)
    assert np.all(sy[0] == -1) and np.all(al // 32 == 16)
    assert np.array_equal(nx[0], [0, 1, 2]) and np.all(ny[0] == 0)
    # bilinear samples of u8 data are exact: equal to the float64 interpolation
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (9, 11)).astype(np.float32)
    M = np.array([[0.97, 0.05, 1.3], [-0.04, 1.02, 0.7]], np.float32)
    sx, sy, al, _, _ = ce.warp_coords(M, 9, 11)
    got = ce.remap_linear(img, sx, sy, al)
    fx, fy = (al % 32) / 32.0, (al // 32) / 32.0

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < 11) & (yy >= 0) & (yy < 9)
        return np.where(ok, img[np.clip(yy, 0, 8), np.clip(xx, 0, 10)].astype(np.float64), 0.0)

    ref = ((1 - fy) * ((1 - fx) * tap(sy, sx) + fx * tap(sy, sx + 1))
           + fy * ((1 - fx) * tap(sy + 1, sx) + fx * tap(sy + 1, sx + 1)))
    assert np.array_equal(got.astype(np.float64), ref)


def test_gradients_reflect101():
    img = np.array([[0, 4, 10, 30], [2, 2, 2, 2], [8, 0, 8, 0]], np.uint8)
    gx, gy = ce.gradients(img)
    assert gx[0].tolist() == [0.0, 5.0, 13.0, 0.0]
    assert gy[:, 0].tolist() == [0.0, 4.0, 0.0] and gy[1, 1] == -2.0


@pytest.mark.parametrize("n", [2, 3, 6])
def test_invert_matches_linalg(n):
    rng = np.random.default_rng(n)
    A = rng.normal(0, 1, (n, n))
    H = (A @ A.T + n * np.eye(n)).astype(np.float32)
    np.testing.assert_allclose(ce.invert(H), np.linalg.inv(H.astype(np.float64)), rtol=2e-4,
                               atol=1e-6)
    assert not ce.invert(np.zeros((n, n), np.float32)).any()


def test_identical_frames_identity():
    g = u8(smooth_scene(108, 192, 3))
    for mode in (0, 1, 2):
        st = {}
        rho, W = ce.find_transform_ecc(g, g, np.eye(2, 3, dtype=np.float32), mode, 100, 1e-5, st)
        assert rho > 0.999999 and st["iters"] <= 3
        np.testing.assert_allclose(W, np.eye(2, 3), atol=1e-6)


@pytest.mark.parametrize("mode,M", [
    (0, [[1, 0, 1.75], [0, 1, -0.8]]),
    (1, [[np.cos(0.02), -np.sin(0.02), 1.2], [np.sin(0.02), np.cos(0.02), 0.6]]),
    (2, [[1.01, 0.02, -0.9], [-0.015, 0.99, 1.4]]),
])
def test_known_motion_recovered(mode, M):
    M = np.array(M)
    g = smooth_scene(160, 240, 7)
    prev = u8(g[20:128, 24:216])
    cur = u8(warp_scene(g, np.linalg.inv(np.vstack([M, [0, 0, 1]]))[:2])[20:128, 24:216])
    # cur(M x) = g(x) on the scene grid; on the crop the template pixel x maps to M (x + o) - o
    o = np.array([24.0, 20.0])
    expect = M.copy()
    expect[:, 2] = M[:, :2] @ o + M[:, 2] - o
    rho, W = ce.find_transform_ecc(prev, cur, np.eye(2, 3, dtype=np.float32), mode, 100, 1e-6)
    assert rho > 0.99
    np.testing.assert_allclose(W[:, :2], expect[:, :2], atol=2e-3)
    np.testing.assert_allclose(W[:, 2], expect[:, 2], atol=0.15)


def test_mot17_frames_converge():
    g = np.load(FIXTURE)
    for key in g.files:
        ims = g[key]
        for i in range(1, 3):
            for mode in (0, 1):
                st = {}
                rho, W = ce.find_transform_ecc(ims[i - 1], ims[i], np.eye(2, 3, dtype=np.float32),
                                               mode, 100, 1e-5, st)
                assert rho > 0.9 and np.abs(W[:, 2]).max() < 5 and 1 <= st["iters"] <= 100


def test_ecc_class_first_frame_scale_and_errors():
    g = smooth_scene(1080 // 4, 1920 // 4, 11, sigma=4)
    big = ndimage.zoom(g, 4, order=1)
    frame = np.repeat(u8(big)[..., None], 3, axis=2)
    shifted = np.repeat(u8(np.roll(big, (-20, 30), axis=(0, 1)))[..., None], 3, axis=2)
    o = ce.ECCOracle()
    W0 = o.apply(frame)
    assert W0.dtype == np.float32 and np.array_equal(W0, np.eye(2, 3))
    assert o.prev_img.shape == (108, 192)
    W = o.apply(shifted)
    assert o.last["outcome"] == 1
    # cur(x) = prev(x - (30, -20)) at full resolution, so cur(x + (30, -20)) = prev(x): the
    # translation comes back in full-resolution pixels (divided by the scale)
    np.testing.assert_allclose(W[:, 2], [30.0, -20.0], atol=1.5)
    prev = o.prev_img.copy()
    # a flat frame: zero variance -> NaN correlation -> OpenCV raises -> identity, prev kept
    flat = np.full_like(frame, 90)
    assert np.array_equal(o.apply(flat), np.eye(2, 3)) and o.last["outcome"] == 2
    assert np.array_equal(o.prev_img, prev)
    with pytest.raises(NotImplementedError):
        ce.ECCOracle(warp_mode=ce.MOTION_HOMOGRAPHY).apply(frame)


def test_uncorrelated_frames_raise():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (60, 80), dtype=np.uint8)
    b = rng.integers(0, 256, (60, 80), dtype=np.uint8)
    for mode in (0, 1, 2):
        with pytest.raises(ce.ECCError):
            ce.find_transform_ecc(a, b, np.eye(2, 3, dtype=np.float32), mode, 100, 1e-5)


def test_warp_affine_u8_identity_and_shift():
    """align=True's warpAffine (INTER_LINEAR, forward matrix inverted first, BORDER_CONSTANT 0):
    the identity returns the image bit for bit; an integer translation moves it with zeros
    entering (dst(x, y) = src(x - tx, y - ty))."""
    img = u8(smooth_scene(37, 53, 3))
    assert np.array_equal(ce.warp_affine_u8(img, np.eye(2, 3, dtype=np.float32), 37, 53), img)
    M = np.array([[1, 0, 5], [0, 1, -3]], np.float32)
    out = ce.warp_affine_u8(img, M, 37, 53)
    want = np.zeros_like(img)
    want[:34, 5:] = img[3:, :48]
    assert np.array_equal(out, want)


def test_warp_affine_u8_rotation_close_to_float_bilinear():
    """A rotation + subpixel shift: within one grey level of a float64 bilinear warp of the same
    inverse map (the 1/32-pixel fixed-point grid and the 15-bit weights are the only differences),
    away from the border; the direction of the map is the forward one (cv2's default)."""
    img = u8(smooth_scene(90, 120, 8))
    th = 0.05
    M = np.array([[np.cos(th), -np.sin(th), 4.3], [np.sin(th), np.cos(th), -2.7]], np.float32)
    out = ce.warp_affine_u8(img, M, 90, 120).astype(np.float64)
    A = np.vstack([M.astype(np.float64), [0, 0, 1]])
    Ai = np.linalg.inv(A)[:2]
    ys, xs = np.mgrid[0:90, 0:120].astype(np.float64)
    sx = Ai[0, 0] * xs + Ai[0, 1] * ys + Ai[0, 2]
    sy = Ai[1, 0] * xs + Ai[1, 1] * ys + Ai[1, 2]
    ref = ndimage.map_coordinates(img.astype(np.float64), [sy, sx], order=1, mode="constant")
    inner = (sx > 1) & (sx < 118) & (sy > 1) & (sy < 88)
    assert np.abs(out - ref)[inner].max() <= 2.0
    assert np.abs(out - ref)[inner].mean() < 0.6


def test_ecc_oracle_align_preview():
    """ECC(align=True) (ecc.py:91-98): after an estimate prev_img_aligned is the previous gray
    frame (its shape) warped by the returned matrix; align=False leaves None; the identity-on-error
    path returns before it and keeps the last preview."""
    big = smooth_scene(1080, 1920, 1)
    frame = np.repeat(u8(big)[..., None], 3, axis=2)
    shifted = np.repeat(u8(np.roll(big, (-20, 30), axis=(0, 1)))[..., None], 3, axis=2)
    o = ce.ECCOracle(align=True)
    o.apply(frame)
    assert o.prev_img_aligned is None
    prev = o.prev_img.copy()
    W = o.apply(shifted)
    assert o.last["outcome"] == 1
    assert o.prev_img_aligned.shape == prev.shape == (108, 192)
    assert np.array_equal(o.prev_img_aligned, ce.warp_affine_u8(prev, W, 108, 192))
    kept = o.prev_img_aligned.copy()
    assert np.array_equal(o.apply(np.full_like(frame, 90)), np.eye(2, 3))
    assert o.last["outcome"] == 2 and np.array_equal(o.prev_img_aligned, kept)
    n = ce.ECCOracle(align=False)
    n.apply(frame)
    n.apply(shifted)
    assert n.prev_img_aligned is None
