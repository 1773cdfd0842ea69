"""GPU: the individual HIP primitives against the reference's known-answer vectors (bit-exact
for IoU / GIoU / DIoU / fuse_score; KF within 1e-9 relative; assignment indices exact)."""
import os

import numpy as np
import pytest

from oracle.lap import lapjv
from yolo_tracking_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kiou(golden_dir):
    return np.load(os.path.join(golden_dir, "kat_iou.npz"))


def test_iou_giou_diou_bit_exact(kiou):
    a, b = kiou["a"], kiou["b"]
    for kind in ("iou", "giou", "diou"):
        got = _lib.box_affinity(a, b, kind)
        assert np.array_equal(got, kiou[kind]), kind


def test_ciou_centroid_close(kiou):
    # arctan / sqrt paths: not correctly rounded on either side -> 1e-12 absolute
    a, b = kiou["a"], kiou["b"]
    np.testing.assert_allclose(_lib.box_affinity(a, b, "ciou"), kiou["ciou"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(_lib.box_affinity(a, b, "centroid", 640, 480), kiou["centroid"],
                               rtol=0, atol=1e-12)


def test_iou_distance_and_fuse_score_bit_exact(kiou):
    a, b = kiou["a"], kiou["b"]
    assert np.array_equal(_lib.iou_distance(a, b), kiou["iou_distance"])
    assert np.array_equal(_lib.iou_distance(a, b, kiou["det_scores"]), kiou["fuse_score"])


def test_giou_degenerate_enclosure_raises():
    a = np.array([[5.0, 5.0, 5.0, 5.0]])
    with pytest.raises(_lib.YTAError):
        _lib.box_affinity(a, a, "giou")


def test_kf_xyah_kat(golden_dir):
    g = np.load(os.path.join(golden_dir, "kat_kf_xyah.npz"))
    m, c = _lib.kf_xyah_initiate(g["meas"])
    assert np.array_equal(m, g["init_mean"]) and np.array_equal(c, g["init_cov"])
    pm, pc = _lib.kf_xyah_predict(g["pred_in_mean"], g["pred_in_cov"])
    assert np.array_equal(pm, g["pred_mean"])
    # packed symmetric covariance: upper triangle bit-exact, lower within 1 ulp-ish
    iu = np.triu_indices(8)
    assert np.array_equal(pc[:, iu[0], iu[1]], g["pred_cov"][:, iu[0], iu[1]])
    np.testing.assert_allclose(pc, g["pred_cov"], rtol=1e-14, atol=0)
    um, uc = _lib.kf_xyah_update(g["pred_mean"], g["pred_cov"], g["z"])
    np.testing.assert_allclose(um, g["upd_mean"], rtol=1e-10, atol=1e-9)
    np.testing.assert_allclose(uc, g["upd_cov"], rtol=1e-8, atol=1e-9)


def test_lap_limited_kat(golden_dir):
    g = np.load(os.path.join(golden_dir, "kat_lap.npz"))
    for k in range(int(g["n_cases"])):
        lim = float(g[f"c{k}__limit"])
        if not np.isfinite(lim):
            continue   # padded (no cost_limit) solves belong to the OCSORT-family dense path
        x, y = _lib.lap_limited(g[f"c{k}__cost"], lim)
        assert np.array_equal(x, g[f"c{k}__x"]), k
        assert np.array_equal(y, g[f"c{k}__y"]), k


@pytest.mark.parametrize("seed", range(6))
def test_lap_limited_random_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    for trial in range(25):
        nr, nc = rng.integers(1, 90, size=2)
        density = rng.choice([0.02, 0.1, 0.5, 1.0])
        cost = np.where(rng.random((nr, nc)) < density, rng.random((nr, nc)) * 0.9, 1.0)
        lim = float(rng.choice([0.3, 0.5, 0.8, 0.95]))
        x, y = _lib.lap_limited(cost, lim)
        _, xo, yo = lapjv(cost, extend_cost=True, cost_limit=lim)
        assert np.array_equal(x, xo), (seed, trial)
        assert np.array_equal(y, yo), (seed, trial)


def test_lap_limited_large_component():
    # one dense 300 x 300 block: exceeds the LDS slab, exercises the global-memory solver
    rng = np.random.default_rng(99)
    cost = rng.random((300, 300)) * 0.5
    x, y = _lib.lap_limited(cost, 0.8)
    _, xo, yo = lapjv(cost, extend_cost=True, cost_limit=0.8)
    assert np.array_equal(x, xo) and np.array_equal(y, yo)


def test_lap_limited_empty():
    x, y = _lib.lap_limited(np.zeros((0, 4)), 0.8)
    assert len(x) == 0 and np.all(y == -1)
    x, y = _lib.lap_limited(np.zeros((3, 0)), 0.8)
    assert np.all(x == -1) and len(y) == 0


def _brute_pairs(a, b, thresh):
    from oracle.geometry import iou_batch
    if len(a) == 0 or len(b) == 0:
        return np.zeros((0, 2), dtype=np.int32)
    d = 1 - iou_batch(a, b)
    i, j = np.nonzero(d < thresh)
    p = np.stack([i, j], 1).astype(np.int32)
    return p[np.lexsort((p[:, 1], p[:, 0]))]


@pytest.mark.parametrize("seed", range(8))
def test_grid_pairs_complete(seed):
    """The grid prunes only non-intersecting pairs: results equal the brute-force IoU test."""
    rng = np.random.default_rng(seed)
    na, nb = rng.integers(1, 400, size=2)
    canvas = rng.choice([60.0, 300.0, 2000.0])
    def boxes(n):
        xy = rng.uniform(0, canvas, size=(n, 2))
        wh = rng.uniform(2, 64, size=(n, 2)) * rng.choice([1, 1, 1, 12], size=(n, 1))
        return np.concatenate([xy, xy + wh], 1)
    a, b = boxes(na), boxes(nb)
    b[:3] = a[:3] + rng.normal(0, 1, size=(3, 4))
    for thresh in (0.15, 0.5, 0.8, 1.0):
        got = _lib.grid_pairs(a, b, thresh)
        assert np.array_equal(got, _brute_pairs(a, b, thresh)), thresh


@pytest.mark.parametrize("seed", range(4))
def test_grid_pairs_near_threshold(seed):
    """The corner-window query (IoU > 1 - thresh) on many jittered copies, IoUs spread across the
    threshold, boxes of mixed sizes (incl. big ones that bypass the grid)."""
    rng = np.random.default_rng(100 + seed)
    n = 600
    xy = rng.uniform(0, 1500, size=(n, 2))
    wh = rng.uniform(8, 120, size=(n, 2)) * rng.choice([1, 1, 1, 1, 10], size=(n, 1))
    a = np.concatenate([xy, xy + wh], 1)
    jit = rng.uniform(0, 0.25, size=(n, 1)) * np.concatenate([wh, wh], 1)
    b = a + rng.uniform(-1, 1, size=(n, 4)) * jit
    b[:, 2:] = np.maximum(b[:, 2:], b[:, :2] + 1)
    for thresh in (0.05, 0.15, 0.3, 0.6):
        got = _lib.grid_pairs(a, b, thresh)
        exp = _brute_pairs(a, b, thresh)
        assert len(exp) > 50 and np.array_equal(got, exp), thresh


def test_grid_pairs_mot17_dedup_case():
    """The lost / tracked boxes of MOT17-02 frame 316 (a duplicate at IoU distance 0.129)."""
    L = np.array([[430.97677576, 457.72682571, 460.54623113, 554.13059315],
                  [848.0807521, 471.72410916, 911.79088983, 560.3342942],
                  [539.63031215, 461.03830408, 563.40578585, 522.46247351],
                  [550.07827234, 461.35683546, 573.58418471, 519.26254885]])
    T = np.array([[548.52661677, 460.85409296, 572.20069217, 518.92964587]])
    got = _lib.grid_pairs(T, L, 0.15)
    assert np.array_equal(got, _brute_pairs(T, L, 0.15)) and len(got) == 1


def test_block_primitives_selftest():
    """DPP wave scans / row and wave reductions behind every block-wide scan and reduction."""
    lib = _lib.load_library()
    _lib.check(lib.yta_selftest(0))
