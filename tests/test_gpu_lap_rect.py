"""GPU: the rectangular solver (lap_rect.hpp) against the restated lapjv (oracle/lapjv.c) on the
padded calls of association.py:20-28.

Where the optimum is unique (continuous random costs) the assignment must be identical to lapjv's;
where many optima exist (integer / zero-heavy costs, all-zero columns as new OCSORT trackers
produce) the solver must return an optimal assignment of the same cost — the engines only use it
where the tracker result does not depend on which optimum is returned."""
import numpy as np
import pytest

from oracle.lap import lapjv
from yolo_tracking_amd import _lib

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1), (1, 9), (9, 1), (2, 3), (5, 5), (7, 4), (37, 53), (53, 37), (64, 64),
          (256, 410), (410, 256), (513, 700), (1000, 1200), (2100, 2500), (300, 5000), (5000, 300)]


def _padded_cost(c, x):
    """Cost of the real pairs of a padded assignment x (row -> column or -1)."""
    r = np.nonzero(x >= 0)[0]
    return float(c[r, x[r]].sum())


def _check_valid(c, x, y):
    nr, nc = c.shape
    assert x.shape == (nr,) and y.shape == (nc,)
    m = np.nonzero(x >= 0)[0]
    assert len(m) == min(nr, nc)
    assert np.array_equal(y[x[m]], m)
    assert (y >= 0).sum() == min(nr, nc)


@pytest.mark.parametrize("shape", SHAPES)
def test_lap_rect_unique_optimum_matches_lapjv(shape):
    rng = np.random.default_rng(shape[0] * 7919 + shape[1])
    c = rng.random(shape) - 0.5
    _, xo, yo = lapjv(c, extend_cost=True)
    x, y = _lib.lap_rect(c)
    _check_valid(c, x, y)
    assert np.array_equal(x, xo), (shape, np.nonzero(x != xo)[0][:10])
    assert np.array_equal(y, yo), shape


def _ocsort_like(rng, n_det, n_trk, zero_cols=0.0):
    """-(iou + angle): a strong pair per detection among the trackers, a small dense angle term,
    births (no strong pair), and optionally all-zero tracker columns (velocity (0, 0), no IoU)."""
    c = -0.1 * (rng.random((n_det, n_trk)) - 0.5)
    perm = rng.permutation(n_trk)
    for i in range(n_det):
        if rng.random() < 0.97:
            c[i, perm[i]] -= 0.3 + 0.7 * rng.random()
    if zero_cols:
        z = rng.random(n_trk) < zero_cols
        c[:, z] = 0.0
    return c


@pytest.mark.parametrize("n_det,n_trk,zc", [(256, 410, 0.0), (256, 410, 0.05), (2048, 2563, 0.0),
                                             (1000, 1000, 0.02), (4096, 4700, 0.0)])
def test_lap_rect_ocsort_shaped(n_det, n_trk, zc):
    rng = np.random.default_rng(n_det + n_trk)
    c = _ocsort_like(rng, n_det, n_trk, zc)
    _, xo, _ = lapjv(c, extend_cost=True)
    x, y = _lib.lap_rect(c)
    _check_valid(c, x, y)
    assert _padded_cost(c, x) == pytest.approx(_padded_cost(c, xo), abs=1e-9)
    if zc == 0.0:
        assert np.array_equal(x, xo)
    else:
        # rows may trade places only among exactly-zero entries
        d = np.nonzero(x != xo)[0]
        assert np.all(c[d, x[d]] == 0.0) and np.all(c[d, xo[d]] == 0.0)


@pytest.mark.parametrize("shape", [(5, 5), (37, 53), (53, 37), (128, 100)])
def test_lap_rect_many_optima(shape):
    rng = np.random.default_rng(11)
    for c in (rng.integers(0, 3, size=shape).astype(np.float64), np.zeros(shape),
              -(rng.random(shape) * (rng.random(shape) < 0.05))):
        _, xo, _ = lapjv(c, extend_cost=True)
        x, y = _lib.lap_rect(c)
        _check_valid(c, x, y)
        assert _padded_cost(c, x) == pytest.approx(_padded_cost(c, xo), abs=1e-9)


def test_lap_rect_empty():
    x, y = _lib.lap_rect(np.zeros((0, 5)))
    assert len(x) == 0 and np.all(y == -1)
    x, y = _lib.lap_rect(np.zeros((4, 0)))
    assert np.all(x == -1) and len(y) == 0
