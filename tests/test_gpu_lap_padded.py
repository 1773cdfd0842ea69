"""GPU: the one-wave dense solver (lap_dense.hpp) against the restated lapjv (oracle/lapjv.c) on
the padded calls of association.py:20-28 — identical x / y (the same operation and tie-breaking
sequence), including tie-heavy integer matrices where many optima exist."""
import numpy as np
import pytest

from oracle.lap import lapjv
from yolo_tracking_amd import _lib

pytestmark = pytest.mark.gpu


def _cases():
    rng = np.random.default_rng(99)
    out = []
    for (nr, nc) in [(1, 1), (2, 3), (5, 5), (7, 4), (4, 9), (37, 53), (64, 64), (65, 63),
                     (128, 100), (100, 128), (257, 256)]:
        out.append(rng.random((nr, nc)))
        out.append(-rng.random((nr, nc)))
        out.append(rng.integers(0, 3, size=(nr, nc)).astype(np.float64))     # many ties
        out.append(np.zeros((nr, nc)))                                       # all tied
    # OCSORT-shaped: -(iou-ish + small angle term), mostly near 0 with a few strong pairs
    for n in (50, 200):
        c = -0.05 * rng.random((n, n + 7))
        idx = rng.permutation(n + 7)[:n]
        c[np.arange(n), idx] -= 0.6 + 0.3 * rng.random(n)
        out.append(c)
    out.append(rng.random((0, 5)))
    out.append(rng.random((6, 0)))
    return out


@pytest.mark.parametrize("k", range(len(_cases())))
def test_lap_padded_matches_oracle(k):
    c = _cases()[k]
    _, xo, yo = lapjv(c, extend_cost=True)
    x, y = _lib.lap_padded(c)
    assert np.array_equal(x, xo), (c.shape, np.nonzero(x != xo)[0][:10])
    assert np.array_equal(y, yo), c.shape


def test_lap_padded_large_global_workspace():
    """n above the LDS limit: the work arrays live in global memory."""
    rng = np.random.default_rng(5)
    c = rng.random((1600, 1700))
    _, xo, yo = lapjv(c, extend_cost=True)
    x, y = _lib.lap_padded(c)
    assert np.array_equal(x, xo) and np.array_equal(y, yo)
