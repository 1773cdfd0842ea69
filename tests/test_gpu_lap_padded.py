"""GPU: the dense replay solver (lap_dense.hpp, phase 3 block-wide from n = 768 in lap_dense_block.hpp) against the restated lapjv (oracle/lapjv.c) on
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


def _surge(rng, na, nb, per_col):
    """GIoU-surge-shaped: every pair that does not overlap costs exactly 0."""
    c = np.zeros((na, nb))
    for j in range(nb):
        rows = rng.choice(na, size=per_col, replace=False)
        c[rows, j] = -rng.random(per_col) * 0.8 - 0.05
    return c


def _mixed(rng, na, nb):
    """Rows of 0-20 nonzero entries of either sign among exact zeros: rows on both sides of the
    sparse sweeps' 16-entry limit, positive entries (a source row maximum above 0)."""
    c = np.zeros((na, nb))
    for i in range(na):
        k = int(rng.integers(0, 21))
        c[i, rng.choice(nb, size=k, replace=False)] = rng.uniform(-0.9, 0.3, k)
    return c


@pytest.mark.parametrize("case", ["ints_900x700", "zeros_1200", "ties_800x1500", "surge_2000x800",
                                  "surge_4000x500", "mixed_1500x900", "mixed_900x1400"])
def test_lap_padded_block_replay_tie_heavy(case):
    """n >= 768: phase 3 runs block-wide (lap_dense_block.hpp); tie-heavy matrices exercise its
    swap-to-front and gather resets, the zero-heavy ones its sparse sweeps; 4000 x 500 also puts
    the work arrays in global memory."""
    rng = np.random.default_rng(sum(map(ord, case)))
    c = {"ints_900x700": lambda: rng.integers(0, 4, size=(900, 700)).astype(np.float64),
         "zeros_1200": lambda: np.zeros((1200, 1200)),
         "ties_800x1500": lambda: -rng.integers(0, 3, size=(800, 1500)).astype(np.float64),
         "surge_2000x800": lambda: _surge(rng, 2000, 800, 3),
         "surge_4000x500": lambda: _surge(rng, 4000, 500, 2),
         "mixed_1500x900": lambda: _mixed(rng, 1500, 900),
         "mixed_900x1400": lambda: _mixed(rng, 900, 1400)}[case]()
    _, xo, yo = lapjv(c, extend_cost=True)
    x, y = _lib.lap_padded(c)
    assert np.array_equal(x, xo), (case, np.nonzero(x != xo)[0][:10])
    assert np.array_equal(y, yo), case
