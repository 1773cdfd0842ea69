"""CPU: the argument behind the reduced -IoU solve (csrc/ocsort_common.hpp iou_lap_reduced).

The BYTE / OCR rounds solve association.py:20-28 (lapjv, extend_cost) on -IoU and keep the pairs
with IoU >= threshold.  Rows / columns without a positive entry can be dropped: the kept pairs of
an optimum of the positive part equal those of an optimum of the whole padded problem (the
oracle's lapjv restatement, oracle/lapjv.c), on sparse random IoU-like matrices with many exact
zeros, in both orientations, with ties only among zero entries.
"""
import numpy as np
import pytest

from oracle.lap import lapjv


def kept(mat, x, thr):
    return sorted((int(i), int(j)) for i, j in enumerate(x) if j >= 0 and mat[i, j] >= thr)


def solve_full(mat):
    _, x, _ = lapjv(-mat, extend_cost=True)
    return x


def solve_reduced(mat):
    rows = np.nonzero((mat > 0).any(axis=1))[0]
    cols = np.nonzero((mat > 0).any(axis=0))[0]
    x = np.full(mat.shape[0], -1, dtype=np.int64)
    if len(rows) == 0:
        return x
    sub = mat[np.ix_(rows, cols)]
    _, xr, _ = lapjv(-sub, extend_cost=True)
    for i, j in enumerate(xr):
        if j >= 0:
            x[rows[i]] = cols[j]
    return x


@pytest.mark.parametrize("shape", [(70, 1150), (40, 1200), (300, 120), (20, 20), (5, 900)])
@pytest.mark.parametrize("seed", range(6))
def test_reduced_solve_keeps_the_same_pairs(shape, seed):
    rng = np.random.default_rng(seed * 97 + shape[0])
    na, nb = shape
    mat = np.zeros(shape)
    nnz = max(1, int(0.01 * na * nb))
    mat[rng.integers(0, na, nnz), rng.integers(0, nb, nnz)] = rng.uniform(0.01, 0.99, nnz)
    thr = 0.3
    full, red = solve_full(mat), solve_reduced(mat)
    assert kept(mat, full, thr) == kept(mat, red, thr)
    # and the kept pairs are a maximum-weight matching's: the reduced optimum's value is the full one's
    val = lambda x: sum(mat[i, j] for i, j in enumerate(x) if j >= 0)
    assert abs(val(full) - val(red)) < 1e-9
