"""Camera-motion correction (SURVEY.md §8(b) affine_apply): BoT-SORT STrack.multi_gmc
(bot_sort.py:95-111) and DeepOCSORT's apply_affine_correction (deepocsort_kf.py:387-405) against
vectors made by calling the reference's own functions (tests/golden/make_affine_golden.py):
the oracle's restatements on the CPU, the engines' device functions through yta_affine_apply on
the GPU.  Bar: 1e-12 relative (the reference's kron(I4, R) products run through BLAS, whose
summation order is not pinned; the device sums in ascending index order without FMA)."""
import os

import numpy as np
import pytest

from oracle.deepocsort import KF8
from oracle.kalman_xywh import gmc

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kat_affine.npz")


def _close(a, b):
    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-9)


def test_oracle_affine_matches_reference_goldens():
    g = np.load(G)
    for i in range(len(g["mean"])):
        m, c = gmc(g["mean"][i].copy(), g["cov"][i].copy(), g["warps"][i])
        _close(m, g["gmc_mean"][i])
        _close(c, g["gmc_cov"][i])
        kf = KF8(np.array([[1.0], [1.0], [1.0], [1.0]]))
        kf.x = g["mean"][i].reshape(8, 1).copy()
        kf.P = g["cov"][i].copy()
        kf.observed = True
        kf.affine(g["warps"][i][:, :2], g["warps"][i][:, 2].reshape(2, 1))
        _close(kf.x.ravel(), g["doc_mean"][i])
        _close(kf.P, g["doc_cov"][i])


@pytest.mark.gpu
@pytest.mark.parametrize("kind,key", [(0, "gmc"), (1, "doc")])
def test_device_affine_matches_reference_goldens(kind, key):
    from yolo_tracking_amd import _lib
    g = np.load(G)
    m, c = _lib.affine_apply(kind, g["warps"], g["mean"], g["cov"])
    _close(m, g[f"{key}_mean"])
    _close(c, g[f"{key}_cov"])
    ident = np.all(g["warps"].reshape(-1, 6) == np.eye(2, 3).ravel(), axis=1)
    assert ident.any() and np.array_equal(m[ident], g["mean"][ident])


@pytest.mark.gpu
def test_device_affine_rejects_coupled_covariance():
    from yolo_tracking_amd import _lib
    g = np.load(G)
    c = g["cov"][:2].copy()
    c[0, 0, 2] = c[0, 2, 0] = 0.5
    with pytest.raises(_lib.YTAError):
        _lib.affine_apply(0, g["warps"][:2], g["mean"][:2], c)
