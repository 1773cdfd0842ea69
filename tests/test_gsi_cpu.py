"""GSI post-processing, CPU side: the oracle (oracle/gsi.py) against the goldens made by importing
the reference (tests/golden/make_gsi_golden.py -> gsi_mot17.npz), the host logic of the package
mirror (band widths, MOT writer).  The GPU path is tested in test_gpu_gsi.py."""
import io
import os

import numpy as np
import pytest

from oracle import gsi as og
import yolo_tracking_amd.postprocessing.gsi as pg  # noqa: E402
from yolo_tracking_amd.postprocessing.mot import write_mot_results


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "gsi_mot17.npz"))


def names(g):
    return sorted({k.split("_", 1)[1] for k in g.files})


def savetxt_ints(a):
    b = io.StringIO()
    np.savetxt(b, a, fmt="%d %d %d %d %d %d %d %d %d")
    return np.loadtxt(io.StringIO(b.getvalue()), dtype=int)


def test_oracle_linear_interpolation_bit_exact(g):
    for n in names(g):
        li = og.linear_interpolation(g["in_" + n], 20)
        assert li.shape == g["li_" + n].shape
        assert np.array_equal(li, g["li_" + n]), n


def test_oracle_gaussian_smooth_bit_exact(g):
    for n in names(g):
        gs = np.asarray(og.gaussian_smooth(g["li_" + n], 10), dtype=np.float64)
        assert np.array_equal(gs, g["gs_" + n]), n
        assert np.array_equal(savetxt_ints(gs), g["out_" + n]), n


def test_golden_covers_edge_cases(g):
    li = g["li_MOT99-11-FRCNN"]
    lens = np.unique(li[:, 1], return_counts=True)[1]
    assert lens.min() == 1 and lens.max() > 1000          # single-row and clipped-scale tracks
    assert len(g["li_MOT99-11-FRCNN"]) > len(g["in_MOT99-11-FRCNN"])


def test_band_width_bounds_the_kernel():
    """Every pair outside the band the host hands the kernel has K < e^-60."""
    rng = np.random.default_rng(3)
    for n in (1, 2, 7, 60, 150, 220, 480, 800, 1100):
        t = np.sort(rng.choice(np.arange(1, 2 * n + 5), n, replace=False)).astype(float)
        ls = float(og.length_scale_of(n, 10))
        w = pg._band_width(t, ls)
        xs = t / ls
        d = xs[:, None] - xs[None, :]
        k = np.exp(-0.5 * d * d)
        i, j = np.tril_indices(n, -1)
        out = (i - j) > w
        assert np.all(k[i[out], j[out]] < np.exp(-60))
        if w > 0:
            assert np.any(d[i[(i - j) == w], j[(i - j) == w]] ** 2 <= pg.BAND_CUTOFF)
        perm = rng.permutation(n)                             # unsorted frames: dense scan
        assert pg._band_width(t[perm], ls) >= 0


def test_write_mot_results(tmp_path):
    """examples/utils.py:8-28: frame_idx + 1, id, ltwh, conf, cls, -1 as '%d', appended."""
    tracks = np.array([[10.7, 20.2, 50.9, 80.4, 3, 0.91, 0, 5],
                       [100.0, 5.5, 140.25, 60.0, 7, 0.55, 2, 1]])
    p = tmp_path / "sub" / "MOT17-02-FRCNN.txt"
    write_mot_results(p, tracks, 0)
    write_mot_results(p, tracks[:1], 4)
    got = np.loadtxt(p, dtype=int)
    exp = np.array([[1, 3, 10, 20, 40, 60, 0, 0, -1],
                    [1, 7, 100, 5, 40, 54, 0, 2, -1],
                    [5, 3, 10, 20, 40, 60, 0, 0, -1]])
    assert np.array_equal(got, exp)
