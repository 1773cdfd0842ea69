"""Gaussian-smoothed interpolation (GSI) of MOT result files, on the MI355X.

Mirror of boxmot/postprocessing/gsi.py: the same functions, arguments and outputs.  The gap
filling and the per-track Gaussian-process smoothing run in libyta.so (csrc/gsi.hip:
yta_gsi_interpolate, yta_gsi_smooth); this module keeps the host logic the reference has around
them: the (id, frame) sort, the grouping of rows by id in `set` iteration order, the length scale
of each track (numpy, gsi.py:40) and the file handling.  There is no CPU fallback.
"""
from pathlib import Path

import numpy as np

from .. import _lib

# pairs with (t_i / l - t_j / l)^2 above this have K < e^-60 and are left out of the band
BAND_CUTOFF = 120.0


def linear_interpolation(input_, interval, device=0):
    """gsi.py:12-30.  Rows [frame, id, ...]; returns the table with every gap of a track shorter
    than `interval` frames filled by linear interpolation, sorted by (id, frame)."""
    input_ = np.asarray(input_)
    input_ = input_[np.lexsort([input_[:, 0], input_[:, 1]])]
    n, ncol = input_.shape
    if n == 0:
        return input_.copy()
    virt0 = int(int(input_[0, 1]) == -1)
    if virt0 and ncol != 10:    # gsi.py:16: the initial zero row has 10 columns
        raise ValueError(f"operands could not be broadcast together with shapes ({ncol},) (10,)")
    rows = np.ascontiguousarray(input_, dtype=np.float64)
    lib = _lib.load_library()
    need = _lib.ctypes.c_longlong(0)
    rc = lib.yta_gsi_interpolate(device, _lib.ptr(rows), n, ncol, int(interval), virt0, None, 0,
                                 _lib.ctypes.byref(need))
    if rc != _lib.YTA_ERR_CAPACITY:
        _lib.check(rc)
    if need.value == n:          # nothing appended: the reference returns the sorted copy as is
        return input_.copy()
    out = np.empty((need.value, ncol), dtype=np.float64)
    _lib.check(lib.yta_gsi_interpolate(device, _lib.ptr(rows), n, ncol, int(interval), virt0,
                                       _lib.ptr(out), need.value, _lib.ctypes.byref(need)))
    if virt0:   # rows interpolated from the zero row carry fractional ids: the final sort moves them
        out = out[np.lexsort([out[:, 0], out[:, 1]])]
    return out


def _band_width(t, length_scale):
    """max(i - j) over the pairs of a track within the band cutoff, with the kernel's float64
    expression (t_i / l - t_j / l)^2.  Frames sorted ascending (the interpolated table is): the
    distance grows with the row offset, so the band ends at the first offset with no pair in it."""
    xs = t / length_scale
    n = len(xs)
    if n <= 1:
        return 0
    if np.all(np.diff(xs) >= 0):
        w = 0
        while w + 1 < n:
            d = xs[w + 1:] - xs[:n - w - 1]
            if not np.any(d * d <= BAND_CUTOFF):
                break
            w += 1
        return w
    d = xs[:, None] - xs[None, :]                 # unsorted input: scan every pair
    ii, jj = np.nonzero(np.tril(d * d <= BAND_CUTOFF))
    return int(np.max(ii - jj))


def gaussian_smooth(input_, tau, device=0):
    """gsi.py:33-59: per id (in set iteration order) a GaussianProcessRegressor with a fixed RBF
    kernel of length scale clip(tau * log(tau**3 / n), 1 / tau, tau**2), fitted to and predicted
    at the track's frames for x, y, w and h; rows [t, id, x, y, w, h, conf, cls, -1]."""
    input_ = np.asarray(input_)
    ids = set(input_[:, 1])
    groups, offs, scales, widths = [], [0], [], []
    for id_ in ids:
        tracks = input_[input_[:, 1] == id_]
        len_scale = np.clip(tau * np.log(tau ** 3 / len(tracks)), tau ** -1, tau ** 2)
        t = tracks[:, 0].astype(np.float64)
        groups.append((id_, tracks))
        offs.append(offs[-1] + len(tracks))
        scales.append(float(len_scale))
        widths.append(_band_width(t, float(len_scale)))
    if not groups:
        return []
    t_all = np.ascontiguousarray(np.concatenate([g[1][:, 0] for g in groups]), dtype=np.float64)
    y_all = np.ascontiguousarray(np.concatenate([g[1][:, 2:6] for g in groups]), dtype=np.float64)
    off = np.asarray(offs, dtype=np.int32)
    ls = np.asarray(scales, dtype=np.float64)
    bw = np.asarray(widths, dtype=np.int32)
    out = np.empty_like(y_all)
    try:
        _lib.check(_lib.load_library().yta_gsi_smooth(device, _lib.ptr(t_all), _lib.ptr(y_all),
                                                      _lib.ptr(off), _lib.ptr(ls), _lib.ptr(bw),
                                                      len(groups), _lib.ptr(out)))
    except _lib.YTAError as e:
        if "positive definite" in str(e):
            raise np.linalg.LinAlgError(str(e)) from e
        raise
    output_ = []
    for k, (id_, tracks) in enumerate(groups):
        sm = out[off[k]:off[k + 1]]
        t = tracks[:, 0]
        output_.extend([[t[j], id_, sm[j, 0], sm[j, 1], sm[j, 2], sm[j, 3], tracks[j, 6],
                         tracks[j, 7], -1] for j in range(len(t))])
    return output_


def gsi(mot_results_folder=Path('examples/runs/val/exp87/labels'), interval=20, tau=10, device=0):
    """gsi.py:62-72: every MOT*FRCNN.txt of the folder is interpolated, smoothed and rewritten
    in place as integers."""
    for p in Path(mot_results_folder).glob('MOT*FRCNN.txt'):
        tracking_results = np.loadtxt(p, dtype=int, delimiter=' ')
        if tracking_results.size != 0:
            li = linear_interpolation(tracking_results, interval, device=device)
            gs = gaussian_smooth(li, tau, device=device)
            np.savetxt(p, gs, fmt='%d %d %d %d %d %d %d %d %d')
        else:
            print('No tracking result in {p}. Skipping...')
