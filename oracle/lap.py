"""ORACLE — test infrastructure only.  ctypes binding of oracle/lapjv.c (restated lapx.lapjv).

Mirrors the two reference call sites:
  * boxmot/utils/matching.py:56-71     linear_assignment(cost, thresh) -> matches, u_a, u_b
  * boxmot/utils/association.py:20-28  linear_assignment(cost) -> [[row, col], ...]
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(path)
        lib.oracle_lapjv.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.oracle_lapjv.restype = ctypes.c_int
        _LIB = lib
    return _LIB


def lapjv(cost, extend_cost=False, cost_limit=np.inf):
    """lapx `lapjv` contract: returns (opt, x, y) with x/y int32, -1 for unassigned."""
    c = np.ascontiguousarray(cost, dtype=np.float64)
    nr, nc = c.shape
    if nr != nc and not extend_cost and not cost_limit < np.inf:
        raise ValueError("Square cost array expected. If cost is intentionally non-square, "
                         "pass extend_cost=True.")
    x = np.empty(nr, dtype=np.int32)
    y = np.empty(nc, dtype=np.int32)
    opt = ctypes.c_double(0.0)
    rc = _lib().oracle_lapjv(nr, nc, c.ctypes.data, int(bool(extend_cost)), float(cost_limit),
                             x.ctypes.data, y.ctypes.data, ctypes.byref(opt))
    if rc != 0:
        raise RuntimeError(f"oracle_lapjv failed ({rc})")
    return opt.value, x, y


def linear_assignment_limited(cost_matrix, thresh):
    """matching.py:56-71 — cost_limit semantics (not a post-filter)."""
    if cost_matrix.size == 0:
        return (np.empty((0, 2), dtype=int), tuple(range(cost_matrix.shape[0])),
                tuple(range(cost_matrix.shape[1])))
    _, x, y = lapjv(cost_matrix, extend_cost=True, cost_limit=thresh)
    rows = np.nonzero(x >= 0)[0]
    matches = np.stack([rows, x[rows]], axis=1) if len(rows) else np.asarray([])
    return matches, np.where(x < 0)[0], np.where(y < 0)[0]


def linear_assignment_padded(cost_matrix):
    """association.py:20-28 — zero-padded square solve, pairs in row order."""
    _, x, y = lapjv(cost_matrix, extend_cost=True)
    return np.array([[y[k], k] for k in x if k >= 0])
