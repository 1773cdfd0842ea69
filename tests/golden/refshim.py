"""Container-only loader for the read-only reference (BoxMOT 10.0.51 at /root/reference).

Used ONLY by tests/golden/make_goldens.py to produce golden vectors; never imported by tests that
run on the GPU box (the reference does not exist there).  Recipe from SURVEY.md §8(c):
  1. a bare `boxmot` package whose __path__ points at the reference, so boxmot/__init__.py
     (ReID / cv2 / gdown imports) is never executed;
  2. a no-op `loguru` (logging only, boxmot/utils/__init__.py:15-19);
  3. `filterpy.common.reshape_z/pretty_str` + `filterpy.stats.logpdf` — shape-only helpers, no
     arithmetic (ocsort_kf.py:105-106);
  4. a `lap` module whose `lapjv` restates lapx's extend_cost / cost_limit contract on top of
     scipy.optimize.linear_sum_assignment (lapx itself is not installed);
  5. for BoT-SORT: a fake `boxmot.appearance.reid_multibackend` whose
     get_features returns harness-supplied rows divided by their global Frobenius norm (as
     reid_multibackend.py:310), and a fake `boxmot.motion.cmc.sof.SparseOptFlow` returning a
     harness-supplied 2x3 warp.
"""
import os
import sys
import types

import numpy as np

REF = os.environ.get("YTA_REFERENCE", "/root/reference")


def _install_shims():
    if "loguru" not in sys.modules:
        lg = types.ModuleType("loguru")

        class _L:
            def __getattr__(self, name):
                return lambda *a, **k: None

        lg.logger = _L()
        sys.modules["loguru"] = lg

    if "filterpy" not in sys.modules:
        fp = types.ModuleType("filterpy")
        common = types.ModuleType("filterpy.common")
        stats = types.ModuleType("filterpy.stats")

        def reshape_z(z, dim_z, ndim):
            z = np.atleast_2d(z)
            if z.shape[1] == dim_z:
                z = z.T
            if z.shape != (dim_z, 1):
                raise ValueError("z must be convertible to shape ({}, 1)".format(dim_z))
            if ndim == 1:
                z = z[:, 0]
            if ndim == 0:
                z = z[0, 0]
            return z

        common.reshape_z = reshape_z
        common.pretty_str = lambda label, arr: f"{label} = {arr}"
        stats.logpdf = lambda *a, **k: 0.0
        fp.common = common
        fp.stats = stats
        sys.modules["filterpy"] = fp
        sys.modules["filterpy.common"] = common
        sys.modules["filterpy.stats"] = stats

    if "lap" not in sys.modules:
        from scipy.optimize import linear_sum_assignment
        lapm = types.ModuleType("lap")

        def lapjv(cost, extend_cost=False, cost_limit=np.inf, return_cost=True):
            c = np.asarray(cost, dtype=np.double)
            nr, nc = c.shape
            if nr != nc and not extend_cost:
                raise ValueError("Square cost array expected.")
            if cost_limit < np.inf:
                n = nr + nc
                e = np.full((n, n), cost_limit / 2.0)
                e[nr:, nc:] = 0
                e[:nr, :nc] = c
            elif extend_cost:
                n = max(nr, nc)
                e = np.zeros((n, n))
                e[:nr, :nc] = c
            else:
                n = nr
                e = c
            r, k = linear_sum_assignment(e)
            x = np.empty(n, dtype=np.int32)
            y = np.empty(n, dtype=np.int32)
            x[r] = k
            y[k] = r
            if cost_limit < np.inf or extend_cost:
                x[x >= nc] = -1
                y[y >= nr] = -1
                x = x[:nr]
                y = y[:nc]
                opt = c[np.nonzero(x != -1)[0], x[x != -1]].sum()
            else:
                opt = c[np.arange(nr), x].sum()
            return (opt, x, y) if return_cost else (x, y)

        lapm.lapjv = lapjv
        sys.modules["lap"] = lapm

    if "boxmot" not in sys.modules:
        pkg = types.ModuleType("boxmot")
        pkg.__path__ = [os.path.join(REF, "boxmot")]
        sys.modules["boxmot"] = pkg


class Harness:
    """Per-frame inputs the fake ReID / CMC modules hand to the reference."""
    feats = None           # (M, D) float32 raw embeddings of the frame's detections
    high_thresh = 0.5      # BoT-SORT track_high_thresh (rows the reference asks features for)
    dets = None
    warp = np.eye(2, 3)
    match_boxes = False    # HybridSORT: get_features sees every row of each per-class call;
                           # its rows are found by box (the global norm is over those rows)


def _install_botsort_shims():
    if "boxmot.appearance.reid_multibackend" in sys.modules:
        return
    app = types.ModuleType("boxmot.appearance")
    app.__path__ = []
    rmb = types.ModuleType("boxmot.appearance.reid_multibackend")

    class ReIDDetectMultiBackend:
        def __init__(self, weights=None, device=None, fp16=False):
            pass

        def get_features(self, xyxys, img):
            if Harness.match_boxes:
                where = {tuple(b): k for k, b in enumerate(Harness.dets[:, :4])}
                idx = [where[tuple(b)] for b in np.asarray(xyxys).reshape(-1, 4)]
                features = Harness.feats[idx]
                return features / np.linalg.norm(features)
            if xyxys.size != 0:
                m = Harness.dets[:, 4] > Harness.high_thresh
                features = Harness.feats[m]
                assert np.array_equal(Harness.dets[m, :4], xyxys)
            else:
                features = np.array([])
            return features / np.linalg.norm(features)          # reid_multibackend.py:310

    rmb.ReIDDetectMultiBackend = ReIDDetectMultiBackend
    cmc = types.ModuleType("boxmot.motion.cmc")
    cmc.__path__ = []
    sof = types.ModuleType("boxmot.motion.cmc.sof")

    class SparseOptFlow:
        def __init__(self, *a, **k):
            pass

        def apply(self, img, dets):
            return np.array(Harness.warp, dtype=np.float64)

    sof.SparseOptFlow = SparseOptFlow
    cmc.get_cmc_method = lambda name: SparseOptFlow       # DeepOCSort: get_cmc_method('sof')()
    sys.modules["boxmot.appearance"] = app
    sys.modules["boxmot.appearance.reid_multibackend"] = rmb
    sys.modules["boxmot.motion.cmc"] = cmc
    sys.modules["boxmot.motion.cmc.sof"] = sof


def load_botsort():
    """Reference BoT-SORT modules (with the fake ReID / CMC of step 5)."""
    _install_shims()
    _install_botsort_shims()
    import importlib
    ns = types.SimpleNamespace()
    ns.bot_sort = importlib.import_module("boxmot.trackers.botsort.bot_sort")
    ns.basetrack = importlib.import_module("boxmot.trackers.botsort.basetrack")
    ns.botsort_kf = importlib.import_module("boxmot.motion.kalman_filters.botsort_kf")
    return ns


def load_deepocsort():
    """Reference DeepOCSORT modules (fake ReID / CMC of step 5)."""
    _install_shims()
    _install_botsort_shims()
    import importlib
    ns = types.SimpleNamespace()
    ns.deep_ocsort = importlib.import_module("boxmot.trackers.deepocsort.deep_ocsort")
    return ns


def load_hybridsort():
    """Reference HybridSORT modules (fake ReID of step 5; its ECC CMC is off, hybridsort.py:360)."""
    _install_shims()
    _install_botsort_shims()
    import importlib
    ns = types.SimpleNamespace()
    ns.hybridsort = importlib.import_module("boxmot.trackers.hybridsort.hybridsort")
    ns.kf = importlib.import_module("boxmot.motion.kalman_filters.hybridsort_kf")
    return ns


def load():
    """Return a namespace with the reference modules needed for goldens."""
    _install_shims()
    import importlib
    ns = types.SimpleNamespace()
    ns.byte_tracker = importlib.import_module("boxmot.trackers.bytetrack.byte_tracker")
    ns.basetrack = importlib.import_module("boxmot.trackers.bytetrack.basetrack")
    ns.bytetrack_kf = importlib.import_module("boxmot.motion.kalman_filters.bytetrack_kf")
    ns.matching = importlib.import_module("boxmot.utils.matching")
    ns.iou = importlib.import_module("boxmot.utils.iou")
    ns.ops = importlib.import_module("boxmot.utils.ops")
    ns.ocsort = importlib.import_module("boxmot.trackers.ocsort.ocsort")
    return ns
