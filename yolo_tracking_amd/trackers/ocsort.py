"""OCSORT on the MI355X: the reference's `OCSort` surface over the HIP engine.

Reference: boxmot/trackers/ocsort/ocsort.py:188-379 (OCSort), :65-186 (KalmanBoxTracker, whose
class-level `count` every OCSort in the process shares and each OCSort constructor resets,
:216).  Tracker state (Kalman filters with their frozen copies, observation rings, velocities)
lives in HBM inside the C-ABI engine (yolo_tracking_amd/csrc/ocsort.hip); this module validates
inputs, passes the frame size the centroid cost reads and returns the (K, 8) result.
"""
import ctypes

import numpy as np

from .. import _lib
from ._streams import StreamSubset


class KalmanBoxTracker:
    """Only the process-wide ID counter of ocsort.py:65-76 (the per-tracker state is on the
    device)."""
    count = 0


class OCSortEngine(StreamSubset):
    """S independent OCSORT streams sharing one device engine."""

    def __init__(self, n_streams=1, det_thresh=0.2, max_age=30, min_hits=3, asso_threshold=0.3,
                 delta_t=3, asso_func="iou", inertia=0.2, use_byte=False, device=0,
                 track_capacity=512, max_dets=256):
        if asso_func not in _lib.ASSO_FUNCS:
            raise KeyError(asso_func)                      # get_asso_func (iou.py:215-224)
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.device = _lib.parse_device(device)
        self.asso_func = asso_func
        prm = _lib.OcParams(float(det_thresh), int(max_age), int(min_hits), float(asso_threshold),
                            int(delta_t), _lib.ASSO_FUNCS[asso_func], float(inertia),
                            int(bool(use_byte)))
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_ocsort_create(self.device, self.n_streams, int(track_capacity),
                                              int(max_dets), ctypes.byref(prm), ctypes.byref(h)))
        self._h = h
        self._out = np.empty((0, 8), dtype=np.float64)
        self._out_off = np.zeros(self.n_streams + 1, dtype=np.int32)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.yta_ocsort_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.yta_ocsort_reset(self._h))

    def reset_stream(self, stream):
        """Reset one stream to a freshly constructed tracker; the others are untouched."""
        _lib.check(self.lib.yta_ocsort_reset_stream(self._h, int(stream)))

    def capacity(self):
        c, d = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.yta_ocsort_capacity(self._h, ctypes.byref(c), ctypes.byref(d)))
        return c.value, d.value

    def lap_stats(self):
        """Solver counters since create / reset (yta_ocsort_lap_stats): first-round solves of the
        transposed problem (more detections than trackers), those not certified unique, and
        lapjv replays, -IoU rounds solved on their positive part."""
        names = ["transposed", "uncertified", "replays", "reduced"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_ocsort_lap_stats(self._h, buf, len(names)))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def stats(self):
        names = ["dets", "high", "second", "trackers", "out", "births", "lap_calls", "fast_path"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_ocsort_stats(self._h, buf))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def update(self, dets_per_stream, img_shapes=None, next_id=None, streams=None):
        """dets_per_stream: S float64 (M_s, 6); img_shapes: S image shapes (h, w, ...) or None;
        next_id: optional int64 (S,) counters (KalmanBoxTracker.count), updated in place.
        streams: update only these stream ids (every per-stream argument and the result then
        follow the listed streams; the others are left as they were)."""
        ids = None
        if streams is not None:
            ids, order = self._subset(streams, len(dets_per_stream))
            dets_per_stream = self._reorder(dets_per_stream, order)
            img_shapes = self._reorder(img_shapes, order)
            nid_user = next_id
            if next_id is not None:
                next_id = np.ascontiguousarray(np.asarray(next_id, np.int64)[order])
        else:
            assert len(dets_per_stream) == self.n_streams
        n = len(dets_per_stream)
        counts = [len(d) for d in dets_per_stream]
        off = np.zeros(n + 1, dtype=np.int32)
        np.cumsum(counts, out=off[1:])
        if off[-1]:
            packed = np.ascontiguousarray(np.concatenate(
                [np.asarray(d, dtype=np.float64).reshape(-1, 6) for d in dets_per_stream]))
        else:
            packed = np.zeros((0, 6))
        wh = None
        if img_shapes is not None:
            wh = np.ascontiguousarray([[int(sh[1]), int(sh[0])] for sh in img_shapes],
                                      dtype=np.int32)
        # every output row is a track matched to or born from one of this frame's detections
        need = max(int(off[-1]), 1)
        if len(self._out) < need:
            self._out = np.empty((2 * need, 8), dtype=np.float64)
        nid = None
        if next_id is not None:
            nid = np.ascontiguousarray(next_id, dtype=np.int64)
        if ids is not None:
            o = np.zeros(n + 1, dtype=np.int32)
            rc = self.lib.yta_ocsort_update_streams(
                self._h, n, _lib.ptr(ids), _lib.ptr(packed), _lib.ptr(off), _lib.ptr(wh),
                _lib.ptr(nid), _lib.ptr(self._out), len(self._out), _lib.ptr(o))
            self._subset_check(rc, order, nid, nid_user)
            return self._subset_result(o, order)
        _lib.check(self.lib.yta_ocsort_update(self._h, _lib.ptr(packed), _lib.ptr(off),
                                              _lib.ptr(wh), _lib.ptr(nid), _lib.ptr(self._out),
                                              len(self._out), _lib.ptr(self._out_off)))
        if next_id is not None:
            next_id[...] = nid
        o = self._out_off
        return [self._out[o[s]:o[s + 1]].copy() for s in range(self.n_streams)]

    def state(self, stream=0):
        """Trackers of one stream in list order: id, age, hits, hit_streak, time_since_update,
        observed, saved; Kalman x (7) and P (7x7)."""
        cap, _ = self.capacity()
        n = ctypes.c_int()
        ints = np.empty((cap, 7), dtype=np.int64)
        x = np.empty((cap, 7))
        P = np.empty((cap, 7, 7))
        _lib.check(self.lib.yta_ocsort_get_state(self._h, int(stream), ctypes.byref(n),
                                                 _lib.ptr(ints), _lib.ptr(x), _lib.ptr(P)))
        k = n.value
        return dict(id=ints[:k, 0], age=ints[:k, 1], hits=ints[:k, 2], hit_streak=ints[:k, 3],
                    time_since_update=ints[:k, 4], observed=ints[:k, 5], saved=ints[:k, 6],
                    x=x[:k], P=P[:k])


class OCSort:
    """Drop-in for boxmot.trackers.ocsort.ocsort.OCSort (ocsort.py:188-379)."""

    def __init__(self, per_class=True, det_thresh=0.2, max_age=30, min_hits=3,
                 asso_threshold=0.3, delta_t=3, asso_func="iou", inertia=0.2, use_byte=False,
                 device=0):
        self.max_age = max_age
        self.min_hits = min_hits
        self.asso_threshold = asso_threshold
        self.frame_count = 0
        self.det_thresh = det_thresh
        self.delta_t = delta_t
        self.asso_func = asso_func
        self.inertia = inertia
        self.use_byte = use_byte
        KalmanBoxTracker.count = 0                                   # :216
        self._engine = OCSortEngine(1, det_thresh, max_age, min_hits, asso_threshold, delta_t,
                                    asso_func, inertia, use_byte, device=device)
        self._nid = np.zeros(1, dtype=np.int64)

    def update(self, dets, img):
        assert isinstance(dets, np.ndarray), \
            f"Unsupported 'dets' input format '{type(dets)}', valid format is np.ndarray"
        assert len(dets.shape) == 2, \
            "Unsupported 'dets' dimensions, valid number of dimensions is two"
        assert dets.shape[1] == 6, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6"
        self.frame_count += 1
        shape = img.shape                                            # :239 (h, w = img.shape[0:2])
        self._nid[0] = KalmanBoxTracker.count
        out = self._engine.update([np.asarray(dets, dtype=np.float64)], [shape],
                                  next_id=self._nid)[0]
        KalmanBoxTracker.count = int(self._nid[0])
        if len(out) == 0:
            return np.array([])                                      # :379
        return out

    @property
    def trackers(self):
        """Snapshot of the device trackers (list order)."""
        return self._engine.state(0)

    def reset(self):
        self._engine.reset()
        self.frame_count = 0


__all__ = ["OCSort", "OCSortEngine", "KalmanBoxTracker"]
