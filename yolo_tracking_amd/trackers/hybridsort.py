"""HybridSORT on the MI355X: the reference's `HybridSORT` surface over the HIP engine.

Reference: boxmot/trackers/hybridsort/hybridsort.py:329-570 (HybridSORT, whose update is wrapped
by boxmot/utils/__init__.py:22-61 PerClassDecorator with per_class hard-wired to True, :339),
:106-326 (KalmanBoxTracker, whose class-level `count` every HybridSORT constructor sets to 0, :361).
Tracker state (9-d Kalman filters with their frozen copies, observation rings, corner velocities,
float32 smoothed appearance features) lives in HBM inside the C-ABI engine
(yolo_tracking_amd/csrc/hybridsort.hip); this module replays the per-class decorator call by call
(each call predicts every tracker, as the reference's does), gets each call's ReID features and
returns the (K, 8) result.

The ReID forward pass (:394 get_features) is not part of the hot path: pass
`reid=` (an object with get_features(xyxys, img) -> (n, D) float32, called once per class call on
that call's boxes, as the reference does) or give `update(..., embs=...)` the get_features rows of
every input detection (each class call then takes its own rows).  ECC camera compensation is off
in the reference (:360) and is not offered.
"""
import ctypes

import numpy as np

from .. import _lib
from ._streams import StreamSubset
from ..appearance import build_reid


class KalmanBoxTracker:
    """Only the process-wide ID counter of hybridsort.py:106-110 (the per-tracker state is on the
    device)."""
    count = 0


class HybridSortEngine(StreamSubset):
    """S independent HybridSORT streams sharing one device engine; one update() = one
    undecorated HybridSORT.update call per stream."""

    def __init__(self, n_streams=1, feat_dim=512, det_thresh=0.0, max_age=30, min_hits=3,
                 iou_threshold=0.3, delta_t=3, asso_func="iou", inertia=0.2, device=0,
                 track_capacity=512, max_dets=256):
        if asso_func not in ("iou", "giou", "diou", "ciou"):
            # get_asso_func (iou.py:215-224); centroid needs the image size HybridSORT never
            # passes (hybridsort.py:516 calls asso_func(left_dets, left_trks))
            raise KeyError(asso_func)
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.device = _lib.parse_device(device)
        self.feat_dim = int(feat_dim)
        prm = _lib.HsParams(float(det_thresh), int(max_age), int(min_hits), float(iou_threshold),
                            int(delta_t), _lib.ASSO_FUNCS[asso_func], float(inertia))
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_hybridsort_create(self.device, self.n_streams, int(track_capacity),
                                                  int(max_dets), self.feat_dim, ctypes.byref(prm),
                                                  ctypes.byref(h)))
        self._h = h
        self._out = np.empty((0, 8), dtype=np.float64)
        self._out_off = np.zeros(self.n_streams + 1, dtype=np.int32)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.yta_hybridsort_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.yta_hybridsort_reset(self._h))

    def reset_stream(self, stream):
        """Reset one stream to a freshly constructed tracker; the others are untouched."""
        _lib.check(self.lib.yta_hybridsort_reset_stream(self._h, int(stream)))

    def capacity(self):
        c, d = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.yta_hybridsort_capacity(self._h, ctypes.byref(c), ctypes.byref(d)))
        return c.value, d.value

    def lap_stats(self):
        """Solver counters since create / reset (yta_hybridsort_lap_stats): first-round solves of the
        transposed problem (more detections than trackers), those not certified unique, and
        lapjv replays, -IoU rounds solved on their positive part."""
        names = ["transposed", "uncertified", "replays", "reduced"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_hybridsort_lap_stats(self._h, buf, len(names)))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def stats(self):
        names = ["dets", "high", "trackers", "out", "births", "lap_calls", "corrections",
                 "feature_jobs"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_hybridsort_stats(self._h, buf))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def update(self, dets_per_stream, feats_per_stream, next_id=None, streams=None):
        """dets_per_stream: S float64 (M_s, 6); feats_per_stream: S float32 (M_s, D), the
        get_features rows of every detection; next_id: optional int64 (S,) counters
        (KalmanBoxTracker.count), updated in place.  streams: update only these stream ids
        (every per-stream argument and the result then follow the listed streams; the others
        are left as they were)."""
        ids = None
        if streams is not None:
            ids, order = self._subset(streams, len(dets_per_stream))
            dets_per_stream = self._reorder(dets_per_stream, order)
            feats_per_stream = self._reorder(feats_per_stream, order)
            nid_user = next_id
            if next_id is not None:
                next_id = np.ascontiguousarray(np.asarray(next_id, np.int64)[order])
        else:
            assert len(dets_per_stream) == self.n_streams
        n = len(dets_per_stream)
        dets = [np.asarray(d, dtype=np.float64).reshape(-1, 6) for d in dets_per_stream]
        off = np.zeros(n + 1, dtype=np.int32)
        np.cumsum([len(d) for d in dets], out=off[1:])
        packed = np.ascontiguousarray(np.concatenate(dets)) if off[-1] else np.zeros((0, 6))
        rows = []
        for s, d in enumerate(dets):
            if not len(d):
                continue
            f = None if feats_per_stream is None else feats_per_stream[s]
            if f is None:
                raise ValueError(f"stream {s}: {len(d)} detections but no embeddings")
            f = np.asarray(f, dtype=np.float32).reshape(-1, self.feat_dim)
            if len(f) != len(d):
                raise ValueError(f"stream {s}: {len(f)} embeddings for {len(d)} detections")
            rows.append(f)
        feats = np.ascontiguousarray(np.concatenate(rows)) if rows else None
        # every output row is a track matched to or born from one of this frame's detections
        need = max(int(off[-1]), 1)
        if len(self._out) < need:
            self._out = np.empty((2 * need, 8), dtype=np.float64)
        nid = None
        if next_id is not None:
            nid = np.ascontiguousarray(next_id, dtype=np.int64)
        if ids is not None:
            o = np.zeros(n + 1, dtype=np.int32)
            rc = self.lib.yta_hybridsort_update_streams(
                self._h, n, _lib.ptr(ids), _lib.ptr(packed), _lib.ptr(off), _lib.ptr(feats),
                _lib.ptr(nid), _lib.ptr(self._out), len(self._out), _lib.ptr(o))
            self._subset_check(rc, order, nid, nid_user)
            return self._subset_result(o, order)
        _lib.check(self.lib.yta_hybridsort_update(
            self._h, _lib.ptr(packed), _lib.ptr(off), _lib.ptr(feats), _lib.ptr(nid),
            _lib.ptr(self._out), len(self._out), _lib.ptr(self._out_off)))
        if next_id is not None:
            next_id[...] = nid
        o = self._out_off
        return [self._out[o[s]:o[s + 1]].copy() for s in range(self.n_streams)]

    def classes(self, stream=0):
        """The cls of every live tracker in list order (PerClassDecorator's active classes)."""
        cap, _ = self.capacity()
        buf = np.empty(max(cap, 1))
        n = ctypes.c_int()
        _lib.check(self.lib.yta_hybridsort_classes(self._h, int(stream), _lib.ptr(buf), len(buf),
                                                   ctypes.byref(n)))
        return [float(v) for v in buf[:n.value]]

    def state(self, stream=0):
        """Trackers of one stream in list order: id, age, hits, hit_streak, time_since_update,
        observed; conf, cls, det_ind; Kalman x (9), P (9x9); float32 smooth features."""
        cap, _ = self.capacity()
        n = ctypes.c_int()
        ints = np.empty((cap, 6), dtype=np.int64)
        dbl = np.empty((cap, 3))
        x = np.empty((cap, 9))
        P = np.empty((cap, 9, 9))
        feat = np.empty((cap, self.feat_dim), dtype=np.float32)
        _lib.check(self.lib.yta_hybridsort_get_state(
            self._h, int(stream), ctypes.byref(n), _lib.ptr(ints), _lib.ptr(dbl), _lib.ptr(x),
            _lib.ptr(P), _lib.ptr(feat)))
        k = n.value
        return dict(id=ints[:k, 0], age=ints[:k, 1], hits=ints[:k, 2], hit_streak=ints[:k, 3],
                    time_since_update=ints[:k, 4], observed=ints[:k, 5], conf=dbl[:k, 0],
                    cls=dbl[:k, 1], det_ind=dbl[:k, 2], x=x[:k], P=P[:k], feat=feat[:k])


class HybridSORT:
    """Drop-in for boxmot.trackers.hybridsort.hybridsort.HybridSORT (hybridsort.py:329-570).

    reid_weights / half name the reference's ReID model, which is outside the hot path: pass
    `reid=` (an object with get_features(xyxys, img) -> (n, D) float32) or give
    `update(..., embs=...)` the get_features rows of every input detection.
    """

    def __init__(self, reid_weights=None, device=0, half=False, det_thresh=0.0, max_age=30,
                 min_hits=3, iou_threshold=0.3, delta_t=3, asso_func="iou", inertia=0.2,
                 use_byte=False, reid=None, feat_dim=None, **kwargs):
        if use_byte and det_thresh > 0.1:
            # hybridsort.py:504-508 calls update(bbox, feature, update_feature=False) with a
            # missing positional argument: the reference raises TypeError once the BYTE round
            # matches (with det_thresh <= 0.1 there are no second-round detections at all)
            raise NotImplementedError("use_byte with det_thresh > 0.1 is not a working path in "
                                      "the reference")
        if asso_func not in ("iou", "giou", "diou", "ciou"):
            raise KeyError(asso_func)
        self.max_age = max_age
        self.min_hits = min_hits
        self.iou_threshold = iou_threshold
        self.per_class = True                                        # :339
        self.frame_count = 0
        self.det_thresh = det_thresh
        self.delta_t = delta_t
        self.asso_func = asso_func
        self.inertia = inertia
        self.use_byte = use_byte
        KalmanBoxTracker.count = 0                                   # :361
        self.model = build_reid(reid, reid_weights, device, half)
        self._kw = dict(det_thresh=det_thresh, max_age=max_age, min_hits=min_hits,
                        iou_threshold=iou_threshold, delta_t=delta_t, asso_func=asso_func,
                        inertia=inertia, device=device)
        self._engine = None
        self._empty_calls = 0           # calls made before the feature width was known
        self._nid = np.zeros(1, dtype=np.int64)
        if feat_dim is not None:
            self._make_engine(int(feat_dim))

    def _make_engine(self, feat_dim):
        self._engine = HybridSortEngine(1, feat_dim=feat_dim, **self._kw)
        for _ in range(self._empty_calls):   # calls before creation had no detection and no
            self._engine.update([np.zeros((0, 6))], [None])   # tracker: they only counted frames
        self._empty_calls = 0

    def _features(self, dets, img, embs, rows):
        if embs is not None:
            return np.asarray(embs, dtype=np.float32)[rows]
        if self.model is None:
            raise RuntimeError("HybridSORT needs a ReID producer: pass reid=<object with "
                               "get_features(xyxys, img)> or update(dets, img, embs=...)")
        return np.asarray(self.model.get_features(dets[:, 0:4], img), dtype=np.float32)

    def _update(self, dets, img, embs, rows):
        """One undecorated HybridSORT.update (hybridsort.py:373-570)."""
        self.frame_count += 1
        dets = np.asarray(dets, dtype=np.float64).reshape(-1, 6)
        feats = self._features(dets, img, embs, rows) if len(dets) else None
        if self._engine is None:
            if feats is None:
                self._empty_calls += 1
                return np.empty((0, 7))
            self._make_engine(feats.shape[1])
        self._nid[0] = KalmanBoxTracker.count
        out = self._engine.update([dets], [feats], next_id=self._nid)[0]
        KalmanBoxTracker.count = int(self._nid[0])
        if len(out) == 0:
            return np.empty((0, 7))                                  # :570
        return out

    def update(self, dets, img, embs=None):
        """PerClassDecorator (boxmot/utils/__init__.py:26-61) around _update."""
        if self.per_class is True and dets.size != 0:
            assert dets.ndim == 2 and dets.shape[1] == 6, "dets must be (M, 6)"
            dets_dict = {class_id: np.array([det for det in dets if det[5] == class_id])
                         for class_id in set(det[5] for det in dets)}
            rows_dict = {class_id: [k for k, det in enumerate(dets) if det[5] == class_id]
                         for class_id in dets_dict}
            detected_classes = set(dets_dict.keys())
            active_classes = set(self._engine.classes(0)) if self._engine is not None else set()
            relevant_classes = active_classes.union(detected_classes)
            mc_dets = np.empty(shape=(0, 8))
            for class_id in relevant_classes:
                d = np.array(dets_dict.get(int(class_id), np.empty((0, 6))))
                rows = rows_dict.get(int(class_id), [])
                out = self._update(d, img, embs, rows)
                if out.size != 0:
                    mc_dets = np.append(mc_dets, out, axis=0)
            return mc_dets
        return self._update(dets, img, embs, slice(None))

    @property
    def trackers(self):
        """Snapshot of the device trackers (list order)."""
        return self._engine.state(0) if self._engine is not None else None

    def reset(self):
        if self._engine is not None:
            self._engine.reset()
        self.frame_count = 0


__all__ = ["HybridSORT", "HybridSortEngine", "KalmanBoxTracker"]
