"""DeepOCSORT on the MI355X: the reference's `DeepOCSort` surface over the HIP engine.

Reference: boxmot/trackers/deepocsort/deep_ocsort.py:308-520 (DeepOCSort), :90-330
(KalmanBoxTracker, whose class-level `count` every DeepOCSort constructor sets to 1, :347).
Tracker state (8-d Kalman filters with their frozen copies, observation rings, velocities,
float64 appearance embeddings) lives in HBM inside the C-ABI engine
(yolo_tracking_amd/csrc/deepocsort.hip); this module validates inputs, gets the frame's ReID
features and camera warp from the pluggable producers and returns the (K, 8) result.

The ReID forward pass (:387 get_features) is the caller's: pass `reid=` (an object with
get_features(xyxys, img) -> (n, D) float32) or give `update(..., embs=...)` the frame's
per-detection embeddings.  The camera warp (:391 cmc.apply) comes from SparseOptFlow on the GPU
(yolo_tracking_amd/motion/sof.py, the reference's estimator, :351) unless `cmc=` (an object with
apply(img, dets) -> 2x3 warp) replaces it.
"""
import ctypes

import numpy as np

from .. import _lib
from ._streams import StreamSubset
from ..appearance import build_reid
from ..motion.cmc import default_cmc


class KalmanBoxTracker:
    """Only the process-wide ID counter of deep_ocsort.py:90-101 (the per-tracker state is on the
    device)."""
    count = 1


class DeepOCSortEngine(StreamSubset):
    """S independent DeepOCSORT streams sharing one device engine."""

    def __init__(self, n_streams=1, feat_dim=512, det_thresh=0.3, max_age=30, min_hits=3,
                 iou_threshold=0.3, delta_t=3, asso_func="iou", inertia=0.2,
                 w_association_emb=0.5, alpha_fixed_emb=0.95, aw_param=0.5, embedding_off=False,
                 cmc_off=False, aw_off=False, device=0, track_capacity=512, max_dets=256):
        if asso_func not in _lib.ASSO_FUNCS:
            raise KeyError(asso_func)                      # get_asso_func (iou.py:215-224)
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.device = _lib.parse_device(device)
        self.det_thresh = float(det_thresh)
        self.embedding_off = bool(embedding_off)
        self.feat_dim = 0 if embedding_off else int(feat_dim)
        prm = _lib.DocParams(float(det_thresh), int(max_age), int(min_hits), float(iou_threshold),
                             int(delta_t), _lib.ASSO_FUNCS[asso_func], float(inertia),
                             float(w_association_emb), float(alpha_fixed_emb), float(aw_param),
                             int(bool(embedding_off)), int(bool(cmc_off)), int(bool(aw_off)))
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_deepocsort_create(self.device, self.n_streams, int(track_capacity),
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
            self.lib.yta_deepocsort_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.yta_deepocsort_reset(self._h))

    def reset_stream(self, stream):
        """Reset one stream to a freshly constructed tracker; the others are untouched."""
        _lib.check(self.lib.yta_deepocsort_reset_stream(self._h, int(stream)))

    def capacity(self):
        c, d = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.yta_deepocsort_capacity(self._h, ctypes.byref(c), ctypes.byref(d)))
        return c.value, d.value

    def lap_stats(self):
        """Solver counters since create / reset (yta_deepocsort_lap_stats): first-round solves of the
        transposed problem (more detections than trackers), those not certified unique, and
        lapjv replays, -IoU rounds solved on their positive part."""
        names = ["transposed", "uncertified", "replays", "reduced"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_deepocsort_lap_stats(self._h, buf, len(names)))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def stats(self):
        names = ["dets", "high", "second", "trackers", "out", "births", "lap_calls", "fast_path"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_deepocsort_stats(self._h, buf))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def update(self, dets_per_stream, feats_per_stream=None, warps=None, img_shapes=None,
               next_id=None, streams=None):
        """streams: update only these stream ids (every per-stream argument and the result then
        follow the listed streams; the others are left as they were).
        dets_per_stream: S float64 (M_s, 6); feats_per_stream: S float32 (K_s, D), the
        embeddings of the detections with conf > det_thresh in input order (None when there are
        none or embeddings are off); warps: (S, 2, 3) float64 camera warps or None (identity);
        img_shapes: S image shapes (h, w, ...) or None; next_id: optional int64 (S,) counters
        (KalmanBoxTracker.count), updated in place."""
        ids = None
        if streams is not None:
            ids, order = self._subset(streams, len(dets_per_stream))
            dets_per_stream = self._reorder(dets_per_stream, order)
            feats_per_stream = self._reorder(feats_per_stream, order)
            img_shapes = self._reorder(img_shapes, order)
            if warps is not None:
                warps = np.asarray(warps, dtype=np.float64).reshape(-1, 6)[order]
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
        feats = None
        if self.feat_dim:
            rows = []
            for s, d in enumerate(dets_per_stream):
                k = int(np.count_nonzero(np.asarray(d, dtype=np.float64).reshape(-1, 6)[:, 4]
                                         > self.det_thresh))
                f = None if feats_per_stream is None else feats_per_stream[s]
                if k == 0:
                    continue
                if f is None:
                    raise ValueError(f"stream {s}: {k} kept detections but no embeddings")
                f = np.asarray(f, dtype=np.float32).reshape(-1, self.feat_dim)
                if len(f) != k:
                    raise ValueError(f"stream {s}: {len(f)} embeddings for {k} kept detections")
                rows.append(f)
            if rows:
                feats = np.ascontiguousarray(np.concatenate(rows))
        wp = None
        if warps is not None:
            wp = np.ascontiguousarray(warps, dtype=np.float64).reshape(n, 6)
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
            rc = self.lib.yta_deepocsort_update_streams(
                self._h, n, _lib.ptr(ids), _lib.ptr(packed), _lib.ptr(off), _lib.ptr(feats),
                _lib.ptr(wp), _lib.ptr(wh), _lib.ptr(nid), _lib.ptr(self._out), len(self._out),
                _lib.ptr(o))
            self._subset_check(rc, order, nid, nid_user)
            return self._subset_result(o, order)
        _lib.check(self.lib.yta_deepocsort_update(
            self._h, _lib.ptr(packed), _lib.ptr(off), _lib.ptr(feats), _lib.ptr(wp),
            _lib.ptr(wh), _lib.ptr(nid), _lib.ptr(self._out), len(self._out),
            _lib.ptr(self._out_off)))
        if next_id is not None:
            next_id[...] = nid
        o = self._out_off
        return [self._out[o[s]:o[s + 1]].copy() for s in range(self.n_streams)]

    def state(self, stream=0):
        """Trackers of one stream in list order: id, age, hits, hit_streak, time_since_update,
        observed, frozen; Kalman x (8), P (8x8) and the float64 embedding."""
        cap, _ = self.capacity()
        n = ctypes.c_int()
        ints = np.empty((cap, 7), dtype=np.int64)
        x = np.empty((cap, 8))
        P = np.empty((cap, 8, 8))
        emb = np.empty((cap, max(self.feat_dim, 1)))
        _lib.check(self.lib.yta_deepocsort_get_state(
            self._h, int(stream), ctypes.byref(n), _lib.ptr(ints), _lib.ptr(x), _lib.ptr(P),
            _lib.ptr(emb) if self.feat_dim else None))
        k = n.value
        return dict(id=ints[:k, 0], age=ints[:k, 1], hits=ints[:k, 2], hit_streak=ints[:k, 3],
                    time_since_update=ints[:k, 4], observed=ints[:k, 5], frozen=ints[:k, 6],
                    x=x[:k], P=P[:k], emb=emb[:k, :self.feat_dim])


class DeepOCSort:
    """Drop-in for boxmot.trackers.deepocsort.deep_ocsort.DeepOCSort (deep_ocsort.py:308-520).

    model_weights / fp16 name the reference's ReID model, which is outside the hot path: pass
    `reid=` (an object with get_features(xyxys, img) -> (n, D) float32) or give
    `update(..., embs=...)` the embeddings of every input detection.  `cmc=` replaces the
    SparseOptFlow estimator, which runs on the GPU by default as in the reference (deep_ocsort.py:351;
    an object with apply(img, dets) -> 2x3 warp, e.g. IdentityCMC() for a static camera).
    """

    def __init__(self, model_weights=None, device=0, fp16=False, per_class=True, det_thresh=0.3,
                 max_age=30, min_hits=3, iou_threshold=0.3, delta_t=3, asso_func="iou",
                 inertia=0.2, w_association_emb=0.5, alpha_fixed_emb=0.95, aw_param=0.5,
                 embedding_off=False, cmc_off=False, aw_off=False, new_kf_off=False, reid=None,
                 cmc=None, feat_dim=None, **kwargs):
        if new_kf_off:
            # deep_ocsort.py:141 names an undefined OCSortKalmanFilterAdapter: the reference
            # raises NameError at the first tracker; only the new KF is a live path
            raise NotImplementedError("new_kf_off=True is not a working path in the reference")
        self.max_age = max_age
        self.min_hits = min_hits
        self.iou_threshold = iou_threshold
        self.frame_count = 0
        self.det_thresh = det_thresh
        self.delta_t = delta_t
        self.asso_func = asso_func
        self.inertia = inertia
        self.w_association_emb = w_association_emb
        self.alpha_fixed_emb = alpha_fixed_emb
        self.aw_param = aw_param
        self.per_class = per_class
        self.embedding_off = embedding_off
        self.cmc_off = cmc_off
        self.aw_off = aw_off
        self.new_kf_off = new_kf_off
        KalmanBoxTracker.count = 1                                   # :347
        self.model = build_reid(reid, model_weights, device, fp16) if not embedding_off else reid
        self.cmc = cmc if cmc is not None or cmc_off else default_cmc("DeepOCSort", device)
        self._kw = dict(det_thresh=det_thresh, max_age=max_age, min_hits=min_hits,
                        iou_threshold=iou_threshold, delta_t=delta_t, asso_func=asso_func,
                        inertia=inertia, w_association_emb=w_association_emb,
                        alpha_fixed_emb=alpha_fixed_emb, aw_param=aw_param,
                        embedding_off=embedding_off, cmc_off=cmc_off, aw_off=aw_off,
                        device=device)
        if asso_func not in _lib.ASSO_FUNCS:
            raise KeyError(asso_func)
        self._engine = None
        self._empty_frames = 0          # frames seen before the feature width was known
        self._nid = np.zeros(1, dtype=np.int64)
        if embedding_off or feat_dim is not None:
            self._make_engine(0 if embedding_off else int(feat_dim))

    def _make_engine(self, feat_dim):
        self._engine = DeepOCSortEngine(1, feat_dim=feat_dim, **self._kw)
        for _ in range(self._empty_frames):   # frames before creation held no kept detection:
            self._engine.update([np.zeros((0, 6))])   # they only advanced frame_count
        self._empty_frames = 0

    def update(self, dets, img, embs=None):
        assert isinstance(dets, np.ndarray), \
            f"Unsupported 'dets' input type '{type(dets)}', valid format is np.ndarray"
        assert isinstance(img, np.ndarray), \
            f"Unsupported 'img' input type '{type(img)}', valid format is np.ndarray"
        assert len(dets.shape) == 2, \
            "Unsupported 'dets' dimensions, valid number of dimensions is two"
        assert dets.shape[1] == 6, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6"
        self.frame_count += 1
        dets = np.asarray(dets, dtype=np.float64)
        keep = dets[:, 4] > self.det_thresh                          # :378-379
        feats = None
        if not self.embedding_off and np.any(keep):                  # :383-387
            if embs is not None:
                feats = np.asarray(embs, dtype=np.float32)[keep]
            else:
                if self.model is None:
                    raise RuntimeError(
                        "DeepOCSort needs a ReID producer: pass reid=<object with "
                        "get_features(xyxys, img)> or update(dets, img, embs=...)")
                feats = np.asarray(self.model.get_features(dets[keep, 0:4], img), np.float32)
            if self._engine is None:
                self._make_engine(feats.shape[1])
        warp = None
        if not self.cmc_off and self.cmc is not None:                # :390-393
            warp = np.asarray(self.cmc.apply(img, dets[keep, :4]), dtype=np.float64)[None]
        if self._engine is None:                                     # no kept detection yet
            self._empty_frames += 1
            return np.array([])
        self._nid[0] = KalmanBoxTracker.count
        out = self._engine.update([dets], [feats], warps=warp, img_shapes=[img.shape],
                                  next_id=self._nid)[0]
        KalmanBoxTracker.count = int(self._nid[0])
        if len(out) == 0:
            return np.array([])                                      # :520
        return out

    @property
    def trackers(self):
        """Snapshot of the device trackers (list order)."""
        return self._engine.state(0) if self._engine is not None else None

    def reset(self):
        if self._engine is not None:
            self._engine.reset()
        self.frame_count = 0


__all__ = ["DeepOCSort", "DeepOCSortEngine", "KalmanBoxTracker"]
