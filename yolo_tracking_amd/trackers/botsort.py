"""BoT-SORT on the MI355X: the reference's `BoTSORT` surface over the HIP engine.

Reference: boxmot/trackers/botsort/bot_sort.py:185-420 (BoTSORT), basetrack.py:15-62 (ID counter,
reset by every BoTSORT constructor).  Per-track state (xywh Kalman filter, smoothed ReID feature,
class histogram) lives in HBM inside the C-ABI engine (yolo_tracking_amd/csrc/bytetrack.hip,
variant BoT-SORT); this module validates inputs, gets the frame's ReID features and camera warp
from the pluggable producers and returns the (K, 8) result.

The ReID forward pass (reid_multibackend.py) is the caller's: pass a `reid` object with
`get_features(xyxys, img)` (or the frame's embeddings to `update(..., embs=...)`).  The camera
warp comes from SparseOptFlow on the GPU (motion/sof.py, the reference's estimator,
bot_sort.py:228) unless a `cmc` object with `apply(img, dets) -> 2x3` is given; the engine applies
it to the predicted pool and the unconfirmed tracks as STrack.multi_gmc does (bot_sort.py:95-111,
290-295).
"""
import ctypes

import numpy as np

from .. import _lib
from ..appearance import build_reid
from ..motion.cmc import IdentityCMC, default_cmc
from .bytetrack import ByteTrackEngine, STrackView


class BaseTrack:
    """boxmot/trackers/botsort/basetrack.py:15-62: one class-level counter for every BoTSORT in
    the process, cleared by each BoTSORT constructor (:205)."""
    _count = 0

    @staticmethod
    def next_id():
        BaseTrack._count += 1
        return BaseTrack._count

    @staticmethod
    def clear_count():
        BaseTrack._count = 0


class TrackState:
    New = 0
    Tracked = 1
    Lost = 2
    LongLost = 3
    Removed = 4




class BoTSORTEngine(ByteTrackEngine):
    """S independent BoT-SORT streams sharing one device engine."""

    def __init__(self, n_streams=1, feat_dim=512, track_high_thresh=0.5, track_low_thresh=0.1,
                 new_track_thresh=0.6, track_buffer=30, match_thresh=0.8, proximity_thresh=0.5,
                 appearance_thresh=0.25, frame_rate=30, fuse_first_associate=False,
                 with_reid=True, device=0, track_capacity=256, max_dets=128):
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.device = _lib.parse_device(device)
        self.feat_dim = int(feat_dim) if with_reid else 0
        self.track_high_thresh = float(track_high_thresh)
        prm = _lib.BotParams(float(track_high_thresh), float(track_low_thresh),
                             float(new_track_thresh), float(match_thresh),
                             float(proximity_thresh), float(appearance_thresh), int(track_buffer),
                             int(frame_rate), int(bool(fuse_first_associate)), int(bool(with_reid)))
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_botsort_create(self.device, self.n_streams, int(track_capacity),
                                               int(max_dets), self.feat_dim, ctypes.byref(prm),
                                               ctypes.byref(h)))
        self._h = h
        self._out = np.empty((0, 8), dtype=np.float64)
        self._out_off = np.zeros(self.n_streams + 1, dtype=np.int32)

    def update(self, dets_per_stream, feats_per_stream=None, warps=None, next_id=None,
               streams=None):
        """dets_per_stream: S float64 (M_s, 6) arrays; feats_per_stream: S float32 (H_s, D)
        arrays, the ReID rows of each stream's high detections (conf > track_high_thresh) in
        detection order; warps: optional S 2x3 affines; next_id: optional int64 (S,) counters,
        updated in place.  Returns S (K_s, 8) arrays.  streams: update only these stream ids
        (every per-stream argument and the result then follow the listed streams)."""
        ids = None
        if streams is not None:
            ids, order = self._subset(streams, len(dets_per_stream))
            dets_per_stream = [dets_per_stream[k] for k in order]
            if feats_per_stream is not None:
                feats_per_stream = [feats_per_stream[k] for k in order]
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
            for d, f in zip(dets_per_stream, feats_per_stream or [None] * n):
                nh = int(np.count_nonzero(np.asarray(d, np.float64).reshape(-1, 6)[:, 4]
                                          > self.track_high_thresh))
                f = np.zeros((0, self.feat_dim), np.float32) if f is None or nh == 0 else f
                f = np.asarray(f, dtype=np.float32).reshape(-1, self.feat_dim)
                if len(f) != nh:
                    raise ValueError(f"expected {nh} feature rows (high detections), got {len(f)}")
                rows.append(f)
            feats = np.ascontiguousarray(np.concatenate(rows)) if rows else None
        w = None
        if warps is not None:
            w = np.ascontiguousarray(np.asarray(warps, dtype=np.float64).reshape(n, 6))
        # every output row is a track matched to or born from one of this frame's detections
        need = max(int(off[-1]), 1)
        if len(self._out) < need:
            self._out = np.empty((2 * need, 8), dtype=np.float64)
        nid = None
        if next_id is not None:
            nid = np.ascontiguousarray(next_id, dtype=np.int64)
        if ids is None:
            _lib.check(self.lib.yta_botsort_update(self._h, _lib.ptr(packed), _lib.ptr(off),
                                                   _lib.ptr(feats), _lib.ptr(w), _lib.ptr(nid),
                                                   _lib.ptr(self._out), len(self._out),
                                                   _lib.ptr(self._out_off)))
            if next_id is not None:
                next_id[...] = nid
            o = self._out_off
            return [self._out[o[s]:o[s + 1]].copy() for s in range(self.n_streams)]
        o = np.zeros(n + 1, dtype=np.int32)
        rc = self.lib.yta_botsort_update_streams(
            self._h, n, _lib.ptr(ids), _lib.ptr(packed), _lib.ptr(off), _lib.ptr(feats),
            _lib.ptr(w), _lib.ptr(nid), _lib.ptr(self._out), len(self._out), _lib.ptr(o))
        self._subset_check(rc, order, nid, nid_user)
        return self._subset_result(o, order)

    def features(self, stream=0):
        """Smoothed features, class histograms (n, 8, 2) and their entry counts of the live
        tracks, in state() order."""
        cap, _ = self.capacity()
        n = ctypes.c_int()
        feats = np.empty((cap, max(self.feat_dim, 1)), dtype=np.float32)
        hist = np.empty((cap, 8, 2))
        ncls = np.empty(cap, dtype=np.int32)
        _lib.check(self.lib.yta_botsort_get_features(self._h, int(stream), ctypes.byref(n),
                                                     _lib.ptr(feats) if self.feat_dim else None,
                                                     _lib.ptr(hist), _lib.ptr(ncls)))
        k = n.value
        return feats[:k, :self.feat_dim], hist[:k], ncls[:k]


class STrackViewXYWH(STrackView):
    @property
    def xyxy(self):
        xc, yc, w, h = self.mean[:4]
        return np.array([xc - w / 2, yc - h / 2, xc + w / 2, yc + h / 2])


class BoTSORT:
    """Drop-in for boxmot.trackers.botsort.bot_sort.BoTSORT (bot_sort.py:185-420).

    model_weights / fp16 name the reference's ReID model, which is outside the hot path: pass
    `reid=` (an object with get_features(xyxys, img) -> (n, D) float32, e.g. a
    ReIDDetectMultiBackend) or give `update(..., embs=...)` the frame's per-detection embeddings.
    Camera motion: SparseOptFlow on the GPU as in the reference (bot_sort.py:228; cmc_method is
    accepted and, as there, not used); `cmc=` replaces it (an object with apply(img, dets) -> 2x3
    warp, e.g. IdentityCMC() for a static camera).
    """

    def __init__(self, model_weights=None, device=0, fp16=False, track_high_thresh=0.5,
                 track_low_thresh=0.1, new_track_thresh=0.6, track_buffer=30, match_thresh=0.8,
                 proximity_thresh=0.5, appearance_thresh=0.25, cmc_method="sparseOptFlow",
                 frame_rate=30, fuse_first_associate=False, with_reid=True, reid=None, cmc=None,
                 feat_dim=None):
        BaseTrack.clear_count()                                   # :205
        self.frame_id = 0
        self.track_high_thresh = track_high_thresh
        self.track_low_thresh = track_low_thresh
        self.new_track_thresh = new_track_thresh
        self.match_thresh = match_thresh
        self.buffer_size = int(frame_rate / 30.0 * track_buffer)
        self.max_time_lost = self.buffer_size
        self.proximity_thresh = proximity_thresh
        self.appearance_thresh = appearance_thresh
        self.with_reid = with_reid
        self.fuse_first_associate = fuse_first_associate
        self.model_weights = model_weights
        if with_reid:
            self.model = build_reid(reid, model_weights, device, fp16)
        self.cmc = cmc if cmc is not None else default_cmc("BoTSORT", device)   # :228
        self._kw = dict(track_high_thresh=track_high_thresh, track_low_thresh=track_low_thresh,
                        new_track_thresh=new_track_thresh, track_buffer=track_buffer,
                        match_thresh=match_thresh, proximity_thresh=proximity_thresh,
                        appearance_thresh=appearance_thresh, frame_rate=frame_rate,
                        fuse_first_associate=fuse_first_associate, with_reid=with_reid,
                        device=device)
        self._engine = None
        self._empty_frames = 0          # frames seen before the feature width was known
        self._feat_dim = feat_dim
        self._nid = np.zeros(1, dtype=np.int64)
        if not with_reid or feat_dim is not None:
            self._make_engine(feat_dim or 0)

    def _make_engine(self, feat_dim):
        self._engine = BoTSORTEngine(1, feat_dim=feat_dim, **self._kw)
        for _ in range(self._empty_frames):   # frames before creation held no high detection:
            self._engine.update([np.zeros((0, 6))], [None])   # they only advanced frame_id
        self._empty_frames = 0

    def update(self, dets, img, embs=None):
        assert isinstance(dets, np.ndarray), \
            f"Unsupported 'dets' input format '{type(dets)}', valid format is np.ndarray"
        assert isinstance(img, np.ndarray), \
            f"Unsupported 'img_numpy' input format '{type(img)}', valid format is np.ndarray"
        assert len(dets.shape) == 2, \
            "Unsupported 'dets' dimensions, valid number of dimensions is two"
        assert dets.shape[1] == 6, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6"
        self.frame_id += 1
        dets = np.asarray(dets, dtype=np.float64)
        high = dets[:, 4] > self.track_high_thresh               # :266-267
        feats = None
        if self.with_reid and np.any(high):                      # :270-271
            if embs is not None:
                feats = np.asarray(embs, dtype=np.float32)[high]
            else:
                if self.model is None:
                    raise RuntimeError(
                        "BoTSORT(with_reid=True) needs a ReID producer: pass reid=<object with "
                        "get_features(xyxys, img)> or update(dets, img, embs=...)")
                feats = np.asarray(self.model.get_features(dets[high, 0:4], img), np.float32)
            if self._engine is None:
                self._make_engine(feats.shape[1])
        warp = np.asarray(self.cmc.apply(img, dets[high]), dtype=np.float64)   # :299
        if self._engine is None:                                  # no high detection yet
            self._empty_frames += 1
            return np.asarray([])
        self._nid[0] = BaseTrack._count
        out = self._engine.update([dets], [feats], warps=warp[None], next_id=self._nid)[0]
        BaseTrack._count = int(self._nid[0])
        if len(out) == 0:
            return np.asarray([])                                 # :418-419
        return out

    # ---- reference-compatible introspection (snapshots; the state itself lives on the GPU)
    def _views(self, which):
        if self._engine is None:
            return []
        st = self._engine.state(0)
        return [STrackViewXYWH(st, i) for i in np.nonzero(st["list"] == which)[0]]

    @property
    def tracked_stracks(self):
        return self._views(0)

    @property
    def lost_stracks(self):
        return self._views(1)

    def reset(self):
        if self._engine is not None:
            self._engine.reset()
        self.frame_id = 0


__all__ = ["BoTSORT", "BoTSORTEngine", "BaseTrack", "TrackState", "IdentityCMC"]
