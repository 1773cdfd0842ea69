"""ByteTrack on the MI355X: the reference's `BYTETracker` surface over the HIP engine.

Reference: boxmot/trackers/bytetrack/byte_tracker.py:114-281 (BYTETracker), basetrack.py:15-40
(process-global ID counter).  All per-track state lives in HBM inside the C-ABI engine
(yolo_tracking_amd/csrc/bytetrack.hip); this module only validates inputs, moves the frame's
detections across the boundary and returns the (K, 8) result.
"""
import ctypes

import numpy as np

from .. import _lib
from ._streams import StreamSubset
from .basetrack import BaseTrack, TrackState


class ByteTrackEngine(StreamSubset):
    """S independent ByteTrack streams sharing one device engine (one launch per kernel covers
    every stream).  Stream s has its own tracks and ID counter."""

    def __init__(self, n_streams=1, track_thresh=0.45, match_thresh=0.8, track_buffer=25,
                 frame_rate=30, device=0, track_capacity=256, max_dets=128):
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.device = _lib.parse_device(device)
        prm = _lib.BtParams(float(track_thresh), float(match_thresh), int(track_buffer),
                            int(frame_rate))
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_bytetrack_create(self.device, self.n_streams, int(track_capacity),
                                                 int(max_dets), ctypes.byref(prm), ctypes.byref(h)))
        self._h = h
        self._out = np.empty((0, 8), dtype=np.float64)
        self._out_off = np.zeros(self.n_streams + 1, dtype=np.int32)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.yta_bytetrack_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.yta_bytetrack_reset(self._h))

    def reset_stream(self, stream):
        """Reset one stream to a fresh tracker; the others are untouched."""
        _lib.check(self.lib.yta_bytetrack_reset_stream(self._h, int(stream)))

    def capacity(self):
        c, d = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.yta_bytetrack_capacity(self._h, ctypes.byref(c), ctypes.byref(d)))
        return c.value, d.value

    def reserve(self, track_capacity, max_dets):
        _lib.check(self.lib.yta_bytetrack_reserve(self._h, int(track_capacity), int(max_dets)))

    def set_lds(self, nbytes):
        """LDS bytes per stream for the association kernels (0: always over global memory)."""
        _lib.check(self.lib.yta_bytetrack_set_lds(self._h, int(nbytes)))

    def stats(self):
        """Last frame's counts summed over streams (see yta_bytetrack_stats)."""
        names = ["dets", "high", "second", "pool", "act", "unc", "left", "rest", "births", "t2",
                 "l2", "tracked", "lost", "out", "edges1", "edges23", "fallback1", "fallback23",
                 "lazy", "res1", "fallback_f"]
        buf = (ctypes.c_longlong * len(names))()
        _lib.check(self.lib.yta_bytetrack_stats(self._h, buf))
        return {k: int(buf[i]) for i, k in enumerate(names)}

    def update(self, dets_per_stream, next_id=None, streams=None):
        """dets_per_stream: list of S float64 (M_s, 6) arrays.  next_id: optional int64 (S,) array
        of last-issued IDs, updated in place.  Returns a list of S (K_s, 8) arrays.
        streams: update only these stream ids (dets_per_stream / next_id / the result then have
        one entry per listed stream, in the listed order); every other stream is left as it was
        (yta_bytetrack_update_streams)."""
        ids = None
        if streams is not None:
            ids, order = self._subset(streams, len(dets_per_stream))
            dets_per_stream = [dets_per_stream[k] for k in order]
            nid_user = next_id
            if next_id is not None:
                next_id = np.ascontiguousarray(np.asarray(next_id, np.int64)[order])
        else:
            assert len(dets_per_stream) == self.n_streams
        n = len(dets_per_stream)
        counts = [len(d) for d in dets_per_stream]
        off = np.zeros(n + 1, dtype=np.int32)
        np.cumsum(counts, out=off[1:])
        # float32 detections (what a float32 detector hands over) cross the link as float32 and
        # are widened on the device, exactly as the reference's promotion (yta_bytetrack_update_f32)
        f32 = ids is None and all(np.asarray(d).dtype == np.float32 for d in dets_per_stream)
        dt = np.float32 if f32 else np.float64
        if off[-1] and n == 1:   # one stream (the drop-in): no concatenation copy
            packed = np.ascontiguousarray(np.asarray(dets_per_stream[0], dtype=dt).reshape(-1, 6))
        elif off[-1]:
            packed = np.ascontiguousarray(np.concatenate(
                [np.asarray(d, dtype=dt).reshape(-1, 6) for d in dets_per_stream]))
        else:
            packed = np.zeros((0, 6), dtype=dt)
        # every output row is a track matched to or born from one of this frame's detections
        need = max(int(off[-1]), 1)
        if len(self._out) < need:
            self._out = np.empty((2 * need, 8), dtype=np.float64)
        nid = None
        if next_id is not None:
            nid = np.ascontiguousarray(next_id, dtype=np.int64)
        if ids is None:
            fn = self.lib.yta_bytetrack_update_f32 if f32 else self.lib.yta_bytetrack_update
            _lib.check(fn(self._h, _lib.ptr(packed), _lib.ptr(off),
                                                     _lib.ptr(nid), _lib.ptr(self._out),
                                                     len(self._out), _lib.ptr(self._out_off)))
            if next_id is not None:
                next_id[...] = nid
            o = self._out_off
            return [self._out[o[s]:o[s + 1]].copy() for s in range(self.n_streams)]
        o = np.zeros(n + 1, dtype=np.int32)
        rc = self.lib.yta_bytetrack_update_streams(
            self._h, n, _lib.ptr(ids), _lib.ptr(packed), _lib.ptr(off), _lib.ptr(nid),
            _lib.ptr(self._out), len(self._out), _lib.ptr(o))
        self._subset_check(rc, order, nid, nid_user)
        return self._subset_result(o, order)

    def submit(self, dets_per_stream, out=None):
        """Pipelined update, first half (yta_bytetrack_submit): enqueue one frame of every stream
        and return at once; at most three frames in flight.  The engine's own ID counters are used.
        out: optional float64 (>= total dets, 8) buffer the matching collect() fills (kept alive
        here until then).  Returns nothing; collect() returns the oldest submitted frame."""
        assert len(dets_per_stream) == self.n_streams
        off = np.zeros(self.n_streams + 1, dtype=np.int32)
        np.cumsum([len(d) for d in dets_per_stream], out=off[1:])
        f32 = all(np.asarray(d).dtype == np.float32 for d in dets_per_stream)
        dt = np.float32 if f32 else np.float64
        packed = (np.ascontiguousarray(np.concatenate(
            [np.asarray(d, dtype=dt).reshape(-1, 6) for d in dets_per_stream]))
            if off[-1] else np.zeros((0, 6), dtype=dt))
        need = max(int(off[-1]), 1)
        if out is None or len(out) < need:
            out = np.empty((need, 8), dtype=np.float64)
        fn = self.lib.yta_bytetrack_submit_f32 if f32 else self.lib.yta_bytetrack_submit
        _lib.check(fn(self._h, _lib.ptr(packed), _lib.ptr(off), None, _lib.ptr(out), len(out)))
        if not hasattr(self, "_inflight"):
            self._inflight = []
        self._inflight.append((packed, out))   # the buffers must outlive the DMA

    def collect(self, next_id=None):
        """Pipelined update, second half: the oldest submitted frame's S (K_s, 8) arrays.
        next_id: optional int64 (S,) array receiving the counters after that frame."""
        if not getattr(self, "_inflight", None):
            raise _lib.YTAError(-1, "collect(): no frame in flight")
        o = np.zeros(self.n_streams + 1, dtype=np.int32)
        nid = None if next_id is None else np.zeros(self.n_streams, np.int64)
        try:
            _lib.check(self.lib.yta_bytetrack_collect(self._h, _lib.ptr(nid), _lib.ptr(o)))
        finally:
            _, out = self._inflight.pop(0)
        if next_id is not None:
            next_id[...] = nid
        return [out[o[s]:o[s + 1]].copy() for s in range(self.n_streams)]

    def state(self, stream=0):
        """Live tracks of one stream (tracked list then lost list) for parity checks."""
        cap, _ = self.capacity()
        n = ctypes.c_int()
        ints = np.empty((cap, 7), dtype=np.int64)
        mean = np.empty((cap, 8))
        cov = np.empty((cap, 8, 8))
        _lib.check(self.lib.yta_bytetrack_get_state(self._h, int(stream), ctypes.byref(n),
                                                    _lib.ptr(ints), _lib.ptr(mean), _lib.ptr(cov)))
        k = n.value
        return dict(list=ints[:k, 0], id=ints[:k, 1], state=ints[:k, 2], activated=ints[:k, 3],
                    frame_id=ints[:k, 4], start_frame=ints[:k, 5], tracklet_len=ints[:k, 6],
                    mean=mean[:k], cov=cov[:k])


class STrackView:
    """Read-only snapshot of one device track with the reference STrack's attribute names."""

    def __init__(self, st, i):
        self.track_id = int(st["id"][i])
        self.state = int(st["state"][i])
        self.is_activated = bool(st["activated"][i])
        self.frame_id = int(st["frame_id"][i])
        self.start_frame = int(st["start_frame"][i])
        self.tracklet_len = int(st["tracklet_len"][i])
        self.mean = st["mean"][i].copy()
        self.covariance = st["cov"][i].copy()

    @property
    def end_frame(self):
        return self.frame_id

    @property
    def xyxy(self):
        xc, yc, a, h = self.mean[:4]
        w = a * h
        return np.array([xc - w / 2, yc - h / 2, xc + w / 2, yc + h / 2])


class BYTETracker:
    """Drop-in for boxmot.trackers.bytetrack.byte_tracker.BYTETracker (byte_tracker.py:114-281).

    IDs come from the process-global `BaseTrack._count`, shared by every BYTETracker in the
    process exactly like the reference (basetrack.py:16, :37-40).
    """

    def __init__(self, track_thresh=0.45, match_thresh=0.8, track_buffer=25, frame_rate=30,
                 device=0):
        self.frame_id = 0
        self.track_buffer = track_buffer
        self.track_thresh = track_thresh
        self.match_thresh = match_thresh
        self.det_thresh = track_thresh
        self.buffer_size = int(frame_rate / 30.0 * track_buffer)
        self.max_time_lost = self.buffer_size
        self._engine = ByteTrackEngine(1, track_thresh, match_thresh, track_buffer, frame_rate,
                                       device=device)
        self._nid = np.zeros(1, dtype=np.int64)

    def update(self, dets, _=None):
        assert isinstance(dets, np.ndarray), \
            f"Unsupported 'dets' input format '{type(dets)}', valid format is np.ndarray"
        assert len(dets.shape) == 2, \
            "Unsupported 'dets' dimensions, valid number of dimensions is two"
        assert dets.shape[1] == 6, "Unsupported 'dets' 2nd dimension lenght, valid lenghts is 6"
        self.frame_id += 1
        self._nid[0] = BaseTrack._count
        out = self._engine.update([dets], next_id=self._nid)[0]
        BaseTrack._count = int(self._nid[0])
        if len(out) == 0:
            return np.asarray([])   # np.asarray([]) for no tracks, as the reference (:280)
        return out

    # ---- reference-compatible introspection (snapshots; the state itself lives on the GPU)
    def _views(self, which):
        st = self._engine.state(0)
        return [STrackView(st, i) for i in np.nonzero(st["list"] == which)[0]]

    @property
    def tracked_stracks(self):
        return self._views(0)

    @property
    def lost_stracks(self):
        return self._views(1)

    def reset(self):
        self._engine.reset()
        self.frame_id = 0


__all__ = ["BYTETracker", "ByteTrackEngine", "STrackView", "TrackState"]
