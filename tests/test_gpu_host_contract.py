"""GPU: the host-buffer update's output-capacity contract (include/yolo_tracking_amd.h,
yta_bytetrack_update): out_capacity >= det_offsets[S] is required and always suffices; a smaller
buffer fails with YTA_ERR_CAPACITY *before* the frame is applied, so retrying the same call gives
exactly what an engine that never saw the failed call gives (tracks, IDs, next_id counters).

The reference has no such failure mode (update() allocates its own result, byte_tracker.py:270-281);
the contract exists so a C caller can size `out` once from the frame it passes in.
"""
import numpy as np
import pytest

from yolo_tracking_amd import _lib
from yolo_tracking_amd.synth import make_frames
from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
from yolo_tracking_amd.trackers.bytetrack import ByteTrackEngine
from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine
from yolo_tracking_amd.trackers.hybridsort import HybridSortEngine
from yolo_tracking_amd.trackers.ocsort import OCSortEngine

pytestmark = pytest.mark.gpu

OC_KW = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
             asso_func="giou", inertia=0.2)


class _TightOut:
    """Library proxy: the tracker's update entry point is called with out_capacity = rows."""

    def __init__(self, eng, lib, fn, cap_arg, rows):
        self._eng, self._lib, self._fn, self._cap_arg, self._rows = eng, lib, fn, cap_arg, rows

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if name != self._fn:
            return f

        def call(*args):
            args = list(args)
            out = self._eng._out
            # (out, out_capacity) must be where we expect them before one is replaced
            assert args[self._cap_arg - 1] == out.ctypes.data and args[self._cap_arg] == len(out)
            args[self._cap_arg] = self._rows
            return f(*args)
        return call


def _norm(e):
    return (e / np.linalg.norm(e, axis=1, keepdims=True)).astype(np.float32)


# name -> (engine factory, update entry point, out_capacity argument index, update(eng, frame, nid))
def _bt(S):
    return ByteTrackEngine(S, track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30,
                           track_capacity=16, max_dets=16)


def _bot(S):
    return BoTSORTEngine(S, feat_dim=16, track_capacity=16, max_dets=16)


def _oc(S):
    kw = dict(OC_KW, asso_threshold=OC_KW["iou_threshold"])   # OCSort's name (ocsort.py:199)
    del kw["iou_threshold"]
    return OCSortEngine(S, **kw, track_capacity=16, max_dets=16)


def _doc(S):
    return DeepOCSortEngine(S, feat_dim=16, **OC_KW, track_capacity=16, max_dets=16)


def _hs(S):
    return HybridSortEngine(S, feat_dim=16, **OC_KW, track_capacity=16, max_dets=16)


def _upd_bt(eng, fr, nid):
    return eng.update([d for d, _ in fr], next_id=nid)


def _upd_bot(eng, fr, nid):
    feats = [_norm(e[d[:, 4] > eng.track_high_thresh]) for d, e in fr]
    return eng.update([d for d, _ in fr], feats, next_id=nid)


def _upd_oc(eng, fr, nid):
    return eng.update([d for d, _ in fr], img_shapes=[(640, 640, 3)] * len(fr), next_id=nid)


def _upd_doc(eng, fr, nid):
    return eng.update([d for d, _ in fr], [_norm(e) for _, e in fr],
                      img_shapes=[(640, 640, 3)] * len(fr), next_id=nid)


def _upd_hs(eng, fr, nid):
    return eng.update([d for d, _ in fr], [_norm(e) for _, e in fr], next_id=nid)


CASES = {
    "bytetrack": (_bt, "yta_bytetrack_update", 5, _upd_bt, 0.1),
    "botsort": (_bot, "yta_botsort_update", 7, _upd_bot, 0.1),
    "ocsort": (_oc, "yta_ocsort_update", 6, _upd_oc, 0.0),
    "deepocsort": (_doc, "yta_deepocsort_update", 8, _upd_doc, 0.0),
    "hybridsort": (_hs, "yta_hybridsort_update", 6, _upd_hs, 0.0),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_short_output_buffer_leaves_the_frame_unapplied(name):
    make, fn, cap_arg, upd, low = CASES[name]
    S, n, nf, bad = 3, 40, 8, 4
    streams = [make_frames(n, nf, 900 + s, emb_dim=16, low_conf_frac=low, drop_frac=0.1)
               for s in range(S)]
    a, b = make(S), make(S)     # b never sees the failed call
    nid_a = np.zeros(S, dtype=np.int64)
    nid_b = np.zeros(S, dtype=np.int64)
    for f in range(nf):
        fr = [streams[s][f] for s in range(S)]
        if f == bad:
            total = sum(len(d) for d, _ in fr)
            real = a.lib
            a.lib = _TightOut(a, real, fn, cap_arg, total - 1)
            before = nid_a.copy()
            try:
                with pytest.raises(_lib.CapacityError):
                    upd(a, fr, nid_a)
            finally:
                a.lib = real
            assert np.array_equal(nid_a, before)
        got = upd(a, fr, nid_a)
        exp = upd(b, fr, nid_b)
        for s in range(S):
            assert np.array_equal(got[s], exp[s]), (name, f, s)
            assert len(got[s]) <= len(fr[s][0])      # the bound the contract rests on
        assert np.array_equal(nid_a, nid_b), (name, f)
    assert nid_a.sum() > 0


def test_pinned_caller_buffers_match_pageable():
    """Page-locked caller buffers (a pinned tensor's NumPy view) are DMA'd directly, without the
    staging copy (bytetrack.hip host_pinned): frame by frame the rows, offsets and IDs equal those
    of the same frames passed in pageable buffers."""
    import torch
    S, N = 5, 300
    streams = [make_frames(N, 8, 700 + s) for s in range(S)]
    a = ByteTrackEngine(S, track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30,
                        track_capacity=3 * N, max_dets=N)
    b = ByteTrackEngine(S, track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30,
                        track_capacity=3 * N, max_dets=N)
    most = max(sum(len(streams[s][f][0]) for s in range(S)) for f in range(8))
    pin_in = torch.empty((most, 6), dtype=torch.float64, pin_memory=True).numpy()
    pin_out = torch.empty((most, 8), dtype=torch.float64, pin_memory=True).numpy()
    off = np.zeros(S + 1, np.int32)
    out_off = np.zeros(S + 1, np.int32)
    nid_a, nid_b = np.zeros(S, np.int64), np.zeros(S, np.int64)
    for f in range(8):
        dets = [streams[s][f][0] for s in range(S)]
        ref = a.update(dets, next_id=nid_a)
        np.cumsum([len(d) for d in dets], out=off[1:])
        pin_in[:off[-1]] = np.concatenate(dets)
        _lib.check(b.lib.yta_bytetrack_update(b.handle, _lib.ptr(pin_in), _lib.ptr(off),
                                              _lib.ptr(nid_b), _lib.ptr(pin_out), len(pin_out),
                                              _lib.ptr(out_off)))
        got = [pin_out[out_off[s]:out_off[s + 1]] for s in range(S)]
        assert np.array_equal(nid_a, nid_b), f
        for s in range(S):
            assert np.array_equal(got[s], ref[s]), (f, s)
