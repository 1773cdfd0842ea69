"""GPU: the pipelined host-buffer update (yta_bytetrack_submit / yta_bytetrack_collect: frame f's
detections in flight while frame f-1's kernels run and frame f-2's rows come back, up to three
frames in flight) gives exactly
the synchronous update's rows and ID counters, frame by frame, with pageable and page-locked
buffers, and when the engine has to grow its capacity while frames are in flight."""
import numpy as np
import pytest

from yolo_tracking_amd import ByteTrackEngine, _lib
from yolo_tracking_amd.synth import make_frames

pytestmark = pytest.mark.gpu

KW = dict(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)


def _streams(S, F, base, seed):
    return [[d for d, _ in make_frames(base + 37 * s, F, seed=seed + s)] for s in range(S)]


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("cap", [64, 2048])
def test_pipelined_equals_synchronous(pinned, cap):
    """cap 64: the engine grows (drains the frames in flight, then reserve) on the first frames."""
    import torch
    S, F = 4, 24
    frames = _streams(S, F, 150, 700)
    ref = ByteTrackEngine(S, track_capacity=cap, max_dets=64, **KW)
    eng = ByteTrackEngine(S, track_capacity=cap, max_dets=64, **KW)
    nid_ref = np.zeros(S, np.int64)
    exp = [ref.update([frames[s][f] for s in range(S)], next_id=nid_ref) + [nid_ref.copy()]
           for f in range(F)]
    outs = None
    if pinned:   # page-locked output buffers, one per slot (DMA'd directly)
        outs = [torch.empty((4096, 8), dtype=torch.float64, pin_memory=True).numpy()
                for _ in range(3)]
    got = []
    nid = np.zeros(S, np.int64)
    for f in range(F):
        eng.submit([frames[s][f] for s in range(S)], out=None if outs is None else outs[f % 3])
        if f >= 2:
            got.append(eng.collect(next_id=nid) + [nid.copy()])
    for _ in range(2):
        got.append(eng.collect(next_id=nid) + [nid.copy()])
    for f in range(F):
        for s in range(S):
            assert np.array_equal(got[f][s], exp[f][s]), (f, s)
        assert np.array_equal(got[f][S], exp[f][S]), f
    for s in range(S):
        a, b = ref.state(s), eng.state(s)
        assert all(np.array_equal(a[k], b[k]) for k in a), s


def test_pipeline_depth_and_sync_calls_refused():
    S = 2
    frames = _streams(S, 5, 60, 800)
    eng = ByteTrackEngine(S, **KW)
    for f in range(3):
        eng.submit([frames[s][f] for s in range(S)])
    with pytest.raises(_lib.YTAError):
        eng.submit([frames[s][3] for s in range(S)])
    with pytest.raises(_lib.YTAError):
        eng.update([frames[s][3] for s in range(S)])
    with pytest.raises(_lib.YTAError):
        eng.reset()
    got = [eng.collect() for _ in range(3)]
    with pytest.raises(_lib.YTAError):
        eng.collect()
    ref = ByteTrackEngine(S, **KW)
    for f in range(3):
        exp = ref.update([frames[s][f] for s in range(S)])
        assert all(np.array_equal(x, y) for x, y in zip(got[f], exp)), f
    out = eng.update([frames[s][3] for s in range(S)])   # the synchronous path works again
    assert all(np.array_equal(x, y) for x, y in zip(out, ref.update([frames[s][3] for s in range(S)])))


@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("pinned", [False, True])
def test_float32_detections_equal_promoted_float64(pipelined, pinned):
    """float32 detections (yta_bytetrack_update_f32 / _submit_f32: half the bytes over PCIe,
    widened on the device) give exactly the float64 call on the promoted rows, as the
    reference's np.hstack promotion does (byte_tracker.py:143)."""
    import torch
    S, F = 3, 16
    frames = [[d.astype(np.float32) for d in fs] for fs in _streams(S, F, 120, 950)]
    ref = ByteTrackEngine(S, **KW)
    eng = ByteTrackEngine(S, **KW)
    exp = [ref.update([frames[s][f].astype(np.float64) for s in range(S)]) for f in range(F)]

    def src(f):
        if not pinned:
            return [frames[s][f] for s in range(S)]
        out = []
        for s in range(S):
            t = torch.empty(frames[s][f].shape, dtype=torch.float32, pin_memory=True).numpy()
            t[:] = frames[s][f]
            out.append(t)
        return out
    got = []
    if pipelined:
        for f in range(F):
            eng.submit(src(f))
            if f >= 2:
                got.append(eng.collect())
        got += [eng.collect(), eng.collect()]
    else:
        got = [eng.update(src(f)) for f in range(F)]
    for f in range(F):
        for s in range(S):
            assert np.array_equal(got[f][s], exp[f][s]), (f, s)
