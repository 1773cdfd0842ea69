"""GPU: the pipelined host-buffer update (yta_bytetrack_submit / yta_bytetrack_collect: frame f's
detections in flight while frame f-1's kernels run and frame f-2's rows come back) gives exactly
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
                for _ in range(2)]
    got = []
    nid = np.zeros(S, np.int64)
    for f in range(F):
        eng.submit([frames[s][f] for s in range(S)], out=None if outs is None else outs[f % 2])
        if f >= 1:
            got.append(eng.collect(next_id=nid) + [nid.copy()])
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
    frames = _streams(S, 4, 60, 800)
    eng = ByteTrackEngine(S, **KW)
    eng.submit([frames[s][0] for s in range(S)])
    eng.submit([frames[s][1] for s in range(S)])
    with pytest.raises(_lib.YTAError):
        eng.submit([frames[s][2] for s in range(S)])
    with pytest.raises(_lib.YTAError):
        eng.update([frames[s][2] for s in range(S)])
    with pytest.raises(_lib.YTAError):
        eng.reset()
    a = eng.collect()
    b = eng.collect()
    with pytest.raises(_lib.YTAError):
        eng.collect()
    ref = ByteTrackEngine(S, **KW)
    assert all(np.array_equal(x, y) for x, y in zip(a, ref.update([frames[s][0] for s in range(S)])))
    assert all(np.array_equal(x, y) for x, y in zip(b, ref.update([frames[s][1] for s in range(S)])))
    out = eng.update([frames[s][2] for s in range(S)])   # the synchronous path works again
    assert all(np.array_equal(x, y) for x, y in zip(out, ref.update([frames[s][2] for s in range(S)])))
