"""GPU: parity of the pipelined host-buffer path at the bench's own shape - the code behind
bench.py's `pcie_inclusive.pipelined` figures (§8(d)'s wall-clock metric).

bench.pcie_pipelined itself runs here (its `check` hook receives every collected frame's packed
rows and, at the end, the engine's ID counters and pipe accounting): one engine of 2048 ByteTrack
streams of 1024 x 1024, track capacity 3N (cap_mult 3), three frames in flight (PIPE_DEPTH),
frames from bench.stage_frames / bench.stream_seeds(1000, 0, 2048); 3 frames submitted and
collected one at a time (the bench's untimed frames), then 45 pipelined frames (past
max_time_lost = 30, so Lost tracks expire inside the pipelined run).  Legs: page-locked float64
buffers (DMA'd directly, rows stored by k_rows_to_host into the caller's buffer), pageable float64
(staged), page-locked float32 detections (widened on the device).

Frame G is one where the capacity bound cannot hold: stream K receives 1100 extra detections on
top of its 1024, so the submit drains the frames in flight and grows the engine (max_dets and
track capacity) while the earlier frames' copy-outs are still queued; pipe_stats must count the
drain.

Bar: every frame's rows of all 2048 streams bit-identical (int64 views) to the device-resident
path (yta_bytetrack_update_device, one engine of 2048 streams sized for the surge, itself checked
against the reference goldens and the oracle at this shape by test_gpu_headline_shape.py) on the
same frames - for the float32 leg, the frames rounded to float32 and promoted back, as the
reference's np.hstack promotion does (byte_tracker.py:143) - the same row offsets, and the same
final ID counters.  Reference: byte_tracker.py:132-281.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 1024
S = 2048
SEED = 1000
FIRST = 3            # submitted and collected one at a time (bench.py's untimed frames)
PIPED = 45           # pipelined, three in flight
F = FIRST + PIPED
G = 20               # the frame whose capacity bound cannot hold
K = 777              # the stream that gets the extra detections
EXTRA = 1100
KW = dict(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)


def _extra_rows():
    rng = np.random.default_rng(4242)
    C = 64.0 * np.sqrt(N)
    xy = rng.uniform(0, C, size=(EXTRA, 2))
    wh = rng.uniform(16, 64, size=(EXTRA, 2))
    d = np.zeros((EXTRA, 6))
    d[:, :2] = xy
    d[:, 2:4] = xy + wh
    d[:, 4] = rng.uniform(0.6, 0.95, size=EXTRA)
    return d


@pytest.fixture(scope="module")
def staged():
    import torch

    import bench
    torch.cuda.set_device(0)
    d_dets, _ = bench.stage_frames(N, F, bench.stream_seeds(SEED, 0, S), 1, "cuda")
    d_dets = d_dets[0]                                         # [F][S*N][6] float64
    extra = torch.from_numpy(_extra_rows()).cuda()
    offs = []
    for f in range(F):
        o = np.arange(S + 1, dtype=np.int64) * N
        if f == G:
            o[K + 1:] += EXTRA
        offs.append(o.astype(np.int32))

    def frame_dev(f, f32=False):
        d = d_dets[f]
        if f == G:
            d = torch.cat([d[:(K + 1) * N], extra, d[(K + 1) * N:]])
        return d.float().double() if f32 else d
    return dict(frame_dev=frame_dev, offs=offs)


def _device_reference(staged, f32):
    """The device-resident path on the same frames: packed rows per frame (on the device), row
    offsets and final ID counters."""
    import torch

    from yolo_tracking_amd import ByteTrackEngine, _lib
    # the surge: stream K peaks at ~1620 tracked + lost plus 1100 births (< 3N); 2124 detections
    CAPR, MAXDR = 3 * N, N + EXTRA + 64
    eng = ByteTrackEngine(S, device=0, track_capacity=CAPR, max_dets=MAXDR, **KW)
    lib = eng.lib
    d_out = torch.empty((S * CAPR, 8), dtype=torch.float64, device="cuda")
    d_cnt = torch.zeros(S, dtype=torch.int32, device="cuda")
    rows = torch.arange(CAPR, device="cuda")
    packed, offsets = [], []
    for f in range(F):
        d = staged["frame_dev"](f, f32).contiguous()
        o = torch.from_numpy(staged["offs"][f]).cuda()
        _lib.check(lib.yta_bytetrack_update_device(
            eng.handle, ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(o.data_ptr()),
            ctypes.c_void_p(d_out.data_ptr()), ctypes.c_void_p(d_cnt.data_ptr())))
        _lib.check(lib.yta_bytetrack_sync(eng.handle))
        mask = rows[None, :] < d_cnt[:, None].long()
        packed.append(d_out.view(S, CAPR, 8)[mask].clone())
        off = np.zeros(S + 1, np.int64)
        np.cumsum(d_cnt.cpu().numpy(), out=off[1:])
        offsets.append(off)
    nid = np.zeros(S, np.int64)
    _lib.check(lib.yta_bytetrack_next_ids(eng.handle, nid.ctypes.data))
    eng.close()
    return packed, offsets, nid


@pytest.fixture(scope="module")
def reference64(staged):
    return _device_reference(staged, False)


@pytest.fixture(scope="module")
def reference32(staged):
    return _device_reference(staged, True)


@pytest.mark.parametrize("leg", ["pinned", "pageable", "pinned_f32"])
def test_pipelined_bench_shape_equals_device_path(leg, staged, request):
    import torch

    import bench
    f32 = leg.endswith("f32")
    packed, offsets, nid_ref = request.getfixturevalue("reference32" if f32 else "reference64")
    seen = {}

    def frame_of(f):
        return staged["frame_dev"](f).cpu().numpy()

    def check(f, rows, out_off, *extra):
        if f is None:
            seen["nid"], seen["stats"] = rows, out_off
            return
        assert np.array_equal(out_off.astype(np.int64), offsets[f]), f
        got = torch.from_numpy(np.ascontiguousarray(rows)).cuda()
        exp = packed[f]
        assert got.shape == exp.shape, (f, tuple(got.shape), tuple(exp.shape))
        bad = (got.view(torch.int64) != exp.view(torch.int64)).any(dim=1)
        if bool(bad.any()):
            r = int(torch.nonzero(bad)[0])
            s = int(np.searchsorted(offsets[f], r, side="right") - 1)
            pytest.fail(f"{leg}: frame {f} row {r} (stream {s}) differs")
        seen[f] = True

    bench.pcie_pipelined(frame_of, S, N, 0, first=FIRST, frames=PIPED, pinned=leg != "pageable",
                         f32=f32, cap_mult=3, check=check,
                         offsets_of=lambda f: staged["offs"][f])
    assert all(seen.get(f) for f in range(F)), sorted(k for k in seen if isinstance(k, int))
    assert np.array_equal(seen["nid"], nid_ref), np.nonzero(seen["nid"] != nid_ref)[0][:8]
    ps = seen["stats"]
    # frame G drained the pipeline and grew the engine; the other frames ran pipelined
    assert ps["capacity_drains"] >= 1, ps
    assert ps["frames"] == PIPED, ps
