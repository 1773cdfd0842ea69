"""GPU: parity of the headline bench's own launch shape (bench.py at the driver's `--steps 20
--warmup 5`): 2048 ByteTrack streams of 1024 x 1024 per GPU in two engines of 1024 streams, each
engine on its own HIP stream, frames staged in HBM by bench.stage_frames (seeds 1000..3047) and run
through yta_bytetrack_update_device exactly as the timed loop does - the 35-frame pre-roll, the 5
warmup and 20 timed frames with both engines' launches interleaved on the chip and phase
profiling on, then 3 frames of engine 0 alone (the isolated leg).  63 frames: Lost tracks expire
(max_time_lost 30, byte_tracker.py:250-253) from frame 32 on.

What only exists at this shape and is checked here: the global arenas and LDS fallbacks at 1024
blocks per launch, the chip-wide kernels' per-stream indexing over 1024 streams, two engines
sharing the chip.

Bar:
* every stream's rows, every frame, bit-identical (int64 views of the float64 rows) to a
  one-stream engine fed that stream's frames from the same staged HBM tensors (the one-stream
  engine is itself bit-exact against the reference's goldens: test_gpu_full_configs.py), and every
  stream's final ID counter equal (yta_bytetrack_next_ids);
* 8 sampled streams (first and last two of each engine) frame by frame against
  oracle.bytetrack.ByteTrackOracle (byte_tracker.py:132-281): ids, scores, classes and det_ind
  exact, boxes within 1e-9 relative (the NumPy restatement's box arithmetic is not the reference's
  operation for operation; the engine is, see test_gpu_full_configs.py), and ID counters equal;
* no stream-frame left the LDS arenas or raised an error flag.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
N = 1024
S = 2048
Q = 2
SQ = S // Q
SEED = 1000
PRE = 35 + 5          # bench.py --preroll 35 + the driver's --warmup 5
STEPS = 20            # the driver's --steps 20
ISO = 3               # bench.py's isolated leg: engine 0 alone
F = PRE + STEPS
FT = F + ISO
CAP = 2 * N           # bench.py: track_capacity 2N, max_dets N
SAMPLED = [0, 1, SQ - 2, SQ - 1, SQ, SQ + 1, S - 2, S - 1]
KW = dict(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)


def frames_of(s):
    """Frames a global stream runs: engine 0's streams also run the isolated leg."""
    return FT if s < SQ else F


@pytest.fixture(scope="module")
def oracle_runs(tmp_path_factory):
    """The sampled streams through the oracle, one CPU process each, started first so they run
    while the GPU works."""
    d = tmp_path_factory.mktemp("oracle_streams")
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1")
    procs = {}
    for s in SAMPLED:
        out = str(d / f"s{s}.npz")
        procs[s] = (out, subprocess.Popen(
            [sys.executable, os.path.join(HERE, "oracle_stream.py"), str(N), str(frames_of(s)),
             str(SEED + s), out], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    yield procs
    for _, p in procs.values():
        if p.poll() is None:
            p.kill()


@pytest.fixture(scope="module")
def headline(oracle_runs):
    import torch

    import bench
    from yolo_tracking_amd import ByteTrackEngine, _lib
    torch.cuda.set_device(0)
    d_dets, d_off = bench.stage_frames(N, FT, bench.stream_seeds(SEED, 0, S), Q, "cuda")
    engs = [ByteTrackEngine(SQ, device=0, track_capacity=CAP, max_dets=N, **KW) for _ in range(Q)]
    assert engs[0].capacity() == (CAP, N)
    lib = engs[0].lib
    # every frame's rows kept (bench.py reuses one output buffer; the kernels are the same)
    d_out = torch.empty((FT, Q, SQ * CAP, 8), dtype=torch.float64, device="cuda")
    d_cnt = torch.zeros((FT, Q, SQ), dtype=torch.int32, device="cuda")
    row_bytes = N * 6 * 8 * SQ

    def step(f, engines):
        for q in engines:
            _lib.check(lib.yta_bytetrack_update_device(
                engs[q].handle, ctypes.c_void_p(d_dets[q].data_ptr() + f * row_bytes),
                ctypes.c_void_p(d_off[q].data_ptr() + f * (SQ + 1) * 4),
                ctypes.c_void_p(d_out[f, q].data_ptr()), ctypes.c_void_p(d_cnt[f, q].data_ptr())))

    torch.cuda.synchronize()
    for f in range(PRE):
        step(f, range(Q))
    for e in engs:
        _lib.check(lib.yta_bytetrack_sync(e.handle))
        _lib.check(lib.yta_bytetrack_profile(e.handle, 1))
    for f in range(PRE, F):                       # the timed loop: no sync between frames
        step(f, range(Q))
    for e in engs:
        _lib.check(lib.yta_bytetrack_sync(e.handle))
    for f in range(F, FT):                        # the isolated leg
        step(f, [0])
    stats = [e.stats() for e in engs]             # synchronises, reports the last frame
    nid = np.zeros(S, np.int64)
    for q, e in enumerate(engs):
        _lib.check(lib.yta_bytetrack_sync(e.handle))
        _lib.check(lib.yta_bytetrack_next_ids(e.handle, nid[q * SQ:].ctypes.data))
    for e in engs:
        e.close()
    return dict(d_dets=d_dets, d_off=d_off, d_out=d_out, d_cnt=d_cnt, stats=stats, nid=nid)


@pytest.fixture(scope="module")
def one_stream(headline):
    """Every stream through a one-stream engine, from the same staged frames (device-resident
    update, 8 engines round robin so their HIP streams overlap).  Rows land at
    ref_out[s][f][:count]."""
    import torch

    from yolo_tracking_amd import ByteTrackEngine, _lib
    R = 8
    engs = [ByteTrackEngine(1, device=0, track_capacity=CAP, max_dets=N, **KW) for _ in range(R)]
    lib = engs[0].lib
    ref_out = torch.empty((S, FT, CAP, 8), dtype=torch.float64, device="cuda")
    ref_cnt = torch.zeros((S, FT), dtype=torch.int32, device="cuda")
    off1 = torch.tensor([0, N], dtype=torch.int32, device="cuda")
    nid = np.zeros(S, np.int64)
    one = np.zeros(1, np.int64)
    d_dets = headline["d_dets"]
    pending = [None] * R
    for s in range(S):
        r = s % R
        e = engs[r]
        if pending[r] is not None:                # the previous stream of this engine: its counter
            _lib.check(lib.yta_bytetrack_next_ids(e.handle, one.ctypes.data))
            nid[pending[r]] = one[0]
        e.reset()
        q, j = divmod(s, SQ)
        base = d_dets[q].data_ptr() + j * N * 48
        for f in range(frames_of(s)):
            _lib.check(lib.yta_bytetrack_update_device(
                e.handle, ctypes.c_void_p(base + f * SQ * N * 48), ctypes.c_void_p(off1.data_ptr()),
                ctypes.c_void_p(ref_out[s, f].data_ptr()),
                ctypes.c_void_p(ref_cnt.data_ptr() + (s * FT + f) * 4)))
        pending[r] = s
    for r, e in enumerate(engs):
        if pending[r] is not None:
            _lib.check(lib.yta_bytetrack_next_ids(e.handle, one.ctypes.data))
            nid[pending[r]] = one[0]
        _lib.check(lib.yta_bytetrack_sync(e.handle))
        e.close()
    torch.cuda.synchronize()
    return dict(ref_out=ref_out, ref_cnt=ref_cnt, nid=nid)


def test_headline_counts_and_arenas(headline):
    """The headline frames ran in the LDS arenas with the steady-state population (bench.py's
    per_stream_last_frame: ~1000 tracked, ~600 lost per stream)."""
    for st in headline["stats"]:
        assert st["fallback1"] == 0 and st["fallback23"] == 0 and st["fallback_f"] == 0, st
    st1 = headline["stats"][1]                    # engine 1's last frame is frame F - 1
    assert st1["dets"] == SQ * N
    assert 900 * SQ < st1["tracked"] < 1100 * SQ and 400 * SQ < st1["lost"] < 800 * SQ, st1


def test_every_stream_equals_one_stream_engine(headline, one_stream):
    import torch
    d_out, d_cnt = headline["d_out"], headline["d_cnt"]
    ref_out, ref_cnt = one_stream["ref_out"], one_stream["ref_cnt"]
    rows_checked = 0
    rows = torch.arange(CAP, device="cuda")
    for f in range(FT):
        ns = S if f < F else SQ                  # the isolated leg: engine 0's streams
        hc = d_cnt[f].reshape(S)[:ns]
        rc = ref_cnt[:ns, f]
        bad = torch.nonzero(hc != rc).flatten()
        assert len(bad) == 0, (f, bad[:8].tolist(), hc[bad[:8]].tolist(), rc[bad[:8]].tolist())
        h = d_out[f].reshape(S, CAP, 8)[:ns].view(torch.int64)
        r = ref_out[:ns, f].view(torch.int64)
        live = (rows[None, :] < hc[:, None].long())[:, :, None]
        diff = ((h != r) & live).any(dim=2).any(dim=1)
        bad = torch.nonzero(diff).flatten()
        assert len(bad) == 0, (f, bad[:8].tolist())
        rows_checked += int(hc.sum())
    assert rows_checked > 0.9 * N * (S * F + SQ * ISO)
    assert np.array_equal(headline["nid"], one_stream["nid"]), np.nonzero(
        headline["nid"] != one_stream["nid"])[0][:8]


def test_sampled_streams_against_oracle(headline, oracle_runs):
    d_out, d_cnt = headline["d_out"], headline["d_cnt"]
    for s in SAMPLED:
        path, p = oracle_runs[s]
        _, err = p.communicate(timeout=600)
        assert p.returncode == 0, err.decode()[-2000:]
        z = np.load(path)
        counts = z["counts"]
        offs = np.concatenate([[0], np.cumsum(counts)])
        q, j = divmod(s, SQ)
        cnt = d_cnt[:, q, j].cpu().numpy()
        for f in range(frames_of(s)):
            exp = z["rows"][offs[f]:offs[f + 1]]
            assert cnt[f] == len(exp), (s, f, int(cnt[f]), len(exp))
            got = d_out[f, q, j * CAP:j * CAP + cnt[f]].cpu().numpy()
            assert np.array_equal(got[:, 4:], exp[:, 4:]), (s, f)
            np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-9, atol=1e-9,
                                       err_msg=f"stream {s} frame {f}")
        assert headline["nid"][s] == int(z["next_id"]), s
