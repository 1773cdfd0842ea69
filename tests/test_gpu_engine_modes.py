"""GPU: the ByteTrack engine's launch modes and teardown.

* Capacity growth mid-run (reserve(): every buffer reallocated, the state copied over, the next
  stage-1 pool rebuilt) on engines created under every combination of YTA_GRAPHS (cached HIP graph
  of a small host-buffer frame, re-captured when an argument changes) and YTA_SPLIT23 (stage 2 and
  stage 3 in two blocks per stream, the 1024-thread stage-1 / finish blocks): rows and ID counters
  bit-identical across the four engines and equal to the oracle (byte_tracker.py:132-281), and
  the mode the kernel arguments carry (with its pooled fallback arenas) still the one chosen at
  create after the growth (yta_bytetrack_modes).  Round 5's reserve() dropped the split mode on growth.
* Destroying an engine with pipelined frames submitted and not collected: the copy streams are
  drained before their buffers are freed; a new engine of the same sizes then runs exactly as a
  fresh one.
"""
import ctypes
import itertools

import numpy as np
import pytest

from oracle.bytetrack import ByteTrackOracle
from yolo_tracking_amd import ByteTrackEngine, _lib
from yolo_tracking_amd.synth import make_frames

pytestmark = pytest.mark.gpu

KW = dict(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)
MODES = ["split23", "args_split23", "ws_slots", "graphs", "bs_split", "captures", "replays", "cap",
         "maxd"]


def modes(eng):
    buf = (ctypes.c_longlong * len(MODES))()
    _lib.check(eng.lib.yta_bytetrack_modes(eng.handle, buf, len(MODES)))
    return {k: int(buf[i]) for i, k in enumerate(MODES)}


def _growing_streams(S, F, grow_at):
    """S streams of 120 objects; before frame grow_at only the first 10 objects are detected, so
    the engine (capacity 32, 32 detections) has to grow mid-run."""
    out = []
    for s in range(S):
        fr = [d for d, _ in make_frames(120, F, seed=910 + s)]
        out.append([d[:10] if f < grow_at else d for f, d in enumerate(fr)])
    return out


def test_growth_under_every_launch_mode(monkeypatch):
    S, F, G = 3, 36, 12
    frames = _growing_streams(S, F, G)
    ors = [ByteTrackOracle(**KW) for _ in range(S)]
    exp = [[ors[s].update(frames[s][f]).reshape(-1, 8) for f in range(F)] for s in range(S)]
    results = {}
    for graphs, split in itertools.product([0, 1], [0, 1]):
        monkeypatch.setenv("YTA_GRAPHS", str(graphs))
        monkeypatch.setenv("YTA_SPLIT23", str(split))
        eng = ByteTrackEngine(S, track_capacity=32, max_dets=32, **KW)
        m0 = modes(eng)
        assert (m0["split23"], m0["args_split23"]) == (split,) * 2, m0
        assert m0["ws_slots"] == (2 * S if split else S), m0   # every block can fall back at once
        assert m0["graphs"] == graphs and (m0["cap"], m0["maxd"]) == (32, 32), m0
        nid = np.zeros(S, np.int64)
        got, caps = [], []
        for f in range(F):
            got.append(eng.update([frames[s][f] for s in range(S)], next_id=nid))
            caps.append(modes(eng)["cap"])
        assert caps[0] == 32 and caps[G - 1] < caps[-1], caps   # grew mid-run
        m1 = modes(eng)
        assert m1["cap"] > 32 and m1["maxd"] >= 120, m1
        # the kernel arguments still carry the mode chosen at create, with its second arena
        assert (m1["split23"], m1["args_split23"]) == (split,) * 2, m1
        assert m1["ws_slots"] == (2 * S if split else S), m1
        if graphs:   # captured at least before and after the growth, then replayed
            assert m1["captures"] >= 2 and m1["replays"] >= F, m1
        else:
            assert m1["captures"] == 0 and m1["replays"] == 0, m1
        results[(graphs, split)] = (got, nid.copy())
        eng.close()
    base_rows, base_nid = results[(1, 1)]
    for key, (rows, nid) in results.items():
        assert np.array_equal(nid, base_nid), key
        for f in range(F):
            for s in range(S):
                assert np.array_equal(rows[f][s].view(np.int64),
                                      base_rows[f][s].view(np.int64)), (key, f, s)
    for f in range(F):
        for s in range(S):
            g, e = base_rows[f][s], exp[s][f]
            assert g.shape == e.shape, (f, s)
            assert np.array_equal(g[:, 4:], e[:, 4:]), (f, s)
            np.testing.assert_allclose(g[:, :4], e[:, :4], rtol=1e-9, atol=1e-9)


def test_reserve_keeps_modes(monkeypatch):
    """yta_bytetrack_reserve (the explicit growth entry point) keeps the create-time modes too."""
    for split in (0, 1):
        monkeypatch.setenv("YTA_SPLIT23", str(split))
        eng = ByteTrackEngine(2, track_capacity=16, max_dets=16, **KW)
        eng.reserve(64, 48)
        m = modes(eng)
        assert (m["split23"], m["args_split23"]) == (split,) * 2, m
        assert m["ws_slots"] == (4 if split else 2), m
        assert (m["cap"], m["maxd"]) == (64, 48), m
        eng.close()


@pytest.mark.parametrize("pinned", [False, True])
def test_destroy_with_frames_in_flight(pinned):
    import torch
    S, N, F = 4, 200, 6
    frames = [[d for d, _ in make_frames(N, F, seed=1300 + s)] for s in range(S)]

    def pbuf(shape):
        if not pinned:
            return np.empty(shape)
        return torch.empty(shape, dtype=torch.float64, pin_memory=True).numpy()
    for rounds in range(3):
        eng = ByteTrackEngine(S, track_capacity=512, max_dets=N, **KW)
        ins = [pbuf((S * N, 6)) for _ in range(2)]
        outs = [pbuf((S * N, 8)) for _ in range(2)]
        for f in range(2):
            ins[f][:] = np.concatenate([frames[s][f] for s in range(S)])
            off = np.arange(S + 1, dtype=np.int32) * N
            _lib.check(eng.lib.yta_bytetrack_submit(eng.handle, ins[f].ctypes.data,
                                                    off.ctypes.data, None, outs[f].ctypes.data,
                                                    S * N))
        eng.close()    # two frames submitted, none collected
        del ins, outs
        # an engine of the same sizes right after: same results as a fresh reference engine
        new = ByteTrackEngine(S, track_capacity=512, max_dets=N, **KW)
        ref = ByteTrackEngine(S, track_capacity=512, max_dets=N, **KW)
        for f in range(F):
            a = new.update([frames[s][f] for s in range(S)])
            b = ref.update([frames[s][f] for s in range(S)])
            for s in range(S):
                assert np.array_equal(a[s].view(np.int64), b[s].view(np.int64)), (rounds, f, s)
        new.close()
        ref.close()


def test_fallback_pool_under_contention(monkeypatch):
    """Every stream-frame on the global fallback arenas (LDS budget 0) with a pool of two arenas
    for eight streams (YTA_WS_POOL=2): every block of a launch queues its stream and the launch's
    two-block redo kernel takes four streams per arena in turn (bytetrack.hip redo_drain; the
    queue cleared by its last block for the next launch), and every row equals the LDS-arena
    engine's."""
    S, F = 8, 14
    frames = [[d for d, _ in make_frames(300, F, seed=1500 + s)] for s in range(S)]
    ref = ByteTrackEngine(S, track_capacity=512, max_dets=300, **KW)
    monkeypatch.setenv("YTA_WS_POOL", "2")
    monkeypatch.setenv("YTA_SPLIT23", "0")
    eng = ByteTrackEngine(S, track_capacity=512, max_dets=300, **KW)
    assert modes(eng)["ws_slots"] == 2
    eng.set_lds(0)
    for f in range(F):
        a = eng.update([frames[s][f] for s in range(S)])
        b = ref.update([frames[s][f] for s in range(S)])
        for s in range(S):
            assert np.array_equal(a[s].view(np.int64), b[s].view(np.int64)), (f, s)
    st = eng.stats()
    assert st["fallback1"] >= S * (F - 1) and st["fallback23"] >= S * F, st


BS_P = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6, track_buffer=30,
            match_thresh=0.8, proximity_thresh=0.5, appearance_thresh=0.25, frame_rate=30)


@pytest.mark.parametrize("case", ["bytetrack_split", "botsort_reid", "botsort_fused",
                                  "botsort_split23_off"])
def test_redo_kernels_every_variant(monkeypatch, case):
    """The redo kernels of every association kernel variant (bytetrack.hip k_redo_s1_lap<1024>,
    k_redo_stage23<V, true / false>, k_redo_finish<V, 1024 / 256>, k_redo_bs_lap,
    k_redo_stage1<BoT-SORT>): ten streams, a pool of two arenas (YTA_WS_POOL=2, so every launch
    has more blocks than arenas and queues), the LDS budget 0 (every stream-frame falls back):
    rows bit-identical to the same engine kind on its LDS arenas, frame by frame.  bytetrack_split:
    the few-stream mode's split stage 2 / 3 and 1024-thread stage-1 / finish blocks;
    botsort_reid: split stage 1 (k_bs_lap) with 32-d embeddings; botsort_fused: the fused
    k_stage1 (YTA_BS_SPLIT=0); botsort_split23_off: one block per stream for stages 2 / 3."""
    from test_oracle_golden import reid_features
    from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
    S, F, n, D = 10, 12, 300, 32
    bot = case.startswith("botsort")
    streams = [make_frames(n, F, 2600 + s, emb_dim=D if bot else 0) for s in range(S)]
    env = {"bytetrack_split": {"YTA_SPLIT23": "1"},
           "botsort_reid": {"YTA_SPLIT23": "1", "YTA_BS_SPLIT": "1"},
           "botsort_fused": {"YTA_SPLIT23": "1", "YTA_BS_SPLIT": "0"},
           "botsort_split23_off": {"YTA_SPLIT23": "0", "YTA_BS_SPLIT": "1"}}[case]
    for k, v in env.items():
        monkeypatch.setenv(k, v)

    def make():
        if bot:
            return BoTSORTEngine(S, feat_dim=D, track_capacity=512, max_dets=n, **BS_P)
        return ByteTrackEngine(S, track_capacity=512, max_dets=n, **KW)
    ref = make()
    monkeypatch.setenv("YTA_WS_POOL", "2")
    eng = make()
    assert modes(eng)["ws_slots"] == 2
    assert modes(eng)["split23"] == int(env["YTA_SPLIT23"])
    eng.set_lds(0)
    for f in range(F):
        dets = [streams[s][f][0] for s in range(S)]
        if bot:
            feats = [reid_features(dets[s], streams[s][f][1], BS_P["track_high_thresh"])
                     for s in range(S)]
            a, b = eng.update(dets, feats), ref.update(dets, feats)
        else:
            a, b = eng.update(dets), ref.update(dets)
        for s in range(S):
            assert np.array_equal(a[s].view(np.int64), b[s].view(np.int64)), (case, f, s)
    st = eng.stats()   # every association that needed an arena ran on a pooled one
    assert st["fallback1"] > 0 and st["fallback23"] > 0, st
    assert st["fallback_f"] >= S * (F - 1), st
