"""GPU: stream-subset updates and per-stream reset (SURVEY.md §8(b) `update(ctx, n_streams,
stream_ids, ...)`).  In the reference every camera stream is its own tracker
(examples/track.py:43-57) and a stream without a new frame is not called at all
(examples/val.py:184-226 runs sequences of different lengths side by side).

Bar: a skipped stream's whole state (tracks, Kalman state, frame and ID counters) is
bit-identical across the call; every stream's rows equal those of a standalone tracker that saw
only that stream's frames (the oracle for ByteTrack, a one-stream engine for BoT-SORT); a reset
stream restarts as a fresh tracker while the others continue.
"""
import ctypes

import numpy as np
import pytest

from oracle.bytetrack import ByteTrackOracle
from test_oracle_golden import reid_features
from yolo_tracking_amd import ByteTrackEngine, _lib
from yolo_tracking_amd.synth import make_frames
from yolo_tracking_amd.trackers.botsort import BoTSORTEngine

pytestmark = pytest.mark.gpu

KW = dict(track_thresh=0.5, match_thresh=0.8, track_buffer=30, frame_rate=30)


def _rows_equal(got, exp, ctx):
    exp = np.asarray(exp, dtype=np.float64).reshape(-1, 8)
    assert got.shape == exp.shape, (ctx, got.shape, exp.shape)
    assert np.array_equal(got[:, 4:], exp[:, 4:]), ctx
    np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-9, atol=1e-6, err_msg=str(ctx))


def _same_state(a, b):
    return all(np.array_equal(a[k], b[k]) for k in a)


@pytest.mark.parametrize("cap", [None, 4096])
def test_bytetrack_subset_schedule_matches_standalone_oracles(cap):
    """Four streams, each frame a random subset of them (incl. single streams and all four),
    listed in a random order: every stream's rows equal its own oracle's, skipped streams are
    bit-identical across the call, and per-stream ID counters follow each stream alone."""
    S, F = 4, 30
    rng = np.random.default_rng(7)
    frames = [[d for d, _ in make_frames(150 + 30 * s, F, seed=300 + s)] for s in range(S)]
    eng = ByteTrackEngine(S, **KW) if cap is None else ByteTrackEngine(
        S, track_capacity=cap, max_dets=512, **KW)
    refs = [ByteTrackOracle(**KW) for _ in range(S)]
    pos = [0] * S
    nid = np.zeros(S, np.int64)
    for step in range(2 * F):
        k = int(rng.integers(1, S + 1))
        ids = [int(i) for i in rng.permutation(S)[:k] if pos[i] < F]
        if not ids:
            continue
        skipped = [s for s in range(S) if s not in ids]
        before = {s: eng.state(s) for s in skipped}
        ids_nid = nid[ids].copy()
        outs = eng.update([frames[s][pos[s]] for s in ids], next_id=ids_nid, streams=ids)
        nid[ids] = ids_nid
        for s, out in zip(ids, outs):
            _rows_equal(out, refs[s].update(frames[s][pos[s]]), (step, s, pos[s]))
            assert nid[s] == refs[s].next_id, (step, s)
            pos[s] += 1
        for s in skipped:
            assert _same_state(before[s], eng.state(s)), (step, s)
    assert min(pos) > 5


def test_bytetrack_reset_stream():
    """reset_stream(1) mid-sequence: stream 1 restarts as a fresh tracker (its next frames equal a
    new oracle's, IDs from 1), streams 0 and 2 continue untouched."""
    S, F = 3, 16
    frames = [[d for d, _ in make_frames(120, F, seed=410 + s)] for s in range(S)]
    eng = ByteTrackEngine(S, **KW)
    refs = [ByteTrackOracle(**KW) for _ in range(S)]
    for f in range(F):
        if f == 9:
            before = [eng.state(s) for s in (0, 2)]
            eng.reset_stream(1)
            assert len(eng.state(1)["id"]) == 0
            assert _same_state(before[0], eng.state(0)) and _same_state(before[1], eng.state(2))
            refs[1] = ByteTrackOracle(**KW)
        outs = eng.update([frames[s][f] for s in range(S)])
        for s in range(S):
            _rows_equal(outs[s], refs[s].update(frames[s][f]), (f, s))


def test_bytetrack_device_masked_matches_host_subset():
    """yta_bytetrack_update_device_masked: the device form of the subset update gives the same
    rows and states as the host-buffer subset update."""
    import torch
    S, N, F = 3, 128, 12
    frames = [[d for d, _ in make_frames(N, F, seed=500 + s)] for s in range(S)]
    host = ByteTrackEngine(S, track_capacity=512, max_dets=N, **KW)
    dev = ByteTrackEngine(S, track_capacity=512, max_dets=N, **KW)
    cap, _ = dev.capacity()
    d_out = torch.empty((S * cap, 8), dtype=torch.float64, device="cuda")
    d_cnt = torch.zeros(S, dtype=torch.int32, device="cuda")
    rng = np.random.default_rng(3)
    pos = [0] * S
    for step in range(2 * F):
        ids = sorted(int(i) for i in rng.permutation(S)[:int(rng.integers(1, S + 1))]
                     if pos[i] < F)
        if not ids:
            continue
        outs = host.update([frames[s][pos[s]] for s in ids], streams=ids)
        mask = np.zeros(S, np.int32)
        mask[ids] = 1
        per = [frames[s][pos[s]] if s in ids else np.zeros((0, 6)) for s in range(S)]
        off = np.zeros(S + 1, np.int32)
        np.cumsum([len(d) for d in per], out=off[1:])
        d_dets = torch.from_numpy(np.ascontiguousarray(np.concatenate(per))).cuda()
        d_off = torch.from_numpy(off).cuda()
        d_mask = torch.from_numpy(mask).cuda()
        torch.cuda.synchronize()
        _lib.check(dev.lib.yta_bytetrack_update_device_masked(
            dev.handle, ctypes.c_void_p(d_mask.data_ptr()), ctypes.c_void_p(d_dets.data_ptr()),
            ctypes.c_void_p(d_off.data_ptr()), ctypes.c_void_p(d_out.data_ptr()),
            ctypes.c_void_p(d_cnt.data_ptr())))
        _lib.check(dev.lib.yta_bytetrack_sync(dev.handle))
        cnt = d_cnt.cpu().numpy()
        rows = d_out.cpu().numpy()
        for s in range(S):
            if s not in ids:
                assert cnt[s] == 0, (step, s)
                continue
            got = rows[s * cap:s * cap + cnt[s]]
            assert np.array_equal(got, outs[ids.index(s)]), (step, s)
            pos[s] += 1
        for s in range(S):
            assert _same_state(host.state(s), dev.state(s)), (step, s)


def test_botsort_subset_with_features_and_warps():
    """BoT-SORT: subset updates with ReID rows and per-stream camera warps equal one-stream
    engines fed the same frames; skipped streams (features included) are untouched."""
    S, N, F, D = 3, 96, 14, 32
    P = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
             track_buffer=30, match_thresh=0.8, proximity_thresh=0.5, appearance_thresh=0.25,
             frame_rate=30)
    frames = [make_frames(N, F, seed=600 + s, emb_dim=D) for s in range(S)]
    warp = np.array([[1.0, 1e-3, 0.5], [-1e-3, 1.0, -0.3]])
    eng = BoTSORTEngine(S, feat_dim=D, **P)
    solo = [BoTSORTEngine(1, feat_dim=D, **P) for _ in range(S)]
    rng = np.random.default_rng(11)
    pos = [0] * S
    for step in range(2 * F):
        ids = [int(i) for i in rng.permutation(S)[:int(rng.integers(1, S + 1))] if pos[i] < F]
        if not ids:
            continue
        skipped = [s for s in range(S) if s not in ids]
        before = {s: (eng.state(s), eng.features(s)[0].copy()) for s in skipped}
        dets = [frames[s][pos[s]][0] for s in ids]
        feats = [reid_features(frames[s][pos[s]][0], frames[s][pos[s]][1], 0.5) for s in ids]
        warps = np.stack([warp if (s + pos[s]) % 3 == 0 else np.eye(2, 3) for s in ids])
        outs = eng.update(dets, feats, warps=warps, streams=ids)
        for k, s in enumerate(ids):
            exp = solo[s].update([dets[k]], [feats[k]], warps=warps[k:k + 1])[0]
            assert np.array_equal(outs[k], exp), (step, s)
            pos[s] += 1
        for s in skipped:
            st, fe = before[s]
            assert _same_state(st, eng.state(s)), (step, s)
            assert np.array_equal(fe, eng.features(s)[0]), (step, s)


def test_subset_rejects_bad_stream_ids():
    eng = ByteTrackEngine(3, **KW)
    d = make_frames(20, 1, seed=1)[0][0]
    with pytest.raises(ValueError):
        eng.update([d, d], streams=[1, 1])
    with pytest.raises(ValueError):
        eng.update([d], streams=[3])
    with pytest.raises(_lib.YTAError):
        eng.reset_stream(5)


# ------------------------------------------------------------------ OCSORT family
OC_KW = dict(det_thresh=0.0, max_age=30, min_hits=1, asso_threshold=0.3, delta_t=3,
             asso_func="giou", inertia=0.2, use_byte=False)
DOC_KW = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2, w_association_emb=0.75, alpha_fixed_emb=0.95,
              aw_param=0.5, embedding_off=False, cmc_off=False, aw_off=False)
HS_KW = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
             asso_func="giou", inertia=0.2)


def _family(kind, S, D=32):
    if kind == "ocsort":
        from yolo_tracking_amd.trackers.ocsort import OCSortEngine
        return lambda n: OCSortEngine(n, **OC_KW)
    if kind == "deepocsort":
        from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine
        return lambda n: DeepOCSortEngine(n, feat_dim=D, **DOC_KW)
    from yolo_tracking_amd.trackers.hybridsort import HybridSortEngine
    return lambda n: HybridSortEngine(n, feat_dim=D, **HS_KW)


def _family_inputs(kind, frame):
    d, e = frame
    if kind == "ocsort":
        return d, None
    f = e if kind == "hybridsort" else e[d[:, 4] > 0.0]
    return d, f / np.linalg.norm(f)


def _family_call(kind, eng, dets, feats, warps, shapes, nid, streams=None):
    if kind == "ocsort":
        return eng.update(dets, shapes, next_id=nid, streams=streams)
    if kind == "deepocsort":
        return eng.update(dets, feats, warps=warps, img_shapes=shapes, next_id=nid,
                          streams=streams)
    return eng.update(dets, feats, next_id=nid, streams=streams)


@pytest.mark.parametrize("kind", ["ocsort", "deepocsort", "hybridsort"])
def test_ocsort_family_subset_and_reset(kind):
    """Random stream subsets (and one reset_stream) against one-stream engines fed each stream's
    own frames: rows and ID counters bit-identical, skipped streams' states untouched."""
    S, F, D = 3, 16, 32
    shape = (1400, 1400, 3)
    frames = [make_frames(100 + 20 * s, F, seed=900 + s, emb_dim=D, low_conf_frac=0.0,
                          drop_frac=0.05, canvas=1400.0) for s in range(S)]
    warp = np.array([[1.0, 1e-3, 0.5], [-1e-3, 1.0, -0.3]])
    make = _family(kind, S, D)
    eng = make(S)
    solo = [make(1) for _ in range(S)]
    nid_solo = [np.zeros(1, np.int64) + (1 if kind == "deepocsort" else 0) for _ in range(S)]
    nid = np.array([int(v[0]) for v in nid_solo])
    rng = np.random.default_rng(21)
    pos = [0] * S
    reset_done = False
    for step in range(3 * F):
        ids = [int(i) for i in rng.permutation(S)[:int(rng.integers(1, S + 1))] if pos[i] < F]
        if not ids:
            continue
        if not reset_done and min(pos) >= 6:   # stream 1 restarts as a fresh tracker
            eng.reset_stream(1)
            solo[1] = make(1)
            nid_solo[1][:] = 1 if kind == "deepocsort" else 0
            nid[1] = nid_solo[1][0]
            reset_done = True
        skipped = [s for s in range(S) if s not in ids]
        before = {s: eng.state(s) for s in skipped}
        ins = [_family_inputs(kind, frames[s][pos[s]]) for s in ids]
        dets = [x[0] for x in ins]
        feats = [x[1] for x in ins]
        warps = np.stack([warp if (s + pos[s]) % 2 else np.eye(2, 3) for s in ids])
        sub_nid = nid[ids].copy()
        outs = _family_call(kind, eng, dets, feats, warps, [shape] * len(ids), sub_nid, ids)
        nid[ids] = sub_nid
        for k, s in enumerate(ids):
            exp = _family_call(kind, solo[s], [dets[k]], [feats[k]], warps[k:k + 1], [shape],
                               nid_solo[s])[0]
            assert np.array_equal(outs[k], exp), (kind, step, s, pos[s])
            assert nid[s] == nid_solo[s][0], (kind, step, s)
            pos[s] += 1
        for s in skipped:
            after = eng.state(s)
            assert all(np.array_equal(before[s][k], after[k]) for k in after), (kind, step, s)
    assert reset_done and min(pos) > 8
