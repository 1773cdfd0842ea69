"""GPU: the device-resident BoT-SORT engine against the reference goldens (G4) and the oracle.

Bar: output rows (ids, boxes, scores, classes, det_ind), track lists and Kalman states bit-exact
on the identity-warp cases (with camera warps: ids / order / scores bit-exact, boxes and states to
1e-9 relative); smoothed features within float32 rounding (the engine sums squares in
float64 where the reference's OpenBLAS sdot sums in float32 lanes: rtol 1e-5, atol 1e-6).
"""
import os

import numpy as np
import pytest

from oracle.botsort import BoTSORTOracle
from test_oracle_golden import botsort_case, reid_features
from yolo_tracking_amd import _lib, create_tracker, get_tracker_config
from yolo_tracking_amd.synth import make_frames
from yolo_tracking_amd.trackers.botsort import BaseTrack, BoTSORT, BoTSORTEngine

pytestmark = pytest.mark.gpu

IDENTITY_CASES = ["bs_n64_d32", "bs_n256_d64", "bs_n128_fuse", "bs_n128_noreid", "bs_n512_d128"]


def _engine(params, D, **kw):
    return BoTSORTEngine(1, feat_dim=max(D, 1), **params, **kw)


def _check_state(eng, g, name, D):
    st = eng.state(0)
    assert np.array_equal(st["list"], g[f"{name}__st_list"])
    assert np.array_equal(st["id"], g[f"{name}__st_id"])
    assert np.array_equal(st["state"], g[f"{name}__st_state"])
    assert np.array_equal(st["activated"], g[f"{name}__st_act"])
    assert np.array_equal(st["frame_id"], g[f"{name}__st_frame"])
    assert np.array_equal(st["start_frame"], g[f"{name}__st_start"])
    assert np.array_equal(st["tracklet_len"], g[f"{name}__st_len"])
    assert np.array_equal(st["mean"], g[f"{name}__st_mean"])
    assert np.array_equal(st["cov"], g[f"{name}__st_cov"])
    if D:
        feats, _, _ = eng.features(0)
        np.testing.assert_allclose(feats, g[f"{name}__st_feat"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", IDENTITY_CASES)
@pytest.mark.parametrize("lds", [None, 0])
def test_botsort_golden(golden_dir, name, lds):
    g = np.load(os.path.join(golden_dir, "botsort_synth.npz"))
    frames, params, warp, D = botsort_case(g, name)
    eng = _engine(params, D)
    if lds is not None:
        eng.set_lds(lds)               # every association over the global-memory arena
    oc, out = g[f"{name}__out_counts"], g[f"{name}__out"]
    r0 = 0
    for f, (dets, embs) in enumerate(frames):
        feats = reid_features(dets, embs, params["track_high_thresh"]) if D else None
        got = eng.update([dets], [feats])[0]
        exp = out[r0:r0 + oc[f]]
        assert got.shape == exp.shape, (name, f, got.shape, exp.shape)
        assert np.array_equal(got, exp), (name, f)
        r0 += oc[f]
    _check_state(eng, g, name, D)


def _close_rows(got, exp, ctx):
    assert got.shape == exp.shape, ctx
    assert np.array_equal(got[:, 4:], exp[:, 4:]), ctx               # ids, scores, cls, det_ind
    np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-9, atol=1e-6, err_msg=str(ctx))


@pytest.mark.parametrize("lds", [None, 0])
def test_botsort_cmc_golden(golden_dir, lds):
    """Camera-motion warps (multi_gmc, bot_sort.py:95-111, 290-295) against the reference: the
    warped covariance couples x with y, so these tracks carry cross terms (kf_xyah.hpp); ids,
    order, scores and det_ind bit-exact, boxes and Kalman states to 1e-9 relative (the dense
    group products sum in a different order than OpenBLAS)."""
    g = np.load(os.path.join(golden_dir, "botsort_synth.npz"))
    name = "bs_n256_d64_cmc"
    frames, params, warp, D = botsort_case(g, name)
    assert not np.allclose(np.asarray(warp), np.eye(2, 3))
    eng = _engine(params, D)
    if lds is not None:
        eng.set_lds(lds)
    oc, out = g[f"{name}__out_counts"], g[f"{name}__out"]
    r0 = 0
    for f, (dets, embs) in enumerate(frames):
        feats = reid_features(dets, embs, params["track_high_thresh"])
        got = eng.update([dets], [feats], warps=np.asarray(warp)[None])[0]
        _close_rows(got, out[r0:r0 + oc[f]], (name, f))
        r0 += oc[f]
    st = eng.state(0)
    for k, gk in (("list", "st_list"), ("id", "st_id"), ("state", "st_state"),
                  ("activated", "st_act"), ("frame_id", "st_frame"), ("start_frame", "st_start"),
                  ("tracklet_len", "st_len")):
        assert np.array_equal(st[k], g[f"{name}__{gk}"]), k
    np.testing.assert_allclose(st["mean"], g[f"{name}__st_mean"], rtol=1e-9, atol=1e-9)
    cov = g[f"{name}__st_cov"]
    assert np.count_nonzero(cov[:, 0, 1]) > 0                          # cross terms present
    np.testing.assert_allclose(st["cov"], cov, rtol=1e-8, atol=1e-12 * np.abs(cov).max())
    feats, _, _ = eng.features(0)
    np.testing.assert_allclose(feats, g[f"{name}__st_feat"], rtol=1e-5, atol=1e-6)


def test_botsort_cmc_multistream_vs_oracle():
    """Per-stream warps changing every frame (identity on some streams and frames) against the
    oracle stream by stream."""
    S, n, nf, D = 3, 96, 14, 32
    params = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
                  track_buffer=30, match_thresh=0.8, proximity_thresh=0.5,
                  appearance_thresh=0.25, frame_rate=30)
    rng = np.random.default_rng(9)
    streams = [make_frames(n, nf, 300 + s, emb_dim=D) for s in range(S)]
    eng = BoTSORTEngine(S, feat_dim=D, **params)
    ors = [BoTSORTOracle(**params) for _ in range(S)]
    for f in range(nf):
        warps = np.tile(np.eye(2, 3), (S, 1, 1))
        for s in range(S):
            if (s + f) % 3:
                a = rng.normal(0, 2e-3)
                warps[s] = [[np.cos(a), -np.sin(a), rng.normal(0, 2)],
                            [np.sin(a), np.cos(a), rng.normal(0, 2)]]
        dets = [streams[s][f][0] for s in range(S)]
        feats = [reid_features(dets[s], streams[s][f][1], 0.5) for s in range(S)]
        got = eng.update(dets, feats, warps=warps)
        for s in range(S):
            exp = ors[s].update(dets[s], feats[s], warp=warps[s]).reshape(-1, 8)
            _close_rows(got[s], exp, (s, f))


def test_botsort_python_surface(golden_dir):
    """create_tracker('botsort') + update(dets, img, embs): the reference's call shape."""
    g = np.load(os.path.join(golden_dir, "botsort_synth.npz"))
    name = "bs_n64_d32"
    frames, params, warp, D = botsort_case(g, name)
    t = BoTSORT(None, "cuda:0", False, **params)
    oc, out = g[f"{name}__out_counts"], g[f"{name}__out"]
    img = np.zeros((8, 8, 3), np.uint8)
    r0 = 0
    for f, (dets, embs) in enumerate(frames):
        hi = dets[:, 4] > params["track_high_thresh"]
        e = np.zeros((len(dets), D), np.float32)
        e[hi] = reid_features(dets, embs, params["track_high_thresh"])
        got = np.asarray(t.update(dets, img, embs=e)).reshape(-1, 8)
        assert np.array_equal(got, out[r0:r0 + oc[f]]), f
        r0 += oc[f]
    assert [v.track_id for v in t.tracked_stracks + t.lost_stracks] == list(g[f"{name}__st_id"])
    # create_tracker wires the YAML keys and a ReID producer passed as reid_weights
    class Reid:
        def get_features(self, xyxys, img):
            return np.ones((len(xyxys), 16), np.float32)
    tz = create_tracker("botsort", get_tracker_config("botsort"), Reid(), "0", False, False)
    r = tz.update(frames[0][0], img)
    assert r.ndim == 2 and r.shape[1] == 8
    assert BaseTrack._count == len(r)


def test_botsort_multistream_matches_oracle():
    """S streams in one engine, each its own seed, against the oracle stream by stream."""
    S, n, nf, D = 4, 64, 12, 32
    params = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
                  track_buffer=30, match_thresh=0.8, proximity_thresh=0.5,
                  appearance_thresh=0.25, frame_rate=30)
    streams = [make_frames(n, nf, 100 + s, emb_dim=D) for s in range(S)]
    eng = BoTSORTEngine(S, feat_dim=D, **params)
    ors = [BoTSORTOracle(**params) for _ in range(S)]
    for f in range(nf):
        dets = [streams[s][f][0] for s in range(S)]
        feats = [reid_features(dets[s], streams[s][f][1], 0.5) for s in range(S)]
        got = eng.update(dets, feats)
        for s in range(S):
            exp = ors[s].update(dets[s], feats[s]).reshape(-1, 8)
            assert np.array_equal(got[s], exp), (s, f)


@pytest.mark.parametrize("crowd", [False, True])
def test_split_stage1_equals_fused(monkeypatch, crowd):
    """Stage 1 with ReID as three launches (k_bs_prep / k_bs_edges chip-wide / k_bs_lap, the
    default for few streams) against the fused k_stage1 (YTA_BS_SPLIT=0): identical rows, states
    features and frame counters every frame.  crowd: objects packed 8x denser than the generator's default, so
    pool rows with more than E_SLOTS candidate edges send k_bs_lap down the fused association."""
    from test_oracle_golden import reid_features
    from yolo_tracking_amd.synth import make_frames
    from yolo_tracking_amd.trackers.botsort import BoTSORTEngine
    n, D = 400, 64
    canvas = 64.0 * np.sqrt(n) / (8.0 if crowd else 1.0)
    frames = make_frames(n, 12, seed=77 if crowd else 78, emb_dim=D, canvas=canvas)
    P = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
             track_buffer=30, match_thresh=0.8, proximity_thresh=0.5, appearance_thresh=0.25,
             frame_rate=30)
    engs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("YTA_BS_SPLIT", mode)
        engs[mode] = BoTSORTEngine(1, feat_dim=D, **P)
    for f, (dets, embs) in enumerate(frames):
        feats = reid_features(dets, embs, P["track_high_thresh"])
        a = engs["1"].update([dets], [feats])[0]
        b = engs["0"].update([dets], [feats])[0]
        assert np.array_equal(a, b), f
        # the frame's counters mean the same in both paths (the LDS-fallback counts aside: the
        # two association bodies size their arenas differently)
        sta, stb = engs["1"].stats(), engs["0"].stats()
        sta.pop("fallback1"), stb.pop("fallback1")
        assert sta == stb, (f, sta, stb)
    sa, sb = engs["1"].state(0), engs["0"].state(0)
    assert all(np.array_equal(sa[k], sb[k]) for k in sa)
    assert np.array_equal(engs["1"].features(0)[0], engs["0"].features(0)[0])
