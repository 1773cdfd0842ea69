"""GPU: the device-resident DeepOCSORT engine against the reference goldens (G6) and the oracle.

Bar: outputs (ids, order, boxes, conf, cls, det_ind) bit-exact against the reference goldens and
the oracle frame by frame.  Kalman state to 1e-10 relative on static-camera streams: the reference
squares NumPy float64 scalars (`(p * w) ** 2`, deep_ocsort.py:76-87), i.e. libm pow, which misses
the correctly rounded square in ~0.1% of calls, where the device squares exactly (x * x); every
other Kalman operation is the reference's, operation for operation.  Under a camera warp the 2x2
blocks of S meet LAPACK's LU and OpenBLAS's products, so x / P agree to 1e-9 relative.
Tracker embeddings agree to 1e-12 (the reference's norm is a BLAS dot product, summed in another
order).  The stage-1 embedding cost is accumulated in float64 where the reference multiplies in
float32 while every tracker embedding is still float32: a ~1e-7 cost difference, below the 1e-6
perturbation the goldens were checked to be insensitive to (make_goldens.py G6).
"""
import os

import numpy as np
import pytest

from oracle.deepocsort import DeepOCSortOracle, Tracker8
from test_oracle_golden import DEEPOCSORT_CASES, deepocsort_case, golden_outputs
from yolo_tracking_amd import _lib, create_tracker, get_tracker_config
from yolo_tracking_amd.synth import make_frames
from yolo_tracking_amd.trackers.deepocsort import DeepOCSortEngine, KalmanBoxTracker

pytestmark = pytest.mark.gpu

KF_RTOL = 1e-9        # camera warp
KF_RTOL_STATIC = 1e-10
EMB_ATOL = 1e-12


def _kat_boxes(rng, n, steps):
    walk = np.cumsum(rng.normal(0, 3, size=(steps + 1, n, 4)), axis=0)
    base = np.column_stack([rng.uniform(50, 900, n), rng.uniform(50, 900, n),
                            rng.uniform(60, 120, n), rng.uniform(60, 120, n)])
    xyxy = np.empty_like(walk)
    for s in range(steps + 1):
        c = base[:, :2] + walk[s, :, :2]
        wh = np.abs(base[:, 2:] + walk[s, :, 2:]) + 5
        xyxy[s] = np.column_stack([c - wh / 2, c + wh / 2])
    return xyxy


def _kat_oracle(xyxy, miss, warps):
    steps, n = miss.shape
    xs, Ps = [], []
    for i in range(n):
        t = Tracker8(np.r_[xyxy[0, i], 0.9, 0.0, 0.0], 1, 3, None)
        for s in range(steps):
            if warps is not None:
                t.affine(warps[s, i])
            t.predict()
            t.update(None if miss[s, i] else np.r_[xyxy[s + 1, i], 0.9, 0.0, 0.0])
        xs.append(t.kf.x.ravel())
        Ps.append(t.kf.P)
    return np.array(xs), np.array(Ps)


@pytest.mark.parametrize("with_warp", [False, True])
def test_kf8_sequences_match_oracle(with_warp):
    rng = np.random.default_rng(5)
    n, steps = 200, 30
    xyxy = _kat_boxes(rng, n, steps)
    miss = rng.random((steps, n)) < 0.3
    miss[:, ::7] = False
    b = xyxy[1:].copy()
    b[miss] = np.nan
    warps = None
    if with_warp:
        ang = rng.normal(0, 0.01, (steps, n))
        sc = 1 + rng.normal(0, 0.01, (steps, n))
        warps = np.empty((steps, n, 2, 3))
        warps[..., 0, 0] = sc * np.cos(ang)
        warps[..., 0, 1] = -sc * np.sin(ang)
        warps[..., 1, 0] = sc * np.sin(ang)
        warps[..., 1, 1] = sc * np.cos(ang)
        warps[..., :, 2] = rng.normal(0, 2, (steps, n, 2))
    x, P = _lib.kf8_run(xyxy[0], b, warps)
    ex, eP = _kat_oracle(xyxy, miss, warps)
    if with_warp:
        np.testing.assert_allclose(x, ex, rtol=KF_RTOL, atol=1e-9)
        np.testing.assert_allclose(P, eP, rtol=KF_RTOL, atol=1e-9)
    else:
        np.testing.assert_allclose(x, ex, rtol=KF_RTOL_STATIC, atol=1e-10)
        np.testing.assert_allclose(P, eP, rtol=KF_RTOL_STATIC, atol=1e-10)


@pytest.mark.parametrize("name", DEEPOCSORT_CASES)
def test_deepocsort_golden(golden_dir, name):
    g = np.load(os.path.join(golden_dir, "deepocsort_synth.npz"))
    frames, img_shape, kw, warp, D = deepocsort_case(g, name)
    eng = DeepOCSortEngine(1, feat_dim=max(D, 1), **kw)
    o = DeepOCSortOracle(**kw)
    exp = golden_outputs(g, name)
    got = []
    for f, (d, feats) in enumerate(frames):
        out = eng.update([d], [feats], warps=None if warp is None else warp[None],
                         img_shapes=[img_shape])[0]
        ref = np.asarray(o.update(d, img_shape, feats, warp), dtype=np.float64).reshape(-1, 8)
        assert np.array_equal(out, ref), (name, f)
        got.append(out)
    assert all(np.array_equal(a, b) for a, b in zip(got, exp))
    st = eng.state(0)
    assert np.array_equal(st["id"], g[f"{name}__st_id"])
    gx, gP = g[f"{name}__st_x"], g[f"{name}__st_P"]
    tol = KF_RTOL_STATIC if warp is None else KF_RTOL
    np.testing.assert_allclose(st["x"], gx, rtol=tol, atol=tol)
    np.testing.assert_allclose(st["P"], gP, rtol=tol, atol=tol)
    if D and not kw["embedding_off"]:
        np.testing.assert_allclose(st["emb"], g[f"{name}__st_emb"], rtol=0, atol=EMB_ATOL)
    s = eng.stats()
    assert s["trackers"] == len(o.trackers)


def test_deepocsort_python_surface(golden_dir):
    g = np.load(os.path.join(golden_dir, "deepocsort_synth.npz"))
    name = "dos_n64_d32"
    frames, img_shape, kw, warp, D = deepocsort_case(g, name)
    assert warp is None
    img = np.zeros((img_shape[0], img_shape[1], 3), np.uint8)

    class Reid:     # replays the golden features for the rows the tracker asks about
        def __init__(self):
            self.f = 0

        def get_features(self, xyxys, im):
            out = frames[self.f][1]
            assert len(out) == len(xyxys)
            self.f += 1
            return out

    from yolo_tracking_amd.trackers.deepocsort import DeepOCSort
    reid = Reid()
    t = DeepOCSort(None, 0, False, reid=reid, **kw)
    assert KalmanBoxTracker.count == 1
    exp = golden_outputs(g, name)
    for f, (d, _) in enumerate(frames):
        got = np.asarray(t.update(d, img)).reshape(-1, 8)
        assert np.array_equal(got, exp[f]), f
    # create_tracker reads deepocsort.yaml (giou, det_thresh 0, min_hits 1)
    class RandomReid:
        def get_features(self, xyxys, im):
            f = np.random.default_rng(len(xyxys)).normal(size=(len(xyxys), 16))
            return (f / np.linalg.norm(f, axis=1, keepdims=True)).astype(np.float32)

    tz = create_tracker("deepocsort", get_tracker_config("deepocsort"), RandomReid(), "0", False,
                        False)
    assert KalmanBoxTracker.count == 1
    d0 = frames[0][0]
    assert (d0[:, 4] > 0).all()
    r = tz.update(d0, img)
    assert r.shape == (len(d0), 8)   # frame_count <= min_hits: frame 1's births reported
    assert KalmanBoxTracker.count == 1 + len(d0)
    assert np.array_equal(np.sort(r[:, 4]), np.arange(1, len(d0) + 1))
    r = tz.update(np.empty((0, 6)), img)
    assert r.shape == (0,)
    with pytest.raises(RuntimeError):
        DeepOCSort(None, 0, False).update(d0, img)   # embeddings on, no producer


def test_deepocsort_multistream_matches_oracle():
    S, n, nf, D = 4, 96, 15, 32
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2)
    raw = [make_frames(n, nf, 300 + s, emb_dim=D, low_conf_frac=0.0, drop_frac=0.1)
           for s in range(S)]
    streams = [[(d, (e / np.linalg.norm(e, axis=1, keepdims=True)).astype(np.float32))
                for d, e in r] for r in raw]
    eng = DeepOCSortEngine(S, feat_dim=D, **kw, track_capacity=64, max_dets=32)   # grows
    ors = [DeepOCSortOracle(**kw) for _ in range(S)]
    shape = (640, 640, 3)
    for f in range(nf):
        got = eng.update([streams[s][f][0] for s in range(S)],
                         [streams[s][f][1] for s in range(S)], img_shapes=[shape] * S)
        for s in range(S):
            d, e = streams[s][f]
            exp = np.asarray(ors[s].update(d, shape, e), dtype=np.float64).reshape(-1, 8)
            assert np.array_equal(got[s], exp), (s, f)


def _crowd(frames, grow):
    """Boxes scaled about their centres: with grow 4 a detection overlaps dozens of trackers."""
    out = []
    for d, e in frames:
        d = d.copy()
        c = (d[:, :2] + d[:, 2:4]) / 2
        h = (d[:, 2:4] - d[:, :2]) / 2 * grow
        d[:, :2], d[:, 2:4] = c - h, c + h
        out.append((d, e))
    return out


def test_deepocsort_dense_embedding_fallback_matches_oracle():
    """A stream whose detections overlap more than 16 trackers each takes the dense embedding
    tiles and AW scans (k_doc_emb, k_doc_aw); the other stream of the same engine the listed
    pairs (k_doc_emb_pairs).  Both against the oracle frame by frame."""
    S, n, nf, D = 2, 96, 12, 32
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2)
    raw = [make_frames(n, nf, 700 + s, emb_dim=D, low_conf_frac=0.0, drop_frac=0.1)
           for s in range(S)]
    streams = [[(d, (e / np.linalg.norm(e, axis=1, keepdims=True)).astype(np.float32))
                for d, e in r] for r in raw]
    streams[0] = _crowd(streams[0], 4.0)
    d0 = streams[0][1][0]
    ov = ((d0[:, None, 0] < d0[None, :, 2]) & (d0[None, :, 0] < d0[:, None, 2]) &
          (d0[:, None, 1] < d0[None, :, 3]) & (d0[None, :, 1] < d0[:, None, 3])).sum(1)
    assert ov.max() > 16   # the crowded stream does list more than POS_K pairs in some row
    eng = DeepOCSortEngine(S, feat_dim=D, **kw, track_capacity=256, max_dets=128)
    ors = [DeepOCSortOracle(**kw) for _ in range(S)]
    shape = (640, 640, 3)
    for f in range(nf):
        got = eng.update([streams[s][f][0] for s in range(S)],
                         [streams[s][f][1] for s in range(S)], img_shapes=[shape] * S)
        for s in range(S):
            d, e = streams[s][f]
            exp = np.asarray(ors[s].update(d, shape, e), dtype=np.float64).reshape(-1, 8)
            assert np.array_equal(got[s], exp), (s, f)


def test_deepocsort_dense_and_listed_paths_agree(monkeypatch):
    """The same frames through an engine forced onto the dense embedding tiles and AW scans for
    every frame (YTA_DOC_DENSE=1: k_doc_emb's f64 MFMA tiles, k_doc_aw) and through the default
    engine, where only the crowded stream takes them (the other lists its pairs: k_doc_emb_pairs,
    k_doc_aw_cols).  The two sum each dot product in a different order (MFMA tiles vs 16-lane
    groups), so an embedding cost may differ in its last bits (<= 1e-15 relative); that can only
    matter on an exact tie or a threshold hit exactly.  Bar: rows, ID counters and every tracker's
    state (ids, counters, x, P, embedding) bit-identical between the two engines on these streams,
    and the oracle agrees with both."""
    S, n, nf, D = 2, 96, 12, 32
    kw = dict(det_thresh=0.0, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2)
    raw = [make_frames(n, nf, 740 + s, emb_dim=D, low_conf_frac=0.0, drop_frac=0.1)
           for s in range(S)]
    streams = [[(d, (e / np.linalg.norm(e, axis=1, keepdims=True)).astype(np.float32))
                for d, e in r] for r in raw]
    streams[0] = _crowd(streams[0], 4.0)
    monkeypatch.setenv("YTA_DOC_DENSE", "1")
    dense = DeepOCSortEngine(S, feat_dim=D, **kw, track_capacity=256, max_dets=128)
    monkeypatch.delenv("YTA_DOC_DENSE")
    listed = DeepOCSortEngine(S, feat_dim=D, **kw, track_capacity=256, max_dets=128)
    ors = [DeepOCSortOracle(**kw) for _ in range(S)]
    shape = (640, 640, 3)
    for f in range(nf):
        args = ([streams[s][f][0] for s in range(S)], [streams[s][f][1] for s in range(S)])
        gd = dense.update(*args, img_shapes=[shape] * S)   # the engines' own ID counters (from 1)
        gl = listed.update(*args, img_shapes=[shape] * S)
        for s in range(S):
            assert np.array_equal(gd[s].view(np.int64), gl[s].view(np.int64)), (s, f)
            d, e = streams[s][f]
            exp = np.asarray(ors[s].update(d, shape, e), dtype=np.float64).reshape(-1, 8)
            assert np.array_equal(gl[s], exp), (s, f)
    for s in range(S):
        a, b = dense.state(s), listed.state(s)
        for k in a:
            if a[k] is not None:
                assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), (s, k)
