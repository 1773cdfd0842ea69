"""GPU: the SparseOptFlow estimator (csrc/cmc.hip through the C ABI) against its restatement
(oracle/cmc_sof.py).  Parity with cv2 itself is unpinned (cv2 is absent); the bar here is the
restatement's, stage by stage and end to end:
  * gray + resize, min-eigenvalue map, corner list (values, order): bit-exact;
  * Lucas-Kanade next points and status: bit-exact (exact integer window sums, float32 updates in
    the restated order, no FMA);
  * RANSAC + LM warp: bit-exact except where a libm log() could move the adaptive iteration count
    (never observed; the test would show it);
  * the engine over several camera streams, frame by frame: warps, stored corners, stored frame.
"""
import ctypes
import functools
import os

import numpy as np
import pytest

from cmc_frames import boxes, sequence
from oracle import cmc_sof as cs
from yolo_tracking_amd import _lib
from yolo_tracking_amd.motion.sof import SofEngine, SparseOptFlow

pytestmark = pytest.mark.gpu

FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "cmc_mot17.npz")


@pytest.fixture(scope="module")
def lib():
    return _lib.load_library()


def kat_pre(lib, frame, scale):
    h, w = frame.shape[:2]
    oh, ow = cs.small_size(h, w, scale)
    out = np.zeros(oh * ow, np.uint8)
    ph, pw = ctypes.c_int(), ctypes.c_int()
    _lib.check(lib.yta_sof_kat_preprocess(0, _lib.ptr(np.ascontiguousarray(frame)), h, w, scale,
                                          _lib.ptr(out), ctypes.byref(ph), ctypes.byref(pw)))
    assert (ph.value, pw.value) == (oh, ow)
    return out.reshape(oh, ow)


@pytest.mark.parametrize("h,w,scale", [(1080, 1920, 0.1), (480, 640, 0.1), (333, 517, 0.1),
                                       (200, 300, 0.25), (120, 160, 0.5), (57, 91, 1.0),
                                       (720, 1280, 0.15)])
def test_preprocess_bit_exact(lib, h, w, scale):
    rng = np.random.default_rng(h * 7 + w)
    frame = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    assert np.array_equal(kat_pre(lib, frame, scale), cs.preprocess(frame, scale))


@functools.lru_cache(maxsize=None)
def gray_cases():
    g = np.load(FIXTURE)
    out = [g["MOT17_13__small"][0], g["MOT17_04__small"][3], g["MOT17_05__small"][0]]
    out.append(cs.preprocess(sequence(300, 400, 1, 3)[0][0], 0.5))
    rng = np.random.default_rng(0)
    out.append(rng.integers(0, 256, (31, 47), dtype=np.uint8))
    out.append(np.full((40, 40), 9, np.uint8))
    return out


@pytest.mark.parametrize("k", range(6))
def test_min_eigen_and_corners_bit_exact(lib, k):
    g = np.ascontiguousarray(gray_cases()[k])
    h, w = g.shape
    eig = np.zeros((h, w), np.float32)
    _lib.check(lib.yta_sof_kat_min_eigen(0, _lib.ptr(g), h, w, _lib.ptr(eig)))
    exp = cs.min_eigen(g)
    assert np.array_equal(eig.view(np.uint32), exp.view(np.uint32))
    for mask in (cs.generate_mask(g, boxes(h * 10, w * 10, 5, k), 0.1),
                 np.full((h, w), 255, np.uint8), np.zeros((h, w), np.uint8)):
        mask = np.ascontiguousarray(mask)
        corners = np.zeros((3000, 2), np.float32)
        n = ctypes.c_int()
        _lib.check(lib.yta_sof_kat_corners(0, _lib.ptr(g), _lib.ptr(mask), h, w,
                                           _lib.ptr(corners), ctypes.byref(n)))
        ref = cs.good_features(g, mask)
        if ref is None:
            assert n.value == 0
        else:
            assert np.array_equal(corners[:n.value], ref)


@functools.lru_cache(maxsize=None)
def lk_cases():
    g = np.load(FIXTURE)
    cases = []
    for key in ("MOT17_13", "MOT17_04", "MOT17_05"):
        fr = g[f"{key}__small"]
        for a, b in ((0, 1), (1, 3), (0, len(fr) - 1)):
            cases.append((fr[a], fr[b]))
    frames, _ = sequence(1080, 1920, 3, 9, step=(0.3, 1.002, 9.0, 5.0))
    small = [cs.preprocess(f, 0.1) for f in frames]
    cases.append((small[0], small[2]))
    return cases


@pytest.mark.parametrize("k", range(10))
def test_lk_bit_exact(lib, k):
    prev, nxt = (np.ascontiguousarray(x) for x in lk_cases()[k])
    h, w = prev.shape
    pts = cs.good_features(prev, cs.generate_mask(prev, None, 0.1))
    # plus points near and beyond the borders (status 0 paths, border reads)
    extra = np.array([[0, 0], [w - 1, h - 1], [-15, 3], [w + 12, h / 2], [w / 2, -30],
                      [3.3, h - 2.7]], np.float32)
    pts = np.ascontiguousarray(np.concatenate([pts, extra]).astype(np.float32))
    n = len(pts)
    out = np.zeros((n, 2), np.float32)
    st = np.zeros(n, np.uint8)
    _lib.check(lib.yta_sof_kat_lk(0, _lib.ptr(prev), _lib.ptr(nxt), h, w, _lib.ptr(pts), n,
                                  _lib.ptr(out), _lib.ptr(st)))
    ref, rst = cs.lk_track(cs.build_pyramid(prev), cs.build_pyramid(nxt), pts)
    assert np.array_equal(st, rst)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


@functools.lru_cache(maxsize=None)
def affine_cases():
    out = []
    for prev, nxt in lk_cases():
        pts = cs.good_features(prev, cs.generate_mask(prev, None, 0.1))
        q, st = cs.lk_track(cs.build_pyramid(prev), cs.build_pyramid(nxt), pts)
        out.append((pts[st == 1], q[st == 1]))
    rng = np.random.default_rng(5)
    f = rng.uniform(0, 190, (400, 2)).astype(np.float32)
    M = np.array([[0.99, -0.03, 4.0], [0.03, 0.99, -2.0]])
    t = (f @ M[:, :2].T + M[:, 2] + rng.normal(0, 0.3, (400, 2))).astype(np.float32)
    t[::3] = rng.uniform(0, 190, (134, 2)).astype(np.float32)       # a third are outliers
    out.append((f, t))
    out.append((f[:2], t[:2]))                                        # count == 2
    out.append((f[:3], t[:3]))
    out.append((f[:1], t[:1]))                                        # no model
    dup = np.repeat(f[:1], 5, axis=0)
    out.append((dup, dup + 1))                                        # degenerate subsets
    return out


@pytest.mark.parametrize("k", range(15))
def test_affine_ransac_lm(lib, k):
    f, t = (np.ascontiguousarray(x, dtype=np.float32) for x in affine_cases()[k])
    n = len(f)
    M = np.zeros(6)
    ok = ctypes.c_int()
    _lib.check(lib.yta_sof_kat_affine(0, _lib.ptr(f), _lib.ptr(t), n, _lib.ptr(M),
                                      ctypes.byref(ok)))
    ref = cs.estimate_affine_partial(f, t)
    if ref is None:
        assert ok.value == 0
        return
    assert ok.value == 1
    assert np.array_equal(M.reshape(2, 3), ref), (M.reshape(2, 3) - ref)


def test_engine_streams_match_oracle():
    """Four camera streams in one engine (different sizes, motions, dets), 7 frames each."""
    specs = [(1080, 1920, (0.2, 1.0, 6.0, -4.0)), (480, 640, (0.0, 1.0, -3.0, 2.0)),
             (720, 1280, (-0.3, 1.003, 2.0, 7.0)), (1080, 1920, (0.0, 1.0, 0.0, 0.0))]
    seqs = [sequence(h, w, 7, 20 + i, step=st)[0] for i, (h, w, st) in enumerate(specs)]
    dets = [boxes(h, w, 8 + 3 * i, i) for i, (h, w, _) in enumerate(specs)]
    eng = SofEngine(len(specs), 0.1, 0, 1080, 1920)
    ors = [cs.SparseOptFlowOracle(0.1) for _ in specs]
    for f in range(7):
        got = eng.apply([seqs[i][f] for i in range(len(specs))], dets)
        oc = eng.outcome()
        for i, o in enumerate(ors):
            exp = o.apply(seqs[i][f], dets[i])
            assert np.array_equal(got[i], exp), (i, f, got[i] - exp)
            st = eng.state(i, with_image=True)
            assert st["initialized"]
            assert np.array_equal(st["keypoints"], o.prev_keypoints)
            assert np.array_equal(st["prev_img"], o.prev_img)
            assert oc[i] == (0 if f == 0 else 1)


def _kp(o):
    return np.zeros((0, 2), np.float32) if o.prev_keypoints is None else o.prev_keypoints


def test_engine_first_frame_without_corners_and_point_loss():
    """A flat first frame finds no corners (no state kept, the next frame detects again); a
    stream whose corners all leave the frame ends with identity warps and an empty corner set."""
    flat = np.full((240, 320, 3), 100, np.uint8)
    frames, _ = sequence(240, 320, 3, 31)
    eng = SofEngine(1, 0.25, 0, 240, 320)
    o = cs.SparseOptFlowOracle(0.25)
    for fr in [flat, frames[0], frames[1]]:
        got = eng.apply([fr], [np.zeros((0, 4))])[0]
        assert np.array_equal(got, o.apply(fr, None))
        assert np.array_equal(eng.state(0)["keypoints"], _kp(o))
    # a frame of noise: LK loses most points; then flat frames: every point fails
    rng = np.random.default_rng(1)
    for fr in [rng.integers(0, 256, (240, 320, 3), dtype=np.uint8), flat, flat]:
        got = eng.apply([fr], [np.zeros((0, 4))])[0]
        assert np.array_equal(got, o.apply(fr, None))
        assert np.array_equal(eng.state(0)["keypoints"], _kp(o))


def test_engine_resolution_switch_mid_sequence():
    """A stream whose frame size changes after the first frame: calcOpticalFlowPyrLK asserts on
    the level sizes and sof.py:105-110 returns the identity with the stored frame and corners
    kept -- for a smaller frame, a larger one that fits the buffers, and one larger than the
    engine was built for (the host path grows the buffers keeping the state).  Frames of the
    stored size then track again."""
    big, _ = sequence(480, 640, 6, 52, step=(0.1, 1.0, 2.0, -1.0))
    small, _ = sequence(240, 320, 2, 53)
    huge, _ = sequence(600, 800, 1, 54)
    seq = [big[0], big[1], small[0], big[2], huge[0], small[1], big[3], big[4], big[5]]
    eng = SofEngine(1, 0.1, 0, 480, 640)
    o = cs.SparseOptFlowOracle(0.1)
    for f, fr in enumerate(seq):
        got = eng.apply([fr], [np.zeros((0, 4))])[0]
        exp = o.apply(fr, None)
        assert np.array_equal(got, exp), (f, got - exp)
        st = eng.state(0, with_image=True)
        assert np.array_equal(st["keypoints"], _kp(o)), f
        assert np.array_equal(st["prev_img"], o.prev_img), f
    assert not np.array_equal(got, np.eye(2, 3))


def test_dropin_sparse_opt_flow_matches_oracle():
    frames, _ = sequence(720, 1280, 4, 44)
    dets = boxes(720, 1280, 10, 4)
    a = SparseOptFlow()
    o = cs.SparseOptFlowOracle()
    for fr in frames:
        H = a.apply(fr, np.hstack([dets, np.ones((len(dets), 3))]))   # 7-column dets_first rows
        assert H.shape == (2, 3) and H.dtype == np.float64
        assert np.array_equal(H, o.apply(fr, dets))


def _moving_camera_case(n_frames=10, n=48, seed=61):
    """Detections from the synthetic stream generator, frames from a moving textured scene."""
    from yolo_tracking_amd.synth import make_frames
    fr = make_frames(n, n_frames, seed, emb_dim=16, low_conf_frac=0.1)
    C = int(64 * np.sqrt(n))
    imgs, _ = sequence(C + 64, C + 64, n_frames, seed, step=(0.1, 1.0, 3.0, -2.0))
    return fr, imgs


def test_botsort_default_cmc_end_to_end():
    """BoTSORT() with no cmc= runs the GPU SparseOptFlow (bot_sort.py:228, :293) on every frame;
    against the oracle tracker fed the restated estimator's warps: ids / scores / det_ind
    bit-exact, boxes to 1e-9 relative (the warped covariance's cross terms)."""
    from oracle.botsort import BoTSORTOracle
    from yolo_tracking_amd.trackers.botsort import BoTSORT
    frames, imgs = _moving_camera_case()
    params = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
                  track_buffer=30, match_thresh=0.8, proximity_thresh=0.5,
                  appearance_thresh=0.25, frame_rate=30)
    t = BoTSORT(None, 0, False, with_reid=False, **params)
    assert isinstance(t.cmc, SparseOptFlow)
    ref = BoTSORTOracle(with_reid=False, **params)
    sof = cs.SparseOptFlowOracle()
    moved = 0
    for f, ((dets, _), img) in enumerate(zip(frames, imgs)):
        got = np.asarray(t.update(dets, img)).reshape(-1, 8)
        warp = sof.apply(img, dets[dets[:, 4] > params["track_high_thresh"]])
        moved += not np.array_equal(warp, np.eye(2, 3))
        exp = ref.update(dets, None, warp).reshape(-1, 8)
        assert got.shape == exp.shape, f
        assert np.array_equal(got[:, 4:], exp[:, 4:]), f
        np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-9, atol=1e-6)
    assert moved >= len(frames) - 1


def test_deepocsort_default_cmc_end_to_end():
    """DeepOCSort() with no cmc= (deep_ocsort.py:351, :391) against the oracle fed the restated
    estimator's warps (on the kept detections' boxes): ids / scores / det_ind bit-exact, boxes to
    1e-9 relative (the warped 2x2 blocks meet LAPACK's LU in the reference)."""
    from oracle.deepocsort import DeepOCSortOracle
    from yolo_tracking_amd.trackers.deepocsort import DeepOCSort
    frames, imgs = _moving_camera_case(seed=62)
    kw = dict(det_thresh=0.3, max_age=30, min_hits=1, iou_threshold=0.3, delta_t=3,
              asso_func="giou", inertia=0.2)
    t = DeepOCSort(None, 0, False, embedding_off=True, **kw)
    assert isinstance(t.cmc, SparseOptFlow)
    ref = DeepOCSortOracle(embedding_off=True, **kw)
    sof = cs.SparseOptFlowOracle()
    for f, ((dets, _), img) in enumerate(zip(frames, imgs)):
        got = np.asarray(t.update(dets, img)).reshape(-1, 8)
        warp = sof.apply(img, dets[dets[:, 4] > kw["det_thresh"], :4])
        exp = np.asarray(ref.update(dets, img.shape, None, warp), dtype=np.float64).reshape(-1, 8)
        assert got.shape == exp.shape, f
        assert np.array_equal(got[:, 4:], exp[:, 4:]), f
        np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-9, atol=1e-6)
