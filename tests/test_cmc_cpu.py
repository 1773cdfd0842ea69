"""CPU: the SparseOptFlow restatement (oracle/cmc_sof.py) on its own terms.  cv2 is absent, so
parity with OpenCV itself is unpinned; these tests pin the restatement's building blocks and its
end-to-end behaviour: exact 2-point similarity, the cv::RNG stream, reflect-101 borders, the
gray / resize fixed point, pyramid sizes, and recovery of known camera motions (synthetic frames
and the MOT17-mini fixture frames)."""
import os

import numpy as np
import pytest

from cmc_frames import boxes, sequence
from oracle import cmc_sof as cs


def test_similarity_2pt_maps_both_points():
    rng = np.random.default_rng(1)
    for _ in range(20):
        f = rng.uniform(0, 200, (2, 2)).astype(np.float32)
        t = rng.uniform(0, 200, (2, 2)).astype(np.float32)
        M = cs.similarity_2pt(f, t)
        assert M[0, 0] == M[1, 1] and M[0, 1] == -M[1, 0]
        got = f.astype(np.float64) @ M[:, :2].T + M[:, 2]
        np.testing.assert_allclose(got, t, atol=1e-9)


def test_cv_rng_stream():
    # multiply-with-carry, seed (uint64)-1: state' = (state & 0xffffffff) * 4164903690 + (state >> 32)
    r = cs.CvRNG()
    s = 0xFFFFFFFFFFFFFFFF
    for _ in range(100):
        s = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & 0xFFFFFFFFFFFFFFFF
        assert r.next() == s & 0xFFFFFFFF
    sub = cs.ransac_subsets(7, 500)
    assert np.all(sub[:, 0] != sub[:, 1]) and sub.min() >= 0 and sub.max() < 7
    assert np.array_equal(sub, cs.ransac_subsets(7, 500))


def test_refl101_and_pyramid_levels():
    assert cs.refl101(np.array([-2, -1, 0, 4, 5, 6]), 5).tolist() == [2, 1, 0, 4, 3, 2]
    assert cs.refl101(np.array([-3, 3]), 1).tolist() == [0, 0]
    assert [l.shape for l in cs.build_pyramid(np.zeros((108, 192), np.uint8))] == \
        [(108, 192), (54, 96), (27, 48)]
    assert [l.shape for l in cs.build_pyramid(np.zeros((48, 64), np.uint8))] == \
        [(48, 64), (24, 32)]
    assert [l.shape for l in cs.build_pyramid(np.zeros((42, 60), np.uint8))] == [(42, 60)]


def test_gray_and_resize_fixed_point():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    g = cs.bgr2gray(img)
    ref = np.rint(img[..., 0] * 0.114 + img[..., 1] * 0.587 + img[..., 2] * 0.299)
    assert np.abs(g.astype(int) - ref).max() <= 1
    # a constant frame stays constant through gray + resize at every scale
    c = np.full((108, 192, 3), 77, np.uint8)
    for sc in (0.1, 0.25, 0.5, 1.0):
        small = cs.preprocess(c, sc)
        assert small.shape == cs.small_size(108, 192, sc) and np.all(small == 77)
    # scale 0.1 of 1080p samples the 2x2 block at (10y + 4, 10x + 4) with weights 1/2, 1/2
    big = rng.integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
    s = cs.preprocess(big, 0.1).astype(int)
    gb = cs.bgr2gray(big).astype(int)
    blk = (gb[4::10, 4::10] + gb[4::10, 5::10] + gb[5::10, 4::10] + gb[5::10, 5::10]) / 4
    assert s.shape == (108, 192) and np.abs(s - blk).max() <= 1


def test_mask_follows_numpy_slicing():
    img = np.zeros((50, 80), np.uint8)
    m = cs.generate_mask(img, np.array([[100., 100., 300., 200.], [-50., 10., 60., 30.]]), 0.1)
    assert m[0].sum() == 0 and m[:, :1].sum() == 0            # 2 % border
    assert np.all(m[10:20, 10:30] == 0)                        # box 1 x 0.1
    # box 2 x 0.1 = (-5, 1, 6, 3): mask[1:3, -5:6] -> columns [75:6), empty: paints nothing
    assert np.all(m[1:3, 1:6] == 255) and np.all(m[1:3, 75:78] == 255) and m[1, 78] == 0


def test_min_eigen_and_corners_properties():
    g = cs.preprocess(sequence(216, 384, 1, 5)[0][0], 0.5)
    eig = cs.min_eigen(g)
    assert eig.dtype == np.float32 and eig.shape == g.shape
    mask = np.full(g.shape, 255, np.uint8)
    kp = cs.good_features(g, mask)
    assert kp is not None and 0 < len(kp) <= 3000
    v = eig[kp[:, 1].astype(int), kp[:, 0].astype(int)]
    assert np.all(np.diff(v.astype(np.float64)) <= 0)          # eigenvalue descending
    assert np.all(v >= np.float32(eig.max() * 0.01))
    assert cs.good_features(np.zeros_like(g), mask) is None     # flat: nothing


@pytest.mark.parametrize("h,w,scale", [(540, 960, 0.2), (1080, 1920, 0.1)])
def test_recovers_known_camera_motion(h, w, scale):
    frames, Ms = sequence(h, w, 4, 11, step=(0.15, 1.0, 5.0, -3.0))
    o = cs.SparseOptFlowOracle(scale)
    dets = boxes(h, w, 6, 2)
    assert np.array_equal(o.apply(frames[0], dets), np.eye(2, 3))
    n0 = len(o.prev_keypoints)
    assert n0 > 100
    for k in range(1, 4):
        H = o.apply(frames[k], dets)
        # the step between consecutive frames: rotation 0.15 deg, translation (5, -3) px, composed
        # about the origin with the previous frames' motion
        step = np.vstack([Ms[k], [0, 0, 1]]) @ np.linalg.inv(np.vstack([Ms[k - 1], [0, 0, 1]]))
        assert abs(H[0, 0] - step[0, 0]) < 2e-3 and abs(H[1, 0] - step[1, 0]) < 2e-3
        # translation at the frame centre within 1.5 px (0.15 px at the estimator's scale)
        c = np.array([w / 2, h / 2, 1.0])
        assert np.abs(H @ c - step[:2] @ c).max() < 1.5 / (scale / 0.1)
    assert len(o.prev_keypoints) <= n0


def test_failure_paths_keep_previous_frame():
    frames, _ = sequence(240, 320, 3, 4)
    o = cs.SparseOptFlowOracle(0.25)
    o.apply(frames[0], None)
    prev = o.prev_img.copy()
    o.prev_keypoints = o.prev_keypoints[:1]          # one point: estimateAffinePartial2D fails
    assert np.array_equal(o.apply(frames[1], None), np.eye(2, 3))
    assert np.array_equal(o.prev_img, prev)
    o.prev_keypoints = o.prev_keypoints[:0]          # none: LK returns None
    assert np.array_equal(o.apply(frames[2], None), np.eye(2, 3))


FIXTURE = os.path.join(os.path.dirname(__file__), "golden", "cmc_mot17.npz")


def test_mot17_fixture_frames():
    """Static sequences give near-identity warps, moving ones a consistent motion."""
    g = np.load(FIXTURE)
    for seq in ("MOT17_04", "MOT17_13"):
        frames = g[f"{seq}__small"]
        o = cs.SparseOptFlowOracle(0.1)
        o.prev_img = frames[0]
        o.prev_pyr = cs.build_pyramid(frames[0])
        o.prev_keypoints = cs.good_features(frames[0], cs.generate_mask(frames[0], None, 0.1))
        for f in frames[1:]:
            pyr = cs.build_pyramid(f)
            nxt, st = cs.lk_track(o.prev_pyr, pyr, o.prev_keypoints)
            M = cs.estimate_affine_partial(o.prev_keypoints[st == 1], nxt[st == 1])
            assert M is not None and abs(M[0, 0] - 1) < 0.02 and abs(M[1, 0]) < 0.02
            if seq == "MOT17_04":
                assert np.abs(M[:, 2]).max() < 0.5      # static camera (at 0.1 scale)
            o.prev_pyr = pyr
