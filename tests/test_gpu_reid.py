"""ReID preprocessing / normalisation on the MI355X (csrc/reid.hip through the C ABI) against the
oracle (oracle/reid.py, a restatement of reid_multibackend.py:189-224 + OpenCV's fixed-point
INTER_LINEAR; parity of the resize step against cv2 itself is unpinned, cv2 being absent).

Bar: crops bit-exact with the oracle (integer resize, then the same float64 expression rounded to
float32 / float16); global normalisation within NORM_RTOL (the sum of squares runs in float64 in a
different order than NumPy's float32 dot)."""
import numpy as np
import pytest

from oracle import reid as orr
from yolo_tracking_amd.appearance import ReIDDetectMultiBackend
from yolo_tracking_amd.appearance.reid_multibackend import normalize_host, preprocess_host
from yolo_tracking_amd._lib import YTAError

pytestmark = pytest.mark.gpu

NORM_RTOL = 2e-6


def boxes_for(rng, h, w, n):
    x1 = rng.uniform(-20, w - 10, n)
    y1 = rng.uniform(-20, h - 10, n)
    bw = rng.uniform(4, 300, n)
    bh = rng.uniform(4, 500, n)
    b = np.stack([x1, y1, x1 + bw, y1 + bh], 1)
    special = np.array([[0, 0, 129, 257],              # 128 x 256 crop: identity
                        [3, 5, 260, 518],              # 256 x 512 crop: INTER_AREA fast path
                        [w - 2, h - 2, w + 50, h + 50],  # 1 x 1 crop at the corner
                        [-50, -50, w + 50, h + 50],    # clamps to (h-1) x (w-1)
                        [10.99, 20.01, 11.5, 400.2],   # width 1
                        [5, 5, 8000, 6]])              # height 1
    return np.concatenate([b, special])


@pytest.mark.parametrize("half", [0, 1])
def test_preprocess_host_bit_exact(half):
    rng = np.random.default_rng(10 + half)
    h, w = 540, 960
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    boxes = boxes_for(rng, h, w, 120)
    rects = [orr.crop_rect(b, h, w) for b in boxes]
    boxes = boxes[[r is not None for r in rects]]
    got = preprocess_host(boxes, img, fp16=bool(half))
    exp = orr.preprocess(boxes, img, fp16=bool(half))
    assert got.dtype == exp.dtype and got.shape == exp.shape
    bad = np.nonzero((got != exp).reshape(len(boxes), -1).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} crops differ, first box {boxes[bad[0]]}"


def test_preprocess_odd_output_width():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (90, 70, 3), dtype=np.uint8)
    boxes = np.array([[1, 2, 60, 80], [10, 10, 30, 20]], dtype=np.float64)
    got = preprocess_host(boxes, img, out_w=37, out_h=19)
    exp = np.stack([((orr.resize_linear_u8(img[y0:y1, x0:x1], 37, 19)[..., ::-1] / 255
                      - orr.MEAN) / orr.STD).astype(np.float32).transpose(2, 0, 1)
                    for y0, y1, x0, x1 in (orr.crop_rect(b, 90, 70) for b in boxes)])
    assert np.array_equal(got, exp)


def test_empty_crop_raises():
    img = np.zeros((50, 50, 3), dtype=np.uint8)
    with pytest.raises(YTAError, match="empty crop"):
        preprocess_host(np.array([[1, 1, 20, 20], [30, 10, 20, 20]]), img)
    assert preprocess_host(np.empty((0, 4)), img).shape == (0, 3, 256, 128)


def test_device_batch_over_images_and_empty_count():
    import ctypes
    import torch
    from yolo_tracking_amd import _lib
    rng = np.random.default_rng(5)
    imgs = [rng.integers(0, 256, s, dtype=np.uint8) for s in [(300, 500, 3), (64, 48, 3),
                                                               (720, 1280, 3)]]
    per = [boxes_for(rng, im.shape[0], im.shape[1], 20) for im in imgs]
    per = [b[[orr.crop_rect(x, im.shape[0], im.shape[1]) is not None for x in b]]
           for b, im in zip(per, imgs)]
    reid = ReIDDetectMultiBackend(device=0, random_init=True)
    got = reid.preprocess_batch(list(zip(per, imgs))).cpu().numpy()
    exp = np.concatenate([orr.preprocess(b, im) for b, im in zip(per, imgs)])
    assert np.array_equal(got, exp)
    # raw device ABI: an empty crop is zero-filled and counted
    d = torch.device("cuda", 0)
    im = imgs[0]
    boxes = np.array([[1, 1, 40, 40], [30, 10, 20, 20], [5, 5, 100, 60]], dtype=np.float64)
    d_img = torch.from_numpy(im.reshape(-1)).to(d)
    d_off = torch.zeros(1, dtype=torch.int64, device=d)
    d_hw = torch.tensor(im.shape[:2], dtype=torch.int32, device=d)
    d_box = torch.from_numpy(boxes).to(d)
    d_cnt = torch.zeros(1, dtype=torch.int32, device=d)
    out = torch.full((3, 3, 256, 128), 7.0, device=d)
    _lib.check(_lib.load_library().yta_reid_preprocess_device(
        ctypes.c_void_p(d_img.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
        ctypes.c_void_p(d_hw.data_ptr()), ctypes.c_void_p(d_box.data_ptr()), None, 3, 256, 128, 0,
        ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(d_cnt.data_ptr()), None))
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert int(d_cnt.item()) == 1
    assert (o[1] == 0).all()
    assert np.array_equal(o[[0, 2]], orr.preprocess(boxes[[0, 2]], im))


@pytest.mark.parametrize("shape", [(1, 512), (37, 512), (1024, 512), (3, 5)])
def test_normalize(shape):
    f = np.random.default_rng(shape[0]).standard_normal(shape).astype(np.float32) * 3
    got = normalize_host(f)
    exp = orr.global_normalize(f)
    assert got.dtype == np.float32
    np.testing.assert_allclose(got, exp, rtol=NORM_RTOL, atol=1e-9)


def test_get_features_with_a_device_network():
    import torch
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.AvgPool2d(8), torch.nn.Flatten(),
                              torch.nn.Linear(3 * 32 * 16, 64)).to("cuda:0").eval()
    reid = ReIDDetectMultiBackend(device="cuda:0", model=net)
    rng = np.random.default_rng(9)
    img = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    boxes = boxes_for(rng, 480, 640, 30)
    boxes = boxes[[orr.crop_rect(b, 480, 640) is not None for b in boxes]]
    feats = reid.get_features(boxes, img)
    crops = torch.from_numpy(orr.preprocess(boxes, img)).to("cuda:0")
    with torch.no_grad():
        raw = net(crops).cpu().numpy()
    np.testing.assert_allclose(feats, orr.global_normalize(raw), rtol=1e-5, atol=1e-7)
    assert reid.get_features(np.empty((0, 4)), img).shape == (0,)


def test_botsort_with_device_reid_matches_oracle():
    """End to end: BoTSORT(reid=ReIDDetectMultiBackend(model=net)) — crops, network and global
    normalisation on the device feeding the device tracker — against the oracle tracker fed with
    the oracle's crops through the same network.  Ids / scores / det_ind bit-exact, boxes to 1e-9
    relative (the features differ only by the normalisation's summation order)."""
    import torch
    from oracle.botsort import BoTSORTOracle
    from yolo_tracking_amd.synth import make_frames
    from yolo_tracking_amd.motion import IdentityCMC
    from yolo_tracking_amd.trackers.botsort import BoTSORT
    torch.manual_seed(1)
    net = torch.nn.Sequential(torch.nn.AvgPool2d(8), torch.nn.Flatten(),
                              torch.nn.Linear(3 * 32 * 16, 128)).to("cuda:0").eval()
    params = dict(track_high_thresh=0.5, track_low_thresh=0.1, new_track_thresh=0.6,
                  track_buffer=30, match_thresh=0.8, proximity_thresh=0.5,
                  appearance_thresh=0.25, frame_rate=30)
    n = 64
    frames = [d for d, _ in make_frames(n, 10, seed=21)]
    C = int(64 * np.sqrt(n))
    rng = np.random.default_rng(4)
    reid = ReIDDetectMultiBackend(device="cuda:0", model=net)
    t = BoTSORT(None, "cuda:0", False, reid=reid, cmc=IdentityCMC(), **params)   # static camera
    ref = BoTSORTOracle(**params)
    for f, dets in enumerate(frames):
        img = rng.integers(0, 256, (C + 128, C + 128, 3), dtype=np.uint8)
        got = np.asarray(t.update(dets, img)).reshape(-1, 8)
        hi = dets[:, 4] > params["track_high_thresh"]
        with torch.no_grad():
            raw = net(torch.from_numpy(orr.preprocess(dets[hi, :4], img)).to("cuda:0"))
        feats = orr.global_normalize(raw.cpu().numpy())
        exp = ref.update(dets, feats).reshape(-1, 8)
        assert got.shape == exp.shape, f
        assert np.array_equal(got[:, 4:], exp[:, 4:]), f
        np.testing.assert_allclose(got[:, :4], exp[:, :4], rtol=1e-9, atol=1e-6)
