"""CPU: the ReID preprocessing oracle (oracle/reid.py) and the package's crop-rectangle logic.

The resize step restates OpenCV's fixed-point INTER_LINEAR; cv2 is not installed here, so it is
PARITY UNPINNED against cv2 itself and cross-checked against an independent float bilinear on the
same sampling grid (agreement within one u8 level).  The float steps after it are NumPy's own
arithmetic (reid_multibackend.py:206-216)."""
import numpy as np
import pytest

from oracle import reid as orr
from yolo_tracking_amd.appearance import crop_rects


@pytest.mark.parametrize("h,w", [(17, 9), (256, 128), (512, 256), (600, 40), (1, 1), (3, 300),
                                 (100, 64), (255, 129), (40, 1000)])
def test_fixed_point_resize_within_one_level_of_float_bilinear(h, w):
    rng = np.random.default_rng(h * 1000 + w)
    c = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    a = orr.resize_linear_u8(c, 128, 256).astype(int)
    b = orr.bilinear_float(c, 128, 256).astype(int)
    assert a.shape == (256, 128, 3)
    assert np.abs(a - b).max() <= 1


def test_same_size_is_identity_and_area_fast_path():
    rng = np.random.default_rng(1)
    c = rng.integers(0, 256, (256, 128, 3), dtype=np.uint8)
    assert np.array_equal(orr.resize_linear_u8(c, 128, 256), c)
    c2 = rng.integers(0, 256, (512, 256, 3), dtype=np.uint8).astype(int)
    s = c2[0::2, 0::2] + c2[0::2, 1::2] + c2[1::2, 0::2] + c2[1::2, 1::2]
    assert np.array_equal(orr.resize_linear_u8(c2.astype(np.uint8), 128, 256), (s + 2) >> 2)


def test_constant_crop_stays_constant():
    c = np.full((37, 23, 3), 200, dtype=np.uint8)
    assert (orr.resize_linear_u8(c, 128, 256) == 200).all()


def test_crop_rect_semantics():
    h, w = 100, 200
    cases = [([10.9, 20.2, 50.7, 60.1], (20, 60, 10, 50)),     # truncation, end-exclusive
             ([-5, -7, 500, 500], (0, 99, 0, 199)),            # clamp to h-1 / w-1 (quirk)
             ([-0.9, 3, 4, 5], (3, 5, 0, 4)),                  # -0.9 truncates to 0
             ([10, 10, -3, 30], (10, 30, 10, 197)),            # negative stop wraps (slice)
             ([150, 10, 120, 30], None),                       # x2 < x1: empty
             ([250, 10, 300, 30], None)]                       # starts past the image
    for box, exp in cases:
        got = orr.crop_rect(box, h, w)
        assert got == exp, (box, got, exp)
        r = crop_rects([box], h, w)[0]
        if exp is None:
            assert r[1] <= r[0] or r[3] <= r[2]
        else:
            assert tuple(int(v) for v in r) == exp


def test_preprocess_float_steps():
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (64, 64, 3), dtype=np.uint8)
    out = orr.preprocess(np.array([[0, 0, 63, 63]]), img)
    crop = orr.resize_linear_u8(img[0:63, 0:63], 128, 256)[..., ::-1]
    exp = ((crop / 255 - orr.MEAN) / orr.STD).astype(np.float32).transpose(2, 0, 1)
    assert out.dtype == np.float32 and out.shape == (1, 3, 256, 128)
    assert np.array_equal(out[0], exp)
    with pytest.raises(ValueError):
        orr.preprocess(np.array([[10, 10, 5, 20]]), img)


def test_global_normalize():
    f = np.random.default_rng(3).standard_normal((7, 512)).astype(np.float32)
    g = orr.global_normalize(f)
    assert g.dtype == np.float32
    assert abs(float(np.sqrt((g.astype(np.float64) ** 2).sum())) - 1) < 1e-6


def test_osnet_graph_matches_reference_module():
    """appearance/osnet.py (folded BatchNorms, batched branches) against the reference's OSNet
    x0.25 module in eval mode (tests/golden/osnet_x0_25.npz, random weights + BN statistics),
    float32 on the CPU."""
    import os
    import torch
    from yolo_tracking_amd.appearance.osnet import OSNetReID
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "osnet_x0_25.npz"))
    sd = {k[4:]: g[k] for k in g.files if k.startswith("sd__")}
    x = np.random.default_rng(int(g["input_seed"])).standard_normal((4, 3, 256, 128))
    y = OSNetReID("osnet_x0_25", sd, device="cpu")(torch.from_numpy(x.astype(np.float32)))
    ref = g["features"]
    assert np.abs(y.numpy() - ref).max() <= 1e-5 * np.abs(ref).max()


def test_osnet_names_and_random_init():
    import torch
    from yolo_tracking_amd.appearance.osnet import OSNetReID, model_name, random_state_dict
    assert model_name("weights/osnet_x0_25_msmt17.pt") == "osnet_x0_25"
    assert model_name("osnet_x1_0_market1501.pt") == "osnet_x1_0"
    assert model_name("resnet50_msmt17.pt") is None
    for name in ("osnet_x0_5", "osnet_x1_0"):
        y = OSNetReID(name, random_state_dict(name), device="cpu")(torch.zeros(2, 3, 256, 128))
        assert y.shape == (2, 512) and torch.isfinite(y).all()
