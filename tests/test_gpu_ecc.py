"""GPU: the ECC estimator (csrc/ecc.hip through the C ABI) against its restatement
(oracle/cmc_ecc.py).  Parity with cv2.findTransformECC itself is unpinned (cv2 is absent); the bar
here is the restatement's, bit for bit: every warp (float32), the outcome (first frame / estimated
/ identity because OpenCV would raise), the iteration count and the final correlation, frame by
frame over several streams, the three motion models, the LDS-staged and the HBM path, frames that
change size, and the identity-on-error path with prev_img kept (ecc.py:82-84)."""
import numpy as np
import pytest
from scipy import ndimage

from oracle import cmc_ecc as ce
from test_ecc_cpu import FIXTURE, smooth_scene, u8, warp_scene
from yolo_tracking_amd.motion.ecc import ECC, EccEngine

pytestmark = pytest.mark.gpu


def gray_bgr(g):
    """A BGR frame whose gray conversion is exactly g (equal channels)."""
    return np.repeat(np.asarray(g, np.uint8)[..., None], 3, axis=2)


def moving_frames(h, w, n, seed, step=(0.002, 3.0, -2.0), sigma=6.0):
    """n BGR frames of a smooth scene under a camera rotating / translating `step` per frame."""
    g = smooth_scene(h + 2 * 64, w + 2 * 64, seed, sigma)
    out = []
    for k in range(n):
        th, tx, ty = step[0] * k, step[1] * k, step[2] * k
        M = np.array([[np.cos(th), -np.sin(th), tx + 64], [np.sin(th), np.cos(th), ty + 64]])
        out.append(gray_bgr(u8(warp_scene(g, M)[:h, :w])))
    return out


def run_pair(frames_per_stream, mode=1, scale=0.1, max_iter=100, eps=1e-5):
    """Run the engine and one oracle per stream over the same frames; assert bit-exact."""
    S = len(frames_per_stream)
    n = len(frames_per_stream[0])
    h0 = max(f.shape[0] for fs in frames_per_stream for f in fs)
    w0 = max(f.shape[1] for fs in frames_per_stream for f in fs)
    eng = EccEngine(S, mode, eps, max_iter, scale, 0, h0, w0)
    oracles = [ce.ECCOracle(warp_mode=mode, eps=eps, max_iter=max_iter, scale=scale)
               for _ in range(S)]
    iters = []
    for k in range(n):
        got = eng.apply([fs[k] for fs in frames_per_stream])
        out, it, rho = eng.outcome()
        for s in range(S):
            want = oracles[s].apply(frames_per_stream[s][k])
            last = oracles[s].last
            assert out[s] == last["outcome"], (k, s)
            assert np.array_equal(got[s], want), (k, s, got[s], want)
            if last["outcome"] == 1:
                assert it[s] == last["iters"] and rho[s] == last["rho"], (k, s)
                iters.append(int(it[s]))
            st = eng.state(s, with_image=True)
            assert np.array_equal(st["prev_img"], oracles[s].prev_img), (k, s)
    eng.close()
    return iters


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_mot17_frames_bit_exact(mode):
    g = np.load(FIXTURE)
    streams = [[gray_bgr(im) for im in g[key]] for key in g.files]
    n = min(len(s) for s in streams)
    iters = run_pair([s[:n] for s in streams], mode=mode, scale=1.0)
    assert iters and max(iters) > 2


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_camera_streams_scaled(mode):
    streams = [moving_frames(1080, 1920, 3, 1),
               moving_frames(480, 640, 3, 2, step=(-0.004, -5.0, 1.0)),
               moving_frames(720, 1280, 3, 3, step=(0.0, 0.0, 0.0))]
    run_pair(streams, mode=mode, scale=0.1)


def test_hbm_path_and_resolution_change():
    # scale 1 on 420 x 400: 168 000 bytes > the 144 KiB LDS stage, so the frame is read from HBM
    fr = moving_frames(420, 400, 3, 5, step=(0.001, 1.5, 0.5), sigma=10.0)
    run_pair([fr], mode=1, scale=1.0, max_iter=30)
    # template and input of different sizes (findTransformECC accepts them)
    a = moving_frames(480, 640, 2, 6)
    b = moving_frames(400, 560, 2, 6)
    run_pair([[a[0], b[1], a[1]]], mode=1, scale=0.25)


def test_identity_on_error_keeps_prev():
    fr = moving_frames(360, 640, 3, 8)
    flat = np.full_like(fr[0], 77)
    run_pair([[fr[0], flat, fr[1], fr[2]], [flat, flat, fr[0], fr[1]]], mode=1, scale=0.25)


def test_max_iter_and_eps_paths():
    fr = moving_frames(540, 960, 3, 9, step=(0.003, 6.0, -3.0))
    run_pair([fr], mode=1, scale=0.2, max_iter=3, eps=1e-12)
    run_pair([fr], mode=2, scale=0.2, max_iter=100, eps=1e-3)


def test_dropin_class_and_growth():
    fr = moving_frames(1080, 1920, 2, 10)
    ecc = ECC()
    o = ce.ECCOracle()
    for f in fr:
        assert np.array_equal(ecc.apply(f, None), o.apply(f))
    big = moving_frames(1200, 2000, 1, 10)[0]   # larger than the engine was created for: grows
    assert np.array_equal(ecc.apply(big, None), o.apply(big))
    with pytest.raises(NotImplementedError):
        ECC(warp_mode=3)


def test_uncorrelated_frames_error_path():
    """Independent noise frames: the step would minimise the correlation (lambda_d <= 0), where
    OpenCV raises; identity, prev_img kept - bit-exact with the restatement for every model."""
    rng = np.random.default_rng(4)
    fr = [gray_bgr(rng.integers(0, 256, (60, 80), dtype=np.uint8)) for _ in range(4)]
    inv = gray_bgr(255 - fr[1][..., 0])
    for mode in (0, 1, 2):
        run_pair([fr, [fr[0], fr[1], inv, fr[3]]], mode=mode, scale=1.0)


def test_capacity_error_leaves_engine_intact():
    """A frame whose scaled size overflows the LDS warp tables is refused (YTA_ERR_CAPACITY) and
    leaves the engine exactly as it was: the next normal frame matches the oracle that never saw
    the refused one (the slots are grown transactionally, csrc/ecc.hip ecc_slots)."""
    from yolo_tracking_amd._lib import YTAError
    frames = moving_frames(120, 160, 3, seed=5)
    eng = EccEngine(1, 1, 1e-5, 100, 0.1, 0, 120, 160)
    o = ce.ECCOracle(warp_mode=1, eps=1e-5, max_iter=100, scale=0.1)
    for k in range(2):
        assert np.array_equal(eng.apply([frames[k]])[0], o.apply(frames[k]))
    huge = np.zeros((1, 190000, 3), np.uint8)
    with pytest.raises(YTAError):
        eng.apply([huge])
    assert np.array_equal(eng.apply([frames[2]])[0], o.apply(frames[2]))
    st = eng.state(0, with_image=True)
    assert np.array_equal(st["prev_img"], o.prev_img)
    eng.close()


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_align_preview_bit_exact(mode):
    """ECC(align=True) (ecc.py:91-98): prev_img_aligned - the previous gray frame warped by the
    returned matrix on the device (k_ecc_align, yta_ecc_aligned) - equals the restatement's
    warpAffine (oracle/cmc_ecc.py warp_affine_u8) bit for bit after every estimate, and the
    identity-on-error path keeps the last preview."""
    fr = moving_frames(540, 960, 4, 11, step=(0.003, 6.0, -3.0))
    ecc = ECC(warp_mode=mode, scale=0.2, align=True)
    o = ce.ECCOracle(warp_mode=mode, scale=0.2, align=True)
    seen = 0
    for f in fr + [np.full_like(fr[0], 90), fr[0]]:
        assert np.array_equal(ecc.apply(f, None), o.apply(f))
        if o.prev_img_aligned is None:
            assert ecc.prev_img_aligned is None
        else:
            assert np.array_equal(ecc.prev_img_aligned, o.prev_img_aligned)
            seen += 1
    assert seen >= 3


def test_align_preview_streams():
    """EccEngine.aligned(s) per stream of a 3-stream engine against one oracle per stream; None
    where the stream's last apply was not an estimate (first frame, identity on error)."""
    a = moving_frames(270, 480, 3, 12)
    b = moving_frames(270, 480, 3, 13, step=(-0.002, -4.0, 2.0))
    eng = EccEngine(3, 2, 1e-5, 100, 0.25, 0, 270, 480)
    oracles = [ce.ECCOracle(warp_mode=2, scale=0.25, align=True) for _ in range(3)]
    for k in range(3):
        frames = [a[k], b[k], b[0] if k < 2 else a[0]]
        got = eng.apply(frames)
        for s in range(3):   # stream 2: the same frame twice, then another scene
            want = oracles[s].apply(frames[s])
            assert np.array_equal(got[s], want), (k, s)
            out, _, _ = eng.outcome()
            al = eng.aligned(s)
            if out[s] == 1:
                assert np.array_equal(al, oracles[s].prev_img_aligned), (k, s)
            else:
                assert al is None, (k, s)
    eng.close()
