"""GPU: the OSNet ReID network (appearance/osnet.py) against the reference's module
(tests/golden/osnet_x0_25.npz: boxmot/appearance/backbones/osnet.py with random weights and
BatchNorm statistics, eval mode), the weight-file path of ReIDDetectMultiBackend, and the trackers
building their ReID producer from reid_weights as the reference does.

Bar: float32 features within 1e-4 of the feature scale (the HIP forward, csrc/osnet.hip, sums its
convolutions and MFMA GEMM tiles in other orders than the CPU's); float16 within 2e-2 relative (the reference's half=True path is
float16 as well)."""
import os

import numpy as np
import pytest
import torch

from yolo_tracking_amd.appearance import ReIDDetectMultiBackend
from yolo_tracking_amd.appearance.osnet import OSNetReID

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "osnet_x0_25.npz"))
    sd = {k[4:]: g[k] for k in g.files if k.startswith("sd__")}
    x = np.random.default_rng(int(g["input_seed"])).standard_normal((4, 3, 256, 128))
    return sd, x.astype(np.float32), g["features"]


def test_osnet_float32_matches_reference(golden):
    sd, x, ref = golden
    y = OSNetReID("osnet_x0_25", sd, device="cuda:0")(torch.from_numpy(x).cuda()).cpu().numpy()
    assert np.abs(y - ref).max() <= 1e-4 * np.abs(ref).max()


def test_osnet_float16(golden):
    sd, x, ref = golden
    y = OSNetReID("osnet_x0_25", sd, device="cuda:0", half=True)(torch.from_numpy(x).cuda())
    assert y.dtype == torch.float16
    y = y.float().cpu().numpy()
    assert np.abs(y - ref).max() <= 2e-2 * np.abs(ref).max()


def test_weight_file_and_get_features(golden, tmp_path):
    """A reference-format checkpoint ({'state_dict': ...} with 'module.' prefixes) loads through
    ReIDDetectMultiBackend(weights); get_features = OSNet(crops) / global norm."""
    sd, _, _ = golden
    w = tmp_path / "osnet_x0_25_msmt17.pt"
    torch.save({"state_dict": {"module." + k: torch.from_numpy(v) for k, v in sd.items()}}, w)
    reid = ReIDDetectMultiBackend(w, device=0, fp16=False)
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (480, 640, 3), dtype=np.uint8)
    boxes = np.array([[10, 20, 110, 300], [300, 50, 380, 250], [500, 100, 639, 479]], np.float64)
    f = reid.get_features(boxes, img)
    crops = reid.preprocess(boxes, img)
    raw = OSNetReID("osnet_x0_25", sd, device="cuda:0")(crops).cpu().numpy()
    np.testing.assert_allclose(f, raw / np.linalg.norm(raw), rtol=1e-5, atol=1e-7)
    reid.warmup()


def test_trackers_build_reid_from_weights(tmp_path):
    """create_tracker('botsort' / 'deepocsort' / 'hybridsort', cfg, reid_weights=<path>) builds
    the OSNet producer (bot_sort.py:217-219); a missing file raises FileNotFoundError, random
    weights only on request (random_init=True)."""
    from yolo_tracking_amd import create_tracker, get_tracker_config
    from yolo_tracking_amd.synth import make_frames
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (640, 640, 3), dtype=np.uint8)
    dets = make_frames(24, 1, 5, canvas=600.0)[0][0]
    from yolo_tracking_amd.appearance.osnet import random_state_dict
    w = tmp_path / "osnet_x0_25_x.pt"
    torch.save({"state_dict": {k: torch.from_numpy(np.asarray(v))
                               for k, v in random_state_dict("osnet_x0_25", 1).items()}}, w)
    for name in ("botsort", "deepocsort", "hybridsort"):
        with pytest.raises(FileNotFoundError):
            create_tracker(name, get_tracker_config(name), tmp_path / "missing_osnet_x0_25.pt",
                           "0", False, False)
        t = create_tracker(name, get_tracker_config(name), w, "0", False, False)
        assert isinstance(t.model, ReIDDetectMultiBackend)
        t.model.warmup()
        r = np.asarray(t.update(dets, img))
        assert r.size == 0 or r.shape[1] == 8


# ---- the block kernels (csrc/osnet.hip) against PyTorch float32 on the same inputs
def _dw_case(n, c, h, w, n_first, half, seed):
    import ctypes
    from yolo_tracking_amd import _lib
    lib = _lib.load_library()
    dt = torch.float16 if half else torch.float32
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((n, c + 3, h, w), generator=g).to(dt).cuda()   # strided view: 3 extra planes
    wt = torch.randn((c, 1, 3, 3), generator=g).cuda()
    b = torch.randn((c,), generator=g).cuda()
    xv = x[:, 2:2 + c]
    yf = torch.full((n, n_first + 1, h, w), 7.0, dtype=dt, device="cuda")
    yr = torch.empty((n, c - n_first, h, w), dtype=dt, device="cuda")
    ps = torch.zeros((n, n_first + 2), dtype=torch.float32, device="cuda")
    _lib.check(lib.yta_osnet_dw3x3(
        ctypes.c_void_p(xv.data_ptr()), (c + 3) * h * w, h * w,
        ctypes.c_void_p(wt.data_ptr()), ctypes.c_void_p(b.data_ptr()), n, c, h, w, int(half),
        ctypes.c_void_p(yf.data_ptr()), (n_first + 1) * h * w, n_first,
        ctypes.c_void_p(yr.data_ptr()) if c > n_first else None, (c - n_first) * h * w,
        ctypes.c_void_p(ps.data_ptr()), n_first + 2, None))
    torch.cuda.synchronize()
    ref = torch.relu(torch.nn.functional.conv2d(xv.float(), wt, b, padding=1, groups=c))
    tol = 2e-3 if half else 1e-5
    scale = ref.abs().max().item()
    def err(a, b):
        return (a.float() - b).abs().max().item() if a.numel() else 0.0
    assert err(yf[:, :n_first], ref[:, :n_first]) <= tol * scale
    assert err(yr, ref[:, n_first:]) <= tol * scale
    assert (yf[:, n_first] == 7.0).all()                    # plane past n_first untouched
    s = yf[:, :n_first].float().sum(dim=(2, 3))              # sums of the stored values
    assert torch.allclose(ps[:, :n_first], s, rtol=1e-5, atol=1e-3)
    assert (ps[:, n_first:] == 0).all()


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("shape", [(2, 12, 64, 32, 4), (3, 20, 16, 8, 5), (1, 6, 5, 3, 6),
                                   (2, 9, 1, 1, 3), (1, 4, 33, 17, 0)])
def test_dw3x3_kernel(shape, half):
    n, c, h, w, nf = shape
    _dw_case(n, c, h, w, nf, half, seed=sum(shape))


@pytest.mark.parametrize("half", [False, True])
def test_gate_sum_kernel(half):
    import ctypes
    from yolo_tracking_amd import _lib
    lib = _lib.load_library()
    dt = torch.float16 if half else torch.float32
    g = torch.Generator().manual_seed(5)
    n, c, p = 3, 24, 16 * 8 + 5
    st = torch.randn((n, 4, c, p), generator=g).to(dt).cuda()
    gate = torch.rand((n, 4, c), generator=g).to(dt).cuda()
    out = torch.empty((n, c, p), dtype=dt, device="cuda")
    _lib.check(lib.yta_osnet_gate_sum(ctypes.c_void_p(st.data_ptr()),
                                      ctypes.c_void_p(gate.data_ptr()), n, c, p, int(half),
                                      ctypes.c_void_p(out.data_ptr()), None))
    torch.cuda.synchronize()
    ref = (st.float() * gate.float()[..., None]).sum(1)
    tol = 2e-3 if half else 1e-6
    assert (out.float() - ref).abs().max().item() <= tol * ref.abs().max().item()


def test_block_kernels_match_torch_graph(golden):
    """The same folded network on PyTorch's kernels (hip=False: MIOpen convolutions) agrees with
    the all-HIP forward."""
    sd, x, _ = golden
    xt = torch.from_numpy(x).cuda()
    a = OSNetReID("osnet_x0_25", sd, device="cuda:0")(xt)
    b = OSNetReID("osnet_x0_25", sd, device="cuda:0", hip=False)(xt)
    assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item()


# ---- the rest of the network's layers as HIP kernels (csrc/osnet.hip k_pw / k_stem / k_pool /
# k_gate) against PyTorch's float32 operators
def _pw_call(x1, w, bias=None, *, k1, G=1, cout_g, P, N, relu, x2=None, k2=0, res=None,
             x1s=None, x2s=None, ys=None, out=None, half=False):
    import ctypes
    from yolo_tracking_amd import _lib
    dt = torch.float16 if half else torch.float32
    if out is None:
        out = torch.full((N, G * cout_g, P), 3.0, dtype=dt, device="cuda")
    a = _lib.PwArgs()
    a.x1 = x1.data_ptr()
    a.x1n, a.x1c, a.x1p = x1s or (G * k1 * P, P, 1)
    if x2 is not None:
        a.x2 = x2.data_ptr()
        a.x2n, a.x2c, a.x2p = x2s or (k2 * P, P, 1)
    wt = w.transpose(1, 2).contiguous()   # (G, cout_g, K) -> the kernel's k-major layout
    a.w = wt.data_ptr()
    a.bias = bias.data_ptr() if bias is not None else None
    if res is not None:
        a.res = res.data_ptr()
        a.rn, a.rc, a.rp = G * cout_g * P, P, 1
    a.y = out.data_ptr()
    a.yn, a.yc, a.yp = ys or (G * cout_g * P, P, 1)
    a.k1, a.k2, a.G, a.cout_g, a.P, a.N, a.relu = k1, k2, G, cout_g, P, N, int(relu)
    _lib.check(_lib.load_library().yta_osnet_pointwise(ctypes.byref(a), int(half), None))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("case", [(2, 16, 16, 1, 2048, 0, False, True),   # conv1 (x0_25 stage 2)
                                  (3, 24, 96, 1, 512, 0, False, False),   # depth 0: mid -> 4 mid
                                  (2, 24, 24, 3, 512, 0, False, False),   # grouped depth 1
                                  (2, 24, 96, 1, 512, 64, True, True),    # conv3 + downsample
                                  (2, 32, 128, 1, 128, 0, True, True),    # conv3 + identity
                                  (1, 130, 70, 1, 37, 0, False, True)])   # ragged M / N / K
def test_pointwise_kernel(case, half):
    n, k1, cout_g, G, P, k2, resid, relu = case
    dt = torch.float16 if half else torch.float32
    g = torch.Generator().manual_seed(sum(case))
    x1 = torch.randn((n, G * k1, P), generator=g).to(dt).cuda()
    w = (torch.randn((G, cout_g, k1 + k2), generator=g) * 0.2).cuda()
    b = torch.randn(G * cout_g, generator=g).cuda()
    x2 = torch.randn((n, k2, P), generator=g).to(dt).cuda() if k2 else None
    res = torch.randn((n, G * cout_g, P), generator=g).to(dt).cuda() if resid and not k2 else None
    out = _pw_call(x1, w, b, k1=k1, G=G, cout_g=cout_g, P=P, N=n, relu=relu, x2=x2, k2=k2,
                   res=res, half=half)
    xs = x1.float().view(n, G, k1, P)
    ref = torch.einsum("gok,ngkp->ngop", w[:, :, :k1], xs).reshape(n, G * cout_g, P)
    if k2:
        ref = ref + torch.einsum("ok,nkp->nop", w[0, :, k1:], x2.float())
    ref = ref + b[None, :, None]
    if res is not None:
        ref = ref + res.float()
    if relu:
        ref = ref.relu()
    tol = 5e-3 if half else 1e-5
    assert (out.float() - ref).abs().max().item() <= tol * ref.abs().max().item()


def test_pointwise_as_linear_over_crops():
    """The fc layer: one 'sample', the crops on the pixel axis (strided input and output)."""
    g = torch.Generator().manual_seed(11)
    n, c, o = 37, 128, 512
    v = torch.randn((n, c), generator=g).cuda()
    w = (torch.randn((1, o, c), generator=g) * 0.1).cuda()
    b = torch.randn(o, generator=g).cuda()
    out = torch.empty((n, o), device="cuda")
    _pw_call(v, w, b, k1=c, cout_g=o, P=n, N=1, relu=True, x1s=(0, 1, c), ys=(0, 1, o), out=out)
    ref = torch.relu(v @ w[0].T + b)
    assert (out - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("shape", [(2, 256, 128, 16), (1, 37, 29, 64)])
def test_stem_kernel(shape, half):
    import ctypes
    from yolo_tracking_amd import _lib
    n, h, w, c0 = shape
    dt = torch.float16 if half else torch.float32
    g = torch.Generator().manual_seed(h + w)
    x = torch.randn((n, 3, h, w), generator=g).to(dt).cuda()
    wt = (torch.randn((c0, 3, 7, 7), generator=g) * 0.1).cuda()
    b = torch.randn(c0, generator=g).cuda()
    y = torch.empty((n, c0, (h - 1) // 2 + 1, (w - 1) // 2 + 1), dtype=dt, device="cuda")
    _lib.check(_lib.load_library().yta_osnet_stem(
        ctypes.c_void_p(x.data_ptr()), n, h, w, ctypes.c_void_p(wt.data_ptr()),
        ctypes.c_void_p(b.data_ptr()), c0, int(half), ctypes.c_void_p(y.data_ptr()), None))
    torch.cuda.synchronize()
    ref = torch.relu(torch.nn.functional.conv2d(x.float(), wt, b, stride=2, padding=3))
    tol = 5e-3 if half else 1e-5
    assert (y.float() - ref).abs().max().item() <= tol * ref.abs().max().item()


@pytest.mark.parametrize("half", [False, True])
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_pool_kernel(kind, half):
    import ctypes
    from yolo_tracking_amd import _lib
    F = torch.nn.functional
    dt = torch.float16 if half else torch.float32
    g = torch.Generator().manual_seed(kind)
    n, c, h, w = 3, 5, 33, 18
    x = torch.randn((n, c, h, w), generator=g).to(dt).cuda()
    if kind == 0:
        ref = F.max_pool2d(x.float(), 3, stride=2, padding=1)
    elif kind == 1:
        ref = F.avg_pool2d(x.float(), 2, stride=2)
    else:
        ref = x.float().mean(dim=(2, 3))
    y = torch.empty(ref.shape, dtype=dt, device="cuda")
    _lib.check(_lib.load_library().yta_osnet_pool(ctypes.c_void_p(x.data_ptr()), n, c, h, w, kind,
                                                  int(half), ctypes.c_void_p(y.data_ptr()), None))
    torch.cuda.synchronize()
    tol = 2e-3 if half else 1e-6
    assert (y.float() - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("half", [False, True])
def test_gate_kernel(half):
    import ctypes
    from yolo_tracking_amd import _lib
    F = torch.nn.functional
    dt = torch.float16 if half else torch.float32
    g = torch.Generator().manual_seed(9)
    n, mid, hid, p = 4, 32, 2, 512
    psum = (torch.randn((n, 4, mid), generator=g) * p).cuda()
    w1 = (torch.randn((hid, mid), generator=g) * 0.3).to(dt).cuda()
    b1 = torch.randn(hid, generator=g).to(dt).cuda()
    w2 = (torch.randn((mid, hid), generator=g) * 0.3).to(dt).cuda()
    b2 = torch.randn(mid, generator=g).to(dt).cuda()
    gate = torch.empty((n, 4, mid), dtype=dt, device="cuda")
    _lib.check(_lib.load_library().yta_osnet_gate(
        ctypes.c_void_p(psum.data_ptr()), n, mid, hid, p, ctypes.c_void_p(w1.data_ptr()),
        ctypes.c_void_p(b1.data_ptr()), ctypes.c_void_p(w2.data_ptr()),
        ctypes.c_void_p(b2.data_ptr()), int(half), ctypes.c_void_p(gate.data_ptr()), None))
    torch.cuda.synchronize()
    pooled = (psum / p).to(dt)
    ref = torch.sigmoid(F.linear(F.relu(F.linear(pooled, w1, b1)), w2, b2)).float()
    tol = 2e-3 if half else 1e-6
    assert (gate.float() - ref).abs().max().item() <= tol
