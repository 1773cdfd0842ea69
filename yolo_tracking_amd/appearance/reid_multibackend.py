"""Device-side ReID preprocessing, mirroring boxmot/appearance/reid_multibackend.py.

The reference crops, resizes (cv2 INTER_LINEAR), colour-converts and standardises every detection
on the CPU in a Python loop (`preprocess`, :189-224), stacks the crops, copies them to the device,
runs the ReID network (`forward`, :226-299) and divides the features by one global norm
(`get_features`, :303-311).  Here the image goes to HBM once and `yta_reid_preprocess_device`
writes every crop of every camera stream in one launch, straight into the NCHW tensor the network
reads; `yta_reid_normalize_device` does the global normalisation before the single copy back.

The network: OSNet (appearance/osnet.py, an eval-mode inference graph with folded BatchNorms,
channels-last, batched branches) built from `weights` as the reference builds it from the weight
file name (reid_multibackend.py:57-80, osnet_x0_25 .. osnet_x1_0); the reference's .pt state dicts
load unchanged (torch.load(weights_only=True)).  A weight file that is not on disk would be
downloaded by the reference (gdown, :61-64) or end the program (:67-72); there is no network here,
so a missing file raises FileNotFoundError.  Freshly initialised weights (benchmarks, plumbing
tests) are an explicit opt-in: `random_init=True`.  `model=` (any torch module on the device
taking (N, 3, 256, 128)) replaces the network; the ONNX / OpenVINO / TensorRT / TFLite export
backends (:82-178) are not rebuilt.  There is no CPU fallback (a missing library raises YTAError).
"""
import warnings
from pathlib import Path
import ctypes

import numpy as np

try:   # before libyta.so loads: the library then binds to torch's HIP runtime (one per process)
    import torch  # noqa: F401
except ImportError:   # pragma: no cover
    torch = None

from .. import _lib

OUT_W, OUT_H = 128, 256   # cv2.resize(crop, (128, 256)) at :200-204


def crop_rects(xyxys, h, w):
    """(n, 4) int rows (y0, y1, x0, x1) of `img[y1:y2, x1:x2]` as :193-199 computes them
    (truncation, clamps, Python slice semantics).  Rows with y1 <= y0 or x1 <= x0 are empty."""
    b = np.asarray(xyxys, dtype=np.float64).reshape(-1, 4).astype("int")
    x1 = np.maximum(0, b[:, 0])
    y1 = np.maximum(0, b[:, 1])
    x2 = np.minimum(w - 1, b[:, 2])
    y2 = np.minimum(h - 1, b[:, 3])

    def stop(s, n):
        s = np.where(s < 0, s + n, s)
        return np.clip(s, 0, n)

    return np.stack([np.minimum(y1, h), stop(y2, h), np.minimum(x1, w), stop(x2, w)], axis=1)


def _check_crops(xyxys, h, w):
    r = crop_rects(xyxys, h, w)
    bad = np.nonzero((r[:, 1] <= r[:, 0]) | (r[:, 3] <= r[:, 2]))[0]
    if len(bad):   # cv2.resize asserts !ssize.empty() (cv2.error in the reference)
        i = int(bad[0])
        raise ValueError(f"box {i} {np.asarray(xyxys)[i].tolist()}: empty crop in a {h}x{w} image")


def preprocess_host(xyxys, img, fp16=False, device=0, out_w=OUT_W, out_h=OUT_H):
    """`preprocess` through the synchronous host-buffer ABI -> (N, 3, out_h, out_w) NumPy array
    (float32, or float16 with fp16)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    assert img.ndim == 3 and img.shape[2] == 3, "img must be H x W x 3 uint8 (BGR)"
    boxes = np.ascontiguousarray(xyxys, dtype=np.float64).reshape(-1, 4)
    out = np.empty((len(boxes), 3, out_h, out_w), dtype=np.float16 if fp16 else np.float32)
    _lib.check(_lib.load_library().yta_reid_preprocess(
        device, _lib.ptr(img), img.shape[0], img.shape[1], _lib.ptr(boxes), len(boxes), out_h,
        out_w, int(bool(fp16)), _lib.ptr(out)))
    return out


def normalize_host(features, device=0):
    """get_features' `features / np.linalg.norm(features)` through yta_reid_normalize."""
    f = np.array(features, dtype=np.float32, order="C")
    _lib.check(_lib.load_library().yta_reid_normalize(device, _lib.ptr(f), f.size))
    return f


class ReIDDetectMultiBackend:
    """reid_multibackend.py:59 ReIDDetectMultiBackend(weights, device, fp16) with a
    caller-supplied network (`model`, a torch module on `device`)."""

    def __init__(self, weights="osnet_x0_25_msmt17.pt", device=0, fp16=False, model=None,
                 random_init=False):
        import torch
        self.torch = torch
        self.weights = weights
        idx = _lib.parse_device(device)
        self.device = torch.device("cuda", idx)
        self.fp16 = bool(fp16)
        self.nhwc = False
        self.lib = _lib.load_library()
        self.random_init = bool(random_init)
        if model is None and weights is not None:
            model = self._build_osnet(weights)
        self.model = model

    def _build_osnet(self, weights):
        """reid_multibackend.py:57-80 for the OSNet family (the trackers' default weights)."""
        from .osnet import OSNetReID, load_checkpoint, model_name
        name = model_name(weights)
        if name is None:
            raise NotImplementedError(
                f"ReID weights {str(weights)!r}: only the OSNet family (osnet_x0_25 .. osnet_x1_0) "
                "is rebuilt on the MI355X path; pass model=<torch module> for other networks")
        w = Path(weights)
        if w.is_file():
            sd = load_checkpoint(w)
        elif self.random_init:
            warnings.warn(f"ReID weights {str(w)!r} not on disk: {name} runs with fresh random "
                          "weights (random_init=True)", RuntimeWarning, stacklevel=3)
            sd = None
        else:
            raise FileNotFoundError(
                f"ReID weights {str(w)!r} not found and there is no network to download them "
                f"(reid_multibackend.py:61-72); pass an existing {name} checkpoint, model=<torch "
                "module>, or random_init=True for untrained weights")
        return OSNetReID(name, sd, device=self.device, half=self.fp16)

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def preprocess_batch(self, items):
        """One launch for the boxes of several images: items = [(xyxys, img), ...] -> (sum n, 3,
        256, 128) device tensor, crops in item order."""
        torch = self.torch
        boxes, owner, offs, hws, bufs = [], [], [], [], []
        off = 0
        for i, (xyxys, img) in enumerate(items):
            img = np.ascontiguousarray(img, dtype=np.uint8)
            h, w = img.shape[:2]
            b = np.asarray(xyxys, dtype=np.float64).reshape(-1, 4)
            _check_crops(b, h, w)
            boxes.append(b)
            owner.append(np.full(len(b), i, dtype=np.int32))
            offs.append(off)
            hws += [h, w]
            bufs.append(img.reshape(-1))
            off += img.size
        boxes = np.concatenate(boxes) if boxes else np.empty((0, 4))
        n = len(boxes)
        dt = torch.half if self.fp16 else torch.float
        out = torch.empty((n, 3, OUT_H, OUT_W), dtype=dt, device=self.device)
        if n == 0:
            return out
        d = self.device
        d_img = torch.from_numpy(np.concatenate(bufs)).to(d, non_blocking=False)
        d_off = torch.tensor(offs, dtype=torch.int64, device=d)
        d_hw = torch.tensor(hws, dtype=torch.int32, device=d)
        d_box = torch.from_numpy(np.ascontiguousarray(boxes)).to(d)
        d_own = torch.from_numpy(np.concatenate(owner)).to(d)
        _lib.check(self.lib.yta_reid_preprocess_device(
            ctypes.c_void_p(d_img.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
            ctypes.c_void_p(d_hw.data_ptr()), ctypes.c_void_p(d_box.data_ptr()),
            ctypes.c_void_p(d_own.data_ptr()), n, OUT_H, OUT_W, int(self.fp16),
            ctypes.c_void_p(out.data_ptr()), None, self._stream()))
        return out

    def preprocess(self, xyxys, img):
        """reid_multibackend.py:189-224 -> (N, 3, 256, 128) tensor on the device."""
        return self.preprocess_batch([(xyxys, img)])

    def forward(self, im_batch):
        """:226-299 for the `pt` backend: the network on the batch -> NumPy."""
        if self.model is None:
            raise RuntimeError("ReIDDetectMultiBackend(weights=None): no network (pass weights "
                               "naming an OSNet variant or model=<torch module>)")
        if self.fp16 and im_batch.dtype != self.torch.float16:
            im_batch = im_batch.half()
        if self.nhwc:
            im_batch = im_batch.permute(0, 2, 3, 1)
        features = self.model(im_batch)
        if isinstance(features, (list, tuple)):
            return (self.to_numpy(features[0]) if len(features) == 1
                    else [self.to_numpy(x) for x in features])
        return self.to_numpy(features)

    def to_numpy(self, x):
        return x.cpu().numpy() if isinstance(x, self.torch.Tensor) else x

    def warmup(self, imgsz=[(256, 128, 3)]):
        im = np.random.randint(0, 255, *imgsz, dtype=np.uint8)
        im = self.preprocess(xyxys=np.array([[0, 0, 128, 256]]), img=im)
        if self.model is not None:
            self.forward(im)

    def normalize_(self, features):
        """In-place global normalisation of a float32 device tensor (get_features :310)."""
        assert features.dtype == self.torch.float32 and features.is_contiguous()
        # partial sums: a fresh block from the caching allocator on the current stream, so calls
        # on different streams (one per camera) never share a workspace
        work = self.torch.empty(256, dtype=self.torch.float64, device=self.device)
        _lib.check(self.lib.yta_reid_normalize_device(
            ctypes.c_void_p(features.data_ptr()), features.numel(),
            ctypes.c_void_p(work.data_ptr()), self._stream()))
        return features

    def get_features(self, xyxys, img):
        """:303-311: features of the crops, divided by their global norm (NumPy (N, D))."""
        torch = self.torch
        if np.asarray(xyxys).size == 0:
            return np.array([])
        with torch.no_grad():
            crops = self.preprocess(xyxys, img)
            if self.model is None:
                self.forward(crops)   # raises
            f = self.model(crops.half() if self.fp16 else crops)
            if isinstance(f, (list, tuple)):
                f = f[0]
            dt = f.dtype
            f = self.normalize_(f.float().contiguous())
            return f.to(dt).cpu().numpy()
