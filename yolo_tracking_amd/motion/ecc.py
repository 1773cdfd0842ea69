"""ECC camera-motion compensation on the MI355X.

Reference: boxmot/motion/cmc/ecc.py:13-104 (ECC: __init__, apply), cmc_interface.py:26-40
(preprocess); get_cmc_method('ecc') (motion/cmc/__init__.py:9-11) is what HybridSORT builds
(hybridsort.py:366) and StrongSORT uses.  `ECC().apply(img, dets)` returns the reference's 2x3
float32 warp: cv2.findTransformECC between the previous and the current gray frame (resized by
`scale`), the translation divided by `scale`, the identity on the first frame and wherever OpenCV
would raise.  The work runs in csrc/ecc.hip (gray + resize, then one 1024-thread block per stream
runs the whole Gauss-Newton loop) through the C ABI.  `EccEngine` runs S camera streams per call.
There is no CPU fallback: without the HIP library or a device this raises YTAError.
"""
import ctypes

import numpy as np

from .. import _lib

MOTION_TRANSLATION, MOTION_EUCLIDEAN, MOTION_AFFINE, MOTION_HOMOGRAPHY = 0, 1, 2, 3


class EccEngine:
    """S independent ECC estimators sharing one device engine."""

    def __init__(self, n_streams=1, warp_mode=MOTION_EUCLIDEAN, eps=1e-5, max_iter=100,
                 scale=0.1, device=0, max_h=1080, max_w=1920):
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.device = _lib.parse_device(device)
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_ecc_create(self.device, self.n_streams, int(warp_mode), float(eps),
                                           int(max_iter), float(scale), int(max_h), int(max_w),
                                           ctypes.byref(h)))
        self._h = h
        self._warps = np.zeros((self.n_streams, 6), dtype=np.float32)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.yta_ecc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.yta_ecc_reset(self._h))

    def apply(self, imgs):
        """imgs: S (h, w, 3) uint8 BGR frames.  Returns (S, 2, 3) float32 warps."""
        assert len(imgs) == self.n_streams
        frames, off = [], np.zeros(self.n_streams, np.int64)
        hw = np.zeros(2 * self.n_streams, np.int32)
        o = 0
        for s, im in enumerate(imgs):
            im = np.ascontiguousarray(im, dtype=np.uint8)
            if im.ndim != 3 or im.shape[2] != 3:
                raise ValueError("ECC needs (h, w, 3) BGR uint8 frames")
            frames.append(im.reshape(-1))
            off[s] = o
            hw[2 * s], hw[2 * s + 1] = im.shape[0], im.shape[1]
            o += im.size
        packed = np.concatenate(frames) if len(frames) > 1 else frames[0]
        _lib.check(self.lib.yta_ecc_apply(self._h, _lib.ptr(packed), _lib.ptr(off), _lib.ptr(hw),
                                          _lib.ptr(self._warps)))
        return self._warps.reshape(self.n_streams, 2, 3).copy()

    def outcome(self):
        """Per stream (outcome, iterations, rho): outcome 0 first frame, 1 estimated, 2 identity
        (findTransformECC would have raised)."""
        out = np.zeros(self.n_streams, np.int32)
        iters = np.zeros(self.n_streams, np.int32)
        rho = np.zeros(self.n_streams, np.float64)
        _lib.check(self.lib.yta_ecc_outcome(self._h, _lib.ptr(out), _lib.ptr(iters),
                                            _lib.ptr(rho)))
        return out, iters, rho

    def aligned(self, stream=0):
        """align=True's preview (ecc.py:91-98): the stream's previous gray frame warped by the
        last returned matrix (cv2.warpAffine INTER_LINEAR), or None when the last apply was not
        an estimate (first frame / identity because OpenCV would have raised)."""
        hh, ww = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.yta_ecc_aligned(self._h, int(stream), None, 0, ctypes.byref(hh),
                                            ctypes.byref(ww)))
        if hh.value == 0:
            return None
        img = np.zeros((hh.value, ww.value), np.uint8)
        _lib.check(self.lib.yta_ecc_aligned(self._h, int(stream), _lib.ptr(img), img.size,
                                            ctypes.byref(hh), ctypes.byref(ww)))
        return img

    def state(self, stream=0, with_image=False):
        init, hh, ww = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.yta_ecc_get_state(self._h, int(stream), ctypes.byref(init),
                                              ctypes.byref(hh), ctypes.byref(ww), None, 0))
        st = {"initialized": bool(init.value)}
        if with_image and init.value:
            img = np.zeros((hh.value, ww.value), np.uint8)
            _lib.check(self.lib.yta_ecc_get_state(self._h, int(stream), ctypes.byref(init),
                                                  ctypes.byref(hh), ctypes.byref(ww),
                                                  _lib.ptr(img), img.size))
            st["prev_img"] = img
        return st


class ECC:
    """Drop-in for boxmot.motion.cmc.ecc.ECC (ecc.py:13-57): same constructor arguments,
    `apply(img, dets) -> 2x3 float32` (dets unused, as in the reference).  align=True keeps the
    previous gray frame warped by each estimate in `prev_img_aligned` (ecc.py:91-98, warped on the
    device: yta_ecc_aligned), None with align=False; MOTION_HOMOGRAPHY and grayscale=False are
    refused."""

    def __init__(self, warp_mode=MOTION_EUCLIDEAN, eps=1e-5, max_iter=100, scale=0.1, align=False,
                 grayscale=True, device=0):
        if warp_mode == MOTION_HOMOGRAPHY or warp_mode not in (0, 1, 2):
            raise NotImplementedError("ECC(warp_mode=MOTION_HOMOGRAPHY): only translation, "
                                      "euclidean and affine models are on the MI355X path")
        if not grayscale:
            raise NotImplementedError("ECC(grayscale=False): findTransformECC needs one channel")
        if scale is None or not 0 < scale <= 1:
            raise ValueError("ECC(scale): a resize factor in (0, 1] (ecc.py:87 compares it to 1)")
        self.warp_mode = warp_mode
        self.termination_criteria = (3, max_iter, eps)   # TERM_CRITERIA_EPS | COUNT
        self.scale = scale
        self.align = align
        self.grayscale = grayscale
        self.prev_img_aligned = None
        self._device = device
        self._engine = None

    def apply(self, img, dets=None):
        img = np.asarray(img)
        if self._engine is None:
            _, max_iter, eps = self.termination_criteria
            self._engine = EccEngine(1, self.warp_mode, eps, max_iter, self.scale, self._device,
                                     img.shape[0], img.shape[1])
        warp = self._engine.apply([img])[0]
        if self.align:   # after an estimate only: the other paths return before ecc.py:91
            aligned = self._engine.aligned(0)
            if aligned is not None:
                self.prev_img_aligned = aligned
        return warp
