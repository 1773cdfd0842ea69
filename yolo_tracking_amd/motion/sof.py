"""SparseOptFlow camera-motion compensation on the MI355X.

Reference: boxmot/motion/cmc/sof.py:15-162 (SparseOptFlow: __init__, apply), cmc_interface.py:13-40
(generate_mask, preprocess).  `SparseOptFlow().apply(img, dets)` returns the reference's 2x3
float64 warp; the work runs in csrc/cmc.hip (gray + resize, goodFeaturesToTrack on the first frame,
pyramidal Lucas-Kanade, RANSAC + LM similarity fit) through the C ABI.  `SofEngine` runs S camera
streams per call (every stream's frame in the same launches); its device form writes the S warps
straight into a device buffer that yta_botsort_update_device / yta_deepocsort_update_device read.
There is no CPU fallback: without the HIP library or a device this raises YTAError.
"""
import ctypes

import numpy as np

from .. import _lib


class SofEngine:
    """S independent SparseOptFlow estimators sharing one device engine."""

    def __init__(self, n_streams=1, scale=0.1, device=0, max_h=1080, max_w=1920):
        self.lib = _lib.load_library()
        self.n_streams = int(n_streams)
        self.scale = float(scale)
        self.device = _lib.parse_device(device)
        h = ctypes.c_void_p()
        _lib.check(self.lib.yta_sof_create(self.device, self.n_streams, self.scale, int(max_h),
                                           int(max_w), ctypes.byref(h)))
        self._h = h
        self._warps = np.zeros((self.n_streams, 6), dtype=np.float64)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.yta_sof_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _lib.check(self.lib.yta_sof_reset(self._h))

    def apply(self, imgs, dets_per_stream):
        """imgs: S (h, w, 3) uint8 BGR frames; dets_per_stream: S (n, >= 4) arrays whose first
        four columns are x1 y1 x2 y2 (the rows the tracker passes to cmc.apply).  Returns
        (S, 2, 3) float64 warps."""
        assert len(imgs) == self.n_streams and len(dets_per_stream) == self.n_streams
        frames, off, hw = [], np.zeros(self.n_streams, np.int64), np.zeros(2 * self.n_streams,
                                                                           np.int32)
        o = 0
        for s, im in enumerate(imgs):
            im = np.ascontiguousarray(im, dtype=np.uint8)
            if im.ndim != 3 or im.shape[2] != 3:
                raise ValueError("SparseOptFlow needs (h, w, 3) BGR uint8 frames")
            frames.append(im.reshape(-1))
            off[s] = o
            hw[2 * s], hw[2 * s + 1] = im.shape[0], im.shape[1]
            o += im.size
        packed = np.concatenate(frames) if len(frames) > 1 else frames[0]
        rows = [np.asarray(d, dtype=np.float64).reshape(len(d), -1)[:, :4] if len(d)
                else np.zeros((0, 4)) for d in dets_per_stream]
        doff = np.zeros(self.n_streams + 1, np.int32)
        np.cumsum([len(r) for r in rows], out=doff[1:])
        dets = np.ascontiguousarray(np.concatenate(rows)) if doff[-1] else np.zeros((1, 4))
        _lib.check(self.lib.yta_sof_apply(self._h, _lib.ptr(packed), _lib.ptr(off), _lib.ptr(hw),
                                          _lib.ptr(dets), 4, _lib.ptr(doff),
                                          _lib.ptr(self._warps)))
        return self._warps.reshape(self.n_streams, 2, 3).copy()

    def outcome(self):
        """Per stream: 0 first frame, 1 estimated, 2 identity (see yta_sof_outcome)."""
        out = np.zeros(self.n_streams, np.int32)
        _lib.check(self.lib.yta_sof_outcome(self._h, _lib.ptr(out)))
        return out

    def state(self, stream=0, with_image=False):
        init, n, hh, ww = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        kp = np.zeros((3000, 2), np.float32)
        _lib.check(self.lib.yta_sof_get_state(self._h, int(stream), ctypes.byref(init),
                                              ctypes.byref(n), _lib.ptr(kp), len(kp),
                                              ctypes.byref(hh), ctypes.byref(ww), None, 0))
        st = {"initialized": bool(init.value), "keypoints": kp[:n.value].copy()}
        if with_image and init.value:
            img = np.zeros((hh.value, ww.value), np.uint8)
            _lib.check(self.lib.yta_sof_get_state(self._h, int(stream), ctypes.byref(init),
                                                  ctypes.byref(n), None, 0, ctypes.byref(hh),
                                                  ctypes.byref(ww), _lib.ptr(img), img.size))
            st["prev_img"] = img
        return st


class SparseOptFlow:
    """Drop-in for boxmot.motion.cmc.sof.SparseOptFlow (sof.py:15-61): same constructor
    arguments (warp_mode / eps / max_iter / align / grayscale / draw_optical_flow are accepted
    and, as in the reference, unused by apply), `apply(img, dets) -> 2x3 float64`."""

    def __init__(self, warp_mode=None, eps=1e-5, max_iter=100, scale=0.1, align=False,
                 grayscale=True, draw_optical_flow=False, device=0):
        if not grayscale:
            raise NotImplementedError("SparseOptFlow(grayscale=False): cvtColor is skipped and "
                                      "goodFeaturesToTrack would receive a 3-channel frame")
        self.scale = scale
        self.align = align
        self.grayscale = grayscale
        self.draw_optical_flow = draw_optical_flow
        self._device = device
        self._engine = None

    def apply(self, img, dets):
        img = np.asarray(img)
        if self._engine is None:
            self._engine = SofEngine(1, self.scale, self._device, img.shape[0], img.shape[1])
        d = np.zeros((0, 4)) if dets is None else np.asarray(dets, dtype=np.float64)
        return self._engine.apply([img], [d])[0]
