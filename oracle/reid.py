"""CPU restatement of BoxMOT's ReID crop preprocessing and feature normalisation.

TEST INFRASTRUCTURE: the checker for yta_reid_* (tests/, tools/bench_reid.py's cpu leg).  The
product path never imports this module.

Follows boxmot/appearance/reid_multibackend.py:
  * preprocess (:189-224): per box `box.astype('int')` (truncation), x1/y1 clamped below at 0,
    x2/y2 clamped above at w-1 / h-1, `img[y1:y2, x1:x2]` with Python slice semantics (a negative
    stop wraps), `cv2.resize(crop, (128, 256), INTER_LINEAR)`, BGR -> RGB, `/ 255`, `- mean`,
    `/ std` in float64, `.float()`, stacked and permuted to (N, 3, H, W);
  * get_features (:303-311): `features / np.linalg.norm(features)` (one Frobenius norm over the
    whole (N, D) batch).

cv2.resize(INTER_LINEAR) on uint8 is OpenCV's fixed-point bilinear (imgproc/src/resize.cpp,
resizeGeneric_ with HResizeLinear + VResizeLinear, INTER_RESIZE_COEF_BITS = 11), restated here from
its published source (OpenCV 4.x; the reference pins `opencv-python>=4.6.0`, requirements.txt):
  x: fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor(fx), fx -= sx; sx < 0 -> (sx, fx) = (0, 0);
     sx >= W-1 -> (sx, fx) = (W-1, 0); alpha = (rint((1 - fx) * 2048), rint(fx * 2048)) as short;
     row value D = S[sx] * a0 + S[sx+1] * a1 (D = S[W-1] * 2048 on the right border)
  y: fy likewise but without border adjustment; the two source rows are clamped to [0, H-1];
     out = ((D0 >> 4) * b0 >> 16) + ((D1 >> 4) * b1 >> 16) + 2 >> 2, saturated to u8 (the SIMD row
     kernel VResizeLinearVec_32s8u, which covers every element when 3 * out_w is a multiple of the
     vector width, as at the reference's 128-wide crops)
  scale_x = 1 / (out_w / W) (double); both scale factors exactly 2 -> INTER_AREA fast path:
     (S00 + S01 + S10 + S11 + 2) >> 2.
OpenCV is not installed in this container, so the resize step is PARITY UNPINNED against cv2
itself; the restatement is cross-checked against a float bilinear of the same sampling grid
(within one u8 level, tests/test_reid_cpu.py).  The float steps after the resize are NumPy's own
arithmetic and are bit-exact.
"""
import numpy as np

MEAN = np.array([0.485, 0.456, 0.406])   # reid_multibackend.py:214 (RGB order)
STD = np.array([0.229, 0.224, 0.225])    # :215
COEF = 2048                              # INTER_RESIZE_COEF_SCALE


def crop_rect(box, h, w):
    """(y0, y1, x0, x1) of img[y1:y2, x1:x2] as reid_multibackend.py:193-199 slices it."""
    x1, y1, x2, y2 = np.asarray(box, dtype=np.float64).astype("int")
    x1 = max(0, x1)
    y1 = max(0, y1)
    x2 = min(w - 1, x2)
    y2 = min(h - 1, y2)
    ys = range(h)[y1:y2]
    xs = range(w)[x1:x2]
    return (ys.start, ys.stop, xs.start, xs.stop) if len(ys) and len(xs) else None


def _axis(ssize, dsize, inv_scale=None):
    # resizeGeneric: scale = 1 / inv_scale, inv_scale = dsize / ssize unless the caller gave fx/fy
    inv = np.float64(dsize) / np.float64(ssize) if inv_scale is None else np.float64(inv_scale)
    scale = 1.0 / inv
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    return s, f, scale


def _sat_short(v):
    return np.rint(v.astype(np.float32)).astype(np.int64)


def resize_linear_u8(crop, out_w, out_h, fx=None, fy=None):
    """cv2.resize(crop, (out_w, out_h), interpolation=cv2.INTER_LINEAR) for an (H, W, C) uint8;
    fx / fy: the scale factors of cv2.resize(crop, (0, 0), fx=, fy=) (out_w / out_h then
    round(W * fx) / round(H * fy))."""
    crop = np.asarray(crop, dtype=np.uint8)
    H, W = crop.shape[:2]
    sx, fx, scx = _axis(W, out_w, fx)
    sy, fy, scy = _axis(H, out_h, fy)
    src = crop.astype(np.int64)
    if abs(scx - 2.0) < np.finfo(np.float64).eps and abs(scy - 2.0) < np.finfo(np.float64).eps:
        s = (src[0:2 * out_h:2, 0:2 * out_w:2] + src[0:2 * out_h:2, 1:2 * out_w:2]
             + src[1:2 * out_h:2, 0:2 * out_w:2] + src[1:2 * out_h:2, 1:2 * out_w:2])
        return ((s + 2) >> 2).astype(np.uint8)
    right = sx >= W - 1
    left = sx < 0
    fx = np.where(left | right, np.float32(0), fx).astype(np.float32)
    sx = np.where(left, 0, np.where(right, W - 1, sx))
    a0 = _sat_short((np.float32(1) - fx) * np.float32(COEF))
    a1 = _sat_short(fx * np.float32(COEF))
    sx1 = np.minimum(sx + 1, W - 1)
    # horizontal pass on every source row: (H, out_w, C) int
    rows = src[:, sx, :] * a0[None, :, None] + src[:, sx1, :] * a1[None, :, None]
    rows = np.where(right[None, :, None], src[:, sx, :] * COEF, rows)
    b0 = _sat_short((np.float32(1) - fy) * np.float32(COEF))
    b1 = _sat_short(fy * np.float32(COEF))
    r0 = rows[np.clip(sy, 0, H - 1)]
    r1 = rows[np.clip(sy + 1, 0, H - 1)]
    v = (((r0 >> 4) * b0[:, None, None]) >> 16) + (((r1 >> 4) * b1[:, None, None]) >> 16)
    return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)


def preprocess(xyxys, img, out_w=128, out_h=256, fp16=False):
    """ReIDDetectMultiBackend.preprocess (reid_multibackend.py:189-224) -> (N, 3, out_h, out_w)
    float32 (float16 if fp16) as a NumPy array.  An empty crop raises ValueError (cv2.resize
    asserts `!ssize.empty()`)."""
    h, w = img.shape[:2]
    crops = []
    for i, box in enumerate(np.asarray(xyxys)):
        r = crop_rect(box, h, w)
        if r is None:
            raise ValueError(f"box {i}: empty crop")
        y0, y1, x0, x1 = r
        c = resize_linear_u8(img[y0:y1, x0:x1], out_w, out_h)
        c = c[..., ::-1]                                   # BGR -> RGB
        c = c / 255
        c = c - MEAN
        c = c / STD
        crops.append(c.astype(np.float32))
    out = np.stack(crops).transpose(0, 3, 1, 2)
    return np.ascontiguousarray(out.astype(np.float16) if fp16 else out)


def bilinear_float(crop, out_w, out_h):
    """Independent float bilinear on OpenCV's sampling grid (edge-clamped), rounded to u8: the
    cross-check for resize_linear_u8 (agreement within one u8 level)."""
    crop = np.asarray(crop, dtype=np.float64)
    H, W = crop.shape[:2]
    x = np.clip((np.arange(out_w) + 0.5) * (W / out_w) - 0.5, 0, W - 1)
    y = np.clip((np.arange(out_h) + 0.5) * (H / out_h) - 0.5, 0, H - 1)
    x0 = np.floor(x).astype(int)
    y0 = np.floor(y).astype(int)
    x1 = np.minimum(x0 + 1, W - 1)
    y1 = np.minimum(y0 + 1, H - 1)
    fx = (x - x0)[None, :, None]
    fy = (y - y0)[:, None, None]
    top = crop[y0][:, x0] * (1 - fx) + crop[y0][:, x1] * fx
    bot = crop[y1][:, x0] * (1 - fx) + crop[y1][:, x1] * fx
    return np.clip(np.rint(top * (1 - fy) + bot * fy), 0, 255).astype(np.uint8)


def global_normalize(features):
    """get_features' `features / np.linalg.norm(features)` (reid_multibackend.py:310)."""
    f = np.asarray(features, dtype=np.float32)
    return f / np.linalg.norm(f)
