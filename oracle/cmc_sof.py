"""CPU restatement of BoxMOT's SparseOptFlow camera-motion estimator.

TEST INFRASTRUCTURE: the checker for yta_sof_* (tests/, tools/bench_cmc.py's cpu leg).  The
product path never imports this module.

Reference: boxmot/motion/cmc/sof.py:64-162 (SparseOptFlow.apply) and cmc_interface.py:13-40
(generate_mask, preprocess); BoTSORT builds SparseOptFlow() (bot_sort.py:228) and calls
apply(img, dets_first) every frame (:293), DeepOCSort builds get_cmc_method('sof')()
(deep_ocsort.py:351) and calls apply(img, dets[:, :4]) (:391).

The arithmetic lives in OpenCV (opencv-python>=4.6.0, requirements.txt; unpinned and NOT
installed here): cvtColor(BGR2GRAY), resize(INTER_LINEAR, fx=fy=scale), goodFeaturesToTrack
(cornerMinEigenVal + threshold + dilate + sort), calcOpticalFlowPyrLK (buildOpticalFlowPyramid,
Scharr derivatives, the fixed-point LKTrackerInvoker) and estimateAffinePartial2D(RANSAC) with its
Levenberg-Marquardt refinement.  They are restated from OpenCV's published algorithms.  PARITY IS
UNPINNED against cv2 itself (no cv2 here, no fixture in the reference holds CMC outputs).  Where
OpenCV's own bits depend on its SIMD lane layout, this restatement fixes one exact order, named in
each function, that the GPU (csrc/cmc.hip) reproduces bit for bit:
  * Sobel / box filter / min-eigenvalue: float32 products in the order written below, the 3x3 box
    sum of the float32 covariance terms in float64 (OpenCV's sumType for float input), rows then
    columns, rounded to float32 once;
  * LK window sums: exact integer sums (OpenCV accumulates in float or int32 SIMD lanes);
  * RANSAC: OpenCV's RNG (multiply-with-carry, seed (uint64)-1), subsets, 2-point similarity,
    float32 reprojection errors, adaptive iteration count;
  * LM refinement: the classic cv::LMSolver iteration (lambda halving / nu growth, 10 iterations)
    with Cholesky solves, every sum over points in the fixed 256-way order of reduce256().
The restatement is validated on its own terms by recovering known camera motions from textured
frames and MOT17-mini images (tests/test_cmc_cpu.py).
"""
import math

import numpy as np

from .reid import resize_linear_u8

F32 = np.float32
WIN = 21                      # calcOpticalFlowPyrLK winSize default (21, 21)
MAX_LEVEL = 3                 # maxLevel default
LK_ITERS = 30                 # TermCriteria(COUNT | EPS, 30, 0.01)
LK_EPS = 0.01
LK_MIN_EIG = F32(1e-4)        # minEigThreshold default
FLT_EPSILON = F32(np.finfo(np.float32).eps)
DBL_EPSILON = np.finfo(np.float64).eps
DBL_MIN = np.finfo(np.float64).tiny
MAX_CORNERS = 3000            # sof.py:83-91
QUALITY = 0.01
RANSAC_THRESH = 3.0           # estimateAffinePartial2D defaults
RANSAC_ITERS = 2000
RANSAC_CONF = 0.99
REFINE_ITERS = 10


# ------------------------------------------------------------------------------ preprocessing
def bgr2gray(img):
    """cvtColor(COLOR_BGR2GRAY) on uint8: fixed point, 14-bit coefficients."""
    img = np.asarray(img, dtype=np.uint8)
    b = img[..., 0].astype(np.int32)
    g = img[..., 1].astype(np.int32)
    r = img[..., 2].astype(np.int32)
    return ((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14).astype(np.uint8)


def small_size(h, w, scale):
    """cv2.resize(img, (0, 0), fx=scale, fy=scale): dsize = (round(w * fx), round(h * fy))."""
    return int(np.rint(h * scale)), int(np.rint(w * scale))


def preprocess(img, scale=0.1):
    """CMCInterface.preprocess (cmc_interface.py:27-40): gray, then resize by `scale`."""
    g = bgr2gray(img)
    if scale is None:
        return g
    oh, ow = small_size(g.shape[0], g.shape[1], scale)
    return resize_linear_u8(g[..., None], ow, oh, fx=scale, fy=scale)[..., 0]


def generate_mask(img, dets, scale):
    """CMCInterface.generate_mask (cmc_interface.py:13-24), NumPy slicing semantics kept."""
    h, w = img.shape
    mask = np.zeros_like(img)
    mask[int(0.02 * h): int(0.98 * h), int(0.02 * w): int(0.98 * w)] = 255
    if dets is not None:
        for det in dets:
            tlbr = np.multiply(det, scale).astype(int)
            mask[tlbr[1]:tlbr[3], tlbr[0]:tlbr[2]] = 0
    return mask


# ------------------------------------------------------------------------------ borders
def refl101(i, n):
    """borderInterpolate(i, n, BORDER_REFLECT_101) for an integer array i."""
    i = np.asarray(i, dtype=np.int64)
    if n == 1:
        return np.zeros_like(i)
    i = i.copy()
    while True:
        lo = i < 0
        hi = i >= n
        if not (lo.any() or hi.any()):
            return i
        i = np.where(lo, -i, i)
        i = np.where(hi, 2 * (n - 1) - i, i)


# ------------------------------------------------------------------------------ corners
def min_eigen(gray):
    """cornerMinEigenVal(gray, blockSize=3, ksize=3) -> float32 (h, w).

    Sobel(CV_32F, scale = 1 / (2^(3-1) * 3 * 255)) with the scale folded into the smoothing
    kernel [k0, k1, k0] = [s, 2s, s] (float32), reflect-101 borders:
      dx = r1 * k1 + (r0 + r2) * k0,   r = s(x+1) - s(x-1)          (column smoothing of row diffs)
      dy = q(y+1) - q(y-1),            q = s * k1 + (s(x-1) + s(x+1)) * k0
    cov = (dx*dx, dx*dy, dy*dy); box 3x3 (unnormalised, reflect-101) summed in float64 as
    ((left + centre) + right) per row, then ((up + centre) + down), rounded to float32;
    lambda_min = (a + c) - sqrt((a - c)^2 + b^2) with a = cov0 / 2, b = cov1, c = cov2 / 2."""
    g = np.asarray(gray, dtype=np.uint8)
    h, w = g.shape
    s = g.astype(F32)
    scale = 1.0 / (4 * 3 * 255)
    k0 = F32(1.0 * scale)
    k1 = F32(2.0 * scale)
    xm, xp = refl101(np.arange(w) - 1, w), refl101(np.arange(w) + 1, w)
    ym, yp = refl101(np.arange(h) - 1, h), refl101(np.arange(h) + 1, h)
    r = s[:, xp] - s[:, xm]
    dx = r * k1 + (r[ym] + r[yp]) * k0
    q = s * k1 + (s[:, xm] + s[:, xp]) * k0
    dy = q[yp] - q[ym]
    cov = [dx * dx, dx * dy, dy * dy]
    box = []
    for c in cov:
        c64 = c.astype(np.float64)
        rs = (c64[:, xm] + c64) + c64[:, xp]
        box.append(((rs[ym] + rs) + rs[yp]).astype(F32))
    a = box[0] * F32(0.5)
    b = box[1]
    c = box[2] * F32(0.5)
    return (a + c) - np.sqrt((a - c) * (a - c) + b * b)


def good_features(gray, mask, max_corners=MAX_CORNERS, quality=QUALITY):
    """goodFeaturesToTrack(gray, mask, maxCorners, qualityLevel, minDistance=1, blockSize=3,
    useHarrisDetector=False) -> float32 (N, 2) [x, y], or None when nothing is found.

    threshold(eig, maxVal * quality, TOZERO) with maxVal = max over mask != 0 (float32 compare
    against the double product cast to float32); 3x3 dilation (out-of-image ignored); candidates
    at interior pixels (1 <= x <= w-2, 1 <= y <= h-2) with eig != 0, eig == dilated, mask != 0;
    sorted by eigenvalue descending, ties by raster position descending (greaterThanPtr compares
    addresses); minDistance = 1 removes nothing (only the same pixel is closer than 1)."""
    eig = min_eigen(gray)
    h, w = eig.shape
    m = np.asarray(mask) != 0
    maxv = float(eig[m].max()) if m.any() else 0.0
    thr = F32(maxv * quality)
    e = np.where(eig > thr, eig, F32(0)).astype(F32)
    pad = np.full((h + 2, w + 2), -np.inf, dtype=F32)
    pad[1:-1, 1:-1] = e
    dil = np.max(np.stack([pad[dy:dy + h, dx:dx + w] for dy in range(3) for dx in range(3)]),
                 axis=0)
    cand = (e != 0) & (e == dil) & m
    cand[0, :] = cand[-1, :] = False
    cand[:, 0] = cand[:, -1] = False
    ys, xs = np.nonzero(cand)
    if len(ys) == 0:
        return None
    idx = ys.astype(np.int64) * w + xs
    vals = e[ys, xs]
    order = np.lexsort((-idx, -vals.astype(np.float64)))[:max_corners]
    return np.stack([xs[order], ys[order]], axis=1).astype(F32)


# ------------------------------------------------------------------------------ pyramids
_K5 = np.array([1, 4, 6, 4, 1], dtype=np.int64)


def pyr_down(img):
    """pyrDown on uint8: 5x5 [1 4 6 4 1]^2 / 256, reflect-101, (sum + 128) >> 8, size
    ((w + 1) / 2, (h + 1) / 2)."""
    img = np.asarray(img, dtype=np.uint8)
    h, w = img.shape
    oh, ow = (h + 1) // 2, (w + 1) // 2
    src = img.astype(np.int64)
    cx = refl101(2 * np.arange(ow)[:, None] + np.arange(-2, 3)[None, :], w)   # (ow, 5)
    cy = refl101(2 * np.arange(oh)[:, None] + np.arange(-2, 3)[None, :], h)
    rows = (src[:, cx] * _K5[None, None, :]).sum(axis=2)                       # (h, ow)
    out = (rows[cy] * _K5[None, :, None]).sum(axis=1)                          # (oh, ow)
    return ((out + 128) >> 8).astype(np.uint8)


def build_pyramid(img, win=WIN, max_level=MAX_LEVEL):
    """buildOpticalFlowPyramid(img, winSize, maxLevel, withDerivatives=False): levels until the
    next level would have a side <= win."""
    levels = [np.asarray(img, dtype=np.uint8)]
    h, w = levels[0].shape
    for level in range(max_level + 1):
        if level != 0:
            levels.append(pyr_down(levels[-1]))
            h, w = levels[-1].shape
        h, w = (h + 1) // 2, (w + 1) // 2
        if w <= win or h <= win:
            return levels
    return levels


def scharr_deriv(img):
    """calcSharrDeriv: int16 (h, w, 2) = (Ix, Iy); vertical (3, 10, 3) smoothing then horizontal
    difference for Ix, vertical difference then horizontal (3, 10, 3) for Iy, reflect-101."""
    s = np.asarray(img, dtype=np.int64)
    h, w = s.shape
    ym, yp = refl101(np.arange(h) - 1, h), refl101(np.arange(h) + 1, h)
    xm, xp = refl101(np.arange(w) - 1, w), refl101(np.arange(w) + 1, w)
    t0 = (s[ym] + s[yp]) * 3 + s * 10
    t1 = s[yp] - s[ym]
    ix = t0[:, xp] - t0[:, xm]
    iy = (t1[:, xp] + t1[:, xm]) * 3 + t1 * 10
    return np.stack([ix, iy], axis=2).astype(np.int16)


# ------------------------------------------------------------------------------ Lucas-Kanade
W_BITS = 14
FLT_SCALE = F32(1.0 / (1 << 20))


def _descale(x, n):
    return (x + (1 << (n - 1))) >> n


def _weights(px, py):
    """Bilinear weights of the fixed-point sampler: (iw00, iw01, iw10, iw11) int64 arrays."""
    ix = np.floor(px).astype(np.int64)
    iy = np.floor(py).astype(np.int64)
    a = (px - ix.astype(F32)).astype(F32)
    b = (py - iy.astype(F32)).astype(F32)
    one = F32(1)
    sc = F32(1 << W_BITS)
    iw00 = np.rint((one - a) * (one - b) * sc).astype(np.int64)
    iw01 = np.rint(a * (one - b) * sc).astype(np.int64)
    iw10 = np.rint((one - a) * b * sc).astype(np.int64)
    iw11 = (1 << W_BITS) - iw00 - iw01 - iw10
    return ix, iy, iw00, iw01, iw10, iw11


def _window(arr, ix, iy, win, border):
    """(n, win+1, win+1, ...) samples of arr at rows iy..iy+win, cols ix..ix+win; border
    'reflect' (pyramid images) or 'zero' (derivative images)."""
    h, w = arr.shape[:2]
    ry = iy[:, None] + np.arange(win + 1)[None, :]
    rx = ix[:, None] + np.arange(win + 1)[None, :]
    if border == "reflect":
        return arr[refl101(ry, h)[:, :, None], refl101(rx, w)[:, None, :]]
    ok = ((ry >= 0) & (ry < h))[:, :, None] & ((rx >= 0) & (rx < w))[:, None, :]
    v = arr[np.clip(ry, 0, h - 1)[:, :, None], np.clip(rx, 0, w - 1)[:, None, :]]
    if v.ndim == 4:
        ok = ok[..., None]
    return np.where(ok, v, 0)


def _bilinear(win_arr, iw00, iw01, iw10, iw11, n_out, shift):
    w00 = iw00[:, None, None]
    w01 = iw01[:, None, None]
    w10 = iw10[:, None, None]
    w11 = iw11[:, None, None]
    v = win_arr.astype(np.int64)
    return _descale(v[:, :n_out, :n_out] * w00 + v[:, :n_out, 1:n_out + 1] * w01 +
                    v[:, 1:n_out + 1, :n_out] * w10 + v[:, 1:n_out + 1, 1:n_out + 1] * w11, shift)


def lk_track(prev_levels, next_levels, pts, win=WIN, max_iter=LK_ITERS, eps=LK_EPS):
    """calcOpticalFlowPyrLK(prev, next, pts, None) with the default winSize 21, maxLevel 3,
    criteria (COUNT | EPS, 30, 0.01), flags 0, minEigThreshold 1e-4 -> (next_pts float32 (n, 2),
    status uint8 (n,)).  The level count is min of the two pyramids' (buildOpticalFlowPyramid)."""
    pts = np.asarray(pts, dtype=F32).reshape(-1, 2)
    n = len(pts)
    status = np.ones(n, dtype=np.uint8)
    nxt = np.zeros((n, 2), dtype=F32)
    max_level = min(len(prev_levels), len(next_levels)) - 1
    half = F32((win - 1) * 0.5)
    eps2 = eps * eps
    for level in range(max_level, -1, -1):
        I = prev_levels[level]
        J = next_levels[level]
        dI = scharr_deriv(I)
        h, w = I.shape
        jh, jw = J.shape
        prev = (pts * F32(1.0 / (1 << level))).astype(F32)
        cur = prev.copy() if level == max_level else (nxt * F32(2)).astype(F32)
        nxt = cur.copy()
        p = (prev - half).astype(F32)
        ipx = np.floor(p[:, 0]).astype(np.int64)
        ipy = np.floor(p[:, 1]).astype(np.int64)
        live = ~((ipx < -win) | (ipx >= w) | (ipy < -win) | (ipy >= h))
        if level == 0:
            status[~live] = 0
        ids = np.nonzero(live)[0]
        if len(ids) == 0:
            continue
        ix, iy, w00, w01, w10, w11 = _weights(p[ids, 0], p[ids, 1])
        ival = _bilinear(_window(I, ix, iy, win, "reflect"), w00, w01, w10, w11, win, W_BITS - 5)
        dwin = _window(dI, ix, iy, win, "zero")
        ixv = _bilinear(dwin[..., 0], w00, w01, w10, w11, win, W_BITS)
        iyv = _bilinear(dwin[..., 1], w00, w01, w10, w11, win, W_BITS)
        a11 = F32((ixv * ixv).sum(axis=(1, 2))) * FLT_SCALE
        a12 = F32((ixv * iyv).sum(axis=(1, 2))) * FLT_SCALE
        a22 = F32((iyv * iyv).sum(axis=(1, 2))) * FLT_SCALE
        a11, a12, a22 = a11.astype(F32), a12.astype(F32), a22.astype(F32)
        D = (a11 * a22 - a12 * a12).astype(F32)
        min_eig = ((a22 + a11 - np.sqrt((a11 - a22) * (a11 - a22) + F32(4) * a12 * a12))
                   / F32(2 * win * win)).astype(F32)
        bad = (min_eig < LK_MIN_EIG) | (D < FLT_EPSILON)
        if level == 0:
            status[ids[bad]] = 0
        keep = ~bad
        ids, ival, ixv, iyv = ids[keep], ival[keep], ixv[keep], iyv[keep]
        a11, a12, a22 = a11[keep], a12[keep], a22[keep]
        D = (F32(1) / D[keep]).astype(F32)
        q = (cur[ids] - half).astype(F32)
        pdx = np.zeros(len(ids), dtype=F32)
        pdy = np.zeros(len(ids), dtype=F32)
        act = np.ones(len(ids), dtype=bool)
        for j in range(max_iter):
            k = np.nonzero(act)[0]
            if len(k) == 0:
                break
            jx = np.floor(q[k, 0]).astype(np.int64)
            jy = np.floor(q[k, 1]).astype(np.int64)
            out = (jx < -win) | (jx >= jw) | (jy < -win) | (jy >= jh)
            if level == 0:
                status[ids[k[out]]] = 0
            act[k[out]] = False
            k = k[~out]
            if len(k) == 0:
                break
            jx, jy, v00, v01, v10, v11 = _weights(q[k, 0], q[k, 1])
            jval = _bilinear(_window(J, jx, jy, win, "reflect"), v00, v01, v10, v11, win, W_BITS - 5)
            diff = jval - ival[k]
            b1 = (F32((diff * ixv[k]).sum(axis=(1, 2))) * FLT_SCALE).astype(F32)
            b2 = (F32((diff * iyv[k]).sum(axis=(1, 2))) * FLT_SCALE).astype(F32)
            dx = ((a12[k] * b2 - a22[k] * b1) * D[k]).astype(F32)
            dy = ((a12[k] * b1 - a11[k] * b2) * D[k]).astype(F32)
            q[k, 0] = (q[k, 0] + dx).astype(F32)
            q[k, 1] = (q[k, 1] + dy).astype(F32)
            nxt[ids[k], 0] = (q[k, 0] + half).astype(F32)
            nxt[ids[k], 1] = (q[k, 1] + half).astype(F32)
            small = dx.astype(np.float64) * dx + dy.astype(np.float64) * dy <= eps2
            osc = np.zeros(len(k), dtype=bool)
            if j > 0:   # std::abs(float) < 0.01 compares in double
                osc = (np.abs((dx + pdx[k]).astype(F32)).astype(np.float64) < 0.01) & \
                      (np.abs((dy + pdy[k]).astype(F32)).astype(np.float64) < 0.01) & ~small
                o = k[osc]
                nxt[ids[o], 0] = (nxt[ids[o], 0] - dx[osc] * F32(0.5)).astype(F32)
                nxt[ids[o], 1] = (nxt[ids[o], 1] - dy[osc] * F32(0.5)).astype(F32)
            act[k[small | osc]] = False
            pdx[k] = dx
            pdy[k] = dy
    return nxt, status


# ------------------------------------------------------------------------------ RANSAC + LM
class CvRNG:
    """cv::RNG: state = (uint64)(unsigned)state * 4164903690 + (state >> 32)."""

    def __init__(self, state=0xFFFFFFFFFFFFFFFF):
        self.state = state if state else 0xFFFFFFFF

    def next(self):
        s = self.state
        self.state = ((s & 0xFFFFFFFF) * 4164903690 + (s >> 32)) & 0xFFFFFFFFFFFFFFFF
        return self.state & 0xFFFFFFFF

    def uniform(self, a, b):
        return a if a == b else (self.next() % (b - a)) + a


def similarity_2pt(f, t):
    """AffinePartial2DEstimatorCallback::runKernel: the exact similarity through two point pairs
    (float32 inputs, float64 arithmetic) -> 2x3 float64."""
    x1, y1 = float(f[0][0]), float(f[0][1])
    x2, y2 = float(f[1][0]), float(f[1][1])
    X1, Y1 = float(t[0][0]), float(t[0][1])
    X2, Y2 = float(t[1][0]), float(t[1][1])
    den = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2)
    d = 1.0 / den if den != 0.0 else math.inf
    S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2))
    S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2))
    S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2)
              - (X1 * x2 - X2 * x1) * (x1 - x2))
    S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2)
              - (Y1 * y2 - Y2 * y1) * (y1 - y2))
    return np.array([[S0, -S1, S2], [S1, S0, S3]])


def reproj_err(M, f, t):
    """Affine2DEstimatorCallback::computeError in float32: ((F0 x + F1 y) + F2) - X, squared sum."""
    F = np.asarray(M, dtype=np.float64).reshape(-1).astype(F32)
    a = (F[0] * f[:, 0] + F[1] * f[:, 1] + F[2] - t[:, 0]).astype(F32)
    b = (F[3] * f[:, 0] + F[4] * f[:, 1] + F[5] - t[:, 1]).astype(F32)
    return (a * a + b * b).astype(F32)


def update_num_iters(p, ep, model_points, max_iters):
    """RANSACUpdateNumIters."""
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, DBL_MIN)
    q = 1.0 - ep
    denom = 1.0 - q * q           # pow(1 - ep, 2)
    if denom < DBL_MIN:
        return 0
    num = math.log(num)
    denom = math.log(denom)
    if denom >= 0 or -num >= max_iters * (-denom):
        return max_iters
    return int(np.rint(num / denom))


def ransac_subsets(count, n_iters=RANSAC_ITERS):
    """The (i0, i1) index pairs getSubset draws for iterations 0..n_iters-1 (the stream of draws
    does not depend on the data: checkSubset never rejects two points)."""
    rng = CvRNG()
    out = np.empty((n_iters, 2), dtype=np.int64)
    for it in range(n_iters):
        i0 = rng.uniform(0, count)
        i1 = rng.uniform(0, count)
        while i1 == i0:
            i1 = rng.uniform(0, count)
        out[it] = (i0, i1)
    return out


def reduce256(v):
    """Sum of a float64 vector in the fixed order the GPU uses: 256 strided partials (element
    e goes to partial e % 256, added in increasing e), then a halving tree (p[i] += p[i + h])."""
    v = np.asarray(v, dtype=np.float64).reshape(-1)
    n = len(v)
    p = np.zeros(256)
    for k in range(0, n, 256):
        seg = v[k:k + 256]
        p[:len(seg)] = p[:len(seg)] + seg
    h = 128
    while h >= 1:
        p = p[:h] + p[h:2 * h]
        h //= 2
    return float(p[0])


def _lm_compute(x, src, dst):
    """AffinePartial2DRefineCallback::compute: residuals (2n,) interleaved (x, y)."""
    Mx = src[:, 0].astype(np.float64)
    My = src[:, 1].astype(np.float64)
    xi = x[0] * Mx - x[1] * My + x[2]
    yi = x[1] * Mx + x[0] * My + x[3]
    r = np.empty(2 * len(src))
    r[0::2] = xi - dst[:, 0].astype(np.float64)
    r[1::2] = yi - dst[:, 1].astype(np.float64)
    return r


def _lm_normal(src, r):
    """A = J^T J (4x4) and v = J^T r for the callback's Jacobian rows (Mx, -My, 1, 0),
    (My, Mx, 0, 1), every sum in reduce256 order over the 2n rows."""
    Mx = src[:, 0].astype(np.float64)
    My = src[:, 1].astype(np.float64)
    n = len(src)
    J = np.zeros((2 * n, 4))
    J[0::2, 0] = Mx
    J[0::2, 1] = -My
    J[0::2, 2] = 1.0
    J[1::2, 0] = My
    J[1::2, 1] = Mx
    J[1::2, 3] = 1.0
    A = np.empty((4, 4))
    for i in range(4):
        for j in range(i, 4):
            A[i, j] = A[j, i] = reduce256(J[:, i] * J[:, j])
    v = np.array([reduce256(J[:, i] * r) for i in range(4)])
    return A, v


def chol_solve4(A, b):
    """Cholesky solve of the 4x4 SPD system A d = b (the restatement's DECOMP_EIG), scalar order."""
    L = [[0.0] * 4 for _ in range(4)]
    for j in range(4):
        s = float(A[j][j])
        for k in range(j):
            s = s - L[j][k] * L[j][k]
        if not s > 0.0:
            return None
        L[j][j] = math.sqrt(s)
        for i in range(j + 1, 4):
            t = float(A[i][j])
            for k in range(j):
                t = t - L[i][k] * L[j][k]
            L[i][j] = t / L[j][j]
    y = [0.0] * 4
    for i in range(4):
        t = float(b[i])
        for k in range(i):
            t = t - L[i][k] * y[k]
        y[i] = t / L[i][i]
    x = [0.0] * 4
    for i in range(3, -1, -1):
        t = y[i]
        for k in range(i + 1, 4):
            t = t - L[k][i] * x[k]
        x[i] = t / L[i][i]
    return np.array(x)


def _dot4(a, b):
    """((a0 b0 + a1 b1) + a2 b2) + a3 b3 in float64 (no BLAS: a fixed order, no FMA)."""
    return ((float(a[0]) * float(b[0]) + float(a[1]) * float(b[1])) + float(a[2]) * float(b[2])) \
        + float(a[3]) * float(b[3])


def lm_refine(x0, src, dst, max_iters=REFINE_ITERS):
    """cv::LMSolver::run on AffinePartial2DRefineCallback (params a, b, tx, ty), epsx = epsf =
    FLT_EPSILON."""
    eps = float(np.finfo(np.float32).eps)
    x = np.asarray(x0, dtype=np.float64).copy()
    r = _lm_compute(x, src, dst)
    S = reduce256(r * r)
    A, v = _lm_normal(src, r)
    D = np.diag(A).copy()
    Rlo, Rhi = 0.25, 0.75
    lam, lc = 1.0, 0.75
    it = 0
    while True:
        Ap = A.copy()
        for i in range(4):
            Ap[i, i] = Ap[i, i] + lam * D[i]
        d = chol_solve4(Ap, v)
        if d is None:
            break
        xd = x - d
        rd = _lm_compute(xd, src, dst)
        Sd = reduce256(rd * rd)
        temp = [-_dot4(A[i], d) + 2.0 * v[i] for i in range(4)]   # gemm(A, d, -1, v, 2)
        dS = _dot4(d, temp)
        R = (S - Sd) / (dS if abs(dS) > DBL_EPSILON else 1.0)
        if R > Rhi:
            lam *= 0.5
            if lam < lc:
                lam = 0.0
        elif R < Rlo:
            t = _dot4(d, v)
            nu = (Sd - S) / (t if abs(t) > DBL_EPSILON else 1.0) + 2.0
            nu = min(max(nu, 2.0), 10.0)
            if lam == 0.0:
                maxval = DBL_EPSILON
                for i in range(4):
                    e = np.zeros(4)
                    e[i] = 1.0
                    col = chol_solve4(A, e)
                    if col is not None:
                        maxval = max(maxval, abs(col[i]))
                lam = lc = 1.0 / maxval
                nu *= 0.5
            lam *= nu
        if Sd < S:
            S = Sd
            x = xd
            r = rd
            A, v = _lm_normal(src, r)
        it += 1
        proceed = it < max_iters and np.max(np.abs(d)) >= eps and np.max(np.abs(r)) >= eps
        if not proceed:
            break
    return x


def estimate_affine_partial(f, t):
    """estimateAffinePartial2D(f, t, RANSAC, 3, 2000, 0.99, 10) -> 2x3 float64 or None."""
    f = np.asarray(f, dtype=F32).reshape(-1, 2)
    t = np.asarray(t, dtype=F32).reshape(-1, 2)
    count = len(f)
    if count < 2:
        return None
    if count == 2:
        return similarity_2pt(f, t)
    subsets = ransac_subsets(count)
    thr = F32(RANSAC_THRESH * RANSAC_THRESH)
    niters = RANSAC_ITERS
    best, best_mask, max_good = None, None, 0
    it = 0
    while it < niters:
        i0, i1 = subsets[it]
        M = similarity_2pt(f[[i0, i1]], t[[i0, i1]])
        mask = reproj_err(M, f, t) <= thr
        good = int(mask.sum())
        if good > max(max_good, 1):
            best, best_mask, max_good = M, mask, good
            niters = update_num_iters(RANSAC_CONF, (count - good) / count, 2, niters)
        it += 1
    if max_good <= 0 or best is None:
        return None
    src, dst = f[best_mask], t[best_mask]
    if len(src) > 0 and REFINE_ITERS:
        x = lm_refine(np.array([best[0, 0], best[1, 0], best[0, 2], best[1, 2]]), src, dst)
        best = np.array([[x[0], -x[1], x[2]], [x[1], x[0], x[3]]])
    return best


# ------------------------------------------------------------------------------ the estimator
class SparseOptFlowOracle:
    """SparseOptFlow(scale=0.1) (sof.py:15-61) .apply(img, dets) (sof.py:64-162), including the
    reference's behaviour that the keypoints are detected once and only ever filtered: `apply`
    stores the tracked positions in `self.prevKeyPoints` (sof.py:155, a different attribute), so
    `prev_keypoints` keeps the first frame's corners, minus every corner LK loses."""

    def __init__(self, scale=0.1):
        self.scale = scale
        self.prev_img = None
        self.prev_keypoints = None
        self.prev_pyr = None

    def apply(self, img, dets):
        H = np.eye(2, 3)
        img = preprocess(img, self.scale)
        mask = generate_mask(img, dets, self.scale)
        if self.prev_img is None:
            kp = good_features(img, mask)
            if kp is None:
                return H
            self.prev_img = img.copy()
            self.prev_pyr = build_pyramid(self.prev_img)
            self.prev_keypoints = kp.copy()
            return H
        if len(self.prev_keypoints) == 0:       # calcOpticalFlowPyrLK returns None outputs
            return H
        if img.shape != self.prev_img.shape:    # calcOpticalFlowPyrLK asserts equal level sizes;
            return H                            # sof.py:105-110 catches it: identity, state kept
        pyr = build_pyramid(img)
        nxt, status = lk_track(self.prev_pyr, pyr, self.prev_keypoints)
        self.prev_keypoints = self.prev_keypoints[status == 1]
        nxt = nxt[status == 1]
        if len(self.prev_keypoints) == 0:       # estimateAffinePartial2D raises (cv2.error)
            return H
        M = estimate_affine_partial(self.prev_keypoints, nxt)
        if M is None:
            return np.eye(2, 3)
        self.prev_img = img.copy()
        self.prev_pyr = pyr
        if self.scale < 1:
            M[0, 2] /= self.scale
            M[1, 2] /= self.scale
        return M
