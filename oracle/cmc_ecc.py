"""CPU restatement of BoxMOT's ECC camera-motion estimator.

TEST INFRASTRUCTURE: the checker for yta_ecc_* (tests/, tools/bench_cmc.py's cpu leg).  The
product path never imports this module.

Reference: boxmot/motion/cmc/ecc.py:13-104 (ECC.__init__ / apply) and cmc_interface.py:26-40
(preprocess); get_cmc_method('ecc') (motion/cmc/__init__.py:9-11) is what HybridSORT builds
(hybridsort.py:366) and StrongSORT uses.  apply() calls cv2.findTransformECC(prev, curr, eye,
warp_mode, (COUNT | EPS, max_iter, eps), None, 1) (ecc.py:73-81), returns the identity when it
raises (ecc.py:82-84, prev_img kept), divides the translation by `scale` (ecc.py:87-89) and keeps
the current frame as prev_img (ecc.py:102).

The arithmetic lives in OpenCV (opencv-python>=4.6.0, unpinned, NOT installed here).  It is
restated from OpenCV's published findTransformECC (imgproc/src/ecc.cpp) with warpAffine's
classic fixed-point path (AB_BITS = 10, INTER_BITS = 5, WARP_INVERSE_MAP, BORDER_CONSTANT 0;
the float32 bilinear table of remap).  PARITY IS UNPINNED against cv2 (no cv2 here and no
reference fixture holds ECC warps).  Where OpenCV's bits depend on its SIMD lanes this restatement
fixes one order that csrc/ecc.hip reproduces:
  * gaussFiltSize = 1 is the identity filter, the all-ones premask survives its rounding, the
    gradients are 0.5 * (I[x+1] - I[x-1]) with reflect-101 borders (exact in float32);
  * bilinear samples of the u8 image and of the gradients are exact in float32 (the table's
    weights are k / 1024), so warped values are order-free;
  * every image sum (meanStdDev's, the Hessian's, the three projections, the correlation) is a
    float64 sum of float32 operands in the fixed order of block_sum(): pixel p belongs to thread
    p % T (T = 1024, 512 for the affine model) which adds its pixels in order, then a halving
    tree over each group of 16 threads and one over the T / 16 group partials;
  * float32 per-pixel arithmetic (zero-mean subtraction, jacobians, the error image) in the order
    written below, no fused multiply-adds;
  * cv::invert (DECOMP_LU) closed forms for 2 x 2 / 3 x 3 (float64 cofactors, stored as float32)
    and hal::LU32f for 6 x 6, gemm with float64 accumulation.
"""
import math

import numpy as np

from .cmc_sof import preprocess

F32 = np.float32
ECC_T = 1024
WAVE = 64
MOTION_TRANSLATION, MOTION_EUCLIDEAN, MOTION_AFFINE, MOTION_HOMOGRAPHY = 0, 1, 2, 3
N_PARAMS = {MOTION_TRANSLATION: 2, MOTION_EUCLIDEAN: 3, MOTION_AFFINE: 6}


def ecc_threads(mode):
    """The device block of a stream: 1024 threads, 512 for the affine model (csrc/ecc.hip)."""
    return 512 if mode == MOTION_AFFINE else ECC_T


AB_BITS, INTER_BITS = 10, 5
AB_SCALE = 1 << AB_BITS
INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1


class ECCError(Exception):
    """cv2.error raised inside findTransformECC (ecc.py:82 catches it)."""


# ------------------------------------------------------------------------------ reductions
def block_sum(v, n_threads=ECC_T):
    """Sum of the last axis of v (float64) in the device's fixed order: thread t accumulates the
    pixels t, t + T, ... in order; a halving tree inside each group of 16 threads; a halving tree
    over the T / 16 group partials (csrc/ecc.hip block_sum)."""
    v = np.asarray(v, dtype=np.float64)
    lead = v.shape[:-1]
    n = v.shape[-1]
    k = max(1, -(-n // n_threads))
    pad = np.zeros(lead + (k * n_threads,))
    pad[..., :n] = v
    rows = pad.reshape(lead + (k, n_threads))
    acc = np.zeros(lead + (n_threads,))
    for r in range(k):
        acc = acc + rows[..., r, :]
    a = acc.reshape(lead + (n_threads // 16, 16))
    while a.shape[-1] > 1:
        h = a.shape[-1] // 2
        a = a[..., :h] + a[..., h:]
    w = a[..., 0]
    while w.shape[-1] > 1:
        h = w.shape[-1] // 2
        w = w[..., :h] + w[..., h:]
    return w[..., 0]


# ------------------------------------------------------------------------------ warpAffine
def cv_round(x):
    """saturate_cast<int>(double): round half to even, saturated to int32."""
    return np.clip(np.rint(x), INT_MIN, INT_MAX).astype(np.int64)


def warp_coords(M, hs, ws):
    """warpAffine's WARP_INVERSE_MAP coordinates (imgwarp.cpp WarpAffineInvoker) for a hs x ws
    output: (sx, sy, alpha index fy * 32 + fx) for INTER_LINEAR and (nx, ny) for INTER_NEAREST,
    both saturated to int16 as the XY map is."""
    M = np.asarray(M, dtype=np.float32).astype(np.float64).ravel()
    x = np.arange(ws, dtype=np.float64)
    y = np.arange(hs, dtype=np.float64)
    adelta = cv_round(M[0] * x * AB_SCALE)
    bdelta = cv_round(M[3] * x * AB_SCALE)
    xr = cv_round((M[1] * y + M[2]) * AB_SCALE)
    yr = cv_round((M[4] * y + M[5]) * AB_SCALE)
    # linear: round_delta = AB_SCALE / INTER_TAB_SIZE / 2
    X = (xr[:, None] + 16 + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (yr[:, None] + 16 + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    alpha = (Y & 31) * 32 + (X & 31)
    # nearest: round_delta = AB_SCALE / 2
    nx = np.clip((xr[:, None] + AB_SCALE // 2 + adelta[None, :]) >> AB_BITS, -32768, 32767)
    ny = np.clip((yr[:, None] + AB_SCALE // 2 + bdelta[None, :]) >> AB_BITS, -32768, 32767)
    return sx, sy, alpha, nx, ny


def bilinear_tab():
    """remap's float32 BilinearTab (initInterTab2D): [vy0 vx0, vy0 vx1, vy1 vx0, vy1 vx1]."""
    t = np.arange(32, dtype=np.float32) * F32(1.0 / 32)
    v = np.stack([F32(1) - t, t], axis=1)                      # interpolateLinear
    tab = np.zeros((32, 32, 4), dtype=np.float32)
    for fy in range(32):
        for fx in range(32):
            tab[fy, fx] = [v[fy, 0] * v[fx, 0], v[fy, 0] * v[fx, 1],
                           v[fy, 1] * v[fx, 0], v[fy, 1] * v[fx, 1]]
    return tab.reshape(1024, 4)


TAB = bilinear_tab()


def remap_linear(src, sx, sy, alpha):
    """remapBilinear (float32, BORDER_CONSTANT 0): ((v00 w0 + v01 w1) + v10 w2) + v11 w3."""
    h, w = src.shape
    w4 = TAB[alpha]

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
        return np.where(ok, src[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)], F32(0))

    v00, v01 = tap(sy, sx), tap(sy, sx + 1)
    v10, v11 = tap(sy + 1, sx), tap(sy + 1, sx + 1)
    r = v00 * w4[..., 0] + v01 * w4[..., 1]
    r = r + v10 * w4[..., 2]
    return (r + v11 * w4[..., 3]).astype(np.float32)


def remap_nearest_ones(h, w, nx, ny):
    """warpAffine(preMask = ones, INTER_NEAREST, BORDER_CONSTANT 0) -> 0/1 mask."""
    return ((nx >= 0) & (nx < w) & (ny >= 0) & (ny < h)).astype(np.float32)


def gradients(img):
    """filter2D(imageFloat, (-0.5, 0, 0.5)) and its transpose, reflect-101 borders (ecc.cpp)."""
    f = img.astype(np.float32)
    h, w = f.shape
    xm = np.abs(np.arange(w) - 1)
    xp = np.arange(w) + 1
    xp = np.where(xp >= w, 2 * (w - 1) - xp, xp) if w > 1 else np.zeros(w, np.int64)
    ym = np.abs(np.arange(h) - 1)
    yp = np.arange(h) + 1
    yp = np.where(yp >= h, 2 * (h - 1) - yp, yp) if h > 1 else np.zeros(h, np.int64)
    if w == 1:
        xm = np.zeros(w, np.int64)
    if h == 1:
        ym = np.zeros(h, np.int64)
    gx = (F32(0.5) * (f[:, xp] - f[:, xm])).astype(np.float32)
    gy = (F32(0.5) * (f[yp, :] - f[ym, :])).astype(np.float32)
    return gx, gy


# ------------------------------------------------------------------------------ small solves
def invert(H):
    """cv::invert(DECOMP_LU) of a float32 matrix -> float32 (zeros when singular)."""
    n = H.shape[0]
    S = H.astype(np.float64)
    D = np.zeros((n, n), dtype=np.float32)
    if n == 2:
        d = S[0, 0] * S[1, 1] - S[0, 1] * S[1, 0]
        if d != 0.0:
            d = 1.0 / d
            D[1, 1] = S[0, 0] * d
            D[0, 0] = S[1, 1] * d
            D[0, 1] = -S[0, 1] * d
            D[1, 0] = -S[1, 0] * d
        return D
    if n == 3:
        d = (S[0, 0] * (S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1])
             - S[0, 1] * (S[1, 0] * S[2, 2] - S[1, 2] * S[2, 0])
             + S[0, 2] * (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]))
        if d != 0.0:
            d = 1.0 / d
            t = [(S[1, 1] * S[2, 2] - S[1, 2] * S[2, 1]) * d,
                 (S[0, 2] * S[2, 1] - S[0, 1] * S[2, 2]) * d,
                 (S[0, 1] * S[1, 2] - S[0, 2] * S[1, 1]) * d,
                 (S[1, 2] * S[2, 0] - S[1, 0] * S[2, 2]) * d,
                 (S[0, 0] * S[2, 2] - S[0, 2] * S[2, 0]) * d,
                 (S[0, 2] * S[1, 0] - S[0, 0] * S[1, 2]) * d,
                 (S[1, 0] * S[2, 1] - S[1, 1] * S[2, 0]) * d,
                 (S[0, 1] * S[2, 0] - S[0, 0] * S[2, 1]) * d,
                 (S[0, 0] * S[1, 1] - S[0, 1] * S[1, 0]) * d]
            D[:] = np.array(t).reshape(3, 3)
        return D
    # hal::LU32f with an identity right-hand side (float32 Gaussian elimination, partial pivot)
    A = H.astype(np.float32).copy()
    b = np.eye(n, dtype=np.float32)
    eps = F32(np.finfo(np.float32).eps * 10)
    for i in range(n):
        k = i
        for j in range(i + 1, n):
            if abs(A[j, i]) > abs(A[k, i]):
                k = j
        if abs(A[k, i]) < eps:
            return np.zeros((n, n), dtype=np.float32)
        if k != i:
            A[[i, k], i:] = A[[k, i], i:]
            b[[i, k]] = b[[k, i]]
        d = F32(-1) / A[i, i]
        for j in range(i + 1, n):
            alpha = F32(A[j, i] * d)
            for kk in range(i + 1, n):
                A[j, kk] = F32(A[j, kk] + F32(alpha * A[i, kk]))
            for kk in range(n):
                b[j, kk] = F32(b[j, kk] + F32(alpha * b[i, kk]))
    for i in range(n - 1, -1, -1):
        for j in range(n):
            s = b[i, j]
            for kk in range(i + 1, n):
                s = F32(s - F32(A[i, kk] * b[kk, j]))
            b[i, j] = F32(s / A[i, i])
    return b


def gemv(A, x):
    """gemm(A (n x n float32), x (n float32)) with float64 accumulation -> float32."""
    out = np.zeros(A.shape[0], dtype=np.float32)
    for i in range(A.shape[0]):
        s = 0.0
        for k in range(A.shape[1]):
            s += float(A[i, k]) * float(x[k])
        out[i] = s
    return out


def dot64(a, b):
    s = 0.0
    for u, v in zip(a, b):
        s += float(u) * float(v)
    return s


# ------------------------------------------------------------------------------ findTransformECC
def jacobian(mode, gx, gy, X, Y, warp):
    """image_jacobian_{translation, euclidean, affine}_ECC (ecc.cpp), float32 per pixel."""
    if mode == MOTION_TRANSLATION:
        return [gx, gy]
    if mode == MOTION_EUCLIDEAN:
        h0, h1 = warp[0, 0], warp[1, 0]                     # cos, sin
        hat_x = (-(X * h1)) - (Y * h0)
        hat_y = (X * h0) - (Y * h1)
        return [(gx * hat_x) + (gy * hat_y), gx, gy]
    return [gx * X, gy * X, gx * Y, gy * Y, gx, gy]


def update_warp(warp, dp, mode):
    """update_warping_matrix_ECC (ecc.cpp): float32 map, float64 trigonometry."""
    w = warp.copy()
    if mode == MOTION_TRANSLATION:
        w[0, 2] += dp[0]
        w[1, 2] += dp[1]
    elif mode == MOTION_AFFINE:
        w[0, 0] += dp[0]
        w[1, 0] += dp[1]
        w[0, 1] += dp[2]
        w[1, 1] += dp[3]
        w[0, 2] += dp[4]
        w[1, 2] += dp[5]
    else:
        theta = float(dp[0]) + math.asin(float(w[1, 0]))
        w[0, 2] += dp[1]
        w[1, 2] += dp[2]
        w[0, 0] = w[1, 1] = F32(math.cos(theta))
        w[1, 0] = F32(math.sin(theta))
        w[0, 1] = -w[1, 0]
    return w


def find_transform_ecc(template, image, warp, mode, max_iter, eps, stats=None):
    """cv2.findTransformECC(template, image, warp, mode, (COUNT|EPS, max_iter, eps), None, 1)
    -> (rho, warp float32 2x3); raises ECCError where OpenCV raises."""
    if mode not in N_PARAMS:
        raise NotImplementedError("MOTION_HOMOGRAPHY is not restated")
    n = N_PARAMS[mode]
    nt = ecc_threads(mode)
    tmpl = np.asarray(template, dtype=np.uint8).astype(np.float32)
    img = np.asarray(image, dtype=np.uint8).astype(np.float32)
    hs, ws = tmpl.shape
    hd, wd = img.shape
    gx, gy = gradients(img)
    X = np.broadcast_to(np.arange(ws, dtype=np.float32)[None, :], (hs, ws)).ravel()
    Y = np.broadcast_to(np.arange(hs, dtype=np.float32)[:, None], (hs, ws)).ravel()
    T = tmpl.ravel()
    warp = np.asarray(warp, dtype=np.float32).copy()
    rho, last_rho = -1.0, -eps
    it = 0
    while it < max_iter and abs(rho - last_rho) >= eps:
        it += 1
        sx, sy, alpha, nx, ny = warp_coords(warp, hs, ws)
        iw = remap_linear(img, sx, sy, alpha).ravel()
        gxw = remap_linear(gx, sx, sy, alpha).ravel()
        gyw = remap_linear(gy, sx, sy, alpha).ravel()
        m = remap_nearest_ones(hd, wd, nx, ny).ravel() != 0
        # pass A: meanStdDev of the warped image and of the template over the mask
        s_i, q_i, s_t, q_t = block_sum(np.stack([
            np.where(m, iw.astype(np.float64), 0.0),
            np.where(m, iw.astype(np.float64) ** 2, 0.0),
            np.where(m, T.astype(np.float64), 0.0),
            np.where(m, T.astype(np.float64) ** 2, 0.0)]), nt)
        cnt = int(m.sum())
        scale = 1.0 / cnt if cnt else 0.0
        img_mean = s_i * scale
        img_std = math.sqrt(max(q_i * scale - img_mean * img_mean, 0.0))
        tmp_mean = s_t * scale
        tmp_std = math.sqrt(max(q_t * scale - tmp_mean * tmp_mean, 0.0))
        iwz = np.where(m, iw - F32(img_mean), iw).astype(np.float32)
        tz = np.where(m, T - F32(tmp_mean), F32(0)).astype(np.float32)
        tmp_norm = math.sqrt(cnt * tmp_std * tmp_std)
        img_norm = math.sqrt(cnt * img_std * img_std)
        J = [j.astype(np.float32) for j in jacobian(mode, gxw, gyw, X, Y, warp)]
        # pass B: Hessian, projections, correlation
        terms = []
        for i in range(n):
            for j in range(i, n):
                terms.append(J[i].astype(np.float64) * J[j])
        for i in range(n):
            terms.append(J[i].astype(np.float64) * iwz)
        for i in range(n):
            terms.append(J[i].astype(np.float64) * tz)
        terms.append(tz.astype(np.float64) * iwz)
        sums = block_sum(np.stack(terms), nt)
        H = np.zeros((n, n), dtype=np.float32)
        k = 0
        for i in range(n):
            for j in range(i, n):
                if i == j:
                    r = math.sqrt(sums[k])
                    H[i, i] = r * r
                else:
                    H[i, j] = H[j, i] = sums[k]
                k += 1
        P = sums[k:k + n].astype(np.float32)
        Q = sums[k + n:k + 2 * n].astype(np.float32)
        corr = float(sums[k + 2 * n])
        Hinv = invert(H)
        last_rho = rho
        with np.errstate(divide="ignore", invalid="ignore"):
            rho = float(np.float64(corr) / np.float64(img_norm * tmp_norm))
        if math.isnan(rho):
            raise ECCError("NaN encountered.")
        iph = gemv(Hinv, P)
        lambda_n = img_norm * img_norm - dot64(P, iph)
        lambda_d = corr - dot64(Q, iph)
        if lambda_d <= 0.0:
            raise ECCError("The algorithm stopped before its convergence.")
        lam = lambda_n / lambda_d
        # pass C: error projection
        err = (lam * tz.astype(np.float64) - iwz).astype(np.float32)
        E = block_sum(np.stack([J[i].astype(np.float64) * err for i in range(n)]), nt)
        E = E.astype(np.float32)
        dp = gemv(Hinv, E)
        warp = update_warp(warp, dp, mode)
    if stats is not None:
        stats["iters"] = it
        stats["rho"] = rho
    return rho, warp


def invert_affine(M):
    """cv::warpAffine without WARP_INVERSE_MAP (imgwarp.cpp): the float32 2x3 matrix widened to
    float64 and inverted in place - D = 1 / (M0 M4 - M1 M3) (0 when singular), M0 = M4 D,
    M1 = -M1 D, M3 = -M3 D, M4 = M0 D, M2 = -M0' M2 - M1' M5, M5 = -M3' M2 - M4' M5."""
    m = [float(v) for v in np.asarray(M, dtype=np.float32).astype(np.float64).ravel()]
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    a11, a22 = m[4] * D, m[0] * D
    m[0] = a11
    m[1] *= -D
    m[3] *= -D
    m[4] = a22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return np.array(m, dtype=np.float64)


def warp_affine_u8(src, M, out_h, out_w):
    """cv2.warpAffine(src, M, (out_w, out_h), flags=INTER_LINEAR) on a uint8 image (ecc.py:97,
    align=True): the inverted map (invert_affine), WarpAffineInvoker's fixed-point coordinates
    (warp_coords, fed the float64 inverse), remapBilinear's integer path - the 15-bit table
    (initInterTab2D fixed point: (32 - fy)(32 - fx) 32 ..., summing to 2^15 exactly), taps outside
    the image read 0 (BORDER_CONSTANT), (sum + 2^14) >> 15.  Integer sums: order-free."""
    src = np.asarray(src, dtype=np.uint8)
    h, w = src.shape
    Minv = invert_affine(M)
    x = np.arange(out_w, dtype=np.float64)
    y = np.arange(out_h, dtype=np.float64)
    adelta = cv_round(Minv[0] * x * AB_SCALE)
    bdelta = cv_round(Minv[3] * x * AB_SCALE)
    xr = cv_round((Minv[1] * y + Minv[2]) * AB_SCALE)
    yr = cv_round((Minv[4] * y + Minv[5]) * AB_SCALE)
    X = (xr[:, None] + 16 + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (yr[:, None] + 16 + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    fx, fy = X & 31, Y & 31
    wts = [(32 - fx) * (32 - fy) * 32, fx * (32 - fy) * 32, (32 - fx) * fy * 32, fx * fy * 32]
    img = src.astype(np.int64)

    def tap(yy, xx):
        ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
        return np.where(ok, img[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)], 0)

    acc = (tap(sy, sx) * wts[0] + tap(sy, sx + 1) * wts[1] + tap(sy + 1, sx) * wts[2] +
           tap(sy + 1, sx + 1) * wts[3])
    return np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


class ECCOracle:
    """ECC (ecc.py:13-104) over the restated OpenCV calls, align=True's preview image included
    (ecc.py:91-100, affine models: warp_affine_u8)."""

    def __init__(self, warp_mode=MOTION_EUCLIDEAN, eps=1e-5, max_iter=100, scale=0.1,
                 align=False, grayscale=True):
        self.warp_mode = warp_mode
        self.eps = eps
        self.max_iter = max_iter
        self.scale = scale
        self.align = align
        self.prev_img = None
        self.prev_img_aligned = None
        self.last = {}

    def apply(self, img, dets=None):
        self.last = {"outcome": 0}
        if self.warp_mode == MOTION_HOMOGRAPHY:
            raise NotImplementedError("MOTION_HOMOGRAPHY is not restated")
        warp = np.eye(2, 3, dtype=np.float32)
        if self.prev_img is None:
            self.prev_img = preprocess(img, self.scale)
            return warp
        curr = preprocess(img, self.scale)
        try:
            _, warp = find_transform_ecc(self.prev_img, curr, warp, self.warp_mode,
                                         self.max_iter, self.eps, self.last)
        except ECCError:
            self.last["outcome"] = 2
            return np.eye(2, 3, dtype=np.float32)
        self.last["outcome"] = 1
        if self.scale < 1:
            warp[0, 2] /= self.scale
            warp[1, 2] /= self.scale
        if self.align:   # ecc.py:91-98: the previous frame warped by the upscaled matrix
            h, w = self.prev_img.shape
            self.prev_img_aligned = warp_affine_u8(self.prev_img, warp, h, w)
        else:
            self.prev_img_aligned = None
        self.prev_img = curr
        return warp
