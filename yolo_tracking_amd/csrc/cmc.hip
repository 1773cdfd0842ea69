// SparseOptFlow camera-motion compensation for S camera streams on gfx950.
//
// Reference: boxmot/motion/cmc/sof.py:64-162 (SparseOptFlow.apply), cmc_interface.py:13-40
// (generate_mask, preprocess); the estimator BoTSORT (bot_sort.py:228, :293) and DeepOCSort
// (deep_ocsort.py:351, :391) call once per frame.  Its arithmetic is OpenCV's (cvtColor, resize,
// goodFeaturesToTrack, calcOpticalFlowPyrLK, estimateAffinePartial2D + LM), restated in
// oracle/cmc_sof.py; every kernel here reproduces that restatement bit for bit (same float32 /
// float64 operation order, exact integer window sums, the same RNG stream).
//
// One frame of every stream = 5 launches:
//   k_sof_small  [grid, pixel/thread]  gray (fixed-point BGR2GRAY) + INTER_LINEAR resize into the
//                                      stream's current pyramid slot; per-stream mode
//   k_sof_pyr    [block/stream]        pyrDown levels (buildOpticalFlowPyramid's level count) and
//                                      the Scharr derivatives of every level (used when this slot
//                                      is the previous frame)
//   k_sof_gftt   [block/stream]        first frame only: mask, min-eigenvalue map, threshold +
//                                      dilate + candidates, bitonic sort (LDS), first 3000 corners
//   k_sof_lk     [wave/point]          pyramidal Lucas-Kanade of every stored corner, levels
//                                      coarse to fine, window sums by DPP wave reductions
//   k_sof_fit    [block/stream]        status compaction (kept: the stored corners shrink),
//                                      RANSAC (64 hypotheses per round, one wave per 16), LM
//                                      refinement with fixed-order block reductions, the warp
//
// HBM layout per stream: two pyramid slots (previous accepted frame / current frame) of uint8
// levels + short2 derivatives, the stored corners (<= 3000 float2), LK results, fit scratch, and
// first-frame scratch (covariance / eigenvalue planes, candidate keys).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "cmc_small.hpp"
#include "common.hpp"

namespace yta {
namespace {
using namespace cmc;

constexpr int SOF_WIN = 21;              // calcOpticalFlowPyrLK winSize (21, 21)
constexpr int SOF_HALF = 10;             // (winSize - 1) / 2
constexpr int SOF_MAX_LEVEL = 3;         // maxLevel
constexpr int SOF_MAXKP = 3000;          // goodFeaturesToTrack maxCorners (sof.py:83-91)
constexpr int SOF_LK_ITERS = 30;         // TermCriteria(COUNT | EPS, 30, 0.01)
constexpr int SOF_RANSAC_ITERS = 2000;   // estimateAffinePartial2D defaults
constexpr int SOF_REFINE_ITERS = 10;
constexpr int SOF_T = 256;               // per-stream block kernels (the 256-way reduce order)
constexpr int GFTT_T = 1024;
constexpr int SORT_CAP = 16384;          // candidate keys sorted in LDS (128 KiB)
constexpr int LK_SLOTS = 7;              // window positions per lane: 441 = 64 * 7 - 7
constexpr int RB = 64;                   // RANSAC hypotheses per round

enum { MODE_GFTT = 0, MODE_LK = 1, MODE_NOKP = 2, MODE_SKIP = 3 };
enum { OUT_FIRST = 0, OUT_EST = 1, OUT_IDENT = 2 };
constexpr int SOF_ERR_SIZE = 1;

struct SofState {
    int init, prev, n_kp, mode;
    int h0[2], w0[2];
    int levels[2];
    int outcome, err;
};

struct SofArgs {
    int S;
    double scale;
    int h0max, w0max;
    long long slot_px;   // pixels per pyramid slot (every level packed)
    long long npx;       // h0max * w0max
    uint8_t *img;        // [S][2][slot_px]
    short2 *der;         // [S][2][slot_px]
    float2 *kp;          // [S][MAXKP] stored corners (prev_keypoints)
    float2 *nxt;         // [S][MAXKP] LK results
    uint8_t *st;         // [S][MAXKP] LK status
    float2 *fit;         // [S][4][MAXKP] compacted src / dst, inlier src / dst
    float *cov;          // [S][3][npx]
    float *eig;          // [S][npx]
    uint8_t *mask;       // [S][npx]
    unsigned long long *keys;   // [S][keys_cap]
    long long keys_cap;
    SofState *state;
    // per frame
    const uint8_t *frames;
    const long long *frame_off;
    const int *frame_hw;
    const double *dets;
    int det_stride;
    const int *det_off;
    double *warps;       // [S][6]
};

struct Lv {
    int h, w;
    long long off;
};

// buildOpticalFlowPyramid's level sizes: level k = ((level k-1) + 1) / 2, stopping when the next
// level would have a side <= winSize.
__host__ __device__ inline int sof_levels(int h, int w, Lv *lv) {
    int n = 0;
    long long off = 0;
    for (int level = 0; level <= SOF_MAX_LEVEL; ++level) {
        if (level != 0) {
            h = (h + 1) / 2;
            w = (w + 1) / 2;
        }
        lv[level].h = h;
        lv[level].w = w;
        lv[level].off = off;
        off += (long long)h * w;
        n = level + 1;
        if ((w + 1) / 2 <= SOF_WIN || (h + 1) / 2 <= SOF_WIN) break;
    }
    return n;
}

__host__ __device__ inline int sof_nlevels(int h, int w) {
    int n = 0;
    for (int level = 0; level <= SOF_MAX_LEVEL; ++level) {
        if (level != 0) {
            h = (h + 1) / 2;
            w = (w + 1) / 2;
        }
        n = level + 1;
        if ((w + 1) / 2 <= SOF_WIN || (h + 1) / 2 <= SOF_WIN) break;
    }
    return n;
}

__host__ __device__ inline long long sof_slot_px(int h, int w) {   // pixels of every level
    const int n = sof_nlevels(h, w);
    long long px = 0;
    for (int l = 0; l < n; ++l) {
        px += (long long)h * w;
        h = (h + 1) / 2;
        w = (w + 1) / 2;
    }
    return px;
}

__device__ __forceinline__ void identity6(double *w) {
    w[0] = 1.0; w[1] = 0.0; w[2] = 0.0;
    w[3] = 0.0; w[4] = 1.0; w[5] = 0.0;
}

// ------------------------------------------------------------------------------- k_sof_small
__global__ __launch_bounds__(256) void k_sof_small(SofArgs a) {
    const int s = blockIdx.y;
    SofState &st = a.state[s];
    const int H = a.frame_hw[2 * s], W = a.frame_hw[2 * s + 1];
    const int h0 = (int)rint(H * a.scale), w0 = (int)rint(W * a.scale);
    const int cur = 1 - st.prev;
    const bool fits = H >= 1 && W >= 1 && h0 >= 1 && w0 >= 1 && h0 <= a.h0max && w0 <= a.w0max;
    // After the first frame a frame of another size makes calcOpticalFlowPyrLK assert on the
    // level sizes; sof.py:105-110 catches it and returns the identity with prev_img and the
    // corners kept (also when the frame exceeds the buffers: that is a size change too).  Only a
    // first frame that does not fit is an error, and it belongs to this frame alone.
    const bool resized = st.init && (!fits || h0 != st.h0[st.prev] || w0 != st.w0[st.prev]);
    const bool ok = fits && !resized;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st.mode = !ok ? MODE_SKIP : (!st.init ? MODE_GFTT : (st.n_kp > 0 ? MODE_LK : MODE_NOKP));
        st.err = !fits && !st.init ? SOF_ERR_SIZE : 0;
        if (ok) {
            st.h0[cur] = h0;
            st.w0[cur] = w0;
        }
    }
    if (!ok) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= h0 * w0) return;
    const int oy = i / w0, ox = i - oy * w0;
    uint8_t *dst = a.img + ((long long)s * 2 + cur) * a.slot_px;
    dst[i] = (uint8_t)small_pixel(a.frames + a.frame_off[s], H, W, a.scale, ox, oy);
}

// --------------------------------------------------------------------------------- k_sof_pyr
// One level's pyrDown ([1 4 6 4 1]^2, reflect-101, (sum + 128) >> 8) and Scharr derivatives
// (calcSharrDeriv) read from `src`: the level staged in LDS, or global memory.
template <typename Src>
__device__ __forceinline__ void pyr_level_work(Src src, int sh, int sw, uint8_t *dst, int h, int w,
                                               short2 *d) {
    const int t = threadIdx.x, nt = blockDim.x;
    if (dst)
        for (int i = t; i < h * w; i += nt) {
            const int y = i / w, x = i - y * w;
            const int x0 = refl(2 * x - 2, sw), x1 = refl(2 * x - 1, sw), x2 = refl(2 * x, sw),
                      x3 = refl(2 * x + 1, sw), x4 = refl(2 * x + 2, sw);
            auto row5 = [&](int r) {
                const int base = refl(2 * y + r - 2, sh) * sw;
                return (int)src[base + x0] + 4 * (int)src[base + x1] + 6 * (int)src[base + x2] +
                       4 * (int)src[base + x3] + (int)src[base + x4];
            };
            const int sum = row5(0) + 4 * row5(1) + 6 * row5(2) + 4 * row5(3) + row5(4);
            dst[i] = (uint8_t)((sum + 128) >> 8);
        }
    for (int i = t; i < sh * sw; i += nt) {
        const int y = i / sw, x = i - y * sw;
        const int ym = refl(y - 1, sh) * sw, yp = refl(y + 1, sh) * sw, yc = y * sw;
        const int xm = refl(x - 1, sw), xp = refl(x + 1, sw);
        auto S = [&](int row, int xx) { return (int)src[row + xx]; };
        const int t0m = (S(ym, xm) + S(yp, xm)) * 3 + S(yc, xm) * 10;
        const int t0p = (S(ym, xp) + S(yp, xp)) * 3 + S(yc, xp) * 10;
        const int t1m = S(yp, xm) - S(ym, xm), t1p = S(yp, xp) - S(ym, xp);
        const int t1c = S(yp, x) - S(ym, x);
        d[i] = make_short2((short)(t0p - t0m), (short)((t1p + t1m) * 3 + t1c * 10));
    }
}

// buildOpticalFlowPyramid + calcSharrDeriv of every level: level l is staged into LDS (when it
// fits lds_cap bytes), then level l + 1 and level l's derivatives are computed from LDS.
__device__ void pyr_levels_body(uint8_t *img, short2 *der, int h0, int w0, uint8_t *lds,
                                int lds_cap) {
    const int t = threadIdx.x, nt = blockDim.x;
    const int nl = sof_nlevels(h0, w0);
    int sh = h0, sw = w0;
    long long off = 0;
    for (int l = 0; l < nl; ++l) {
        const int h = (sh + 1) / 2, w = (sw + 1) / 2;
        const long long noff = off + (long long)sh * sw;
        uint8_t *dst = l + 1 < nl ? img + noff : nullptr;
        const uint8_t *src = img + off;
        const int n = sh * sw;
        if (n <= lds_cap) {
            const int nw = (n + 3) / 4;   // slot levels are not word aligned: byte copy in words
            for (int k = t; k < nw; k += nt) {
                unsigned v = 0;
                for (int b = 0; b < 4; ++b) {
                    const int q = 4 * k + b;
                    if (q < n) v |= (unsigned)src[q] << (8 * b);
                }
                reinterpret_cast<unsigned *>(lds)[k] = v;
            }
            __syncthreads();
            pyr_level_work(lds, sh, sw, dst, h, w, der + off);
        } else {
            pyr_level_work(src, sh, sw, dst, h, w, der + off);
        }
        block_sync();
        off = noff;
        sh = h;
        sw = w;
    }
}

constexpr int PYR_T = 1024;
constexpr int PYR_LDS = 64 * 1024;

__global__ __launch_bounds__(PYR_T) void k_sof_pyr(SofArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int s = blockIdx.x;
    const SofState &st = a.state[s];
    if (st.mode != MODE_GFTT && st.mode != MODE_LK) return;
    const int cur = 1 - st.prev;
    const long long slot = (long long)s * 2 + cur;
    pyr_levels_body(a.img + slot * a.slot_px, a.der + slot * a.slot_px, st.h0[cur], st.w0[cur],
                    smem, PYR_LDS);
    if (threadIdx.x == 0) a.state[s].levels[cur] = sof_nlevels(st.h0[cur], st.w0[cur]);
}

// -------------------------------------------------------------------------------- k_sof_gftt
struct GfttShared {
    double red[16];
    int cnt;
    int any;
};

// cornerMinEigenVal + goodFeaturesToTrack on one gray image (oracle/cmc_sof.py min_eigen /
// good_features).  cov (3 planes) / eig: scratch of h * w floats; keys: scratch of >= next_pow2(
// candidates) (only used past SORT_CAP); lds_keys: SORT_CAP keys of dynamic LDS.
__device__ void gftt_body(const uint8_t *g, const uint8_t *mask, int h, int w, float *cov,
                          float *eig, unsigned long long *keys, long long keys_cap,
                          unsigned long long *lds_keys, float2 *out, int *n_out, GfttShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x;
    const int n = h * w;
    const double scale = 1.0 / (4 * 3 * 255);
    const float k0 = (float)(1.0 * scale), k1 = (float)(2.0 * scale);
    float *c0 = cov, *c1 = cov + n, *c2 = cov + 2 * n;
    for (int i = t; i < n; i += nt) {   // Sobel dx / dy (scale folded into the smoothing taps)
        const int y = i / w, x = i - y * w;
        const int ym = refl(y - 1, h), yp = refl(y + 1, h);
        const int xm = refl(x - 1, w), xp = refl(x + 1, w);
        auto S = [&](int yy, int xx) { return (float)g[(long long)yy * w + xx]; };
        const float r0 = S(ym, xp) - S(ym, xm), r1 = S(y, xp) - S(y, xm), r2 = S(yp, xp) - S(yp, xm);
        const float dx = r1 * k1 + (r0 + r2) * k0;
        const float qm = S(ym, x) * k1 + (S(ym, xm) + S(ym, xp)) * k0;
        const float qp = S(yp, x) * k1 + (S(yp, xm) + S(yp, xp)) * k0;
        const float dy = qp - qm;
        c0[i] = dx * dx;
        c1[i] = dx * dy;
        c2[i] = dy * dy;
    }
    if (t == 0) {
        sh.cnt = 0;
        sh.any = 0;
    }
    block_sync();
    double mx = -INFINITY;
    int any = 0;
    for (int i = t; i < n; i += nt) {   // 3x3 box in float64, min eigenvalue in float32
        const int y = i / w, x = i - y * w;
        const int ys[3] = {refl(y - 1, h), y, refl(y + 1, h)};
        const int xs[3] = {refl(x - 1, w), x, refl(x + 1, w)};
        float bx[3];
        const float *cs[3] = {c0, c1, c2};
        for (int c = 0; c < 3; ++c) {
            double rs[3];
            for (int r = 0; r < 3; ++r) {
                const float *row = cs[c] + (long long)ys[r] * w;
                rs[r] = ((double)row[xs[0]] + (double)row[xs[1]]) + (double)row[xs[2]];
            }
            bx[c] = (float)((rs[0] + rs[1]) + rs[2]);
        }
        const float A = bx[0] * 0.5f, B = bx[1], C = bx[2] * 0.5f;
        const float e = (A + C) - sqrtf((A - C) * (A - C) + B * B);
        eig[i] = e;
        if (mask[i]) {
            mx = fmax(mx, (double)e);
            any = 1;
        }
    }
    mx = wave_reduce(RED_MAX, mx);
    if (__any(any) && lane_id() == 0) atomicOr(&sh.any, 1);
    if (lane_id() == 0) sh.red[t / WAVE] = mx;
    block_sync();
    double maxv = -INFINITY;
    for (int k = 0; k < nt / WAVE; ++k) maxv = fmax(maxv, sh.red[k]);
    if (!sh.any) maxv = 0.0;
    const float thr = (float)(maxv * 0.01);
    auto T = [&](int j) {
        const float v = eig[j];
        return v > thr ? v : 0.f;
    };
    for (int i = t; i < n; i += nt) {   // threshold + 3x3 dilate + candidates
        const int y = i / w, x = i - y * w;
        if (y < 1 || y > h - 2 || x < 1 || x > w - 2 || !mask[i]) continue;
        const float e = T(i);
        if (e == 0.f) continue;
        float d = e;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) d = fmaxf(d, T(i + dy * w + dx));
        if (e != d) continue;
        const int p = atomicAdd(&sh.cnt, 1);
        keys[p] = ((unsigned long long)__float_as_uint(e) << 32) | (unsigned)i;
    }
    block_sync();
    const int nc = sh.cnt;
    int P = 1;
    while (P < nc) P <<= 1;
    const bool in_lds = P <= SORT_CAP;
    unsigned long long *K = in_lds ? lds_keys : keys;
    if (!in_lds && P > keys_cap) P = 0;   // cannot happen: keys_cap >= next_pow2(h * w)
    for (int i = t; i < P; i += nt) K[i] = i < nc ? keys[i] : 0ull;
    block_sync();
    // bitonic sort, descending: eigenvalue bits (positive floats order as integers), then index
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = t; i < P; i += nt) {
                const int ij = i ^ j;
                if (ij > i) {
                    const unsigned long long x = K[i], y = K[ij];
                    const bool desc = (i & k) == 0;
                    if (desc ? x < y : x > y) {
                        K[i] = y;
                        K[ij] = x;
                    }
                }
            }
            block_sync();
        }
    const int m = nc < SOF_MAXKP ? nc : SOF_MAXKP;
    for (int i = t; i < m; i += nt) {
        const int idx = (int)(unsigned)(K[i] & 0xFFFFFFFFull);
        const int y = idx / w;
        out[i] = make_float2((float)(idx - y * w), (float)y);
    }
    if (t == 0) *n_out = m;
    block_sync();
}

// NumPy slice [a:b) of an axis of length n (Python semantics, step 1)
__device__ __forceinline__ int2 py_slice(long long a, long long b, int n) {
    if (a < 0) a += n;
    if (a < 0) a = 0;
    if (a > n) a = n;
    if (b < 0) b += n;
    if (b < 0) b = 0;
    if (b > n) b = n;
    return make_int2((int)a, (int)(b > a ? b : a));
}

__global__ __launch_bounds__(GFTT_T) void k_sof_gftt(SofArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ GfttShared sh;
    const int s = blockIdx.x;
    const SofState &st = a.state[s];
    if (st.mode != MODE_GFTT) return;
    const int t = threadIdx.x, nt = blockDim.x;
    const int cur = 1 - st.prev, h = st.h0[cur], w = st.w0[cur];
    uint8_t *mask = a.mask + (long long)s * a.npx;
    // generate_mask (cmc_interface.py:13-24)
    const int y0 = (int)(0.02 * h), y1 = (int)(0.98 * h), x0 = (int)(0.02 * w), x1 = (int)(0.98 * w);
    for (int i = t; i < h * w; i += nt) {
        const int y = i / w, x = i - y * w;
        mask[i] = (y >= y0 && y < y1 && x >= x0 && x < x1) ? 255 : 0;
    }
    block_sync();
    const int d0 = a.det_off[s], nd = a.det_off[s + 1] - d0;
    for (int k = t; k < nd; k += nt) {
        const double *d = a.dets + (long long)(d0 + k) * a.det_stride;
        long long tl[4];
        for (int q = 0; q < 4; ++q) {
            const double v = d[q] * a.scale;
            tl[q] = isfinite(v) ? (long long)v : 0;   // astype(int) truncates
        }
        const int2 ry = py_slice(tl[1], tl[3], h), rx = py_slice(tl[0], tl[2], w);
        for (int y = ry.x; y < ry.y; ++y)
            for (int x = rx.x; x < rx.y; ++x) mask[(long long)y * w + x] = 0;
    }
    block_sync();
    const long long slot = (long long)s * 2 + cur;
    int n_kp = 0;
    gftt_body(a.img + slot * a.slot_px, mask, h, w, a.cov + (long long)s * 3 * a.npx,
              a.eig + (long long)s * a.npx, a.keys + (long long)s * a.keys_cap, a.keys_cap,
              (unsigned long long *)smem, a.kp + (long long)s * SOF_MAXKP, &a.state[s].n_kp, sh);
    n_kp = a.state[s].n_kp;
    if (t == 0) {
        SofState &o = a.state[s];
        if (n_kp > 0) {   // sof.py:94-101: keep the frame and its corners
            o.init = 1;
            o.prev = cur;
        }
        o.outcome = OUT_FIRST;
        identity6(a.warps + 6LL * s);
    }
}

// ---------------------------------------------------------------------------------- k_sof_lk
// LKTrackerInvoker for one point (one wave): levels maxLevel .. 0.  Window position k = lane +
// 64 m (m < 7, k < 441) at (k / 21, k % 21).  Returns (next point, status).
struct LkLevel {
    const uint8_t *I;
    const short2 *dI;
    const uint8_t *J;
    int hI, wI, hJ, wJ;
};

// The two pyramids of one LK call: slot bases and level-0 dims (levels derived on the fly, so no
// per-level array lives in private memory).
struct LkPyr {
    const uint8_t *I;
    const short2 *dI;
    const uint8_t *J;
    int hI, wI, hJ, wJ;
};

__device__ __forceinline__ void level_dims(int h, int w, int level, int &lh, int &lw,
                                           long long &off) {
    off = 0;
    for (int l = 0; l < level; ++l) {
        off += (long long)h * w;
        h = (h + 1) / 2;
        w = (w + 1) / 2;
    }
    lh = h;
    lw = w;
}

__device__ __forceinline__ LkLevel lk_level(const LkPyr &p, int level) {
    LkLevel L;
    long long oi, oj;
    level_dims(p.hI, p.wI, level, L.hI, L.wI, oi);
    level_dims(p.hJ, p.wJ, level, L.hJ, L.wJ, oj);
    L.I = p.I + oi;
    L.dI = p.dI + oi;
    L.J = p.J + oj;
    return L;
}

__device__ __forceinline__ void lk_weights(float px, float py, int &ix, int &iy, int &w00, int &w01,
                                           int &w10, int &w11) {
    ix = (int)floorf(px);
    iy = (int)floorf(py);
    const float a = px - (float)ix, b = py - (float)iy;
    w00 = (int)rintf((1.f - a) * (1.f - b) * 16384.f);
    w01 = (int)rintf(a * (1.f - b) * 16384.f);
    w10 = (int)rintf((1.f - a) * b * 16384.f);
    w11 = 16384 - w00 - w01 - w10;
}

__device__ __forceinline__ void lk_point(const LkPyr &pyr, int max_level, float2 pt, float2 &out,
                                         int &status) {
    const int lane = lane_id();
    const float FLT_SCALE = 1.f / (1 << 20);
    float nx = 0.f, ny = 0.f;
    status = 1;
    for (int level = max_level; level >= 0; --level) {
        const LkLevel L = lk_level(pyr, level);
        const float lsc = (float)(1.0 / (1 << level));
        const float px0 = pt.x * lsc, py0 = pt.y * lsc;
        float cx, cy;
        if (level == max_level) {
            cx = px0;
            cy = py0;
        } else {
            cx = nx * 2.f;
            cy = ny * 2.f;
        }
        nx = cx;
        ny = cy;
        const float px = px0 - (float)SOF_HALF, py = py0 - (float)SOF_HALF;
        int ix, iy, w00, w01, w10, w11;
        lk_weights(px, py, ix, iy, w00, w01, w10, w11);
        if (ix < -SOF_WIN || ix >= L.wI || iy < -SOF_WIN || iy >= L.hI) {
            if (level == 0) status = 0;
            continue;
        }
        int ival[LK_SLOTS], ixv[LK_SLOTS], iyv[LK_SLOTS];
        int s11 = 0, s12 = 0, s22 = 0;
        const bool inside = ix >= 0 && iy >= 0 && ix + SOF_WIN < L.wI && iy + SOF_WIN < L.hI;
#pragma unroll
        for (int m = 0; m < LK_SLOTS; ++m) {
            const int k = lane + WAVE * m;
            ival[m] = ixv[m] = iyv[m] = 0;
            if (k >= SOF_WIN * SOF_WIN) continue;
            const int wy = k / SOF_WIN, wx = k - wy * SOF_WIN;
            const int y = iy + wy, x = ix + wx;
            short2 d00, d01, d10, d11;
            if (inside) {   // the window and its +1 taps lie inside the level
                const uint8_t *r0 = L.I + y * L.wI + x, *r1 = r0 + L.wI;
                ival[m] = ((int)r0[0] * w00 + (int)r0[1] * w01 + (int)r1[0] * w10 +
                           (int)r1[1] * w11 + (1 << 8)) >> 9;
                const short2 *q0 = L.dI + y * L.wI + x, *q1 = q0 + L.wI;
                d00 = q0[0];
                d01 = q0[1];
                d10 = q1[0];
                d11 = q1[1];
            } else {
                const int ry0 = refl(y, L.hI), ry1 = refl(y + 1, L.hI);
                const int rx0 = refl(x, L.wI), rx1 = refl(x + 1, L.wI);
                const uint8_t *r0 = L.I + ry0 * L.wI, *r1 = L.I + ry1 * L.wI;
                ival[m] = ((int)r0[rx0] * w00 + (int)r0[rx1] * w01 + (int)r1[rx0] * w10 +
                           (int)r1[rx1] * w11 + (1 << 8)) >> 9;
                auto D = [&](int yy, int xx) {
                    return (yy >= 0 && yy < L.hI && xx >= 0 && xx < L.wI) ? L.dI[yy * L.wI + xx]
                                                                        : make_short2(0, 0);
                };
                d00 = D(y, x);
                d01 = D(y, x + 1);
                d10 = D(y + 1, x);
                d11 = D(y + 1, x + 1);
            }
            ixv[m] = ((int)d00.x * w00 + (int)d01.x * w01 + (int)d10.x * w10 + (int)d11.x * w11 +
                      (1 << 13)) >> 14;
            iyv[m] = ((int)d00.y * w00 + (int)d01.y * w01 + (int)d10.y * w10 + (int)d11.y * w11 +
                      (1 << 13)) >> 14;
            s11 += ixv[m] * ixv[m];
            s12 += ixv[m] * iyv[m];
            s22 += iyv[m] * iyv[m];
        }
        const float A11 = (float)wave_reduce(RED_SUM, (double)s11) * FLT_SCALE;
        const float A12 = (float)wave_reduce(RED_SUM, (double)s12) * FLT_SCALE;
        const float A22 = (float)wave_reduce(RED_SUM, (double)s22) * FLT_SCALE;
        float Dt = A11 * A22 - A12 * A12;
        const float min_eig =
            (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) / (float)(2 * SOF_WIN * SOF_WIN);
        if (min_eig < 1e-4f || Dt < FLT_EPSILON) {
            if (level == 0) status = 0;
            continue;
        }
        Dt = 1.f / Dt;
        float qx = cx - (float)SOF_HALF, qy = cy - (float)SOF_HALF;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < SOF_LK_ITERS; ++j) {
            int jx, jy, v00, v01, v10, v11;
            lk_weights(qx, qy, jx, jy, v00, v01, v10, v11);
            if (jx < -SOF_WIN || jx >= L.wJ || jy < -SOF_WIN || jy >= L.hJ) {
                if (level == 0) status = 0;
                break;
            }
            int p1 = 0, p2 = 0;
            if (jx >= 0 && jy >= 0 && jx + SOF_WIN < L.wJ && jy + SOF_WIN < L.hJ) {
                // the window and its +1 taps lie inside the level: no border handling
                const uint8_t *b = L.J + jy * L.wJ + jx;
#pragma unroll
                for (int m = 0; m < LK_SLOTS; ++m) {
                    const int k = lane + WAVE * m;
                    if (k >= SOF_WIN * SOF_WIN) continue;
                    const int wy = k / SOF_WIN, wx = k - wy * SOF_WIN;
                    const uint8_t *r0 = b + wy * L.wJ + wx, *r1 = r0 + L.wJ;
                    const int jv = ((int)r0[0] * v00 + (int)r0[1] * v01 + (int)r1[0] * v10 +
                                    (int)r1[1] * v11 + (1 << 8)) >> 9;
                    const int diff = jv - ival[m];
                    p1 += diff * ixv[m];
                    p2 += diff * iyv[m];
                }
            } else {
#pragma unroll
                for (int m = 0; m < LK_SLOTS; ++m) {
                    const int k = lane + WAVE * m;
                    if (k >= SOF_WIN * SOF_WIN) continue;
                    const int wy = k / SOF_WIN, wx = k - wy * SOF_WIN;
                    const int ry0 = refl(jy + wy, L.hJ), ry1 = refl(jy + wy + 1, L.hJ);
                    const int rx0 = refl(jx + wx, L.wJ), rx1 = refl(jx + wx + 1, L.wJ);
                    const uint8_t *r0 = L.J + ry0 * L.wJ, *r1 = L.J + ry1 * L.wJ;
                    const int jv = ((int)r0[rx0] * v00 + (int)r0[rx1] * v01 + (int)r1[rx0] * v10 +
                                    (int)r1[rx1] * v11 + (1 << 8)) >> 9;
                    const int diff = jv - ival[m];
                    p1 += diff * ixv[m];
                    p2 += diff * iyv[m];
                }
            }
            const float b1 = (float)wave_reduce(RED_SUM, (double)p1) * FLT_SCALE;
            const float b2 = (float)wave_reduce(RED_SUM, (double)p2) * FLT_SCALE;
            const float dx = (A12 * b2 - A22 * b1) * Dt;
            const float dy = (A12 * b1 - A11 * b2) * Dt;
            qx += dx;
            qy += dy;
            nx = qx + (float)SOF_HALF;
            ny = qy + (float)SOF_HALF;
            if ((double)dx * dx + (double)dy * dy <= 0.01 * 0.01) break;
            if (j > 0 && (double)fabsf(dx + pdx) < 0.01 && (double)fabsf(dy + pdy) < 0.01) {
                nx -= dx * 0.5f;
                ny -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }
    }
    out = make_float2(nx, ny);
}

__device__ __forceinline__ int lk_pyr(const SofArgs &a, int s, const SofState &st, LkPyr &P) {
    const int p = st.prev, c = 1 - st.prev;
    const int np_ = sof_nlevels(st.h0[p], st.w0[p]);
    const int nc = sof_nlevels(st.h0[c], st.w0[c]);
    const long long sp = ((long long)s * 2 + p) * a.slot_px, sc = ((long long)s * 2 + c) * a.slot_px;
    P.I = a.img + sp;
    P.dI = a.der + sp;
    P.J = a.img + sc;
    P.hI = st.h0[p];
    P.wI = st.w0[p];
    P.hJ = st.h0[c];
    P.wJ = st.w0[c];
    return np_ < nc ? np_ : nc;
}

// 8 points per block (one wave each).  LDSJ: the current frame's pyramid (every level, the
// image each Lucas-Kanade iteration samples) is staged in LDS first, so the iterations' bilinear
// taps are LDS reads; the previous frame and its derivatives are read once per level from HBM.
constexpr int LKB = 512;

template <bool LDSJ>
__global__ __launch_bounds__(LKB) void k_sof_lk(SofArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int s = blockIdx.y;
    const SofState &st = a.state[s];
    if (st.mode != MODE_LK) return;
    const int n_kp = st.n_kp;
    const int first = blockIdx.x * (LKB / WAVE);
    if (first >= n_kp) return;   // block-uniform
    LkPyr P;
    const int nl = lk_pyr(a, s, st, P);
    if (LDSJ) {
        const long long n16 = (sof_slot_px(P.hJ, P.wJ) + 15) / 16;
        const uint4 *src = reinterpret_cast<const uint4 *>(P.J);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        for (long long k = threadIdx.x; k < n16; k += LKB) dst[k] = src[k];
        __syncthreads();
        P.J = smem;
    }
    const int i = first + threadIdx.x / WAVE;
    if (i >= n_kp) return;
    float2 out;
    int status;
    lk_point(P, nl - 1, a.kp[(long long)s * SOF_MAXKP + i], out, status);
    if (lane_id() == 0) {
        a.nxt[(long long)s * SOF_MAXKP + i] = out;
        a.st[(long long)s * SOF_MAXKP + i] = (uint8_t)status;
    }
}

// --------------------------------------------------------------------------------- k_sof_fit
// cv::RNG
__device__ __forceinline__ unsigned rng_next(unsigned long long &state) {
    state = (unsigned long long)(unsigned)state * 4164903690ull + (unsigned)(state >> 32);
    return (unsigned)state;
}
__device__ __forceinline__ int rng_uniform(unsigned long long &state, int n) {
    return (int)(rng_next(state) % (unsigned)n);
}

// AffinePartial2DEstimatorCallback::runKernel (oracle similarity_2pt)
__device__ __forceinline__ void similarity_2pt(float2 f0, float2 f1, float2 t0, float2 t1,
                                               double *M) {
    const double x1 = f0.x, y1 = f0.y, x2 = f1.x, y2 = f1.y;
    const double X1 = t0.x, Y1 = t0.y, X2 = t1.x, Y2 = t1.y;
    const double den = (x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2);
    const double d = 1.0 / den;
    const double S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2));
    const double S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2));
    const double S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) -
                           (X1 * x2 - X2 * x1) * (x1 - x2));
    const double S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) -
                           (Y1 * y2 - Y2 * y1) * (y1 - y2));
    M[0] = S0; M[1] = -S1; M[2] = S2;
    M[3] = S1; M[4] = S0; M[5] = S3;
}

__device__ __forceinline__ bool inlier(const float *F, float2 f, float2 t) {
    const float a = ((F[0] * f.x + F[1] * f.y) + F[2]) - t.x;
    const float b = ((F[3] * f.x + F[4] * f.y) + F[5]) - t.y;
    return a * a + b * b <= 9.0f;   // (float)(3 * 3)
}

__device__ int update_num_iters(double p, double ep, int max_iters) {   // RANSACUpdateNumIters
    p = fmin(fmax(p, 0.0), 1.0);
    ep = fmin(fmax(ep, 0.0), 1.0);
    double num = fmax(1.0 - p, DBL_MIN);
    const double q = 1.0 - ep;
    double denom = 1.0 - q * q;
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

constexpr int FIT_K = 15;   // values reduced together by lm_normal: A (10), v (4), S

struct FitShared {
    double red[SOF_T];
    double redk[FIT_K][SOF_T];
    double models[RB][6];
    int counts[RB];
    double best[6];
    double x[4], d[4], A[16], v[4];
    int max_good, niters, it0, ok;
    double S, Sd, lam, lc;
    int wsum[16];
};

// reduce256: strided partials (element e -> partial e % 256, increasing e), halving tree
__device__ __forceinline__ double reduce256(double p, FitShared &sh) {
    const int t = threadIdx.x;
    sh.red[t] = p;
    __syncthreads();
    for (int h = SOF_T / 2; h > 0; h >>= 1) {
        if (t < h) sh.red[t] = sh.red[t] + sh.red[t + h];
        __syncthreads();
    }
    const double r = sh.red[0];
    __syncthreads();
    return r;
}

// K independent reduce256 sums sharing each tree step's barrier (same order per value)
template <int K>
__device__ __forceinline__ void reduce256_k(const double *p, double *out, FitShared &sh) {
    const int t = threadIdx.x;
    for (int k = 0; k < K; ++k) sh.redk[k][t] = p[k];
    __syncthreads();
    for (int h = SOF_T / 2; h > 0; h >>= 1) {
        if (t < h)
            for (int k = 0; k < K; ++k) sh.redk[k][t] = sh.redk[k][t] + sh.redk[k][t + h];
        __syncthreads();
    }
    for (int k = 0; k < K; ++k) out[k] = sh.redk[k][0];
    __syncthreads();
}

// residual row e of AffinePartial2DRefineCallback::compute (x rows even, y rows odd)
__device__ __forceinline__ double lm_res(const double *x, const float2 *src, const float2 *dst,
                                         int e) {
    const float2 M = src[e >> 1], m = dst[e >> 1];
    const double Mx = M.x, My = M.y;
    if ((e & 1) == 0) return ((x[0] * Mx - x[1] * My) + x[2]) - (double)m.x;
    return ((x[1] * Mx + x[0] * My) + x[3]) - (double)m.y;
}
__device__ __forceinline__ void lm_jrow(const float2 *src, int e, double *J) {
    const float2 M = src[e >> 1];
    const double Mx = M.x, My = M.y;
    if ((e & 1) == 0) {
        J[0] = Mx; J[1] = -My; J[2] = 1.0; J[3] = 0.0;
    } else {
        J[0] = My; J[1] = Mx; J[2] = 0.0; J[3] = 1.0;
    }
}

// Cholesky solve of a 4x4 SPD system (oracle chol_solve4); false if not positive definite.
__device__ bool chol_solve4(const double *A, const double *b, double *x) {
    double L[4][4] = {};
    for (int j = 0; j < 4; ++j) {
        double s = A[4 * j + j];
        for (int k = 0; k < j; ++k) s = s - L[j][k] * L[j][k];
        if (!(s > 0.0)) return false;
        L[j][j] = sqrt(s);
        for (int i = j + 1; i < 4; ++i) {
            double t = A[4 * i + j];
            for (int k = 0; k < j; ++k) t = t - L[i][k] * L[j][k];
            L[i][j] = t / L[j][j];
        }
    }
    double y[4];
    for (int i = 0; i < 4; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t = t - L[i][k] * y[k];
        y[i] = t / L[i][i];
    }
    for (int i = 3; i >= 0; --i) {
        double t = y[i];
        for (int k = i + 1; k < 4; ++k) t = t - L[k][i] * x[k];
        x[i] = t / L[i][i];
    }
    return true;
}

__device__ __forceinline__ double dot4(const double *a, const double *b) {
    return ((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3];
}

// A = J^T J, v = J^T r over the 2n rows of the inliers (reduce256 order); r from x.
__device__ void lm_normal(const double *x, const float2 *src, const float2 *dst, int rows,
                          FitShared &sh, double *A, double *v, double *S, double *rmax) {
    const int t = threadIdx.x;
    double pa[10] = {}, pv[4] = {}, ps = 0.0, pm = 0.0;
    for (int e = t; e < rows; e += SOF_T) {
        double J[4];
        lm_jrow(src, e, J);
        const double r = lm_res(x, src, dst, e);
        int q = 0;
        for (int i = 0; i < 4; ++i)
            for (int j = i; j < 4; ++j) pa[q] = pa[q] + J[i] * J[j], ++q;
        for (int i = 0; i < 4; ++i) pv[i] = pv[i] + J[i] * r;
        ps = ps + r * r;
        pm = fmax(pm, fabs(r));
    }
    double vals[FIT_K], sums[FIT_K];
    for (int k = 0; k < 10; ++k) vals[k] = pa[k];
    for (int k = 0; k < 4; ++k) vals[10 + k] = pv[k];
    vals[14] = ps;
    reduce256_k<FIT_K>(vals, sums, sh);
    int q = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j, ++q) A[4 * i + j] = A[4 * j + i] = sums[q];
    for (int i = 0; i < 4; ++i) v[i] = sums[10 + i];
    *S = sums[14];
    // max |r|: order-free
    pm = wave_reduce(RED_MAX, pm);
    if (lane_id() == 0) sh.red[t / WAVE] = pm;
    __syncthreads();
    double m = 0.0;
    for (int k = 0; k < SOF_T / WAVE; ++k) m = fmax(m, sh.red[k]);
    *rmax = m;
    __syncthreads();
}

__device__ void lm_sum_sq(const double *x, const float2 *src, const float2 *dst, int rows,
                          FitShared &sh, double *S) {
    double ps = 0.0;
    for (int e = threadIdx.x; e < rows; e += SOF_T) {
        const double r = lm_res(x, src, dst, e);
        ps = ps + r * r;
    }
    *S = reduce256(ps, sh);
}

// cv::LMSolver::run (oracle lm_refine) on the block; x in/out (every thread holds it).
__device__ void lm_refine(double *x, const float2 *src, const float2 *dst, int n, FitShared &sh) {
    const int t = threadIdx.x, rows = 2 * n;
    const double eps = (double)FLT_EPSILON;
    double A[16], v[4], S, rmax, D[4];
    lm_normal(x, src, dst, rows, sh, A, v, &S, &rmax);
    for (int i = 0; i < 4; ++i) D[i] = A[4 * i + i];
    double lam = 1.0, lc = 0.75;
    int it = 0;
    for (;;) {
        double Ap[16], d[4];
        for (int k = 0; k < 16; ++k) Ap[k] = A[k];
        for (int i = 0; i < 4; ++i) Ap[4 * i + i] = Ap[4 * i + i] + lam * D[i];
        if (!chol_solve4(Ap, v, d)) break;
        double xd[4];
        for (int i = 0; i < 4; ++i) xd[i] = x[i] - d[i];
        double Sd;
        lm_sum_sq(xd, src, dst, rows, sh, &Sd);
        double temp[4];
        for (int i = 0; i < 4; ++i) temp[i] = -dot4(A + 4 * i, d) + 2.0 * v[i];
        const double dS = dot4(d, temp);
        const double R = (S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1.0);
        if (R > 0.75) {
            lam *= 0.5;
            if (lam < lc) lam = 0.0;
        } else if (R < 0.25) {
            const double tt = dot4(d, v);
            double nu = (Sd - S) / (fabs(tt) > DBL_EPSILON ? tt : 1.0) + 2.0;
            nu = fmin(fmax(nu, 2.0), 10.0);
            if (lam == 0.0) {
                double maxval = DBL_EPSILON;
                for (int i = 0; i < 4; ++i) {
                    double e[4] = {0.0, 0.0, 0.0, 0.0}, col[4];
                    e[i] = 1.0;
                    if (chol_solve4(A, e, col)) maxval = fmax(maxval, fabs(col[i]));
                }
                lam = lc = 1.0 / maxval;
                nu *= 0.5;
            }
            lam *= nu;
        }
        if (Sd < S) {
            S = Sd;
            for (int i = 0; i < 4; ++i) x[i] = xd[i];
            double Sx;
            lm_normal(x, src, dst, rows, sh, A, v, &Sx, &rmax);
        }
        ++it;
        double dmax = 0.0;
        for (int i = 0; i < 4; ++i) dmax = fmax(dmax, fabs(d[i]));
        if (!(it < SOF_REFINE_ITERS && dmax >= eps && rmax >= eps)) break;
    }
    (void)t;
}

// estimateAffinePartial2D(src, dst, RANSAC) + refinement over n >= 3 pairs; M out; false: none.
__device__ bool ransac_fit(const float2 *src, const float2 *dst, int n, float2 *isrc,
                           float2 *idst, double *M, FitShared &sh) {
    const int t = threadIdx.x, lane = lane_id(), wv = t / WAVE;
    unsigned long long rng = 0xFFFFFFFFFFFFFFFFull;   // RNG((uint64)-1)
    if (t == 0) {
        sh.max_good = 0;
        sh.niters = SOF_RANSAC_ITERS;
        sh.it0 = 0;
    }
    __syncthreads();
    while (sh.it0 < sh.niters) {
        if (t == 0)
            for (int b = 0; b < RB; ++b) {   // getSubset: two distinct indices
                const int i0 = rng_uniform(rng, n);
                int i1 = rng_uniform(rng, n);
                while (i1 == i0) i1 = rng_uniform(rng, n);
                similarity_2pt(src[i0], src[i1], dst[i0], dst[i1], sh.models[b]);
            }
        __syncthreads();
        for (int b = wv * (RB / 4); b < (wv + 1) * (RB / 4); ++b) {
            float F[6];
            for (int k = 0; k < 6; ++k) F[k] = (float)sh.models[b][k];
            int cnt = 0;
            for (int i0 = 0; i0 < n; i0 += WAVE) {
                const int i = i0 + lane;
                const bool in = i < n && inlier(F, src[i], dst[i]);
                cnt += __popcll(__ballot(in));
            }
            if (lane == 0) sh.counts[b] = cnt;
        }
        __syncthreads();
        if (t == 0) {
            for (int b = 0; b < RB; ++b) {
                if (sh.it0 + b >= sh.niters) break;
                const int g = sh.counts[b];
                if (g > (sh.max_good > 1 ? sh.max_good : 1)) {
                    sh.max_good = g;
                    for (int k = 0; k < 6; ++k) sh.best[k] = sh.models[b][k];
                    sh.niters = update_num_iters(0.99, (double)(n - g) / n, sh.niters);
                }
            }
            sh.it0 += RB;
        }
        __syncthreads();
    }
    if (sh.max_good <= 0) return false;
    float F[6];
    for (int k = 0; k < 6; ++k) F[k] = (float)sh.best[k];
    const int ni = block_compact(
        n, sh.wsum, [&](int i) { return inlier(F, src[i], dst[i]); },
        [&](int i, int pos) {
            isrc[pos] = src[i];
            idst[pos] = dst[i];
        });
    block_sync();
    double x[4] = {sh.best[0], sh.best[3], sh.best[2], sh.best[5]};
    if (ni > 0) lm_refine(x, isrc, idst, ni, sh);
    M[0] = x[0]; M[1] = -x[1]; M[2] = x[2];
    M[3] = x[1]; M[4] = x[0]; M[5] = x[3];
    return true;
}

__global__ __launch_bounds__(SOF_T) void k_sof_fit(SofArgs a) {
    __shared__ FitShared sh;
    const int s = blockIdx.x, t = threadIdx.x;
    const SofState &st = a.state[s];
    double *W = a.warps + 6LL * s;
    if (st.mode == MODE_NOKP || st.mode == MODE_SKIP) {   // sof.py:106-111 (no points: identity)
        if (t == 0) {
            identity6(W);
            a.state[s].outcome = OUT_IDENT;
        }
        return;
    }
    if (st.mode != MODE_LK) return;
    float2 *kp = a.kp + (long long)s * SOF_MAXKP;
    const float2 *nx = a.nxt + (long long)s * SOF_MAXKP;
    const uint8_t *stt = a.st + (long long)s * SOF_MAXKP;
    float2 *csrc = a.fit + (long long)s * 4 * SOF_MAXKP, *cdst = csrc + SOF_MAXKP;
    float2 *isrc = cdst + SOF_MAXKP, *idst = isrc + SOF_MAXKP;
    // sof.py:119-121: keep the points LK tracked (the stored corners shrink for good)
    const int m = block_compact(
        st.n_kp, sh.wsum, [&](int i) { return stt[i] == 1; },
        [&](int i, int pos) {
            csrc[pos] = kp[i];
            cdst[pos] = nx[i];
        });
    block_sync();
    for (int i = t; i < m; i += SOF_T) kp[i] = csrc[i];
    double M[6];
    bool ok = false;
    if (m == 2) {   // count == modelPoints: the 2-point model, no refinement
        similarity_2pt(csrc[0], csrc[1], cdst[0], cdst[1], M);
        ok = true;
    } else if (m > 2) {
        ok = ransac_fit(csrc, cdst, m, isrc, idst, M, sh);
    }
    if (t == 0) {
        SofState &o = a.state[s];
        o.n_kp = m;
        if (ok) {   // sof.py:153-160
            o.prev = 1 - st.prev;
            M[2] /= a.scale;
            M[5] /= a.scale;
            for (int k = 0; k < 6; ++k) W[k] = M[k];
            o.outcome = OUT_EST;
        } else {
            identity6(W);
            o.outcome = OUT_IDENT;
        }
    }
}

// ------------------------------------------------------------------------------- KAT kernels
__global__ __launch_bounds__(GFTT_T) void k_kat_gftt(const uint8_t *g, const uint8_t *mask, int h,
                                                    int w, float *cov, float *eig,
                                                    unsigned long long *keys, long long keys_cap,
                                                    float2 *out, int *n_out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ GfttShared sh;
    gftt_body(g, mask, h, w, cov, eig, keys, keys_cap, (unsigned long long *)smem, out, n_out, sh);
}

__global__ __launch_bounds__(PYR_T) void k_kat_pyr(uint8_t *img, short2 *der, int h, int w) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    pyr_levels_body(img, der, h, w, smem, PYR_LDS);
}

__global__ __launch_bounds__(256) void k_kat_lk(const uint8_t *pimg, const short2 *pder,
                                                const uint8_t *nimg, int h, int w,
                                                const float2 *pts, int n, float2 *out,
                                                uint8_t *status) {
    const int i = blockIdx.x * (256 / WAVE) + threadIdx.x / WAVE;
    if (i >= n) return;
    const int nl = sof_nlevels(h, w);
    const LkPyr P{pimg, pder, nimg, h, w, h, w};
    float2 o;
    int stv;
    lk_point(P, nl - 1, pts[i], o, stv);
    if (lane_id() == 0) {
        out[i] = o;
        status[i] = (uint8_t)stv;
    }
}

__global__ __launch_bounds__(SOF_T) void k_kat_affine(const float2 *src, const float2 *dst, int n,
                                                      float2 *isrc, float2 *idst, double *M,
                                                      int *ok) {
    __shared__ FitShared sh;
    double m[6];
    bool r = false;
    if (n == 2) {
        similarity_2pt(src[0], src[1], dst[0], dst[1], m);
        r = true;
    } else if (n > 2) {
        r = ransac_fit(src, dst, n, isrc, idst, m, sh);
    }
    if (threadIdx.x == 0) {
        *ok = r ? 1 : 0;
        for (int k = 0; k < 6; ++k) M[k] = r ? m[k] : 0.0;
    }
}

__global__ __launch_bounds__(256) void k_kat_small(const uint8_t *f, int H, int W, double scale,
                                                   int h0, int w0, uint8_t *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= h0 * w0) return;
    const int oy = i / w0, ox = i - oy * w0;
    out[i] = (uint8_t)small_pixel(f, H, W, scale, ox, oy);
}

__global__ __launch_bounds__(GFTT_T) void k_kat_eig(const uint8_t *g, int h, int w, float *cov,
                                                   float *eig) {
    // the eigenvalue stage of gftt_body alone (mask = nothing; candidates are not needed)
    __shared__ GfttShared sh;
    const int t = threadIdx.x, nt = blockDim.x, n = h * w;
    const double scale = 1.0 / (4 * 3 * 255);
    const float k0 = (float)(1.0 * scale), k1 = (float)(2.0 * scale);
    float *c0 = cov, *c1 = cov + n, *c2 = cov + 2 * n;
    for (int i = t; i < n; i += nt) {
        const int y = i / w, x = i - y * w;
        const int ym = refl(y - 1, h), yp = refl(y + 1, h);
        const int xm = refl(x - 1, w), xp = refl(x + 1, w);
        auto S = [&](int yy, int xx) { return (float)g[(long long)yy * w + xx]; };
        const float r0 = S(ym, xp) - S(ym, xm), r1 = S(y, xp) - S(y, xm), r2 = S(yp, xp) - S(yp, xm);
        const float dx = r1 * k1 + (r0 + r2) * k0;
        const float qm = S(ym, x) * k1 + (S(ym, xm) + S(ym, xp)) * k0;
        const float qp = S(yp, x) * k1 + (S(yp, xm) + S(yp, xp)) * k0;
        const float dy = qp - qm;
        c0[i] = dx * dx;
        c1[i] = dx * dy;
        c2[i] = dy * dy;
    }
    block_sync();
    (void)sh;
    for (int i = t; i < n; i += nt) {
        const int y = i / w, x = i - y * w;
        const int ys[3] = {refl(y - 1, h), y, refl(y + 1, h)};
        const int xs[3] = {refl(x - 1, w), x, refl(x + 1, w)};
        float bx[3];
        const float *cs[3] = {c0, c1, c2};
        for (int c = 0; c < 3; ++c) {
            double rs[3];
            for (int r = 0; r < 3; ++r) {
                const float *row = cs[c] + (long long)ys[r] * w;
                rs[r] = ((double)row[xs[0]] + (double)row[xs[1]]) + (double)row[xs[2]];
            }
            bx[c] = (float)((rs[0] + rs[1]) + rs[2]);
        }
        const float A = bx[0] * 0.5f, B = bx[1], C = bx[2] * 0.5f;
        eig[i] = (A + C) - sqrtf((A - C) * (A - C) + B * B);
    }
}

}  // namespace
}  // namespace yta

using namespace yta;

struct yta_sof {
    int device = 0, S = 0;
    double scale = 0.1;
    int max_h = 0, max_w = 0;
    hipStream_t stream = nullptr;
    SofArgs a{};
    std::vector<void *> allocs;
    // host staging
    uint8_t *d_frames = nullptr;
    long long frames_cap = 0;
    long long *d_frame_off = nullptr;
    int *d_frame_hw = nullptr;
    double *d_dets = nullptr;
    long long dets_cap = 0;
    int *d_det_off = nullptr;
    double *d_warps = nullptr;
    SofState *h_state = nullptr;
};

namespace {

template <typename T>
int sof_alloc(yta_sof *e, T **p, long long n) {
    void *q = nullptr;
    if (n <= 0) n = 1;
    hipError_t err = hipMalloc(&q, sizeof(T) * (size_t)n);
    if (err != hipSuccess) {
        set_error("hipMalloc(%lld bytes) failed: %s", (long long)(sizeof(T) * n),
                  hipGetErrorString(err));
        return YTA_ERR_NOMEM;
    }
    e->allocs.push_back(q);
    *p = static_cast<T *>(q);
    return YTA_OK;
}
#define SOF_ALLOC(ptr, n)                     \
    do {                                      \
        int _rc = sof_alloc(e, &(ptr), (n));  \
        if (_rc) return _rc;                  \
    } while (0)

long long next_pow2(long long v) {
    long long p = 1;
    while (p < v) p <<= 1;
    return p;
}

void sof_free(yta_sof *e) {
    for (void *p : e->allocs) (void)hipFree(p);
    e->allocs.clear();
    if (e->d_frames) (void)hipFree(e->d_frames);
    if (e->d_dets) (void)hipFree(e->d_dets);
    if (e->h_state) (void)hipHostFree(e->h_state);
    e->d_frames = nullptr;
    e->d_dets = nullptr;
    e->h_state = nullptr;
    e->frames_cap = e->dets_cap = 0;
}

int sof_buffers(yta_sof *e) {
    SofArgs &a = e->a;
    const long long S = e->S;
    a.S = e->S;
    a.scale = e->scale;
    a.h0max = (int)std::rint(e->max_h * e->scale);
    a.w0max = (int)std::rint(e->max_w * e->scale);
    YTA_CHECK(a.h0max >= 1 && a.w0max >= 1, YTA_ERR_INVALID, "frames scale to an empty image");
    a.npx = (long long)a.h0max * a.w0max;
    a.slot_px = (sof_slot_px(a.h0max, a.w0max) + 15) & ~15LL;
    a.keys_cap = next_pow2(a.npx);
    SOF_ALLOC(a.img, S * 2 * a.slot_px);
    SOF_ALLOC(a.der, S * 2 * a.slot_px);
    SOF_ALLOC(a.kp, S * SOF_MAXKP);
    SOF_ALLOC(a.nxt, S * SOF_MAXKP);
    SOF_ALLOC(a.st, S * SOF_MAXKP);
    SOF_ALLOC(a.fit, S * 4 * SOF_MAXKP);
    SOF_ALLOC(a.cov, S * 3 * a.npx);
    SOF_ALLOC(a.eig, S * a.npx);
    SOF_ALLOC(a.mask, S * a.npx);
    SOF_ALLOC(a.keys, S * a.keys_cap);
    SOF_ALLOC(a.state, S);
    SOF_ALLOC(e->d_frame_off, S);
    SOF_ALLOC(e->d_frame_hw, 2 * S);
    SOF_ALLOC(e->d_det_off, S + 1);
    SOF_ALLOC(e->d_warps, 6 * S);
    YTA_HIP(hipHostMalloc((void **)&e->h_state, sizeof(SofState) * S, hipHostMallocDefault));
    return YTA_OK;
}

int sof_launch(yta_sof *e) {
    SofArgs &a = e->a;
    const int blocks = (int)((a.npx + 255) / 256);
    hipLaunchKernelGGL(k_sof_small, dim3(blocks, a.S), dim3(256), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_sof_pyr, dim3(a.S), dim3(PYR_T), PYR_LDS, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_sof_gftt, dim3(a.S), dim3(GFTT_T), SORT_CAP * 8, e->stream, a);
    YTA_HIP(hipGetLastError());
    const dim3 glk((SOF_MAXKP + LKB / WAVE - 1) / (LKB / WAVE), a.S);
    if (a.slot_px <= PYR_LDS)
        hipLaunchKernelGGL(k_sof_lk<true>, glk, dim3(LKB), (size_t)a.slot_px, e->stream, a);
    else
        hipLaunchKernelGGL(k_sof_lk<false>, glk, dim3(LKB), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_sof_fit, dim3(a.S), dim3(SOF_T), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int set_sof_lds() {
    static bool done = false;
    if (done) return YTA_OK;
    YTA_HIP(hipFuncSetAttribute((const void *)k_sof_gftt,
                                hipFuncAttributeMaxDynamicSharedMemorySize, SORT_CAP * 8));
    YTA_HIP(hipFuncSetAttribute((const void *)k_kat_gftt,
                                hipFuncAttributeMaxDynamicSharedMemorySize, SORT_CAP * 8));
    for (const void *k : {(const void *)k_sof_pyr, (const void *)k_kat_pyr,
                          (const void *)k_sof_lk<true>})
        YTA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, PYR_LDS));
    done = true;
    return YTA_OK;
}

// frame / det sizes of a host-buffer call
int check_frames(yta_sof *e, const long long *frame_off, const int *frame_hw, long long *bytes) {
    long long b = 0;
    for (int s = 0; s < e->S; ++s) {
        const int h = frame_hw[2 * s], w = frame_hw[2 * s + 1];
        YTA_CHECK(h >= 1 && w >= 1 && frame_off[s] >= 0, YTA_ERR_INVALID,
                  "stream %d: bad frame %d x %d at offset %lld", s, h, w, frame_off[s]);
        b = std::max(b, frame_off[s] + (long long)h * w * 3);
    }
    *bytes = b;
    return YTA_OK;
}

}  // namespace

namespace {
// ------------------------------------------------------------------------------------- KATs
int kat_copy_in(void **d, const void *h, size_t bytes) {
    YTA_HIP(hipMalloc(d, bytes ? bytes : 1));
    if (bytes) YTA_HIP(hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice));
    return YTA_OK;
}

struct KatMem {
    std::vector<void *> p;
    ~KatMem() {
        for (void *q : p) (void)hipFree(q);
    }
    template <typename T>
    int alloc(T **d, long long n) {
        void *q = nullptr;
        YTA_HIP(hipMalloc(&q, sizeof(T) * (size_t)(n > 0 ? n : 1)));
        p.push_back(q);
        *d = (T *)q;
        return YTA_OK;
    }
    template <typename T, typename U>
    int in(T **d, const U *h, long long n) {
        void *q = nullptr;
        int rc = kat_copy_in(&q, h, sizeof(U) * (size_t)(n > 0 ? n : 0));
        if (rc) return rc;
        p.push_back(q);
        *d = (T *)q;
        return YTA_OK;
    }
};
#define KAT(x)             \
    do {                   \
        int _r = (x);      \
        if (_r) return _r; \
    } while (0)

}  // namespace

extern "C" {

int yta_sof_create(int device, int n_streams, double scale, int max_h, int max_w,
                   yta_sof **engine) {
    YTA_CHECK(engine, YTA_ERR_INVALID, "null engine");
    *engine = nullptr;
    YTA_CHECK(n_streams > 0 && max_h > 0 && max_w > 0, YTA_ERR_INVALID,
              "n_streams, max_h and max_w must be positive");
    YTA_CHECK(scale > 0.0 && scale <= 1.0, YTA_ERR_INVALID, "scale must be in (0, 1]");
    int rc = select_device(device);
    if (rc) return rc;
    rc = set_sof_lds();
    if (rc) return rc;
    yta_sof *e = new (std::nothrow) yta_sof();
    YTA_CHECK(e, YTA_ERR_NOMEM, "out of host memory");
    e->device = device;
    e->S = n_streams;
    e->scale = scale;
    e->max_h = max_h;
    e->max_w = max_w;
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        set_error("hipStreamCreate: %s", hipGetErrorString(he));
        delete e;
        return YTA_ERR_HIP;
    }
    rc = sof_buffers(e);
    if (!rc) rc = yta_sof_reset(e);
    if (rc) {
        yta_sof_destroy(e);
        return rc;
    }
    *engine = e;
    return YTA_OK;
}

int yta_sof_destroy(yta_sof *e) {
    if (!e) return YTA_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)host_wait(e->stream);
    sof_free(e);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return YTA_OK;
}

int yta_sof_reset(yta_sof *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(hipMemsetAsync(e->a.state, 0, sizeof(SofState) * e->S, e->stream));
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

int yta_sof_apply_device(yta_sof *e, const uint8_t *d_frames, const long long *d_frame_off,
                         const int *d_frame_hw, const double *d_dets, int det_stride,
                         const int *d_det_off, double *d_warps) {
    YTA_CHECK(e && d_frames && d_frame_off && d_frame_hw && d_det_off && d_warps, YTA_ERR_INVALID,
              "null argument");
    YTA_CHECK(det_stride >= 4, YTA_ERR_INVALID, "det_stride must be >= 4");
    YTA_HIP(hipSetDevice(e->device));
    SofArgs &a = e->a;
    a.frames = d_frames;
    a.frame_off = d_frame_off;
    a.frame_hw = d_frame_hw;
    a.dets = d_dets;
    a.det_stride = det_stride;
    a.det_off = d_det_off;
    a.warps = d_warps;
    return sof_launch(e);
}

int yta_sof_sync(yta_sof *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(hipMemcpyAsync(e->h_state, e->a.state, sizeof(SofState) * e->S, hipMemcpyDeviceToHost,
                           e->stream));
    YTA_HIP(host_wait(e->stream));
    for (int s = 0; s < e->S; ++s)
        YTA_CHECK(!(e->h_state[s].err & SOF_ERR_SIZE), YTA_ERR_CAPACITY,
                  "stream %d: frame larger than the engine's max_h x max_w", s);
    return YTA_OK;
}

int yta_sof_apply(yta_sof *e, const uint8_t *frames, const long long *frame_off,
                  const int *frame_hw, const double *dets, int det_stride, const int *det_off,
                  double *warps) {
    YTA_CHECK(e && frames && frame_off && frame_hw && det_off && warps, YTA_ERR_INVALID,
              "null argument");
    YTA_CHECK(det_stride >= 4, YTA_ERR_INVALID, "det_stride must be >= 4");
    YTA_CHECK(det_off[0] == 0, YTA_ERR_INVALID, "det_off[0] must be 0");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    long long bytes = 0;
    int rc = check_frames(e, frame_off, frame_hw, &bytes);
    if (rc) return rc;
    int mh = e->max_h, mw = e->max_w;
    for (int s = 0; s < S; ++s) {
        mh = std::max(mh, frame_hw[2 * s]);
        mw = std::max(mw, frame_hw[2 * s + 1]);
        YTA_CHECK(det_off[s + 1] >= det_off[s], YTA_ERR_INVALID, "det_off must be non-decreasing");
    }
    if (mh > e->max_h || mw > e->max_w) {
        // grow, keeping every stream's state: the stored frame's pyramid and derivatives (packed
        // from the slot start at the stored frame's own size), the corners and SofState
        YTA_HIP(host_wait(e->stream));
        const SofArgs old = e->a;
        std::vector<void *> old_allocs;
        old_allocs.swap(e->allocs);
        if (e->h_state) (void)hipHostFree(e->h_state);
        e->h_state = nullptr;
        e->max_h = mh;
        e->max_w = mw;
        rc = sof_buffers(e);
        if (!rc) rc = yta_sof_reset(e);
        if (!rc) {
            SofArgs &a = e->a;
            const size_t rows = (size_t)S * 2;
            YTA_HIP(hipMemcpy2DAsync(a.img, a.slot_px, old.img, old.slot_px, old.slot_px, rows,
                                     hipMemcpyDeviceToDevice, e->stream));
            YTA_HIP(hipMemcpy2DAsync(a.der, a.slot_px * sizeof(short2), old.der,
                                     old.slot_px * sizeof(short2), old.slot_px * sizeof(short2),
                                     rows, hipMemcpyDeviceToDevice, e->stream));
            YTA_HIP(hipMemcpyAsync(a.kp, old.kp, sizeof(float2) * S * SOF_MAXKP,
                                   hipMemcpyDeviceToDevice, e->stream));
            YTA_HIP(hipMemcpyAsync(a.state, old.state, sizeof(SofState) * S,
                                   hipMemcpyDeviceToDevice, e->stream));
            rc = host_wait(e->stream) == hipSuccess ? YTA_OK : YTA_ERR_HIP;
        }
        for (void *p : old_allocs) (void)hipFree(p);
        if (rc) return rc;
    }
    if (bytes > e->frames_cap) {
        if (e->d_frames) (void)hipFree(e->d_frames);
        e->d_frames = nullptr;
        e->frames_cap = 0;
        YTA_HIP(hipMalloc((void **)&e->d_frames, (size_t)bytes));
        e->frames_cap = bytes;
    }
    const long long nd = det_off[S];
    if (nd * det_stride > e->dets_cap) {
        if (e->d_dets) (void)hipFree(e->d_dets);
        e->d_dets = nullptr;
        e->dets_cap = 0;
        YTA_HIP(hipMalloc((void **)&e->d_dets, sizeof(double) * (size_t)std::max(1LL, nd * det_stride)));
        e->dets_cap = std::max(1LL, nd * det_stride);
    }
    YTA_CHECK(nd == 0 || dets, YTA_ERR_INVALID, "null dets");
    YTA_HIP(hipMemcpyAsync(e->d_frames, frames, (size_t)bytes, hipMemcpyHostToDevice, e->stream));
    if (nd)
        YTA_HIP(hipMemcpyAsync(e->d_dets, dets, sizeof(double) * nd * det_stride,
                               hipMemcpyHostToDevice, e->stream));
    YTA_HIP(hipMemcpyAsync(e->d_frame_off, frame_off, sizeof(long long) * S, hipMemcpyHostToDevice,
                           e->stream));
    YTA_HIP(hipMemcpyAsync(e->d_frame_hw, frame_hw, sizeof(int) * 2 * S, hipMemcpyHostToDevice,
                           e->stream));
    YTA_HIP(hipMemcpyAsync(e->d_det_off, det_off, sizeof(int) * (S + 1), hipMemcpyHostToDevice,
                           e->stream));
    rc = yta_sof_apply_device(e, e->d_frames, e->d_frame_off, e->d_frame_hw, e->d_dets, det_stride,
                              e->d_det_off, e->d_warps);
    if (rc) return rc;
    YTA_HIP(hipMemcpyAsync(warps, e->d_warps, sizeof(double) * 6 * S, hipMemcpyDeviceToHost,
                           e->stream));
    return yta_sof_sync(e);
}

int yta_sof_get_state(yta_sof *e, int stream, int *initialized, int *n_kp, float *kp, int cap,
                      int *h, int *w, uint8_t *prev_img, int img_cap) {
    YTA_CHECK(e && initialized && n_kp && h && w, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream out of range");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(host_wait(e->stream));
    SofState st;
    YTA_HIP(hipMemcpy(&st, e->a.state + stream, sizeof(st), hipMemcpyDeviceToHost));
    *initialized = st.init;
    *n_kp = st.n_kp;
    *h = st.init ? st.h0[st.prev] : 0;
    *w = st.init ? st.w0[st.prev] : 0;
    if (kp && st.n_kp > 0) {
        YTA_CHECK(cap >= st.n_kp, YTA_ERR_CAPACITY, "kp holds %d points, %d stored", cap, st.n_kp);
        YTA_HIP(hipMemcpy(kp, e->a.kp + (long long)stream * SOF_MAXKP, sizeof(float2) * st.n_kp,
                          hipMemcpyDeviceToHost));
    }
    if (prev_img && st.init) {
        const long long n = (long long)(*h) * (*w);
        YTA_CHECK(img_cap >= n, YTA_ERR_CAPACITY, "prev_img holds %d bytes, %lld needed", img_cap, n);
        YTA_HIP(hipMemcpy(prev_img, e->a.img + ((long long)stream * 2 + st.prev) * e->a.slot_px,
                          (size_t)n, hipMemcpyDeviceToHost));
    }
    return YTA_OK;
}

int yta_sof_outcome(yta_sof *e, int *outcome) {
    YTA_CHECK(e && outcome, YTA_ERR_INVALID, "null argument");
    int rc = yta_sof_sync(e);
    if (rc) return rc;
    for (int s = 0; s < e->S; ++s) outcome[s] = e->h_state[s].outcome;
    return YTA_OK;
}

int yta_sof_hip_stream(yta_sof *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

int yta_sof_kat_preprocess(int device, const uint8_t *frame, int h, int w, double scale,
                           uint8_t *out, int *out_h, int *out_w) {
    YTA_CHECK(frame && out && out_h && out_w && h > 0 && w > 0 && scale > 0, YTA_ERR_INVALID,
              "bad argument");
    KAT(select_device(device));
    const int h0 = (int)std::rint(h * scale), w0 = (int)std::rint(w * scale);
    YTA_CHECK(h0 >= 1 && w0 >= 1, YTA_ERR_INVALID, "empty output");
    KatMem m;
    const uint8_t *df;
    uint8_t *dout;
    KAT(m.in(&df, frame, 3LL * h * w));
    KAT(m.alloc(&dout, (long long)h0 * w0));
    hipLaunchKernelGGL(k_kat_small, dim3((h0 * w0 + 255) / 256), dim3(256), 0, 0, df, h, w, scale,
                       h0, w0, dout);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(out, dout, (size_t)h0 * w0, hipMemcpyDeviceToHost));
    *out_h = h0;
    *out_w = w0;
    return YTA_OK;
}

int yta_sof_kat_min_eigen(int device, const uint8_t *gray, int h, int w, float *eig) {
    YTA_CHECK(gray && eig && h > 0 && w > 0, YTA_ERR_INVALID, "bad argument");
    KAT(select_device(device));
    KatMem m;
    const uint8_t *dg;
    float *dcov, *deig;
    KAT(m.in(&dg, gray, (long long)h * w));
    KAT(m.alloc(&dcov, 3LL * h * w));
    KAT(m.alloc(&deig, (long long)h * w));
    hipLaunchKernelGGL(k_kat_eig, dim3(1), dim3(GFTT_T), 0, 0, dg, h, w, dcov, deig);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(eig, deig, sizeof(float) * h * w, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_sof_kat_corners(int device, const uint8_t *gray, const uint8_t *mask, int h, int w,
                        float *corners, int *n) {
    YTA_CHECK(gray && mask && corners && n && h > 0 && w > 0, YTA_ERR_INVALID, "bad argument");
    KAT(select_device(device));
    KAT(set_sof_lds());
    KatMem m;
    const uint8_t *dg, *dm;
    float *dcov, *deig;
    unsigned long long *dk;
    float2 *dout;
    int *dn;
    const long long cap = next_pow2((long long)h * w);
    KAT(m.in(&dg, gray, (long long)h * w));
    KAT(m.in(&dm, mask, (long long)h * w));
    KAT(m.alloc(&dcov, 3LL * h * w));
    KAT(m.alloc(&deig, (long long)h * w));
    KAT(m.alloc(&dk, cap));
    KAT(m.alloc(&dout, SOF_MAXKP));
    KAT(m.alloc(&dn, 1));
    hipLaunchKernelGGL(k_kat_gftt, dim3(1), dim3(GFTT_T), SORT_CAP * 8, 0, dg, dm, h, w, dcov, deig,
                       dk, cap, dout, dn);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(n, dn, sizeof(int), hipMemcpyDeviceToHost));
    if (*n > 0) YTA_HIP(hipMemcpy(corners, dout, sizeof(float2) * *n, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_sof_kat_lk(int device, const uint8_t *prev, const uint8_t *next, int h, int w,
                   const float *pts, int n, float *next_pts, uint8_t *status) {
    YTA_CHECK(prev && next && h > 0 && w > 0 && n >= 0 && (n == 0 || (pts && next_pts && status)),
              YTA_ERR_INVALID, "bad argument");
    KAT(select_device(device));
    KAT(set_sof_lds());
    if (n == 0) return YTA_OK;
    KatMem m;
    const long long px = sof_slot_px(h, w);
    uint8_t *pi, *ni;
    short2 *pd, *nd;
    const float2 *dp;
    float2 *dout;
    uint8_t *dst;
    KAT(m.alloc(&pi, px));
    KAT(m.alloc(&ni, px));
    KAT(m.alloc(&pd, px));
    KAT(m.alloc(&nd, px));
    KAT(m.in(&dp, (const float2 *)pts, n));
    KAT(m.alloc(&dout, n));
    KAT(m.alloc(&dst, n));
    YTA_HIP(hipMemcpy(pi, prev, (size_t)h * w, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(ni, next, (size_t)h * w, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_kat_pyr, dim3(1), dim3(PYR_T), PYR_LDS, 0, pi, pd, h, w);
    hipLaunchKernelGGL(k_kat_pyr, dim3(1), dim3(PYR_T), PYR_LDS, 0, ni, nd, h, w);
    hipLaunchKernelGGL(k_kat_lk, dim3((n + 3) / 4), dim3(256), 0, 0, pi, pd, ni, h, w, dp, n, dout,
                       dst);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(next_pts, dout, sizeof(float2) * n, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(status, dst, (size_t)n, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_sof_kat_affine(int device, const float *src, const float *dst, int n, double *M, int *ok) {
    YTA_CHECK(M && ok && n >= 0 && (n == 0 || (src && dst)), YTA_ERR_INVALID, "bad argument");
    KAT(select_device(device));
    KatMem m;
    const float2 *ds, *dd;
    float2 *is, *id;
    double *dM;
    int *dok;
    KAT(m.in(&ds, (const float2 *)src, n));
    KAT(m.in(&dd, (const float2 *)dst, n));
    KAT(m.alloc(&is, n));
    KAT(m.alloc(&id, n));
    KAT(m.alloc(&dM, 6));
    KAT(m.alloc(&dok, 1));
    hipLaunchKernelGGL(k_kat_affine, dim3(1), dim3(SOF_T), 0, 0, ds, dd, n, is, id, dM, dok);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(M, dM, sizeof(double) * 6, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(ok, dok, sizeof(int), hipMemcpyDeviceToHost));
    return YTA_OK;
}

}  // extern "C"
