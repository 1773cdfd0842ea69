// ECC camera-motion compensation for S camera streams on gfx950.
//
// Reference: boxmot/motion/cmc/ecc.py:13-104 (ECC.apply: preprocess, cv2.findTransformECC(prev,
// curr, eye, warp_mode, (COUNT | EPS, max_iter, eps), None, 1), identity when it raises, the
// translation divided by `scale`), cmc_interface.py:26-40 (preprocess); get_cmc_method('ecc')
// (motion/cmc/__init__.py:9-11) is what HybridSORT builds (hybridsort.py:366).  OpenCV's
// findTransformECC (Gauss-Newton on the enhanced correlation coefficient, warpAffine with
// WARP_INVERSE_MAP) is restated in oracle/cmc_ecc.py; this file reproduces that restatement: the
// same fixed-point warp coordinates, exact float32 bilinear samples, float32 per-pixel arithmetic
// without fused multiply-adds (the Makefile's -ffp-contract=off) and float64 image sums in the
// fixed order oracle/cmc_ecc.py block_sum() names.
//
// One frame of every stream = 2 launches:
//   k_ecc_small  [grid, pixel/thread]  gray + INTER_LINEAR resize into the stream's current slot
//   k_ecc        [block/stream, 1024]  the whole Gauss-Newton loop of one stream in one block:
//                                      the current frame staged in LDS (u8; gradients are
//                                      0.5 * (I[x+1] - I[x-1]) with reflect-101 borders, formed
//                                      from the staged bytes where a bilinear tap needs them), the
//                                      template (previous accepted frame) read from HBM/L2 at its
//                                      own pixel; per iteration three passes over the template
//                                      grid (masked moments; Hessian, projections, correlation;
//                                      error projection), each closed by a block reduction, and
//                                      the small solves done redundantly by every thread so that
//                                      the loop's exit is block-uniform.
// align=True's preview image (ecc.py:91-98) is a third, on-demand launch: k_ecc_align
// [grid, pixel/thread] warps the retired template with the returned matrix (yta_ecc_aligned).
//
// HBM layout per stream: two u8 slots (previous accepted frame / current frame) of
// round(max_h * scale) x round(max_w * scale) bytes, EccState, the 2x3 float32 warp.
#include <algorithm>
#include <type_traits>
#include <cfloat>
#include <cmath>
#include <new>
#include <vector>

#include "cmc_small.hpp"
#include "common.hpp"

namespace yta {
namespace {
using namespace cmc;

constexpr int ECC_LDS = 144 * 1024;         // k_ecc's dynamic LDS (warp tables + packed frame)

enum { ECC_TRANSLATION = 0, ECC_EUCLIDEAN = 1, ECC_AFFINE = 2 };
enum { ECC_OUT_FIRST = 0, ECC_OUT_EST = 1, ECC_OUT_FAIL = 2 };
constexpr int ECC_ERR_SIZE = 1;

struct EccState {
    int init, prev;
    int h[2], w[2];
    int outcome, iters, err, pad;
    double rho;
};

struct EccArgs {
    int S;
    double scale;
    int hmax, wmax;
    long long slot_px;
    int mode, max_iter;
    double eps;
    uint8_t *img;        // [S][2][slot_px]
    EccState *state;
    const uint8_t *frames;
    const long long *frame_off;
    const int *frame_hw;
    float *warps;        // [S][6]
};

__host__ __device__ constexpr int ecc_nparams(int mode) {
    return mode == ECC_TRANSLATION ? 2 : mode == ECC_EUCLIDEAN ? 3 : 6;
}

// k_ecc's block: 1024 threads, 512 for the affine model (34 float64 sums per thread in pass B)
#ifndef ECC_T1
#define ECC_T1 1024
#endif
__host__ __device__ constexpr int ecc_threads(int mode) {
    return mode == ECC_AFFINE ? 512 : mode == ECC_EUCLIDEAN ? ECC_T1 : 1024;
}
// unrolling of the three pixel loops (moments; Hessian + projections; error projection)
#ifndef ECC_UA
#define ECC_UA 4
#endif
#ifndef ECC_UB
#define ECC_UB 1
#endif
#ifndef ECC_UC
#define ECC_UC 2
#endif
#define ECC_PRAGMA(x) _Pragma(#x)
#define ECC_UNROLL(n) ECC_PRAGMA(unroll n)

// ------------------------------------------------------------------------------- k_ecc_small
__global__ __launch_bounds__(256) void k_ecc_small(EccArgs a) {
    const int s = blockIdx.y;
    EccState &st = a.state[s];
    const int H = a.frame_hw[2 * s], W = a.frame_hw[2 * s + 1];
    const int h0 = (int)rint(H * a.scale), w0 = (int)rint(W * a.scale);
    const int cur = 1 - st.prev;
    // findTransformECC takes template and input of different sizes: only a frame larger than the
    // slots is refused (an error for this frame; the host-buffer path grows the slots first)
    const bool fits = H >= 1 && W >= 1 && h0 >= 1 && w0 >= 1 && h0 <= a.hmax && w0 <= a.wmax;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st.err = fits ? 0 : ECC_ERR_SIZE;
        if (fits) {
            st.h[cur] = h0;
            st.w[cur] = w0;
        }
    }
    if (!fits) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= h0 * w0) return;
    const int oy = i / w0, ox = i - oy * w0;
    uint8_t *dst = a.img + ((long long)s * 2 + cur) * a.slot_px;
    dst[i] = (uint8_t)small_pixel(a.frames + a.frame_off[s], H, W, a.scale, ox, oy);
}

// ------------------------------------------------------------------------------------ k_ecc
// warpAffine's fixed-point coordinates (WarpAffineInvoker, WARP_INVERSE_MAP): AB_BITS = 10,
// INTER_BITS = 5; cvRound = round half to even, saturated to int32; the XY map is int16.
__device__ __forceinline__ int cv_round(double v) {
    const double r = rint(v);
    return r <= -2147483648.0 ? INT_MIN : r >= 2147483647.0 ? INT_MAX : (int)r;
}

__device__ __forceinline__ int sat16(int v) { return min(max(v, -32768), 32767); }

// block-uniform values pinned to scalar registers (they come from LDS, which the compiler does not
// know to be uniform)
__device__ __forceinline__ float uni(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double uni(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

struct Warped {
    float iw, gx, gy;   // bilinear samples of the image and its gradients (BORDER_CONSTANT 0)
    bool m;             // nearest sample of the all-ones premask
};

// The current frame in LDS, one word per pixel: the byte, and 2 x the x / y gradients (the
// filter2D (-0.5, 0, 0.5) responses with reflect-101 borders are half-integers in
// [-127.5, 127.5]) biased by 255 in 9 bits each.  One LDS read per bilinear tap.
struct PackedSrc {
    const unsigned *p;
    int hd, wd;
    // pixel q: the byte and 2 x the gradients (integers)
    __device__ __forceinline__ void tap(int q, int &v, int &g2x, int &g2y) const {
        const unsigned w = p[q];
        v = (int)(w & 255u);
        g2x = (int)__builtin_amdgcn_ubfe(w, 8, 9) - 255;
        g2y = (int)__builtin_amdgcn_ubfe(w, 17, 9) - 255;
    }
};

__device__ __forceinline__ unsigned pack_px(const uint8_t *img, int hd, int wd, int q) {
    const int r = q / wd, u = q - r * wd, row = r * wd;
    const int gx2 = (int)img[row + refl(u + 1, wd)] - (int)img[row + refl(u - 1, wd)];
    const int gy2 = (int)img[refl(r + 1, hd) * wd + u] - (int)img[refl(r - 1, hd) * wd + u];
    return (unsigned)img[q] | ((unsigned)(gx2 + 255) << 8) | ((unsigned)(gy2 + 255) << 17);
}

// The current frame's bytes in HBM (frames too large for the LDS stage): gradients formed from
// the neighbouring bytes at every tap.
struct RawSrc {
    const uint8_t *p;
    int hd, wd;
    __device__ __forceinline__ void tap(int q, int &v, int &g2x, int &g2y) const {
        const int r = q / wd, u = q - r * wd, row = r * wd;
        v = p[q];
        g2x = (int)p[row + refl(u + 1, wd)] - (int)p[row + refl(u - 1, wd)];
        g2y = (int)p[refl(r + 1, hd) * wd + u] - (int)p[refl(r - 1, hd) * wd + u];
    }
};

// warpAffine's per-row and per-column fixed-point terms of one iteration's map (LDS):
// xr / yr[y] = cvRound((M1 y + M2) 1024) / cvRound((M4 y + M5) 1024),
// ad / bd[x] = cvRound(M0 x 1024) / cvRound(M3 x 1024) (WarpAffineInvoker's adelta / bdelta).
struct WarpTabs {
    int *xr, *yr, *ad, *bd;
};

// One template pixel (x, y) warped into the current frame.  remapBilinear's float32 sum
// ((v00 w0 + v01 w1) + v10 w2) + v11 w3 with the table's weights (32 - f)(32 - g) / 1024 ... is
// exact here (u8 or half-integer values, 11-bit weights, < 2^24 in every partial sum), so it is
// formed as the integer sum of weight numerators x values, scaled by 2^-10 (2^-11 for the
// gradients, which are stored doubled): the same float32 bits in any order.
template <bool GRAD, typename Src>
__device__ __forceinline__ Warped warp_px(const Src &src, const WarpTabs &tb, int x, int y) {
    const int xr = tb.xr[y], yr = tb.yr[y], ad = tb.ad[x], bd = tb.bd[x];
    const int X = (xr + 16 + ad) >> 5, Y = (yr + 16 + bd) >> 5;
    const int sx = sat16(X >> 5), sy = sat16(Y >> 5);
    const int nx = sat16((xr + 512 + ad) >> 10), ny = sat16((yr + 512 + bd) >> 10);
    const int fx = X & 31, fy = Y & 31;
    const int wn[4] = {(32 - fx) * (32 - fy), fx * (32 - fy), (32 - fx) * fy, fx * fy};
    const int wd = src.wd, hd = src.hd;
    int si = 0, sgx = 0, sgy = 0;
    const int q0 = sy * wd + sx;
    if ((unsigned)sx < (unsigned)(wd - 1) && (unsigned)sy < (unsigned)(hd - 1)) {   // interior
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int v, g2x, g2y;
            src.tap(q0 + (k & 1) + (k >> 1) * wd, v, g2x, g2y);
            si += wn[k] * v;
            if (GRAD) {
                sgx += wn[k] * g2x;
                sgy += wn[k] * g2y;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int u = sx + (k & 1), r = sy + (k >> 1);
            if ((unsigned)u < (unsigned)wd && (unsigned)r < (unsigned)hd) {
                int v, g2x, g2y;
                src.tap(r * wd + u, v, g2x, g2y);
                si += wn[k] * v;
                if (GRAD) {
                    sgx += wn[k] * g2x;
                    sgy += wn[k] * g2y;
                }
            }
        }
    }
    Warped o;
    o.iw = (float)si * (1.f / 1024);
    o.gx = GRAD ? (float)sgx * (1.f / 2048) : 0.f;
    o.gy = GRAD ? (float)sgy * (1.f / 2048) : 0.f;
    o.m = (unsigned)nx < (unsigned)wd && (unsigned)ny < (unsigned)hd;
    return o;
}

// pixels t, t + T, ... of a w-wide grid in raster order, (x, y) stepped without divisions
struct PixIter {
    int x, y, dx, dy, w;
    __device__ __forceinline__ PixIter(int p0, int step, int w_) : w(w_) {
        y = p0 / w_;
        x = p0 - y * w_;
        dy = step / w_;
        dx = step - dy * w_;
    }
    __device__ __forceinline__ void next() {
        x += dx;
        y += dy;
        if (x >= w) {
            x -= w;
            ++y;
        }
    }
};

// image_jacobian_{translation, euclidean, affine}_ECC (ecc.cpp) at one pixel, float32
template <int MODE>
__device__ __forceinline__ void jac(float gx, float gy, float X, float Y, float c, float s,
                                    float *J) {
    if constexpr (MODE == ECC_TRANSLATION) {
        J[0] = gx;
        J[1] = gy;
    } else if constexpr (MODE == ECC_EUCLIDEAN) {
        const float hx = (-(X * s)) - (Y * c), hy = (X * c) - (Y * s);
        J[0] = (gx * hx) + (gy * hy);
        J[1] = gx;
        J[2] = gy;
    } else {
        J[0] = gx * X;
        J[1] = gy * X;
        J[2] = gx * Y;
        J[3] = gy * Y;
        J[4] = gx;
        J[5] = gy;
    }
}

// Block sum of K float64 values over T threads, identical in every thread: a halving tree inside
// each 16-lane row (DPP row shifts), the T / 16 row partials through LDS, then for each value one
// wave runs the halving tree over its row partials (lane i holds partial i; bpermute for the
// cross-row strides, DPP within rows) - oracle/cmc_ecc.py block_sum.  red: K x T/16 doubles.
template <int T, int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double *red, double *tot) {
    constexpr int NR = T / 16, NW = T / WAVE;
    const int t = threadIdx.x, lane = t & (WAVE - 1), wave = t / WAVE;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v[k] = v[k] + dpp_f64<0x108>(v[k]);   // row_shl:8
        v[k] = v[k] + dpp_f64<0x104>(v[k]);
        v[k] = v[k] + dpp_f64<0x102>(v[k]);
        v[k] = v[k] + dpp_f64<0x101>(v[k]);
    }
    if ((t & 15) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[k * NR + (t >> 4)] = v[k];
    __syncthreads();
    for (int k = wave; k < K; k += NW) {   // wave-uniform
        double x = lane < NR ? red[k * NR + lane] : 0.0;
        if (NR > 32) x = x + __shfl_down(x, 32, WAVE);
        if (NR > 16) x = x + __shfl_down(x, 16, WAVE);
        x = x + dpp_f64<0x108>(x);
        x = x + dpp_f64<0x104>(x);
        x = x + dpp_f64<0x102>(x);
        x = x + dpp_f64<0x101>(x);
        if (lane == 0) tot[k] = x;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = tot[k];
}

// cv::invert(DECOMP_LU) of the float32 Hessian: closed forms for n <= 3 (float64 cofactors),
// hal::LU32f (float32 elimination with partial pivoting) for n = 6; zeros when singular.
template <int N>
__device__ __forceinline__ void invert(const float (*H)[6], float (*D)[6], float (*A)[6]) {
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) D[i][j] = 0.f;
    if constexpr (N == 2) {
        double d = (double)H[0][0] * H[1][1] - (double)H[0][1] * H[1][0];
        if (d != 0.0) {
            d = 1.0 / d;
            D[1][1] = (float)(H[0][0] * d);
            D[0][0] = (float)(H[1][1] * d);
            D[0][1] = (float)(-H[0][1] * d);
            D[1][0] = (float)(-H[1][0] * d);
        }
    } else if constexpr (N == 3) {
        const float(*S)[6] = H;
        double d = S[0][0] * ((double)S[1][1] * S[2][2] - (double)S[1][2] * S[2][1]) -
                   S[0][1] * ((double)S[1][0] * S[2][2] - (double)S[1][2] * S[2][0]) +
                   S[0][2] * ((double)S[1][0] * S[2][1] - (double)S[1][1] * S[2][0]);
        if (d != 0.0) {
            d = 1.0 / d;
            float(*R)[6] = D;
            R[0][0] = (float)(((double)S[1][1] * S[2][2] - (double)S[1][2] * S[2][1]) * d);
            R[0][1] = (float)(((double)S[0][2] * S[2][1] - (double)S[0][1] * S[2][2]) * d);
            R[0][2] = (float)(((double)S[0][1] * S[1][2] - (double)S[0][2] * S[1][1]) * d);
            R[1][0] = (float)(((double)S[1][2] * S[2][0] - (double)S[1][0] * S[2][2]) * d);
            R[1][1] = (float)(((double)S[0][0] * S[2][2] - (double)S[0][2] * S[2][0]) * d);
            R[1][2] = (float)(((double)S[0][2] * S[1][0] - (double)S[0][0] * S[1][2]) * d);
            R[2][0] = (float)(((double)S[1][0] * S[2][1] - (double)S[1][1] * S[2][0]) * d);
            R[2][1] = (float)(((double)S[0][1] * S[2][0] - (double)S[0][0] * S[2][1]) * d);
            R[2][2] = (float)(((double)S[0][0] * S[1][1] - (double)S[0][1] * S[1][0]) * d);
        }
    } else {
        for (int i = 0; i < N; ++i)
            for (int j = 0; j < N; ++j) {
                A[i][j] = H[i][j];
                D[i][j] = i == j ? 1.f : 0.f;
            }
        const float eps = FLT_EPSILON * 10;
        for (int i = 0; i < N; ++i) {
            int k = i;
            for (int j = i + 1; j < N; ++j)
                if (fabsf(A[j][i]) > fabsf(A[k][i])) k = j;
            if (fabsf(A[k][i]) < eps) {
                for (int p = 0; p < N; ++p)
                    for (int q = 0; q < N; ++q) D[p][q] = 0.f;
                return;
            }
            if (k != i) {
                for (int j = i; j < N; ++j) {
                    const float tmp = A[i][j];
                    A[i][j] = A[k][j];
                    A[k][j] = tmp;
                }
                for (int j = 0; j < N; ++j) {
                    const float tmp = D[i][j];
                    D[i][j] = D[k][j];
                    D[k][j] = tmp;
                }
            }
            const float dd = -1.f / A[i][i];
            for (int j = i + 1; j < N; ++j) {
                const float alpha = A[j][i] * dd;
                for (int q = i + 1; q < N; ++q) A[j][q] = A[j][q] + alpha * A[i][q];
                for (int q = 0; q < N; ++q) D[j][q] = D[j][q] + alpha * D[i][q];
            }
        }
        for (int i = N - 1; i >= 0; --i)
            for (int j = 0; j < N; ++j) {
                float sacc = D[i][j];
                for (int q = i + 1; q < N; ++q) sacc = sacc - A[i][q] * D[q][j];
                D[i][j] = sacc / A[i][i];
            }
    }
}

template <int N>
__device__ __forceinline__ void gemv(const float (*A)[6], const float *x, float *y) {
    for (int i = 0; i < N; ++i) {
        double acc = 0.0;
        for (int k = 0; k < N; ++k) acc = acc + (double)A[i][k] * (double)x[k];
        y[i] = (float)acc;
    }
}

template <int N>
__device__ __forceinline__ double dot64(const float *a, const float *b) {
    double acc = 0.0;
    for (int k = 0; k < N; ++k) acc = acc + (double)a[k] * (double)b[k];
    return acc;
}

// The whole findTransformECC loop of stream blockIdx.x (oracle/cmc_ecc.py find_transform_ecc).
// Thread 0 does the small solves in LDS between the passes; the loop's control values are read
// back by every thread after a barrier, so its exit is block-uniform.
#ifdef YTA_STAMPS
// diagnostic build: block 0's time per phase of the loop, summed over iterations (100 MHz ticks)
#define ECC_PH(k)                                                 \
    do {                                                          \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                \
            const unsigned long long now = wall_clock64();        \
            ph[k] += now - ph_t;                                  \
            ph_t = now;                                           \
        }                                                         \
    } while (0)
#else
#define ECC_PH(k) \
    do {          \
    } while (0)
#endif

struct EccSolve {
    float H[6][6], Hi[6][6], A[6][6];
    float P[6], Q[6], iph[6], E[6], dp[6];
    float m[6];
    double lam, rho;
    int fail;
};

template <bool PACKED, int MODE>
__global__ __launch_bounds__(ecc_threads(MODE)) void k_ecc(EccArgs a) {
    constexpr int T = ecc_threads(MODE);
    constexpr int N = ecc_nparams(MODE);
    constexpr int NB = N * (N + 1) / 2 + 2 * N + 1;   // pass B sums
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[NB * (T / 16)], tot[NB];
    __shared__ EccSolve sv;
    const int s = blockIdx.x, t = threadIdx.x;
    EccState &st = a.state[s];
    const EccState st0 = st;
    float *W = a.warps + 6 * (long long)s;
    __syncthreads();   // every thread holds st0 before thread 0 rewrites the state
    if (st0.err) {
        if (t < 6) W[t] = (t == 0 || t == 4) ? 1.f : 0.f;
        return;
    }
    const int cur = 1 - st0.prev;
    if (!st0.init) {   // ecc.py:66-68: the first frame becomes prev_img, the identity returned
        if (t < 6) W[t] = (t == 0 || t == 4) ? 1.f : 0.f;
        if (t == 0) {
            st.init = 1;
            st.prev = cur;
            st.outcome = ECC_OUT_FIRST;
            st.iters = 0;
            st.rho = 0.0;
        }
        return;
    }
    // (selects, not indexing: a dynamically indexed local array would live in scratch)
    const int hs = st0.prev ? st0.h[1] : st0.h[0], ws = st0.prev ? st0.w[1] : st0.w[0];
    const int hd = cur ? st0.h[1] : st0.h[0], wd = cur ? st0.w[1] : st0.w[0];
    const uint8_t *gtmpl = a.img + ((long long)s * 2 + st0.prev) * a.slot_px;
    const uint8_t *gimg = a.img + ((long long)s * 2 + cur) * a.slot_px;
    const int npx = hs * ws, nd = hd * wd;
    // LDS: the warp tables, then (PACKED) the current frame's words and the template's bytes
    WarpTabs tb;
    tb.xr = reinterpret_cast<int *>(smem);
    tb.yr = tb.xr + hs;
    tb.ad = tb.yr + hs;
    tb.bd = tb.ad + ws;
    const long long tab_bytes = ((2LL * (hs + ws) * 4) + 15) & ~15LL;
    unsigned *words = reinterpret_cast<unsigned *>(smem + tab_bytes);
    uint8_t *ltmpl = reinterpret_cast<uint8_t *>(words + nd);
    if (PACKED) {
        for (int q = t; q < nd; q += T) words[q] = pack_px(gimg, hd, wd, q);
        for (int q = t; q < npx; q += T) ltmpl[q] = gtmpl[q];
    }
    if (t < 6) sv.m[t] = (t == 0 || t == 4) ? 1.f : 0.f;
    const uint8_t *tmpl = PACKED ? (const uint8_t *)ltmpl : gtmpl;
    using Src = typename std::conditional<PACKED, PackedSrc, RawSrc>::type;
    Src src;
    if constexpr (PACKED) src.p = words;
    else src.p = gimg;
    src.hd = hd;
    src.wd = wd;
    float m[6] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f};
    double rho = -1.0, last_rho = -a.eps;
    int it = 0;
    bool fail = false;
#ifdef YTA_STAMPS
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ph_t = wall_clock64();
    const unsigned long long clk0 = clock64();
#endif
    __syncthreads();
    ECC_PH(0);
    while (it < a.max_iter && fabs(rho - last_rho) >= a.eps) {
        ++it;
        {   // this iteration's warp tables
            const double M[6] = {uni((double)m[0]), uni((double)m[1]), uni((double)m[2]),
                                 uni((double)m[3]), uni((double)m[4]), uni((double)m[5])};
            for (int k = t; k < hs; k += T) {
                tb.xr[k] = cv_round((M[1] * k + M[2]) * 1024.0);
                tb.yr[k] = cv_round((M[4] * k + M[5]) * 1024.0);
            }
            for (int k = t; k < ws; k += T) {
                tb.ad[k] = cv_round(M[0] * k * 1024.0);
                tb.bd[k] = cv_round(M[3] * k * 1024.0);
            }
            __syncthreads();
        }
        ECC_PH(1);
        // pass A: meanStdDev of the warped image and of the template over the warped mask
        double va[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        PixIter pa(t, T, ws);
        ECC_UNROLL(ECC_UA)
        for (int p = t; p < npx; p += T, pa.next()) {
            const int x = pa.x, y = pa.y;
            const Warped q = warp_px<false>(src, tb, x, y);
            if (q.m) {
                const double iw = q.iw, tv = (double)tmpl[p];
                va[0] = va[0] + iw;
                va[1] = fma(iw, iw, va[1]);   // products of float32 values are exact in float64
                va[2] = va[2] + tv;
                va[3] = fma(tv, tv, va[3]);
                va[4] = va[4] + 1.0;
            }
        }
        ECC_PH(2);
        block_sum<T>(va, red, tot);
        ECC_PH(3);
#pragma unroll
        for (int k = 0; k < 5; ++k) va[k] = uni(va[k]);
        const double cnt = va[4];
        const double sc = cnt != 0.0 ? 1.0 / cnt : 0.0;
        const double img_mean = va[0] * sc, tmp_mean = va[2] * sc;
        const double img_std = sqrt(fmax(va[1] * sc - img_mean * img_mean, 0.0));
        const double tmp_std = sqrt(fmax(va[3] * sc - tmp_mean * tmp_mean, 0.0));
        const float img_mean_f = uni((float)img_mean), tmp_mean_f = uni((float)tmp_mean);
        const double tmp_norm = sqrt(cnt * tmp_std * tmp_std);
        const double img_norm = sqrt(cnt * img_std * img_std);
        const float c = uni(m[0]), sn = uni(m[3]);
        // pass B: Hessian (upper triangle), image / template projections, correlation
        double vb[NB];
#pragma unroll
        for (int k = 0; k < NB; ++k) vb[k] = 0.0;
        PixIter pb(t, T, ws);
        ECC_UNROLL(ECC_UB)
        for (int p = t; p < npx; p += T, pb.next()) {
            const int x = pb.x, y = pb.y;
            const Warped q = warp_px<true>(src, tb, x, y);
            const float tv = (float)tmpl[p];
            const float iwz = q.m ? q.iw - img_mean_f : q.iw;
            const float tz = q.m ? tv - tmp_mean_f : 0.f;
            float J[N];
            jac<MODE>(q.gx, q.gy, (float)x, (float)y, c, sn, J);
            int k = 0;
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int j = i; j < N; ++j, ++k) vb[k] = fma((double)J[i], (double)J[j], vb[k]);
#pragma unroll
            for (int i = 0; i < N; ++i) vb[k + i] = fma((double)J[i], (double)iwz, vb[k + i]);
#pragma unroll
            for (int i = 0; i < N; ++i) vb[k + N + i] = fma((double)J[i], (double)tz, vb[k + N + i]);
            vb[k + 2 * N] = fma((double)tz, (double)iwz, vb[k + 2 * N]);
        }
        ECC_PH(4);
        block_sum<T>(vb, red, tot);
        ECC_PH(3);
        if (t == 0) {
            int k = 0;
            for (int i = 0; i < N; ++i)
                for (int j = i; j < N; ++j, ++k) {
                    if (i == j) {
                        const double r = sqrt(tot[k]);
                        sv.H[i][i] = (float)(r * r);
                    } else {
                        sv.H[i][j] = sv.H[j][i] = (float)tot[k];
                    }
                }
            for (int i = 0; i < N; ++i) {
                sv.P[i] = (float)tot[k + i];
                sv.Q[i] = (float)tot[k + N + i];
            }
            const double corr = tot[k + 2 * N];
            invert<N>(sv.H, sv.Hi, sv.A);
            const double r = corr / (img_norm * tmp_norm);
            sv.rho = r;
            sv.fail = 0;
            if (isnan(r)) {
                sv.fail = 1;
            } else {
                gemv<N>(sv.Hi, sv.P, sv.iph);
                const double lambda_n = img_norm * img_norm - dot64<N>(sv.P, sv.iph);
                const double lambda_d = corr - dot64<N>(sv.Q, sv.iph);
                if (lambda_d <= 0.0) sv.fail = 1;
                else sv.lam = lambda_n / lambda_d;
            }
        }
        __syncthreads();
        ECC_PH(5);
        last_rho = rho;
        rho = sv.rho;
        if (sv.fail) {
            fail = true;
            break;
        }
        const double lam = uni(sv.lam);
        // pass C: projection of the error image lambda * templateZM - imageWarped
        double vc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) vc[k] = 0.0;
        PixIter pc(t, T, ws);
        ECC_UNROLL(ECC_UC)
        for (int p = t; p < npx; p += T, pc.next()) {
            const int x = pc.x, y = pc.y;
            const Warped q = warp_px<true>(src, tb, x, y);
            const float tv = (float)tmpl[p];
            const float iwz = q.m ? q.iw - img_mean_f : q.iw;
            const float tz = q.m ? tv - tmp_mean_f : 0.f;
            const float e = (float)(lam * (double)tz - (double)iwz);
            float J[N];
            jac<MODE>(q.gx, q.gy, (float)x, (float)y, c, sn, J);
#pragma unroll
            for (int i = 0; i < N; ++i) vc[i] = fma((double)J[i], (double)e, vc[i]);
        }
        ECC_PH(6);
        block_sum<T>(vc, red, tot);
        ECC_PH(3);
        if (t == 0) {   // update_warping_matrix_ECC
            for (int i = 0; i < N; ++i) sv.E[i] = (float)tot[i];
            gemv<N>(sv.Hi, sv.E, sv.dp);
            float *w = sv.m;
            const float *dp = sv.dp;
            if (MODE == ECC_TRANSLATION) {
                w[2] = w[2] + dp[0];
                w[5] = w[5] + dp[1];
            } else if (MODE == ECC_AFFINE) {
                w[0] = w[0] + dp[0];
                w[3] = w[3] + dp[1];
                w[1] = w[1] + dp[2];
                w[4] = w[4] + dp[3];
                w[2] = w[2] + dp[4];
                w[5] = w[5] + dp[5];
            } else {
                const double theta = (double)dp[0] + asin((double)w[3]);
                w[2] = w[2] + dp[1];
                w[5] = w[5] + dp[2];
                w[0] = w[4] = (float)cos(theta);
                w[3] = (float)sin(theta);
                w[1] = -w[3];
            }
        }
        __syncthreads();
        ECC_PH(5);
#pragma unroll
        for (int k = 0; k < 6; ++k) m[k] = uni(sv.m[k]);
    }
#ifdef YTA_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int k = 0; k < 9; ++k)
            g_stamps[k] = k == 7 ? (unsigned long long)it : k == 8 ? clock64() - clk0 : ph[k];
#endif
    if (fail) {   // ecc.py:82-84: the identity, prev_img kept
        if (t < 6) W[t] = (t == 0 || t == 4) ? 1.f : 0.f;
        if (t == 0) {
            st.outcome = ECC_OUT_FAIL;
            st.iters = it;
            st.rho = rho;
        }
        return;
    }
    if (t == 0 && a.scale < 1.0) {   // ecc.py:87-89 (float32 division, NumPy's float32 scalars)
        sv.m[2] = sv.m[2] / (float)a.scale;
        sv.m[5] = sv.m[5] / (float)a.scale;
    }
    __syncthreads();
    if (t < 6) W[t] = sv.m[t];
    if (t == 0) {
        st.prev = cur;   // ecc.py:102
        st.outcome = ECC_OUT_EST;
        st.iters = it;
        st.rho = rho;
    }
}

// --------------------------------------------------------------------------------- k_ecc_align
// align=True (ecc.py:91-98): cv2.warpAffine(prev_img, warp, (w, h), INTER_LINEAR) of the template
// the last estimate registered against - the slot that estimate retired (1 - prev), intact until
// the next frame's k_ecc_small - with the returned warp (translation already divided by the
// scale).  Without WARP_INVERSE_MAP warpAffine inverts the float64-widened matrix first
// (imgwarp.cpp), then the same WarpAffineInvoker fixed-point map as warp_px, and remapBilinear's
// u8 path: the 15-bit integer table ((32 - fy)(32 - fx) 32, ...), taps outside the image 0
// (BORDER_CONSTANT), (sum + 2^14) >> 15.  One pixel per thread; streams whose last outcome was
// not an estimate are skipped (the reference returns before ecc.py:91 there).
__global__ __launch_bounds__(256) void k_ecc_align(EccArgs a, int s, uint8_t *out) {
    const EccState &st = a.state[s];
    if (!st.init || st.outcome != ECC_OUT_EST) return;
    const int slot = 1 - st.prev;
    const int h = st.h[slot], w = st.w[slot];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= h * w) return;
    const int y = i / w, x = i - y * w;
    double M[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) M[k] = (double)a.warps[6 * s + k];
    double D = M[0] * M[4] - M[1] * M[3];
    D = D != 0.0 ? 1.0 / D : 0.0;
    const double A11 = M[4] * D, A22 = M[0] * D;
    M[0] = A11;
    M[1] *= -D;
    M[3] *= -D;
    M[4] = A22;
    const double b1 = -M[0] * M[2] - M[1] * M[5];
    const double b2 = -M[3] * M[2] - M[4] * M[5];
    M[2] = b1;
    M[5] = b2;
    const int xr = cv_round((M[1] * y + M[2]) * 1024.0), yr = cv_round((M[4] * y + M[5]) * 1024.0);
    const int ad = cv_round(M[0] * x * 1024.0), bd = cv_round(M[3] * x * 1024.0);
    const int X = (xr + 16 + ad) >> 5, Y = (yr + 16 + bd) >> 5;
    const int sx = sat16(X >> 5), sy = sat16(Y >> 5);
    const int fx = X & 31, fy = Y & 31;
    const int wn[4] = {(32 - fx) * (32 - fy) * 32, fx * (32 - fy) * 32, (32 - fx) * fy * 32,
                       fx * fy * 32};
    const uint8_t *p = a.img + ((long long)s * 2 + slot) * a.slot_px;
    int acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int xx = sx + (k & 1), yy = sy + (k >> 1);
        if ((unsigned)xx < (unsigned)w && (unsigned)yy < (unsigned)h) acc += (int)p[yy * w + xx] * wn[k];
    }
    out[i] = (uint8_t)min(max((acc + (1 << 14)) >> 15, 0), 255);
}

}  // namespace
}  // namespace yta

using namespace yta;

struct yta_ecc {
    int device = 0, S = 0;
    int mode = ECC_EUCLIDEAN, max_iter = 100;
    double eps = 1e-5, scale = 0.1;
    int max_h = 0, max_w = 0;
    hipStream_t stream = nullptr;
    EccArgs a{};
    uint8_t *img = nullptr;
    EccState *state = nullptr;
    float *d_warps = nullptr;
    uint8_t *d_frames = nullptr;
    long long frames_cap = 0;
    long long *d_frame_off = nullptr;
    int *d_frame_hw = nullptr;
    EccState *h_state = nullptr;
    uint8_t *d_aligned = nullptr;   // align=True preview image (yta_ecc_aligned), slot_px bytes
    long long aligned_cap = 0;
};

namespace {

void ecc_free_slots(yta_ecc *e) {
    if (e->img) (void)hipFree(e->img);
    e->img = nullptr;
}

// Allocate the two image slots per stream for frames up to mh x mw.  Transactional: the engine
// (max_h / max_w, the slot geometry in e->a, e->img) changes only on success; the caller frees
// the previous slots (returned in *old) after copying what it keeps out of them.
int ecc_slots(yta_ecc *e, int mh, int mw, uint8_t **old, long long *old_px) {
    EccArgs &a = e->a;
    const int hmax = (int)std::rint(mh * e->scale);
    const int wmax = (int)std::rint(mw * e->scale);
    YTA_CHECK(hmax >= 1 && wmax >= 1, YTA_ERR_INVALID, "frames scale to an empty image");
    YTA_CHECK(8LL * (hmax + wmax) + 16 <= ECC_LDS, YTA_ERR_CAPACITY,
              "scaled frames of %d x %d: the warp tables exceed the LDS stage", hmax, wmax);
    const long long slot_px = ((long long)hmax * wmax + 15) & ~15LL;
    uint8_t *img = nullptr;
    YTA_HIP(hipMalloc((void **)&img, (size_t)(2LL * e->S * slot_px)));
    if (old) *old = e->img;
    if (old_px) *old_px = a.slot_px;
    e->max_h = mh;
    e->max_w = mw;
    a.hmax = hmax;
    a.wmax = wmax;
    a.slot_px = slot_px;
    a.img = e->img = img;
    return YTA_OK;
}

template <bool LDS>
const void *ecc_kernel(int mode) {
    return mode == ECC_TRANSLATION ? (const void *)k_ecc<LDS, ECC_TRANSLATION>
           : mode == ECC_EUCLIDEAN ? (const void *)k_ecc<LDS, ECC_EUCLIDEAN>
                                   : (const void *)k_ecc<LDS, ECC_AFFINE>;
}

int set_ecc_lds() {
    static bool done = false;
    if (done) return YTA_OK;
    for (int mode = 0; mode < 3; ++mode)
        for (const void *k : {ecc_kernel<true>(mode), ecc_kernel<false>(mode)})
            YTA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, ECC_LDS));
    done = true;
    return YTA_OK;
}

int ecc_launch(yta_ecc *e) {
    EccArgs &a = e->a;
    a.state = e->state;
    a.mode = e->mode;
    a.max_iter = e->max_iter;
    a.eps = e->eps;
    a.scale = e->scale;
    a.S = e->S;
    const int blocks = (int)((a.slot_px + 255) / 256);
    hipLaunchKernelGGL(k_ecc_small, dim3(blocks, a.S), dim3(256), 0, e->stream, a);
    YTA_HIP(hipGetLastError());
    // dynamic LDS: the warp tables, then (packed path) 4 B per current-frame pixel + the template
    const long long tab = ((2LL * (a.hmax + a.wmax) * 4) + 15) & ~15LL;
    const bool packed = tab + 5 * a.slot_px <= ECC_LDS;
    const size_t lds = (size_t)(packed ? tab + 5 * a.slot_px : tab);
    void *args[] = {&a};
    YTA_HIP(hipLaunchKernel(packed ? ecc_kernel<true>(e->mode) : ecc_kernel<false>(e->mode),
                            dim3(a.S), dim3(ecc_threads(e->mode)), args, lds, e->stream));
    return YTA_OK;
}

}  // namespace

extern "C" {

int yta_ecc_create(int device, int n_streams, int warp_mode, double eps, int max_iter,
                   double scale, int max_h, int max_w, yta_ecc **engine) {
    YTA_CHECK(engine, YTA_ERR_INVALID, "null engine");
    *engine = nullptr;
    YTA_CHECK(n_streams > 0 && max_h > 0 && max_w > 0, YTA_ERR_INVALID,
              "n_streams, max_h and max_w must be positive");
    YTA_CHECK(warp_mode >= ECC_TRANSLATION && warp_mode <= ECC_AFFINE, YTA_ERR_INVALID,
              "warp_mode %d: MOTION_TRANSLATION (0), MOTION_EUCLIDEAN (1) or MOTION_AFFINE (2)",
              warp_mode);
    YTA_CHECK(scale > 0.0 && scale <= 1.0, YTA_ERR_INVALID, "scale must be in (0, 1]");
    int rc = select_device(device);
    if (rc) return rc;
    rc = set_ecc_lds();
    if (rc) return rc;
    yta_ecc *e = new (std::nothrow) yta_ecc();
    YTA_CHECK(e, YTA_ERR_NOMEM, "out of host memory");
    e->device = device;
    e->S = n_streams;
    e->mode = warp_mode;
    e->eps = eps;
    e->max_iter = max_iter;
    e->scale = scale;
    e->max_h = 0;
    e->max_w = 0;
    hipError_t he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (he != hipSuccess) {
        set_error("hipStreamCreate: %s", hipGetErrorString(he));
        delete e;
        return YTA_ERR_HIP;
    }
    auto fail = [&](int code) {
        yta_ecc_destroy(e);
        return code;
    };
    rc = ecc_slots(e, max_h, max_w, nullptr, nullptr);
    if (rc) return fail(rc);
    if (hipMalloc((void **)&e->state, sizeof(EccState) * n_streams) != hipSuccess ||
        hipMalloc((void **)&e->d_warps, sizeof(float) * 6 * n_streams) != hipSuccess ||
        hipMalloc((void **)&e->d_frame_off, sizeof(long long) * n_streams) != hipSuccess ||
        hipMalloc((void **)&e->d_frame_hw, sizeof(int) * 2 * n_streams) != hipSuccess ||
        hipHostMalloc((void **)&e->h_state, sizeof(EccState) * n_streams,
                      hipHostMallocDefault) != hipSuccess) {
        set_error("ECC engine allocation failed");
        return fail(YTA_ERR_NOMEM);
    }
    rc = yta_ecc_reset(e);
    if (rc) return fail(rc);
    *engine = e;
    return YTA_OK;
}

int yta_ecc_destroy(yta_ecc *e) {
    if (!e) return YTA_OK;
    (void)hipSetDevice(e->device);
    if (e->stream) (void)host_wait(e->stream);
    ecc_free_slots(e);
    for (void *p : {(void *)e->state, (void *)e->d_warps, (void *)e->d_frames,
                    (void *)e->d_frame_off, (void *)e->d_frame_hw, (void *)e->d_aligned})
        if (p) (void)hipFree(p);
    if (e->h_state) (void)hipHostFree(e->h_state);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return YTA_OK;
}

int yta_ecc_reset(yta_ecc *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(hipMemsetAsync(e->state, 0, sizeof(EccState) * e->S, e->stream));
    YTA_HIP(host_wait(e->stream));
    return YTA_OK;
}

int yta_ecc_apply_device(yta_ecc *e, const uint8_t *d_frames, const long long *d_frame_off,
                         const int *d_frame_hw, float *d_warps) {
    YTA_CHECK(e && d_frames && d_frame_off && d_frame_hw && d_warps, YTA_ERR_INVALID,
              "null argument");
    YTA_HIP(hipSetDevice(e->device));
    EccArgs &a = e->a;
    a.frames = d_frames;
    a.frame_off = d_frame_off;
    a.frame_hw = d_frame_hw;
    a.warps = d_warps;
    return ecc_launch(e);
}

int yta_ecc_sync(yta_ecc *e) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null engine");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(hipMemcpyAsync(e->h_state, e->state, sizeof(EccState) * e->S, hipMemcpyDeviceToHost,
                           e->stream));
    YTA_HIP(host_wait(e->stream));
    for (int s = 0; s < e->S; ++s)
        YTA_CHECK(!(e->h_state[s].err & ECC_ERR_SIZE), YTA_ERR_CAPACITY,
                  "stream %d: frame larger than the engine's max_h x max_w", s);
    return YTA_OK;
}

int yta_ecc_apply(yta_ecc *e, const uint8_t *frames, const long long *frame_off,
                  const int *frame_hw, float *warps) {
    YTA_CHECK(e && frames && frame_off && frame_hw && warps, YTA_ERR_INVALID, "null argument");
    YTA_HIP(hipSetDevice(e->device));
    const int S = e->S;
    long long bytes = 0;
    int mh = e->max_h, mw = e->max_w;
    for (int s = 0; s < S; ++s) {
        const int h = frame_hw[2 * s], w = frame_hw[2 * s + 1];
        YTA_CHECK(h >= 1 && w >= 1 && frame_off[s] >= 0, YTA_ERR_INVALID,
                  "stream %d: bad frame %d x %d at offset %lld", s, h, w, frame_off[s]);
        bytes = std::max(bytes, frame_off[s] + (long long)h * w * 3);
        mh = std::max(mh, h);
        mw = std::max(mw, w);
    }
    if (mh > e->max_h || mw > e->max_w) {
        // grow the slots, keeping every stream's previous frame (packed from the slot start);
        // on failure the engine keeps its previous slots and size untouched
        YTA_HIP(host_wait(e->stream));
        uint8_t *old = nullptr;
        long long old_px = 0;
        int rc = ecc_slots(e, mh, mw, &old, &old_px);
        if (rc) return rc;
        if (old) {
            if (hipMemcpy2DAsync(e->img, e->a.slot_px, old, old_px, old_px, (size_t)S * 2,
                                 hipMemcpyDeviceToDevice, e->stream) != hipSuccess ||
                host_wait(e->stream) != hipSuccess)
                rc = YTA_ERR_HIP;
            (void)hipFree(old);
        }
        if (rc) return rc;
    }
    if (bytes > e->frames_cap) {
        if (e->d_frames) (void)hipFree(e->d_frames);
        e->d_frames = nullptr;
        e->frames_cap = 0;
        YTA_HIP(hipMalloc((void **)&e->d_frames, (size_t)bytes));
        e->frames_cap = bytes;
    }
    YTA_HIP(hipMemcpyAsync(e->d_frames, frames, (size_t)bytes, hipMemcpyHostToDevice, e->stream));
    YTA_HIP(hipMemcpyAsync(e->d_frame_off, frame_off, sizeof(long long) * S, hipMemcpyHostToDevice,
                           e->stream));
    YTA_HIP(hipMemcpyAsync(e->d_frame_hw, frame_hw, sizeof(int) * 2 * S, hipMemcpyHostToDevice,
                           e->stream));
    int rc = yta_ecc_apply_device(e, e->d_frames, e->d_frame_off, e->d_frame_hw, e->d_warps);
    if (rc) return rc;
    YTA_HIP(hipMemcpyAsync(warps, e->d_warps, sizeof(float) * 6 * S, hipMemcpyDeviceToHost,
                           e->stream));
    return yta_ecc_sync(e);
}

int yta_ecc_outcome(yta_ecc *e, int *outcome, int *iters, double *rho) {
    YTA_CHECK(e, YTA_ERR_INVALID, "null argument");
    int rc = yta_ecc_sync(e);
    if (rc) return rc;
    for (int s = 0; s < e->S; ++s) {
        if (outcome) outcome[s] = e->h_state[s].outcome;
        if (iters) iters[s] = e->h_state[s].iters;
        if (rho) rho[s] = e->h_state[s].rho;
    }
    return YTA_OK;
}

int yta_ecc_get_state(yta_ecc *e, int stream, int *initialized, int *h, int *w,
                      uint8_t *prev_img, int img_cap) {
    YTA_CHECK(e && initialized && h && w, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream out of range");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(host_wait(e->stream));
    EccState st;
    YTA_HIP(hipMemcpy(&st, e->state + stream, sizeof(st), hipMemcpyDeviceToHost));
    *initialized = st.init;
    *h = st.init ? st.h[st.prev] : 0;
    *w = st.init ? st.w[st.prev] : 0;
    if (prev_img && st.init) {
        const long long n = (long long)(*h) * (*w);
        YTA_CHECK(img_cap >= n, YTA_ERR_CAPACITY, "prev_img holds %d bytes, %lld needed", img_cap, n);
        YTA_HIP(hipMemcpy(prev_img, e->img + ((long long)stream * 2 + st.prev) * e->a.slot_px,
                          (size_t)n, hipMemcpyDeviceToHost));
    }
    return YTA_OK;
}

int yta_ecc_aligned(yta_ecc *e, int stream, uint8_t *out, long long cap, int *h, int *w) {
    YTA_CHECK(e && h && w, YTA_ERR_INVALID, "null argument");
    YTA_CHECK(stream >= 0 && stream < e->S, YTA_ERR_INVALID, "stream out of range");
    YTA_HIP(hipSetDevice(e->device));
    YTA_HIP(host_wait(e->stream));
    EccState st;
    YTA_HIP(hipMemcpy(&st, e->state + stream, sizeof(st), hipMemcpyDeviceToHost));
    *h = 0;
    *w = 0;
    if (!st.init || st.outcome != ECC_OUT_EST || !e->a.warps) return YTA_OK;
    const int slot = 1 - st.prev;
    const long long n = (long long)st.h[slot] * st.w[slot];
    YTA_CHECK(n > 0 && n <= e->a.slot_px, YTA_ERR_INVALID, "stream %d: bad template size", stream);
    if (!out) {   // size query
        *h = st.h[slot];
        *w = st.w[slot];
        return YTA_OK;
    }
    YTA_CHECK(cap >= n, YTA_ERR_CAPACITY, "out holds %lld bytes, %lld needed", cap, n);
    if (e->aligned_cap < e->a.slot_px) {
        if (e->d_aligned) (void)hipFree(e->d_aligned);
        e->d_aligned = nullptr;
        e->aligned_cap = 0;
        YTA_HIP(hipMalloc((void **)&e->d_aligned, (size_t)e->a.slot_px));
        e->aligned_cap = e->a.slot_px;
    }
    hipLaunchKernelGGL(k_ecc_align, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, e->stream, e->a,
                       stream, e->d_aligned);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpyAsync(out, e->d_aligned, (size_t)n, hipMemcpyDeviceToHost, e->stream));
    YTA_HIP(host_wait(e->stream));
    *h = st.h[slot];
    *w = st.w[slot];
    return YTA_OK;
}

#ifdef YTA_STAMPS
// diagnostic build only: block 0's phase ticks of the last k_ecc (setup, tables, pass A, the
// three block sums, pass B, the solves, pass C, iterations)
int yta_ecc_debug_stamps(yta_ecc *e, unsigned long long *out) {
    YTA_HIP(host_wait(e->stream));
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), 9 * sizeof(unsigned long long)));
    return YTA_OK;
}
#endif

int yta_ecc_hip_stream(yta_ecc *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

}  // extern "C"
