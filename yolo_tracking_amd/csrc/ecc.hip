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
//
// HBM layout per stream: two u8 slots (previous accepted frame / current frame) of
// round(max_h * scale) x round(max_w * scale) bytes, EccState, the 2x3 float32 warp.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <new>
#include <vector>

#include "cmc_small.hpp"
#include "common.hpp"

namespace yta {
namespace {
using namespace cmc;

constexpr int ECC_LDS = 144 * 1024;         // current frame bytes staged in LDS

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
__host__ __device__ constexpr int ecc_threads(int mode) { return mode == ECC_AFFINE ? 512 : 1024; }

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

// One template pixel (x, y) warped into the current frame `img` (hd x wd).  Every bilinear
// sample is exact in float32 (u8 or half-integer values times k / 1024 weights), the sum order
// is remapBilinear's ((v00 w0 + v01 w1) + v10 w2) + v11 w3.
template <bool GRAD, typename P>
__device__ __forceinline__ Warped warp_px(P img, int hd, int wd, const double (&M)[6], int x,
                                          int y) {
    const int xr = cv_round((M[1] * y + M[2]) * 1024.0), yr = cv_round((M[4] * y + M[5]) * 1024.0);
    const int ad = cv_round(M[0] * x * 1024.0), bd = cv_round(M[3] * x * 1024.0);
    const int X = (xr + 16 + ad) >> 5, Y = (yr + 16 + bd) >> 5;
    const int sx = sat16(X >> 5), sy = sat16(Y >> 5);
    const int nx = sat16((xr + 512 + ad) >> 10), ny = sat16((yr + 512 + bd) >> 10);
    const float tx = (float)(X & 31) * (1.f / 32), ty = (float)(Y & 31) * (1.f / 32);
    const float vx0 = 1.f - tx, vy0 = 1.f - ty;
    const float w[4] = {vy0 * vx0, vy0 * tx, ty * vx0, ty * tx};
    Warped o;
    o.iw = o.gx = o.gy = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {   // taps accumulated in remapBilinear's order
        const int u = sx + (k & 1), r = sy + (k >> 1);
        const bool in = (unsigned)u < (unsigned)wd && (unsigned)r < (unsigned)hd;
        float v = 0.f, gx = 0.f, gy = 0.f;
        if (in) {
            const int row = r * wd;
            v = (float)img[row + u];
            if (GRAD) {
                gx = 0.5f * ((float)img[row + refl(u + 1, wd)] - (float)img[row + refl(u - 1, wd)]);
                gy = 0.5f * ((float)img[refl(r + 1, hd) * wd + u] - (float)img[refl(r - 1, hd) * wd + u]);
            }
        }
        if (k == 0) {
            o.iw = v * w[0];
            o.gx = gx * w[0];
            o.gy = gy * w[0];
        } else {
            o.iw = o.iw + v * w[k];
            o.gx = o.gx + gx * w[k];
            o.gy = o.gy + gy * w[k];
        }
    }
    o.m = (unsigned)nx < (unsigned)wd && (unsigned)ny < (unsigned)hd;
    return o;
}

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

// Block sum of K float64 values over T threads, identical in every thread: halving tree over each
// wave's lanes, then thread k < K runs the halving tree over the waves of value k
// (oracle/cmc_ecc.py block_sum); red holds K x T/64 wave sums, tot the K totals.
template <int T, int K>
__device__ __forceinline__ void block_sum(double (&v)[K], double *red, double *tot) {
    constexpr int NW = T / WAVE;
    const int t = threadIdx.x, lane = t & (WAVE - 1), wave = t / WAVE;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int off = WAVE / 2; off >= 1; off >>= 1) v[k] = v[k] + __shfl_down(v[k], off, WAVE);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[k * NW + wave] = v[k];
    __syncthreads();
    if (t < K) {
        double w[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) w[i] = red[t * NW + i];
#pragma unroll
        for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int i = 0; i < h; ++i) w[i] = w[i] + w[i + h];
        tot[t] = w[0];
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
struct EccSolve {
    float H[6][6], Hi[6][6], A[6][6];
    float P[6], Q[6], iph[6], E[6], dp[6];
    float m[6];
    double lam, rho;
    int fail;
};

template <bool LDS, int MODE>
__global__ __launch_bounds__(ecc_threads(MODE)) void k_ecc(EccArgs a) {
    constexpr int T = ecc_threads(MODE);
    constexpr int N = ecc_nparams(MODE);
    constexpr int NB = N * (N + 1) / 2 + 2 * N + 1;   // pass B sums
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[NB * (T / WAVE)], tot[NB];
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
    const int hs = st0.h[st0.prev], ws = st0.w[st0.prev], hd = st0.h[cur], wd = st0.w[cur];
    const uint8_t *tmpl = a.img + ((long long)s * 2 + st0.prev) * a.slot_px;
    const uint8_t *gimg = a.img + ((long long)s * 2 + cur) * a.slot_px;
    const int npx = hs * ws, nd = hd * wd;
    if (LDS) {
        const uint4 *src = reinterpret_cast<const uint4 *>(gimg);
        uint4 *dst = reinterpret_cast<uint4 *>(smem);
        for (int k = t; k < (nd + 15) / 16; k += T) dst[k] = src[k];
    }
    if (t < 6) sv.m[t] = (t == 0 || t == 4) ? 1.f : 0.f;
    __syncthreads();
    const uint8_t *img = LDS ? (const uint8_t *)smem : gimg;
    float m[6] = {1.f, 0.f, 0.f, 0.f, 1.f, 0.f};
    double rho = -1.0, last_rho = -a.eps;
    int it = 0;
    bool fail = false;
    while (it < a.max_iter && fabs(rho - last_rho) >= a.eps) {
        ++it;
        const double M[6] = {uni((double)m[0]), uni((double)m[1]), uni((double)m[2]),
                             uni((double)m[3]), uni((double)m[4]), uni((double)m[5])};
        // pass A: meanStdDev of the warped image and of the template over the warped mask
        double va[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
        for (int p = t; p < npx; p += T) {
            const int y = p / ws, x = p - y * ws;
            const Warped q = warp_px<false>(img, hd, wd, M, x, y);
            if (q.m) {
                const double iw = q.iw, tv = (double)tmpl[p];
                va[0] = va[0] + iw;
                va[1] = va[1] + iw * iw;
                va[2] = va[2] + tv;
                va[3] = va[3] + tv * tv;
                va[4] = va[4] + 1.0;
            }
        }
        block_sum<T>(va, red, tot);
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
        for (int p = t; p < npx; p += T) {
            const int y = p / ws, x = p - y * ws;
            const Warped q = warp_px<true>(img, hd, wd, M, x, y);
            const float tv = (float)tmpl[p];
            const float iwz = q.m ? q.iw - img_mean_f : q.iw;
            const float tz = q.m ? tv - tmp_mean_f : 0.f;
            float J[N];
            jac<MODE>(q.gx, q.gy, (float)x, (float)y, c, sn, J);
            int k = 0;
#pragma unroll
            for (int i = 0; i < N; ++i)
#pragma unroll
                for (int j = i; j < N; ++j, ++k) vb[k] = vb[k] + (double)J[i] * (double)J[j];
#pragma unroll
            for (int i = 0; i < N; ++i) vb[k + i] = vb[k + i] + (double)J[i] * (double)iwz;
#pragma unroll
            for (int i = 0; i < N; ++i) vb[k + N + i] = vb[k + N + i] + (double)J[i] * (double)tz;
            vb[k + 2 * N] = vb[k + 2 * N] + (double)tz * (double)iwz;
        }
        block_sum<T>(vb, red, tot);
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
        for (int p = t; p < npx; p += T) {
            const int y = p / ws, x = p - y * ws;
            const Warped q = warp_px<true>(img, hd, wd, M, x, y);
            const float tv = (float)tmpl[p];
            const float iwz = q.m ? q.iw - img_mean_f : q.iw;
            const float tz = q.m ? tv - tmp_mean_f : 0.f;
            const float e = (float)(lam * (double)tz - (double)iwz);
            float J[N];
            jac<MODE>(q.gx, q.gy, (float)x, (float)y, c, sn, J);
#pragma unroll
            for (int i = 0; i < N; ++i) vc[i] = vc[i] + (double)J[i] * (double)e;
        }
        block_sum<T>(vc, red, tot);
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
#pragma unroll
        for (int k = 0; k < 6; ++k) m[k] = uni(sv.m[k]);
    }
    if (fail) {   // ecc.py:82-84: the identity, prev_img kept
        if (t < 6) W[t] = (t == 0 || t == 4) ? 1.f : 0.f;
        if (t == 0) {
            st.outcome = ECC_OUT_FAIL;
            st.iters = it;
            st.rho = rho;
        }
        return;
    }
    if (a.scale < 1.0) {   // ecc.py:87-89 (float32 division, NumPy's float32 scalar rules)
        m[2] = m[2] / (float)a.scale;
        m[5] = m[5] / (float)a.scale;
    }
    if (t < 6) W[t] = m[t];
    if (t == 0) {
        st.prev = cur;   // ecc.py:102
        st.outcome = ECC_OUT_EST;
        st.iters = it;
        st.rho = rho;
    }
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
};

namespace {

void ecc_free_slots(yta_ecc *e) {
    if (e->img) (void)hipFree(e->img);
    e->img = nullptr;
}

int ecc_slots(yta_ecc *e) {
    EccArgs &a = e->a;
    a.hmax = (int)std::rint(e->max_h * e->scale);
    a.wmax = (int)std::rint(e->max_w * e->scale);
    YTA_CHECK(a.hmax >= 1 && a.wmax >= 1, YTA_ERR_INVALID, "frames scale to an empty image");
    a.slot_px = ((long long)a.hmax * a.wmax + 15) & ~15LL;
    YTA_HIP(hipMalloc((void **)&e->img, (size_t)(2LL * e->S * a.slot_px)));
    a.img = e->img;
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
        YTA_HIP(hipFuncSetAttribute(ecc_kernel<true>(mode),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, ECC_LDS));
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
    const bool lds = a.slot_px <= ECC_LDS;
    void *args[] = {&a};
    YTA_HIP(hipLaunchKernel(lds ? ecc_kernel<true>(e->mode) : ecc_kernel<false>(e->mode),
                            dim3(a.S), dim3(ecc_threads(e->mode)), args, lds ? (size_t)a.slot_px : 0, e->stream));
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
    e->max_h = max_h;
    e->max_w = max_w;
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
    rc = ecc_slots(e);
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
                    (void *)e->d_frame_off, (void *)e->d_frame_hw})
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
        // grow the slots, keeping every stream's previous frame (packed from the slot start)
        YTA_HIP(host_wait(e->stream));
        uint8_t *old = e->img;
        const long long old_px = e->a.slot_px;
        e->img = nullptr;
        e->max_h = mh;
        e->max_w = mw;
        int rc = ecc_slots(e);
        if (!rc) {
            YTA_HIP(hipMemcpy2DAsync(e->img, e->a.slot_px, old, old_px, old_px, (size_t)S * 2,
                                     hipMemcpyDeviceToDevice, e->stream));
            rc = host_wait(e->stream) == hipSuccess ? YTA_OK : YTA_ERR_HIP;
        }
        (void)hipFree(old);
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

int yta_ecc_hip_stream(yta_ecc *e, void **stream) {
    YTA_CHECK(e && stream, YTA_ERR_INVALID, "null argument");
    *stream = (void *)e->stream;
    return YTA_OK;
}

}  // extern "C"
