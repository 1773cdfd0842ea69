// ReID crop preprocessing and feature normalisation on gfx950: the work
// boxmot/appearance/reid_multibackend.py does per crop on the CPU before and after the ReID
// forward pass.
//
//   k_reid_crops   [block = (box, band of ROWS output rows), 256 threads]
//                  preprocess (:189-224): crop rectangle with the reference's truncation / clamp /
//                  slice semantics, cv2.resize(INTER_LINEAR) in OpenCV's fixed-point form (or the
//                  INTER_AREA fast path when both scale factors are exactly 2), BGR -> RGB,
//                  (v / 255 - mean) / std through a compile-time table (IEEE float64), float32 or
//                  float16 stores into out[box][c][y][x] (NCHW), 4 consecutive x per thread;
//                  the horizontal pass runs once per source row of a band when the band's
//                  resized rows fit in LDS (int16 D >> 4), else per output row
//   k_feat_sumsq   [grid]  per-block float64 partial sums of squares of the (n, D) features
//   k_feat_scale   [grid]  every block folds the partials in the same order, norm -> float32,
//                  features / norm (get_features :310)
//
// Output stores are nontemporal (the 393 KB per crop stream past L2; measured 1.14 -> 0.90 ms per
// 8192-crop launch; -DYTA_REID_CACHED_STORES restores plain stores).
//
// Multi-image batches: box b reads image box_img[b] (HxWx3 uint8 BGR at imgs + img_off[i], dims
// img_hw[2i], img_hw[2i+1]).  The kernel is HBM-write bound: each 128 x 256 crop writes 393 KB of
// float32 and reads a few KB of source pixels (which stay in L2).
#include <hip/hip_fp16.h>

#include <vector>

#include "common.hpp"

namespace yta {
namespace {

constexpr int RP_T = 256;       // threads per block
constexpr int RP_ROWS = 32;     // output rows per block
constexpr int COEF = 2048;      // INTER_RESIZE_COEF_SCALE
constexpr int MAX_OUT_W = 1024;
constexpr int STAGE_BYTES = 24 * 1024;   // LDS for the block's source rows
constexpr int STAGE_ROWS = 96;

// (v / 255 - mean[c]) / std[c] rounded to float32, v = 0..255, c in RGB order
// (reid_multibackend.py:211-216: crop / 255, - mean, / std in float64, then .float()).  Evaluated
// by the compiler in IEEE double, so every entry equals NumPy's.
struct Lut {
    float v[3 * 256];
};
constexpr Lut make_lut() {
    Lut l{};
    constexpr double mean[3] = {0.485, 0.456, 0.406};   // :214
    constexpr double stdv[3] = {0.229, 0.224, 0.225};   // :215
    for (int c = 0; c < 3; ++c)
        for (int v = 0; v < 256; ++v)
            l.v[c * 256 + v] = (float)(((double)v / 255.0 - mean[c]) / stdv[c]);
    return l;
}
__constant__ Lut c_lut = make_lut();

struct Rect {
    int y0, y1, x0, x1;   // rows y0..y1-1, columns x0..x1-1; empty when y1 <= y0 or x1 <= x0
};

// Python slice stop: a negative stop counts from the end (clamped at 0); a stop past the end is
// the end.
__host__ __device__ inline int slice_stop(int stop, int n) {
    if (stop < 0) stop += n;
    if (stop < 0) stop = 0;
    return stop > n ? n : stop;
}
__host__ __device__ inline int slice_start(int start, int n) { return start > n ? n : start; }

// reid_multibackend.py:193-199: box.astype('int') (C truncation), max(0, x1), min(w - 1, x2),
// img[y1:y2, x1:x2]
__host__ __device__ inline Rect crop_rect(const double *box, int h, int w) {
    int x1 = (int)box[0], y1 = (int)box[1], x2 = (int)box[2], y2 = (int)box[3];
    x1 = x1 > 0 ? x1 : 0;
    y1 = y1 > 0 ? y1 : 0;
    x2 = x2 < w - 1 ? x2 : w - 1;
    y2 = y2 < h - 1 ? y2 : h - 1;
    Rect r;
    r.x0 = slice_start(x1, w);
    r.x1 = slice_stop(x2, w);
    r.y0 = slice_start(y1, h);
    r.y1 = slice_stop(y2, h);
    return r;
}

struct RpArgs {
    const uint8_t *imgs;
    const long long *img_off;
    const int *img_hw;
    const double *boxes;
    const int *box_img;   // nullable: every box reads image 0
    int n, out_h, out_w, half;
    void *out;
    int *n_empty;         // nullable: count of empty crops (their output is zero-filled)
};

__device__ __forceinline__ void store4(void *out, long long idx, float a, float b, float c, float d,
                                       int half) {
    if (half) {
        __half2 p0 = __halves2half2(__float2half_rn(a), __float2half_rn(b));
        __half2 p1 = __halves2half2(__float2half_rn(c), __float2half_rn(d));
        uint2 v;
        v.x = *reinterpret_cast<unsigned *>(&p0);
        v.y = *reinterpret_cast<unsigned *>(&p1);
#ifndef YTA_REID_CACHED_STORES
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(u2{v.x, v.y}, reinterpret_cast<u2 *>((__half *)out + idx));
#else
        *reinterpret_cast<uint2 *>((__half *)out + idx) = v;
#endif
    } else {
#ifndef YTA_REID_CACHED_STORES
        typedef float f4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(f4{a, b, c, d}, reinterpret_cast<f4 *>((float *)out + idx));
#else
        *reinterpret_cast<float4 *>((float *)out + idx) = make_float4(a, b, c, d);
#endif
    }
}

__device__ __forceinline__ void store1(void *out, long long idx, float a, int half) {
    if (half)
        ((__half *)out)[idx] = __float2half_rn(a);
    else
        ((float *)out)[idx] = a;
}

// cv2 INTER_LINEAR y sampling of output row dy (no border adjustment; rows clamped on use)
__device__ __forceinline__ void y_sample(int dy, double scale_y, int &sy, int &b0, int &b1) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    sy = (int)floorf(fy);
    fy -= (float)sy;
    b0 = (int)rintf((1.f - fy) * (float)COEF);
    b1 = (int)rintf(fy * (float)COEF);
}

// One output row group (V columns from dx0) of the bilinear path; q0 / q1 address the two source
// rows (global memory or the LDS copy), crop-relative columns.
template <int V, typename P>
__device__ __forceinline__ void bilinear_group(P q0, P q1, int dx0, int b0, int b1, int cw,
                                               const int *s_sx, const int *s_a, const float *lut,
                                               float (&res)[3][V]) {
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int dx = dx0 + k;
        const int sx = s_sx[dx], aa = s_a[dx];
        const int a0 = aa & 0xffff, a1 = aa >> 16;
        const int sx1 = min(sx + 1, cw - 1);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int sc = 2 - c;   // BGR -> RGB
            const int d0 = (int)q0[sx * 3 + sc] * a0 + (int)q0[sx1 * 3 + sc] * a1;
            const int d1 = (int)q1[sx * 3 + sc] * a0 + (int)q1[sx1 * 3 + sc] * a1;
            int v = ((((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16) + 2) >> 2;
            v = min(max(v, 0), 255);
            res[c][k] = lut[c * 256 + v];
        }
    }
}

template <int V>
__device__ __forceinline__ void store_group(void *out, long long obase, long long plane, int dy,
                                            int OW, int dx0, const float (&res)[3][V], int half) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const long long idx = obase + c * plane + (long long)dy * OW + dx0;
        if (V == 4)
            store4(out, idx, res[c][0], res[c][V > 1 ? 1 : 0], res[c][V > 2 ? 2 : 0],
                   res[c][V > 3 ? 3 : 0], half);
        else
            store1(out, idx, res[c][0], half);
    }
}

// V = consecutive output columns per thread (4 when out_w % 4 == 0, else 1)
template <int V>
__global__ __launch_bounds__(RP_T) void k_reid_crops(RpArgs a) {
    __shared__ float s_lut[3 * 256];
    __shared__ int s_sx[MAX_OUT_W];           // source column (crop-relative)
    __shared__ int s_a[MAX_OUT_W];            // a0 | a1 << 16
    __shared__ int s_lead[STAGE_ROWS];        // byte offset of each staged row in its dword run
    // either the band's raw source rows (dword runs) or its horizontally resized rows (int16)
    __shared__ __attribute__((aligned(16))) uint8_t s_rows[STAGE_BYTES];

    const int b = blockIdx.x;
    const int img = a.box_img ? a.box_img[b] : 0;
    const int h = a.img_hw[2 * img], w = a.img_hw[2 * img + 1];
    const uint8_t *base = a.imgs + a.img_off[img];
    const Rect r = crop_rect(a.boxes + 4 * (long long)b, h, w);
    const int ch = r.y1 - r.y0, cw = r.x1 - r.x0;
    const int OW = a.out_w, OH = a.out_h;
    const long long plane = (long long)OH * OW;
    const long long obase = (long long)b * 3 * plane;
    const int row0 = blockIdx.y * RP_ROWS;
    const int nrows = min(RP_ROWS, OH - row0);

    if (ch <= 0 || cw <= 0) {   // cv2.resize refuses an empty source: zero crop, count it
        for (int e = threadIdx.x; e < 3 * nrows * OW; e += RP_T) {
            const int c = e / (nrows * OW), rem = e - c * nrows * OW;
            store1(a.out, obase + c * plane + (long long)row0 * OW + rem, 0.f, a.half);
        }
        if (a.n_empty && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(a.n_empty, 1);
        return;
    }

    for (int e = threadIdx.x; e < 3 * 256; e += RP_T) s_lut[e] = c_lut.v[e];
    // resize.cpp resizeGeneric_ setup (INTER_LINEAR); both factors exactly 2 -> INTER_AREA
    const double scale_x = 1.0 / ((double)OW / (double)cw);
    const double scale_y = 1.0 / ((double)OH / (double)ch);
    const bool area2 = fabs(scale_x - 2.0) < 2.220446049250313e-16 &&
                       fabs(scale_y - 2.0) < 2.220446049250313e-16;
    const int groups = OW / V;                 // column groups per row

    if (area2) {
        __syncthreads();
        for (int e = threadIdx.x; e < nrows * groups; e += RP_T) {
            const int ry = e / groups, dy = row0 + ry, dx0 = (e - ry * groups) * V;
            float res[3][V];
            const uint8_t *p0 = base + ((long long)(r.y0 + 2 * dy) * w + r.x0) * 3;
            const uint8_t *p1 = p0 + (long long)w * 3;
#pragma unroll
            for (int k = 0; k < V; ++k) {
                const int sx = 2 * (dx0 + k);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const int sc = 2 - c;
                    const int sm = p0[sx * 3 + sc] + p0[sx * 3 + 3 + sc] + p1[sx * 3 + sc] +
                                   p1[sx * 3 + 3 + sc];
                    res[c][k] = s_lut[c * 256 + ((sm + 2) >> 2)];
                }
            }
            store_group<V>(a.out, obase, plane, dy, OW, dx0, res, a.half);
        }
        return;
    }

    for (int dx = threadIdx.x; dx < OW; dx += RP_T) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= (float)sx;
        int a0, a1;
        if (sx >= cw - 1) {          // right border: D = S[W-1] * ONE
            sx = cw - 1;
            a0 = COEF;
            a1 = 0;
        } else {
            if (sx < 0) {
                sx = 0;
                fx = 0.f;
            }
            a0 = (int)rintf((1.f - fx) * (float)COEF);
            a1 = (int)rintf(fx * (float)COEF);
        }
        s_sx[dx] = sx;
        s_a[dx] = a0 | (a1 << 16);
    }

    // source rows this block reads: clamp(sy(row0)) .. clamp(sy(last) + 1)
    int sy_a, sy_b, t0, t1;
    y_sample(row0, scale_y, sy_a, t0, t1);
    y_sample(row0 + nrows - 1, scale_y, sy_b, t0, t1);
    const int lo = min(max(sy_a, 0), ch - 1), hi = min(max(sy_b + 1, 0), ch - 1);
    const int R = hi - lo + 1;
    if (V == 4 && R <= STAGE_BYTES / (6 * OW)) {
        // Horizontal pass once per source row of the band (HResizeLinear), kept as D >> 4 in
        // int16 (the SIMD row kernel's v_pack input; <= 255 * 2048 >> 4 fits), then the vertical
        // pass per output row reads two 8-byte runs per channel.
        short *hb = reinterpret_cast<short *>(s_rows);   // [R][3][OW]
        __syncthreads();                                  // x tables
        for (int e = threadIdx.x; e < R * groups; e += RP_T) {
            const int rr = e / groups, dx0 = (e - rr * groups) * V;
            const uint8_t *q = base + ((long long)(r.y0 + lo + rr) * w + r.x0) * 3;
            short o[3][4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int dx = dx0 + k;
                const int sx = s_sx[dx], aa = s_a[dx];
                const int a0 = aa & 0xffff, a1 = aa >> 16;
                const int sx1 = min(sx + 1, cw - 1);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const int sc = 2 - c;   // BGR -> RGB
                    o[c][k] = (short)(((int)q[sx * 3 + sc] * a0 + (int)q[sx1 * 3 + sc] * a1) >> 4);
                }
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                uint2 v;
                v.x = (unsigned)(unsigned short)o[c][0] | ((unsigned)(unsigned short)o[c][1] << 16);
                v.y = (unsigned)(unsigned short)o[c][2] | ((unsigned)(unsigned short)o[c][3] << 16);
                *reinterpret_cast<uint2 *>(hb + ((long long)rr * 3 + c) * OW + dx0) = v;
            }
        }
        __syncthreads();
        for (int e = threadIdx.x; e < nrows * groups; e += RP_T) {
            const int ry = e / groups, dy = row0 + ry, dx0 = (e - ry * groups) * V;
            int sy, b0, b1;
            y_sample(dy, scale_y, sy, b0, b1);
            const int y0 = min(max(sy, 0), ch - 1) - lo, y1 = min(max(sy + 1, 0), ch - 1) - lo;
            float res[3][V];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const uint2 u0 = *reinterpret_cast<const uint2 *>(hb + (y0 * 3 + c) * OW + dx0);
                const uint2 u1 = *reinterpret_cast<const uint2 *>(hb + (y1 * 3 + c) * OW + dx0);
                const int h0[4] = {(int)(short)(u0.x & 0xffff), (int)(short)(u0.x >> 16),
                                   (int)(short)(u0.y & 0xffff), (int)(short)(u0.y >> 16)};
                const int h1[4] = {(int)(short)(u1.x & 0xffff), (int)(short)(u1.x >> 16),
                                   (int)(short)(u1.y & 0xffff), (int)(short)(u1.y >> 16)};
#pragma unroll
                for (int k = 0; k < V; ++k) {
                    int v = (((h0[k] * b0) >> 16) + ((h1[k] * b1) >> 16) + 2) >> 2;
                    v = min(max(v, 0), 255);
                    res[c][k] = s_lut[c * 256 + v];
                }
            }
            store_group<V>(a.out, obase, plane, dy, OW, dx0, res, a.half);
        }
        return;
    }
    const int rs = ((cw * 3 + 3 + 3) / 4) * 4;   // LDS stride: the row's dword run
    const bool staged = R <= STAGE_ROWS && (long long)R * rs <= STAGE_BYTES;
    if (staged) {   // dword-aligned runs covering each row's cw * 3 bytes, coalesced
        const int ndw = rs / 4;
        for (int e = threadIdx.x; e < R * ndw; e += RP_T) {
            const int rr = e / ndw, k = e - rr * ndw;
            const uint8_t *rp = base + ((long long)(r.y0 + lo + rr) * w + r.x0) * 3;
            const uintptr_t al = (uintptr_t)rp & ~(uintptr_t)3;
            if (k == 0) s_lead[rr] = (int)((uintptr_t)rp - al);
            reinterpret_cast<unsigned *>(s_rows + rr * rs)[k] = ((const unsigned *)al)[k];
        }
    }
    __syncthreads();

    for (int e = threadIdx.x; e < nrows * groups; e += RP_T) {
        const int ry = e / groups, dy = row0 + ry, dx0 = (e - ry * groups) * V;
        int sy, b0, b1;
        y_sample(dy, scale_y, sy, b0, b1);
        const int y0 = min(max(sy, 0), ch - 1), y1 = min(max(sy + 1, 0), ch - 1);
        float res[3][V];
        if (staged) {
            const uint8_t *q0 = s_rows + (y0 - lo) * rs + s_lead[y0 - lo];
            const uint8_t *q1 = s_rows + (y1 - lo) * rs + s_lead[y1 - lo];
            bilinear_group<V>(q0, q1, dx0, b0, b1, cw, s_sx, s_a, s_lut, res);
        } else {
            const uint8_t *q0 = base + ((long long)(r.y0 + y0) * w + r.x0) * 3;
            const uint8_t *q1 = base + ((long long)(r.y0 + y1) * w + r.x0) * 3;
            bilinear_group<V>(q0, q1, dx0, b0, b1, cw, s_sx, s_a, s_lut, res);
        }
        store_group<V>(a.out, obase, plane, dy, OW, dx0, res, a.half);
    }
}

constexpr int FN_T = 256, FN_G = 256;

__device__ __forceinline__ double block_sum(double v, double *sh) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (ln == 0) sh[wv] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0)
        for (int i = 0; i < FN_T / 64; ++i) t += sh[i];
    __syncthreads();
    return t;   // valid in thread 0
}

__global__ __launch_bounds__(FN_T) void k_feat_sumsq(const float *f, long long n, double *part) {
    __shared__ double sh[FN_T / 64];
    double s = 0.0;
    for (long long i = blockIdx.x * (long long)FN_T + threadIdx.x; i < n;
         i += (long long)gridDim.x * FN_T) {
        const double v = f[i];
        s += v * v;
    }
    s = block_sum(s, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(FN_T) void k_feat_scale(float *f, long long n, const double *part,
                                                     int nparts) {
    __shared__ double sh[FN_T / 64];
    __shared__ float s_norm;
    double s = threadIdx.x < nparts ? part[threadIdx.x] : 0.0;
    s = block_sum(s, sh);
    if (threadIdx.x == 0) s_norm = (float)sqrt(s);
    __syncthreads();
    const float nrm = s_norm;
    for (long long i = blockIdx.x * (long long)FN_T + threadIdx.x; i < n;
         i += (long long)gridDim.x * FN_T)
        f[i] = f[i] / nrm;
}

int launch_crops(const RpArgs &a, hipStream_t st) {
    YTA_CHECK(a.out_w > 0 && a.out_w <= MAX_OUT_W && a.out_h > 0, YTA_ERR_INVALID,
              "output size %d x %d (width 1..%d)", a.out_w, a.out_h, MAX_OUT_W);
    if (a.n == 0) return YTA_OK;
    dim3 grid(a.n, (a.out_h + RP_ROWS - 1) / RP_ROWS);
    if (a.out_w % 4 == 0)
        hipLaunchKernelGGL(k_reid_crops<4>, grid, dim3(RP_T), 0, st, a);
    else
        hipLaunchKernelGGL(k_reid_crops<1>, grid, dim3(RP_T), 0, st, a);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int launch_normalize(float *d_f, long long n, double *d_part, hipStream_t st) {
    if (n == 0) return YTA_OK;
    hipLaunchKernelGGL(k_feat_sumsq, dim3(FN_G), dim3(FN_T), 0, st, d_f, n, d_part);
    YTA_HIP(hipGetLastError());
    const int g = (int)((n + FN_T * 4 - 1) / (FN_T * 4));
    hipLaunchKernelGGL(k_feat_scale, dim3(g < 1024 ? g : 1024), dim3(FN_T), 0, st, d_f, n,
                       d_part, FN_G);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

struct DevBuf {
    std::vector<void *> ptrs;
    ~DevBuf() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    hipError_t get(void **p, size_t bytes) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, bytes ? bytes : 1);
        if (e == hipSuccess) ptrs.push_back(q);
        *p = q;
        return e;
    }
};

}  // namespace
}  // namespace yta

using namespace yta;

extern "C" {

int yta_reid_preprocess(int device, const uint8_t *img, int h, int w, const double *xyxys, int n,
                        int out_h, int out_w, int half, void *out) {
    YTA_CHECK(n >= 0 && h > 0 && w > 0 && (half == 0 || half == 1), YTA_ERR_INVALID,
              "bad arguments (n %d, image %d x %d, half %d)", n, h, w, half);
    YTA_CHECK(out_w > 0 && out_w <= MAX_OUT_W && out_h > 0, YTA_ERR_INVALID,
              "output size %d x %d (width 1..%d)", out_w, out_h, MAX_OUT_W);
    if (n == 0) return YTA_OK;
    YTA_CHECK(img && xyxys && out, YTA_ERR_INVALID, "null buffer");
    for (int i = 0; i < n; ++i) {   // cv2.resize asserts !ssize.empty()
        const Rect r = crop_rect(xyxys + 4 * i, h, w);
        YTA_CHECK(r.y1 > r.y0 && r.x1 > r.x0, YTA_ERR_INVALID,
                  "box %d (%g, %g, %g, %g): empty crop in a %d x %d image", i, xyxys[4 * i],
                  xyxys[4 * i + 1], xyxys[4 * i + 2], xyxys[4 * i + 3], h, w);
    }
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    void *d_img, *d_boxes, *d_out, *d_meta;
    const size_t img_bytes = (size_t)h * w * 3;
    const size_t out_bytes = (size_t)n * 3 * out_h * out_w * (half ? 2 : 4);
    YTA_HIP(m.get(&d_img, img_bytes));
    YTA_HIP(m.get(&d_boxes, sizeof(double) * 4 * n));
    YTA_HIP(m.get(&d_out, out_bytes));
    YTA_HIP(m.get(&d_meta, 16));
    const long long off0 = 0;
    const int hw[2] = {h, w};
    YTA_HIP(hipMemcpy(d_img, img, img_bytes, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_boxes, xyxys, sizeof(double) * 4 * n, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(d_meta, &off0, 8, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy((char *)d_meta + 8, hw, 8, hipMemcpyHostToDevice));
    RpArgs a{(const uint8_t *)d_img, (const long long *)d_meta, (const int *)((char *)d_meta + 8),
             (const double *)d_boxes, nullptr, n, out_h, out_w, half, d_out, nullptr};
    rc = launch_crops(a, 0);
    if (rc) return rc;
    YTA_HIP(hipMemcpy(out, d_out, out_bytes, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_reid_preprocess_device(const uint8_t *d_imgs, const long long *d_img_off,
                               const int *d_img_hw, const double *d_xyxys, const int *d_box_img,
                               int n, int out_h, int out_w, int half, void *d_out, int *d_n_empty,
                               void *stream) {
    YTA_CHECK(n >= 0 && (half == 0 || half == 1), YTA_ERR_INVALID, "bad arguments (n %d, half %d)",
              n, half);
    if (n == 0) return YTA_OK;
    YTA_CHECK(d_imgs && d_img_off && d_img_hw && d_xyxys && d_out, YTA_ERR_INVALID,
              "null buffer");
    RpArgs a{d_imgs, d_img_off, d_img_hw, d_xyxys, d_box_img, n, out_h, out_w, half, d_out,
             d_n_empty};
    return launch_crops(a, (hipStream_t)stream);
}

int yta_reid_normalize(int device, float *feats, long long count) {
    YTA_CHECK(count >= 0, YTA_ERR_INVALID, "bad count %lld", count);
    if (count == 0) return YTA_OK;
    YTA_CHECK(feats, YTA_ERR_INVALID, "null features");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    void *d_f, *d_part;
    YTA_HIP(m.get(&d_f, sizeof(float) * count));
    YTA_HIP(m.get(&d_part, sizeof(double) * FN_G));
    YTA_HIP(hipMemcpy(d_f, feats, sizeof(float) * count, hipMemcpyHostToDevice));
    rc = launch_normalize((float *)d_f, count, (double *)d_part, 0);
    if (rc) return rc;
    YTA_HIP(hipMemcpy(feats, d_f, sizeof(float) * count, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_reid_normalize_device(float *d_feats, long long count, double *d_work, void *stream) {
    YTA_CHECK(count >= 0, YTA_ERR_INVALID, "bad count %lld", count);
    if (count == 0) return YTA_OK;
    YTA_CHECK(d_feats && d_work, YTA_ERR_INVALID, "null buffer");
    return launch_normalize(d_feats, count, d_work, (hipStream_t)stream);
}

}  // extern "C"
