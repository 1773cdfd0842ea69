// OSNet omni-scale block kernels on gfx950 (the ReID network's forward).
//
// Reference: boxmot/appearance/backbones/osnet.py LightConv3x3 (depthwise 3x3 + BatchNorm + ReLU
// after the 1x1) and OSBlock.forward (x2 = gate(x2a) + gate(x2b) + gate(x2c) + gate(x2d), the
// ChannelGate's global average pool).  appearance/osnet.py runs the four branches batched and
// folds every BatchNorm; MIOpen has no fast depthwise path for these shapes (its naive kernel
// took 37 % of the forward), so the two bandwidth-bound steps are written here:
//   k_dw3x3    one (sample, channel) plane per block: depthwise 3x3 (zero padding 1) + bias +
//              ReLU, the output plane routed to one of two tensors (the branch that ends at this
//              depth goes into the block's branch stack, the rest feeds the next depth), and the
//              plane's sum for the channel gate's average pool (float32, block reduction);
//   k_gate_sum x2[n, c] = sum_b stack[n, b, c] * gate[n, b, c] over the four branches.
//   k_pw       every 1x1 convolution (conv1, the branches' pointwise layers, conv3 + downsample
//              + residual, the transition convs, conv5, the fc) as a GEMM on v_mfma_f32_32x32x2_f32:
//              one wave per 32 (output channels) x 32 (pixels) tile, operands straight from
//              global memory (the pixel axis is contiguous: B fragments are coalesced rows), groups,
//              a second input segment (the downsample branch joins conv3's sum), bias, identity
//              residual and ReLU fused in the epilogue;
//   k_stem     conv 7x7 stride 2 pad 3 (3 -> C0) + bias + ReLU, input tile + halo in LDS,
//              16 output channels per pass in registers, weights broadcast from LDS;
//   k_pool     max 3x3 stride 2 pad 1 / average 2x2 stride 2 / global mean (OSNet's pools);
//   k_gate     ChannelGate's two 1x1 layers on the pooled branch planes (fc1 + ReLU, fc2 +
//              sigmoid), one block per sample.
// NCHW planes, float32 or float16 storage, float32 arithmetic.
#include <algorithm>

#include "common.hpp"
#include "../../include/yolo_tracking_amd.h"

namespace yta {
namespace {

constexpr int DW_T = 256;

template <typename T>
__device__ __forceinline__ float ld(const T *p) { return (float)*p; }

template <typename T>
__global__ __launch_bounds__(DW_T) void k_dw3x3(const T *x, long long xn, long long xc,
                                                 const float *w, const float *b, int C, int H,
                                                 int W, T *yf, long long yfn, int n_first, T *yr,
                                                 long long yrn, float *psum, long long psn) {
    __shared__ float red[DW_T / WAVE];
    const int c = blockIdx.x, n = blockIdx.y;
    const T *src = x + n * xn + c * xc;
    const bool first = c < n_first;
    T *dst = first ? yf + n * yfn + (long long)c * H * W
                   : yr + n * yrn + (long long)(c - n_first) * H * W;
    float k[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) k[q] = w[c * 9 + q];
    const float bias = b[c];
    float acc = 0.f;
    for (int i = threadIdx.x; i < H * W; i += DW_T) {
        const int y = i / W, xx = i - y * W;
        float s = 0.f;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy) {
            const int yy = y + dy;
            if (yy < 0 || yy >= H) continue;
            const T *row = src + (long long)yy * W;
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const int xq = xx + dx;
                if (xq < 0 || xq >= W) continue;
                s += k[(dy + 1) * 3 + (dx + 1)] * ld(row + xq);
            }
        }
        const float v = fmaxf(s + bias, 0.f);
        const T o = (T)v;
        dst[i] = o;
        acc += (float)o;
    }
    if (first && psum) {   // the channel gate's average pool reads the stored values
        acc = (float)wave_reduce(RED_SUM, (double)acc);
        if (lane_id() == 0) red[threadIdx.x / WAVE] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            float s = 0.f;
            for (int k2 = 0; k2 < DW_T / WAVE; ++k2) s += red[k2];
            psum[n * psn + c] = s;
        }
    }
}

// The same for planes that fit LDS: a block takes ppb consecutive planes of a sample (about 4096
// pixels together, so small late-stage planes do not leave most of a block idle), stages them in
// LDS with coalesced loads and computes every output from LDS; a first-branch plane's sum of its
// stored outputs is reduced in a fixed order (thread partials, waves, then wave 0: deterministic
// gate inputs).
constexpr int DW_LDS_PX = 4096;
template <typename T>
__global__ __launch_bounds__(DW_T) void k_dw3x3_lds(const T *x, long long xn, long long xc,
                                                     const float *w, const float *b, int C, int H,
                                                     int W, int ppb, T *yf, long long yfn,
                                                     int n_first, T *yr, long long yrn,
                                                     float *psum, long long psn) {
    __shared__ float in[DW_LDS_PX];
    __shared__ float red[DW_T / WAVE];
    const int n = blockIdx.y, c0 = blockIdx.x * ppb;
    const int np = C - c0 < ppb ? C - c0 : ppb;
    const int HW = H * W;
    const float invW = 1.0f / (float)W;   // q / W for q < 2^22: (q + 0.5) / W rounds to the quotient
    for (int j = 0; j < np; ++j) {
        const T *src = x + n * xn + (long long)(c0 + j) * xc;
        for (int q = threadIdx.x; q < HW; q += DW_T) in[j * HW + q] = (float)src[q];
    }
    __syncthreads();
    for (int j = 0; j < np; ++j) {
        const int c = c0 + j;
        const float *pl = in + j * HW;
        float k[9];
#pragma unroll
        for (int u = 0; u < 9; ++u) k[u] = w[c * 9 + u];
        const float bias = b[c];
        const bool first = c < n_first;
        T *dst = first ? yf + n * yfn + (long long)c * HW : yr + n * yrn + (long long)(c - n_first) * HW;
        float acc = 0.f;
        for (int q = threadIdx.x; q < HW; q += DW_T) {
            const int y = (int)(((float)q + 0.5f) * invW), xx = q - y * W;
            float s = 0.f;
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy) {
                const int yy = y + dy;
                if (yy < 0 || yy >= H) continue;
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx) {
                    const int xq = xx + dx;
                    if (xq < 0 || xq >= W) continue;
                    s += k[(dy + 1) * 3 + (dx + 1)] * pl[yy * W + xq];
                }
            }
            const T o = (T)fmaxf(s + bias, 0.f);
            dst[q] = o;
            acc += (float)o;
        }
        if (first && psum) {   // block-uniform
            acc = (float)wave_reduce(RED_SUM, (double)acc);
            if (lane_id() == 0) red[threadIdx.x / WAVE] = acc;
            __syncthreads();
            if (threadIdx.x == 0) {
                float t = 0.f;
                for (int u = 0; u < DW_T / WAVE; ++u) t += red[u];
                psum[n * psn + c] = t;
            }
            __syncthreads();
        }
    }
}

// x2[n][c][p] = sum_b stack[n][b][c][p] * gate[n][b][c]   (stack: N x 4 x C x P contiguous)
template <typename T>
__global__ __launch_bounds__(256) void k_gate_sum(const T *stack, const T *gate, int C, int P,
                                                  T *out) {
    const int c = blockIdx.x, n = blockIdx.y;
    const long long base = (long long)n * 4 * C;
    float g[4];
#pragma unroll
    for (int br = 0; br < 4; ++br) g[br] = (float)gate[base + br * C + c];
    const T *s0 = stack + (base + c) * P;
    const long long bs = (long long)C * P;
    T *o = out + ((long long)n * C + c) * P;
    for (int p = threadIdx.x; p < P; p += 256) {
        float v = 0.f;
#pragma unroll
        for (int br = 0; br < 4; ++br) v += (float)s0[br * bs + p] * g[br];
        o[p] = (T)v;
    }
}


// ---------------------------------------------------------------------------------------- k_pw
// D[co][p] = sum_k W[co][k] X[k][p] per (sample, group): A = W (f32, row-major [cout_g][K]),
// B = X.  v_mfma_f32_32x32x2_f32: lane l holds A[l & 31][k = l >> 5] and B[k = l >> 5][l & 31];
// D register r of lane l is row (r & 3) + 8 (r >> 2) + 4 (l >> 5), column l & 31.
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int PW_T = 256;           // 4 waves: 32 channels x 128 pixels per block
constexpr int PW_KU = 8;            // k-steps (of 2) whose loads are issued together

// A wave computes MB 32 x 32 tiles (up to 128 output channels) for its 32 pixels, so each
// X element is read once per 128 output channels.
template <typename T, int MB>
__global__ __launch_bounds__(PW_T) void k_pw(yta_pw_args a) {
    const int lane = lane_id(), wv = threadIdx.x / WAVE;
    const int mt = (a.cout_g + 31) / 32, mg = (mt + MB - 1) / MB;
    const int g = blockIdx.y / mg, co0 = (blockIdx.y - g * mg) * MB * 32;
    const long long n = blockIdx.z;
    const int p0 = (blockIdx.x * (PW_T / WAVE) + wv) * 32;
    if (p0 >= a.P) return;                                   // wave-uniform
    const int K = a.k1 + a.k2;
    const int r = lane & 31, h = lane >> 5;
    const int p = p0 + r;
    const bool p_ok = p < a.P;
    const float *wg = a.w + (long long)g * K * a.cout_g;   // [K][cout_g]: lanes read along co
    bool co_ok[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) co_ok[m] = co0 + 32 * m + r < a.cout_g;
    const T *x1 = (const T *)a.x1 + n * a.x1n + (long long)g * a.k1 * a.x1c + (long long)(p_ok ? p : 0) * a.x1p;
    const T *x2 = a.x2 ? (const T *)a.x2 + n * a.x2n + (long long)(p_ok ? p : 0) * a.x2p : nullptr;
    f32x16 acc[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[m][q] = 0.f;
    for (int k0 = 0; k0 < K; k0 += 2 * PW_KU) {
        float av[MB][PW_KU], bv[PW_KU];
#pragma unroll
        for (int u = 0; u < PW_KU; ++u) {
            const int k = k0 + 2 * u + h;
#pragma unroll
            for (int m = 0; m < MB; ++m)
                av[m][u] = co_ok[m] && k < K ? wg[(long long)k * a.cout_g + co0 + 32 * m + r] : 0.f;
            float b = 0.f;
            if (p_ok && k < a.k1) b = (float)x1[(long long)k * a.x1c];
            else if (p_ok && k < K) b = (float)x2[(long long)(k - a.k1) * a.x2c];
            bv[u] = b;
        }
#pragma unroll
        for (int u = 0; u < PW_KU; ++u)
#pragma unroll
            for (int m = 0; m < MB; ++m)
                acc[m] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m][u], bv[u], acc[m], 0, 0, 0);
    }
    T *y = (T *)a.y + n * a.yn;
    const T *res = a.res ? (const T *)a.res + n * a.rn : nullptr;
    if (!p_ok) return;   // this lane's D column is pixel p
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = co0 + 32 * m + (q & 3) + 8 * (q >> 2) + 4 * h;
            if (c >= a.cout_g) continue;
            const long long ch = (long long)g * a.cout_g + c;
            float v = acc[m][q];
            if (a.bias) v += a.bias[ch];
            if (res) v += (float)res[ch * a.rc + (long long)p * a.rp];
            if (a.relu) v = fmaxf(v, 0.f);
            y[ch * a.yc + (long long)p * a.yp] = (T)v;
        }
}

// --------------------------------------------------------------------------------------- k_stem
// conv1 (osnet.py ConvLayer(3, C0, 7, stride=2, padding=3) + folded BatchNorm + ReLU): a block
// computes a 16 x 16 tile of output pixels; the input tile (3 x 37 x 37 with the halo) sits in
// LDS, each thread keeps the C0 (a multiple of 16, <= 64 per pass) accumulators of its pixel in
// registers and reads every input value once per pass, the weights being uniform across the block
// (scalar loads).
constexpr int ST_TILE = 16, ST_IN = 2 * ST_TILE + 5;   // 37 input rows / columns per tile
template <typename T, int CB>
__global__ __launch_bounds__(256) void k_stem(const T *x, int H, int W, const float *w,
                                              const float *b, int C0, T *y, int Ho, int Wo) {
    __shared__ float tile[3][ST_IN][ST_IN + 1];
    extern __shared__ __attribute__((aligned(16))) float swt[];   // [147][C0]
    const int n = blockIdx.z, t = threadIdx.x;
    const int oy0 = blockIdx.y * ST_TILE, ox0 = blockIdx.x * ST_TILE;
    const int iy0 = 2 * oy0 - 3, ix0 = 2 * ox0 - 3;
    for (int i = t; i < 147 * C0; i += 256) {
        const int k = i / C0, co = i - k * C0;
        swt[i] = w[co * 147 + k];
    }
    for (int i = t; i < 3 * ST_IN * ST_IN; i += 256) {
        const int c = i / (ST_IN * ST_IN), rem = i - c * ST_IN * ST_IN;
        const int yy = rem / ST_IN, xx = rem - yy * ST_IN;
        const int gy = iy0 + yy, gx = ix0 + xx;
        tile[c][yy][xx] = gy >= 0 && gy < H && gx >= 0 && gx < W
                              ? (float)x[((long long)n * 3 + c) * H * W + (long long)gy * W + gx]
                              : 0.f;
    }
    __syncthreads();
    const int ty = t / ST_TILE, tx = t - ty * ST_TILE;
    const int oy = oy0 + ty, ox = ox0 + tx;
    const bool on = oy < Ho && ox < Wo;
    for (int cb = 0; cb < C0; cb += CB) {   // block-uniform
        float acc[CB];
#pragma unroll
        for (int q = 0; q < CB; ++q) acc[q] = b[cb + q];
#pragma unroll 1
        for (int c = 0; c < 3; ++c)
#pragma unroll 1
            for (int ky = 0; ky < 7; ++ky)
#pragma unroll
                for (int kx = 0; kx < 7; ++kx) {
                    const float v = tile[c][2 * ty + ky][2 * tx + kx];
                    const float4 *wk = reinterpret_cast<const float4 *>(
                        swt + (c * 49 + ky * 7 + kx) * C0 + cb);
#pragma unroll
                    for (int q = 0; q < CB / 4; ++q) {
                        const float4 w4 = wk[q];
                        acc[4 * q] += w4.x * v;
                        acc[4 * q + 1] += w4.y * v;
                        acc[4 * q + 2] += w4.z * v;
                        acc[4 * q + 3] += w4.w * v;
                    }
                }
        if (on)
#pragma unroll
            for (int q = 0; q < CB; ++q)
                y[(((long long)n * C0 + cb + q) * Ho + oy) * Wo + ox] = (T)fmaxf(acc[q], 0.f);
    }
}

// --------------------------------------------------------------------------------------- k_pool
// kind 0: max 3x3 stride 2 pad 1 (F.max_pool2d(x, 3, 2, 1)); 1: average 2x2 stride 2
// (F.avg_pool2d(x, 2, 2)); 2: mean over the plane -> y[n][c] (the global average pool, summed in
// float32).  One block per (sample, channel) plane.
template <typename T>
__global__ __launch_bounds__(256) void k_pool(const T *x, int C, int H, int W, int kind, T *y,
                                              int Ho, int Wo) {
    __shared__ float red[256 / WAVE];
    const int c = blockIdx.x, n = blockIdx.y;
    const T *src = x + ((long long)n * C + c) * H * W;
    if (kind == 2) {
        float s = 0.f;
        for (int i = threadIdx.x; i < H * W; i += 256) s += (float)src[i];
        s = (float)wave_reduce(RED_SUM, (double)s);
        if (lane_id() == 0) red[threadIdx.x / WAVE] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            float tot = 0.f;
            for (int k = 0; k < 256 / WAVE; ++k) tot += red[k];
            y[(long long)n * C + c] = (T)(tot / (float)(H * W));
        }
        return;
    }
    T *dst = y + ((long long)n * C + c) * Ho * Wo;
    for (int i = threadIdx.x; i < Ho * Wo; i += 256) {
        const int oy = i / Wo, ox = i - oy * Wo;
        float v;
        if (kind == 0) {
            v = -INFINITY;
            for (int dy = -1; dy <= 1; ++dy) {
                const int yy = 2 * oy + dy;
                if (yy < 0 || yy >= H) continue;
                for (int dx = -1; dx <= 1; ++dx) {
                    const int xx = 2 * ox + dx;
                    if (xx < 0 || xx >= W) continue;
                    v = fmaxf(v, (float)src[yy * W + xx]);
                }
            }
        } else {
            const T *q = src + 2 * oy * W + 2 * ox;
            v = (((float)q[0] + (float)q[1]) + ((float)q[W] + (float)q[W + 1])) * 0.25f;
        }
        dst[i] = (T)v;
    }
}

// --------------------------------------------------------------------------------------- k_gate
// ChannelGate (osnet.py): pooled = plane sums / P (rounded to T, as the graph's .to(dtype)),
// hidden = relu(W1 pooled + b1), gate = sigmoid(W2 hidden + b2), for the four branches of a
// sample.  Block per sample; mid <= 512, hid <= 64.
template <typename T>
__global__ __launch_bounds__(256) void k_gate(const float *psum, float inv_p, const T *w1,
                                              const T *b1, const T *w2, const T *b2, int mid,
                                              int hid, T *gate) {
    __shared__ float pooled[4 * 512];
    __shared__ float hidden[4 * 64];
    const int n = blockIdx.x;
    for (int i = threadIdx.x; i < 4 * mid; i += 256)
        pooled[i] = (float)(T)(psum[(long long)n * 4 * mid + i] * inv_p);
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * hid; i += 256) {
        const int br = i / hid, j = i - br * hid;
        float s = (float)b1[j];
        for (int k = 0; k < mid; ++k) s += (float)w1[j * mid + k] * pooled[br * mid + k];
        hidden[i] = (float)(T)fmaxf((float)(T)s, 0.f);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 4 * mid; i += 256) {
        const int br = i / mid, c = i - br * mid;
        float s = (float)b2[c];
        for (int j = 0; j < hid; ++j) s += (float)w2[c * hid + j] * hidden[br * hid + j];
        s = (float)(T)s;
        gate[(long long)n * 4 * mid + i] = (T)(1.f / (1.f + expf(-s)));
    }
}
}  // namespace
}  // namespace yta

using namespace yta;

extern "C" {

int yta_osnet_dw3x3(const void *x, long long x_n_stride, long long x_c_stride, const float *w,
                    const float *b, int N, int C, int H, int W, int half, void *y_first,
                    long long yf_n_stride, int n_first, void *y_rest, long long yr_n_stride,
                    float *plane_sum, long long ps_n_stride, void *stream) {
    YTA_CHECK(x && w && b && N > 0 && C > 0 && H > 0 && W > 0 && n_first >= 0 && n_first <= C,
              YTA_ERR_INVALID, "bad argument");
    YTA_CHECK((n_first == 0 || y_first) && (n_first == C || y_rest), YTA_ERR_INVALID,
              "null output");
    if (H * W <= DW_LDS_PX) {
        const int ppb = std::max(1, std::min(C, DW_LDS_PX / (H * W)));
        const dim3 gl((C + ppb - 1) / ppb, N);
        if (half)
            hipLaunchKernelGGL(k_dw3x3_lds<_Float16>, gl, dim3(DW_T), 0, (hipStream_t)stream,
                               (const _Float16 *)x, x_n_stride, x_c_stride, w, b, C, H, W, ppb,
                               (_Float16 *)y_first, yf_n_stride, n_first, (_Float16 *)y_rest,
                               yr_n_stride, plane_sum, ps_n_stride);
        else
            hipLaunchKernelGGL(k_dw3x3_lds<float>, gl, dim3(DW_T), 0, (hipStream_t)stream,
                               (const float *)x, x_n_stride, x_c_stride, w, b, C, H, W, ppb,
                               (float *)y_first, yf_n_stride, n_first, (float *)y_rest,
                               yr_n_stride, plane_sum, ps_n_stride);
        YTA_HIP(hipGetLastError());
        return YTA_OK;
    }
    const dim3 g(C, N);
    if (half)
        hipLaunchKernelGGL(k_dw3x3<_Float16>, g, dim3(DW_T), 0, (hipStream_t)stream,
                           (const _Float16 *)x, x_n_stride, x_c_stride, w, b, C, H, W,
                           (_Float16 *)y_first, yf_n_stride, n_first, (_Float16 *)y_rest,
                           yr_n_stride, plane_sum, ps_n_stride);
    else
        hipLaunchKernelGGL(k_dw3x3<float>, g, dim3(DW_T), 0, (hipStream_t)stream, (const float *)x,
                           x_n_stride, x_c_stride, w, b, C, H, W, (float *)y_first, yf_n_stride,
                           n_first, (float *)y_rest, yr_n_stride, plane_sum, ps_n_stride);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int yta_osnet_gate_sum(const void *stack, const void *gate, int N, int C, int P, int half,
                       void *out, void *stream) {
    YTA_CHECK(stack && gate && out && N > 0 && C > 0 && P > 0, YTA_ERR_INVALID, "bad argument");
    const dim3 g(C, N);
    if (half)
        hipLaunchKernelGGL(k_gate_sum<_Float16>, g, dim3(256), 0, (hipStream_t)stream,
                           (const _Float16 *)stack, (const _Float16 *)gate, C, P, (_Float16 *)out);
    else
        hipLaunchKernelGGL(k_gate_sum<float>, g, dim3(256), 0, (hipStream_t)stream,
                           (const float *)stack, (const float *)gate, C, P, (float *)out);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int yta_osnet_pointwise(const yta_pw_args *args, int half, void *stream) {
    YTA_CHECK(args, YTA_ERR_INVALID, "null argument");
    const yta_pw_args &a = *args;
    YTA_CHECK(a.x1 && a.w && a.y && a.G > 0 && a.cout_g > 0 && a.k1 >= 0 && a.k2 >= 0 &&
                  a.k1 + a.k2 > 0 && a.P > 0 && a.N > 0 && (a.k2 == 0 || a.x2),
              YTA_ERR_INVALID, "bad pointwise arguments");
    const int mt = (a.cout_g + 31) / 32, MB = mt >= 3 ? 4 : mt;
    const dim3 g((a.P + 32 * (PW_T / WAVE) - 1) / (32 * (PW_T / WAVE)),
                 a.G * ((mt + MB - 1) / MB), a.N);
    YTA_CHECK(g.y <= 65535 && g.z <= 65535, YTA_ERR_INVALID, "grid too large");
    hipStream_t st = (hipStream_t)stream;
    if (half) {
        if (MB == 1) hipLaunchKernelGGL((k_pw<_Float16, 1>), g, dim3(PW_T), 0, st, a);
        else if (MB == 2) hipLaunchKernelGGL((k_pw<_Float16, 2>), g, dim3(PW_T), 0, st, a);
        else hipLaunchKernelGGL((k_pw<_Float16, 4>), g, dim3(PW_T), 0, st, a);
    } else {
        if (MB == 1) hipLaunchKernelGGL((k_pw<float, 1>), g, dim3(PW_T), 0, st, a);
        else if (MB == 2) hipLaunchKernelGGL((k_pw<float, 2>), g, dim3(PW_T), 0, st, a);
        else hipLaunchKernelGGL((k_pw<float, 4>), g, dim3(PW_T), 0, st, a);
    }
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int yta_osnet_stem(const void *x, int N, int H, int W, const float *w, const float *b, int C0,
                   int half, void *y, void *stream) {
    YTA_CHECK(x && w && b && y && N > 0 && H > 0 && W > 0 && C0 > 0 && C0 % 16 == 0,
              YTA_ERR_INVALID, "bad stem arguments (C0 a multiple of 16)");
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const dim3 g((Wo + ST_TILE - 1) / ST_TILE, (Ho + ST_TILE - 1) / ST_TILE, N);
    const size_t lds = sizeof(float) * 147 * C0;
    if (half)
        hipLaunchKernelGGL((k_stem<_Float16, 16>), g, dim3(256), lds, (hipStream_t)stream,
                           (const _Float16 *)x, H, W, w, b, C0, (_Float16 *)y, Ho, Wo);
    else
        hipLaunchKernelGGL((k_stem<float, 16>), g, dim3(256), lds, (hipStream_t)stream,
                           (const float *)x, H, W, w, b, C0, (float *)y, Ho, Wo);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int yta_osnet_pool(const void *x, int N, int C, int H, int W, int kind, int half, void *y,
                   void *stream) {
    YTA_CHECK(x && y && N > 0 && C > 0 && H > 0 && W > 0 && kind >= 0 && kind <= 2,
              YTA_ERR_INVALID, "bad pool arguments");
    const int Ho = kind == 0 ? (H - 1) / 2 + 1 : H / 2, Wo = kind == 0 ? (W - 1) / 2 + 1 : W / 2;
    YTA_CHECK(kind == 2 || (Ho > 0 && Wo > 0), YTA_ERR_INVALID, "plane too small");
    const dim3 g(C, N);
    if (half)
        hipLaunchKernelGGL(k_pool<_Float16>, g, dim3(256), 0, (hipStream_t)stream,
                           (const _Float16 *)x, C, H, W, kind, (_Float16 *)y, Ho, Wo);
    else
        hipLaunchKernelGGL(k_pool<float>, g, dim3(256), 0, (hipStream_t)stream, (const float *)x, C,
                           H, W, kind, (float *)y, Ho, Wo);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

int yta_osnet_gate(const float *plane_sum, int N, int mid, int hid, int P, const void *w1,
                   const void *b1, const void *w2, const void *b2, int half, void *gate,
                   void *stream) {
    YTA_CHECK(plane_sum && w1 && b1 && w2 && b2 && gate && N > 0 && mid > 0 && mid <= 512 &&
                  hid > 0 && hid <= 64 && P > 0,
              YTA_ERR_INVALID, "bad gate arguments");
    const float inv = 1.0f / (float)P;
    if (half)
        hipLaunchKernelGGL(k_gate<_Float16>, dim3(N), dim3(256), 0, (hipStream_t)stream, plane_sum,
                           inv, (const _Float16 *)w1, (const _Float16 *)b1, (const _Float16 *)w2,
                           (const _Float16 *)b2, mid, hid, (_Float16 *)gate);
    else
        hipLaunchKernelGGL(k_gate<float>, dim3(N), dim3(256), 0, (hipStream_t)stream, plane_sum,
                           inv, (const float *)w1, (const float *)b1, (const float *)w2,
                           (const float *)b2, mid, hid, (float *)gate);
    YTA_HIP(hipGetLastError());
    return YTA_OK;
}

}  // extern "C"
