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
// NCHW planes, float32 or float16 storage, float32 arithmetic.
#include "common.hpp"

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

}  // extern "C"
