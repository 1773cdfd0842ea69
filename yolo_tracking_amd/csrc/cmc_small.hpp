// Frame preprocessing shared by the camera-motion estimators (cmc.hip: SparseOptFlow, ecc.hip:
// ECC): CMCInterface.preprocess (boxmot/motion/cmc/cmc_interface.py:26-40) = cvtColor(BGR2GRAY)
// + cv2.resize(fx = fy = scale, INTER_LINEAR), restated in oracle/cmc_sof.py (preprocess), and
// borderInterpolate(BORDER_REFLECT_101).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <cstdint>

namespace yta {
namespace cmc {

// borderInterpolate(p, n, BORDER_REFLECT_101)
__device__ __forceinline__ int refl(int p, int n) {
    if ((unsigned)p < (unsigned)n) return p;
    if (n == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * (n - 1) - p;
    } while ((unsigned)p >= (unsigned)n);
    return p;
}

// cvtColor(BGR2GRAY) (8u fixed point) + cv2.resize(img, (0, 0), fx=scale, fy=scale,
// INTER_LINEAR) (oracle/reid.py resize_linear_u8 with fx / fy) for one output pixel.
__device__ __forceinline__ int bgr_gray(const uint8_t *p) {
    return ((int)p[0] * 1868 + (int)p[1] * 9617 + (int)p[2] * 4899 + (1 << 13)) >> 14;
}

__device__ __forceinline__ int small_pixel(const uint8_t *f, int H, int W, double inv, int ox,
                                           int oy) {
    const double sc = 1.0 / inv;
    auto g = [&](int y, int x) { return bgr_gray(f + ((long long)y * W + x) * 3); };
    if (fabs(sc - 2.0) < DBL_EPSILON) {   // INTER_AREA fast path (exact 2x)
        const int x0 = min(2 * ox, W - 1), x1 = min(2 * ox + 1, W - 1);
        const int y0 = min(2 * oy, H - 1), y1 = min(2 * oy + 1, H - 1);
        return (g(y0, x0) + g(y0, x1) + g(y1, x0) + g(y1, x1) + 2) >> 2;
    }
    float fx = (float)((ox + 0.5) * sc - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) {
        sx = 0;
        fx = 0.f;
    }
    if (sx >= W - 1) {
        sx = W - 1;
        fx = 0.f;
    }
    const int a0 = (int)rintf((1.f - fx) * 2048.f), a1 = (int)rintf(fx * 2048.f);
    const int sx1 = min(sx + 1, W - 1);
    float fy = (float)((oy + 0.5) * sc - 0.5);
    const int sy = (int)floorf(fy);
    fy -= (float)sy;
    const int b0 = (int)rintf((1.f - fy) * 2048.f), b1 = (int)rintf(fy * 2048.f);
    const int r0 = min(max(sy, 0), H - 1), r1 = min(max(sy + 1, 0), H - 1);
    const int D0 = g(r0, sx) * a0 + g(r0, sx1) * a1;
    const int D1 = g(r1, sx) * a0 + g(r1, sx1) * a1;
    const int v = (((D0 >> 4) * b0) >> 16) + (((D1 >> 4) * b1) >> 16);
    return min(max((v + 2) >> 2, 0), 255);
}

}  // namespace cmc
}  // namespace yta
