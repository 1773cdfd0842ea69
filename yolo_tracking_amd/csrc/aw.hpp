// compute_aw_max_metric building blocks (boxmot/utils/association.py:79-108), shared by the
// DeepOCSORT engine (deepocsort.hip) and its known-answer entry point (kat.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace yta {

// Running top two of a row or column: argsort(-x)[0:2] picks the largest value and the second in
// sorted order, which equals the largest when it occurs twice; selection is order-free.
__device__ __forceinline__ void top2_push(double v, double &m1, double &m2) {
    if (v > m1) {
        m2 = m1;
        m1 = v;
    } else if (v > m2) {
        m2 = v;
    }
}
__device__ __forceinline__ double aw_weight(double m1, double m2, double bottom, int n) {
    if (n < 2) return 1.0;
    if (m1 == 0) return 0.0;
    double ex = (m2 / m1) - bottom;
    ex = ex > 0 ? ex : 0.0;   // max(..., 0)
    return 1 - ex / (1 - bottom);
}

}  // namespace yta
