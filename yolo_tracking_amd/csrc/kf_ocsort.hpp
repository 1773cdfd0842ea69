// OCSORT's Kalman filter (boxmot/motion/kalman_filters/ocsort_kf.py: predict :339-380, update
// :437-526, freeze :383-387, unfreeze :390-434) as set up by KalmanBoxTracker (ocsort.py:76-106):
// state x = (u, v, s, r, u', v', s'), F adds velocity i+4 to position i (i < 3), H picks x[0..3],
// P0 = 10 I with the velocity block x1000, Q = I with Q[4:,4:] x0.01 and Q[6,6] x0.01 once more,
// R = diag(1, 1, 10, 10).
//
// Layout.  P0, Q and R are diagonal and F / H only couple i with i+4, so every covariance the
// reference forms is zero outside the 2x2 blocks {0,4}, {1,5}, {2,6} and the 1x1 block {3}: S is
// diagonal, inv(S) = diag(1/S_ii) (LAPACK's LU of a diagonal matrix), and each block evolves on
// its own.  13 doubles per covariance (block g: P_aa, P_ab, P_ba, P_bb; then P_33), with the
// reference's operation order on the full matrices kept term by term (zero terms of its products
// add exactly): e.g. predict P'_aa = ((P_aa + P_ba) + (P_ab + P_bb)) + Q_a, and the Joseph form
// (I-KH) P (I-KH)^T + K R K^T expanded per block.  KAT: tests/test_gpu_ocsort.py (sequences of
// predict / update / missed updates / re-acquisitions against oracle/ocsort.py's KF7).
#pragma once
#include "common.hpp"

namespace yta {

struct Kf7 {
    double x[7];
    double p[13];
};

constexpr double OC_Q_VEL = 0.01;              // Q[4:, 4:] *= 0.01
constexpr double OC_Q_S = 0.01 * 0.01;         // Q[6, 6] *= 0.01, then *= 0.01 again
__host__ __device__ __forceinline__ double oc_r(int m) { return m < 2 ? 1.0 : 10.0; }
__host__ __device__ __forceinline__ double oc_qv(int g) { return g == 2 ? OC_Q_S : OC_Q_VEL; }

// ocsort.py:25-37 convert_bbox_to_z
__host__ __device__ __forceinline__ void oc_bbox_to_z(const double *b, double *z) {
    const double w = b[2] - b[0];
    const double h = b[3] - b[1];
    z[0] = b[0] + w / 2.0;
    z[1] = b[1] + h / 2.0;
    z[2] = w * h;
    z[3] = w / (h + 1e-6);
}

// ocsort.py:40-54 convert_x_to_bbox
__host__ __device__ __forceinline__ void oc_x_to_bbox(const double *x, double *b) {
    const double w = sqrt(x[2] * x[3]);
    const double h = x[2] / w;
    b[0] = x[0] - w / 2.0;
    b[1] = x[1] - h / 2.0;
    b[2] = x[0] + w / 2.0;
    b[3] = x[1] + h / 2.0;
}

// ocsort.py:101-108: x[:4] = z, P = 10 * (I with P[4:,4:] *= 1000)
__host__ __device__ inline void kf7_init(const double *z, Kf7 &s) {
    for (int i = 0; i < 4; ++i) s.x[i] = z[i];
    for (int i = 4; i < 7; ++i) s.x[i] = 0.0;
    for (int g = 0; g < 3; ++g) {
        s.p[4 * g + 0] = 1.0 * 10.0;
        s.p[4 * g + 1] = 0.0;
        s.p[4 * g + 2] = 0.0;
        s.p[4 * g + 3] = (1.0 * 1000.0) * 10.0;
    }
    s.p[12] = 1.0 * 10.0;
}

// x = F x; P = 1.0 * (F P) F^T + Q
__host__ __device__ inline void kf7_predict(Kf7 &s) {
    for (int g = 0; g < 3; ++g) {
        const double aa = s.p[4 * g], ab = s.p[4 * g + 1], ba = s.p[4 * g + 2], bb = s.p[4 * g + 3];
        s.p[4 * g + 0] = ((aa + ba) + (ab + bb)) + 1.0;
        s.p[4 * g + 1] = (ab + bb) + 0.0;
        s.p[4 * g + 2] = (ba + bb) + 0.0;
        s.p[4 * g + 3] = bb + oc_qv(g);
        s.x[g] = s.x[g] + s.x[g + 4];
    }
    s.p[12] = s.p[12] + 1.0;
}

// The measurement step for z (ocsort_kf.py:478-526).
__host__ __device__ inline void kf7_correct(Kf7 &s, const double *z) {
    for (int g = 0; g < 3; ++g) {
        const double R = oc_r(g);
        const double aa = s.p[4 * g], ab = s.p[4 * g + 1], ba = s.p[4 * g + 2], bb = s.p[4 * g + 3];
        const double si = 1.0 / (aa + R);
        const double ka = aa * si, kb = ba * si;
        const double y = z[g] - s.x[g];
        s.x[g] = s.x[g] + ka * y;
        s.x[g + 4] = s.x[g + 4] + kb * y;
        const double ia = 1.0 - ka, ib = 0.0 - kb;   // (I - KH) entries (a, a), (b, a)
        const double caa = ia * aa, cab = ia * ab;    // C = (I - KH) P
        const double cba = ib * aa + ba, cbb = ib * ab + bb;
        const double daa = caa * ia, dab = caa * ib + cab;   // D = C (I - KH)^T
        const double dba = cba * ia, dbb = cba * ib + cbb;
        const double ea = ka * R, eb = kb * R;        // K R, then (K R) K^T
        s.p[4 * g + 0] = daa + ea * ka;
        s.p[4 * g + 1] = dab + ea * kb;
        s.p[4 * g + 2] = dba + eb * ka;
        s.p[4 * g + 3] = dbb + eb * kb;
    }
    const double pp = s.p[12], R = oc_r(3);
    const double k = pp * (1.0 / (pp + R));
    const double y = z[3] - s.x[3];
    s.x[3] = s.x[3] + k * y;
    const double i = 1.0 - k;
    s.p[12] = ((i * pp) * i) + (k * R) * k;
}

// unfreeze's virtual trajectory (ocsort_kf.py:399-434): from the last observation kept in the
// filter's history (z1) to the new one (z2), `gap` steps apart, with update / predict pairs.
__host__ __device__ inline void kf7_replay(Kf7 &s, const double *z1, const double *z2, int gap,
                                           double *last_z) {
    const double w1 = sqrt(z1[2] * z1[3]), h1 = sqrt(z1[2] / z1[3]);
    const double w2 = sqrt(z2[2] * z2[3]), h2 = sqrt(z2[2] / z2[3]);
    const double g = (double)gap;
    const double dx = (z2[0] - z1[0]) / g, dy = (z2[1] - z1[1]) / g;
    const double dw = (w2 - w1) / g, dh = (h2 - h1) / g;
    for (int i = 0; i < gap; ++i) {
        const double t = (double)(i + 1);
        const double w = w1 + t * dw, h = h1 + t * dh;
        double v[4];
        v[0] = z1[0] + t * dx;
        v[1] = z1[1] + t * dy;
        v[2] = w * h;
        v[3] = w / h;
        kf7_correct(s, v);
        if (i == gap - 1)
            for (int k = 0; k < 4; ++k) last_z[k] = v[k];
        else
            kf7_predict(s);
    }
}

// numpy's sum of a 5-vector, a left-to-right running sum below 8 elements (checked against
// np.sum) - last_observation.sum() (ocsort.py:137, :355)
__host__ __device__ __forceinline__ double np_sum5(const double *a) {
    return (((a[0] + a[1]) + a[2]) + a[3]) + a[4];
}

}  // namespace yta
