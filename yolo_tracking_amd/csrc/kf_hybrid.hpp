// HybridSORT's Kalman filter (boxmot/motion/kalman_filters/hybridsort_kf.py: predict :339-380,
// update :439-528, freeze :383-387, unfreeze :390-436) as set up by KalmanBoxTracker
// (boxmot/trackers/hybridsort/hybridsort.py:130-156): state x = (u, v, s, c, r, u', v', s', c'),
// F adds velocity i+5 to position i (i < 4), H picks x[0..4] (z = (u, v, s, score, r)),
// P0 = 10 I with the velocity block x1000, Q = I with Q[5:,5:] x0.01 and Q[7,7], Q[8,8] x0.01
// once more, R = diag(1, 1, 10, 10, 10).
//
// Layout.  As for OCSORT's filter (kf_ocsort.hpp): P0, Q and R are diagonal and F / H couple only
// i with i+5, so every covariance the reference forms is zero outside the 2x2 blocks {0,5},
// {1,6}, {2,7}, {3,8} and the 1x1 block {4}; inv(S) of the diagonal S is diag(1/S_ii) (LAPACK's LU
// of a diagonal matrix), and each block evolves on its own with the reference's operation order
// kept term by term (zero terms of its products add exactly).  17 doubles per covariance.
// KAT: tests/test_gpu_hybridsort.py (yta_kf9_run against oracle/hybridsort.py's KF9).
#pragma once
#include "common.hpp"

namespace yta {

struct Kf9 {
    double x[9];
    double p[17];   // block g < 4: P_aa, P_ab, P_ba, P_bb (a = g, b = g + 5); p[16] = P_44
};

__host__ __device__ __forceinline__ double hs_r(int m) { return m < 2 ? 1.0 : 10.0; }
// Q of velocity g: Q[5:,5:] *= 0.01 after Q[7,7] and Q[8,8] were scaled by 0.01 (hybridsort.py:152-154)
__host__ __device__ __forceinline__ double hs_qv(int g) { return g >= 2 ? (1.0 * 0.01) * 0.01 : 0.01; }

// hybridsort.py:33-49 convert_bbox_to_z (score non-zero: the 5-vector form)
__host__ __device__ __forceinline__ void hs_bbox_to_z(const double *b, double *z) {
    const double w = b[2] - b[0];
    const double h = b[3] - b[1];
    z[0] = b[0] + w / 2.0;
    z[1] = b[1] + h / 2.0;
    z[2] = w * h;
    z[3] = b[4];
    z[4] = w / (h + 1e-6);
}

// hybridsort.py:52-63 convert_x_to_bbox (box; the score column is x[3])
__host__ __device__ __forceinline__ void hs_x_to_bbox(const double *x, double *b) {
    const double w = sqrt(x[2] * x[4]);
    const double h = x[2] / w;
    b[0] = x[0] - w / 2.0;
    b[1] = x[1] - h / 2.0;
    b[2] = x[0] + w / 2.0;
    b[3] = x[1] + h / 2.0;
}

// hybridsort.py:131-156: x[:5] = z, P = 10 * (I with P[5:,5:] *= 1000)
__host__ __device__ inline void kf9_init(const double *z, Kf9 &s) {
    for (int i = 0; i < 5; ++i) s.x[i] = z[i];
    for (int i = 5; i < 9; ++i) s.x[i] = 0.0;
    for (int g = 0; g < 4; ++g) {
        s.p[4 * g + 0] = 1.0 * 10.0;
        s.p[4 * g + 1] = 0.0;
        s.p[4 * g + 2] = 0.0;
        s.p[4 * g + 3] = (1.0 * 1000.0) * 10.0;
    }
    s.p[16] = 1.0 * 10.0;
}

// x = F x; P = 1.0 * (F P) F^T + Q
__host__ __device__ inline void kf9_predict(Kf9 &s) {
    for (int g = 0; g < 4; ++g) {
        const double aa = s.p[4 * g], ab = s.p[4 * g + 1], ba = s.p[4 * g + 2], bb = s.p[4 * g + 3];
        s.p[4 * g + 0] = ((aa + ba) + (ab + bb)) + 1.0;
        s.p[4 * g + 1] = (ab + bb) + 0.0;
        s.p[4 * g + 2] = (ba + bb) + 0.0;
        s.p[4 * g + 3] = bb + hs_qv(g);
        s.x[g] = s.x[g] + s.x[g + 5];
    }
    s.p[16] = s.p[16] + 1.0;
}

// The measurement step for z (hybridsort_kf.py:492-528).
__host__ __device__ inline void kf9_correct(Kf9 &s, const double *z) {
    for (int g = 0; g < 4; ++g) {
        const double R = hs_r(g);
        const double aa = s.p[4 * g], ab = s.p[4 * g + 1], ba = s.p[4 * g + 2], bb = s.p[4 * g + 3];
        const double si = 1.0 / (aa + R);
        const double ka = aa * si, kb = ba * si;
        const double y = z[g] - s.x[g];
        s.x[g] = s.x[g] + ka * y;
        s.x[g + 5] = s.x[g + 5] + kb * y;
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
    const double pp = s.p[16], R = hs_r(4);
    const double k = pp * (1.0 / (pp + R));
    const double y = z[4] - s.x[4];
    s.x[4] = s.x[4] + k * y;
    const double i = 1.0 - k;
    s.p[16] = ((i * pp) * i) + (k * R) * k;
}

// unfreeze's virtual trajectory (hybridsort_kf.py:397-436): from the last measurement kept in the
// filter's history (z1) to the new one (z2), `gap` steps apart, with update / predict pairs.  The
// stored (u, v, s, c, r) is unpacked as (x, y, s, r, c): w = sqrt(s c), h = sqrt(s / c), and the
// replayed measurement is (x, y, w h, w / h, interpolated r).
__host__ __device__ inline void kf9_replay(Kf9 &s, const double *z1, const double *z2, int gap,
                                           double *last_z) {
    const double w1 = sqrt(z1[2] * z1[3]), h1 = sqrt(z1[2] / z1[3]);
    const double w2 = sqrt(z2[2] * z2[3]), h2 = sqrt(z2[2] / z2[3]);
    const double g = (double)gap;
    const double dx = (z2[0] - z1[0]) / g, dy = (z2[1] - z1[1]) / g;
    const double dw = (w2 - w1) / g, dh = (h2 - h1) / g;
    const double dc = (z2[4] - z1[4]) / g;
    for (int i = 0; i < gap; ++i) {
        const double t = (double)(i + 1);
        const double w = w1 + t * dw, h = h1 + t * dh;
        double v[5];
        v[0] = z1[0] + t * dx;
        v[1] = z1[1] + t * dy;
        v[2] = w * h;
        v[3] = w / h;
        v[4] = z1[4] + t * dc;
        kf9_correct(s, v);
        if (i == gap - 1)
            for (int k = 0; k < 5; ++k) last_z[k] = v[k];
        else
            kf9_predict(s);
    }
}

}  // namespace yta
