// DeepOCSORT's Kalman filter, "new KF" branch (boxmot/trackers/deepocsort/deep_ocsort.py:103-136,
// :76-87; boxmot/motion/kalman_filters/deepocsort_kf.py: predict :340-379, apply_affine_correction
// :387-407, unfreeze :433-478, update :480-580): state (x, y, w, h, x', y', w', h').
//
// Layout.  F couples i with i+4, H picks x[0..3], Q and R are diagonal, and the camera-motion
// correction multiplies (x, y), (w, h), (x', y'), (w', h') by the same 2x2 matrix, so every
// covariance the reference forms is zero outside two 4x4 groups: A = {x, y, x', y'} (global
// indices 0, 1, 4, 5) and B = {w, h, w', h'} (2, 3, 6, 7).  Each group is stored as a full 4x4
// (local order = ascending global index).  Every product is a plain sum over ascending global k
// (no fused multiply-add), so with the zero terms the reference's 8x8 products contain - exact
// no-ops - a stream without camera motion is bit-identical to NumPy / OpenBLAS; under a camera
// warp (2x2 blocks inside S, LAPACK's LU inverse) the state agrees to rounding (parity tolerance).
#pragma once
#include "common.hpp"

namespace yta {

struct Kf8 {
    double x[8];
    double p[2][16];   // group g, local (i, j) at 4 * i + j
};

constexpr double DK_P = 1.0 / 20, DK_V = 1.0 / 160;   // deep_ocsort.py:76
__host__ __device__ __forceinline__ int dk_glob(int g, int l) {   // local -> global index
    return (l & 1) + 2 * g + 4 * (l >> 1);
}

// deep_ocsort.py:76-80 (Q(w, h)) diagonal entry of global index i
__host__ __device__ __forceinline__ double dk_q(int i, double w, double h) {
    const double wh = (i & 1) ? h : w;
    const double f = i < 4 ? DK_P : DK_V;
    const double v = f * wh;
    return v * v;
}

__host__ __device__ inline void kf8_init(const double *z, Kf8 &s) {   // :103-116
    for (int i = 0; i < 4; ++i) s.x[i] = z[i];
    for (int i = 4; i < 8; ++i) s.x[i] = 0.0;
    for (int g = 0; g < 2; ++g)
        for (int k = 0; k < 16; ++k) {
            const int i = k >> 2, j = k & 3;
            double v = 0.0;
            if (i == j) {
                const int gi = dk_glob(g, i);
                v = dk_q(gi, z[2], z[3]) * (gi < 4 ? 4.0 : 100.0);
            }
            s.p[g][k] = v;
        }
}

// x = F x; P = 1.0 * (F P) F^T + Q, Q given by its diagonal (qd[8], global order)
__host__ __device__ inline void kf8_predict(Kf8 &s, const double *qd) {
    for (int g = 0; g < 2; ++g) {
        double *P = s.p[g];
        double FP[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                FP[4 * i + j] = i < 2 ? P[4 * i + j] + P[4 * (i + 2) + j] : P[4 * i + j];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const double v = j < 2 ? FP[4 * i + j] + FP[4 * i + j + 2] : FP[4 * i + j];
                P[4 * i + j] = v + (i == j ? qd[dk_glob(g, i)] : 0.0);
            }
    }
    for (int i = 0; i < 4; ++i) s.x[i] = s.x[i] + s.x[i + 4];
}

// Inverse of a 2x2 block [[a, b], [c, d]] the way LAPACK's getrf / getrs does it on a
// block-diagonal matrix: partial pivoting, multiplier, back substitution of the identity.
__host__ __device__ inline void inv2_lu(double a, double b, double c, double d, double *o) {
    const bool sw = fabs(c) > fabs(a);
    const double p = sw ? c : a, q = sw ? d : b, r = sw ? a : c, t = sw ? b : d;
    const double l = r / p;
    const double u = t - l * q;
    // columns e0, e1 of the (row-swapped) identity
    double e[2][2] = {{sw ? 0.0 : 1.0, sw ? 1.0 : 0.0}, {sw ? 1.0 : 0.0, sw ? 0.0 : 1.0}};
    for (int col = 0; col < 2; ++col) {
        const double y0 = e[0][col];
        const double y1 = e[1][col] - l * y0;
        const double x1 = y1 / u;
        const double x0 = (y0 - q * x1) / p;
        o[0 * 2 + col] = x0;
        o[1 * 2 + col] = x1;
    }
}

// Measurement step for z = (x, y, w, h) with R given by its diagonal rd[4] (deepocsort_kf.py:
// 531-580): y = z - Hx, S = H P H^T + R, K = P H^T inv(S), x += K y, Joseph-form P.
__host__ __device__ inline void kf8_correct(Kf8 &s, const double *z, const double *rd) {
    for (int g = 0; g < 2; ++g) {
        double *P = s.p[g];
        const int m0 = 2 * g;   // measurement rows of this group: m0, m0 + 1
        double S[4];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j) S[2 * i + j] = P[4 * i + j] + (i == j ? rd[m0 + i] : 0.0);
        double SI[4];
        inv2_lu(S[0], S[1], S[2], S[3], SI);
        double K[8];   // 4 x 2
        for (int i = 0; i < 4; ++i)
            for (int m = 0; m < 2; ++m) K[2 * i + m] = P[4 * i + 0] * SI[m] + P[4 * i + 1] * SI[2 + m];
        const double y0 = z[m0] - s.x[dk_glob(g, 0)], y1 = z[m0 + 1] - s.x[dk_glob(g, 1)];
        for (int i = 0; i < 4; ++i) {
            const int gi = dk_glob(g, i);
            s.x[gi] = s.x[gi] + (K[2 * i] * y0 + K[2 * i + 1] * y1);
        }
        double IKH[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const double kh = j < 2 ? K[2 * i + j] : 0.0;
                IKH[4 * i + j] = (i == j ? 1.0 : 0.0) - kh;
            }
        double C[16], D[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double acc = IKH[4 * i] * P[j];
                for (int k = 1; k < 4; ++k) acc = acc + IKH[4 * i + k] * P[4 * k + j];
                C[4 * i + j] = acc;
            }
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double acc = C[4 * i] * IKH[4 * j];
                for (int k = 1; k < 4; ++k) acc = acc + C[4 * i + k] * IKH[4 * j + k];
                D[4 * i + j] = acc;
            }
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                const double kr0 = K[2 * i] * rd[m0], kr1 = K[2 * i + 1] * rd[m0 + 1];
                const double krk = kr0 * K[2 * j] + kr1 * K[2 * j + 1];
                P[4 * i + j] = D[4 * i + j] + krk;
            }
    }
}

// Camera-motion correction of a state (deepocsort_kf.py:393-397): x <- B x, x[:2] += t,
// P <- B P B^T with B = kron(I4, m).
__host__ __device__ inline void kf8_affine(Kf8 &s, const double *m, const double *t) {
    double nx[8];
    for (int p = 0; p < 4; ++p) {   // pairs (0,1), (2,3), (4,5), (6,7)
        const double a = s.x[2 * p], b = s.x[2 * p + 1];
        nx[2 * p] = m[0] * a + m[1] * b;
        nx[2 * p + 1] = m[2] * a + m[3] * b;
    }
    nx[0] = nx[0] + t[0];
    nx[1] = nx[1] + t[1];
    for (int i = 0; i < 8; ++i) s.x[i] = nx[i];
    for (int g = 0; g < 2; ++g) {
        double *P = s.p[g];
        double BP[16];
        // B restricted to the group: diag(m, m) in local order (pairs (0,1) and (2,3))
        auto Bl = [&](int i, int k) {
            if ((i >> 1) != (k >> 1)) return 0.0;
            return m[2 * (i & 1) + (k & 1)];
        };
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double acc = Bl(i, 0) * P[j];
                for (int k = 1; k < 4; ++k) acc = acc + Bl(i, k) * P[4 * k + j];
                BP[4 * i + j] = acc;
            }
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                double acc = BP[4 * i] * Bl(j, 0);
                for (int k = 1; k < 4; ++k) acc = acc + BP[4 * i + k] * Bl(j, k);
                P[4 * i + j] = acc;
            }
    }
}

// unfreeze's replay (deepocsort_kf.py:433-478): the stored measurement (x, y, w, h) read as
// (x, y, s, r), virtual boxes z = (x, y, w h, w / h), updates with R = I, predicts with Q = I.
__host__ __device__ inline void kf8_replay(Kf8 &s, const double *z1, const double *z2, int gap,
                                           double *last_z) {
    const double w1 = sqrt(z1[2] * z1[3]), h1 = sqrt(z1[2] / z1[3]);
    const double w2 = sqrt(z2[2] * z2[3]), h2 = sqrt(z2[2] / z2[3]);
    const double g = (double)gap;
    const double dx = (z2[0] - z1[0]) / g, dy = (z2[1] - z1[1]) / g;
    const double dw = (w2 - w1) / g, dh = (h2 - h1) / g;
    const double one4[4] = {1.0, 1.0, 1.0, 1.0};
    const double one8[8] = {1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0};
    for (int i = 0; i < gap; ++i) {
        const double t = (double)(i + 1);
        const double w = w1 + t * dw, h = h1 + t * dh;
        double v[4];
        v[0] = z1[0] + t * dx;
        v[1] = z1[1] + t * dy;
        v[2] = w * h;
        v[3] = w / h;
        kf8_correct(s, v, one4);
        if (i == gap - 1)
            for (int k = 0; k < 4; ++k) last_z[k] = v[k];
        else
            kf8_predict(s, one8);
    }
}

}  // namespace yta
