// ByteTrack constant-velocity Kalman filter in (xc, yc, a, h) space, float64, one track per thread.
// Follows boxmot/motion/kalman_filters/bytetrack_kf.py:40-226.  The covariance is stored as the
// packed upper triangle (36 doubles): F P F^T + Q and P - K S K^T are symmetric, and the packed
// form moves 352 B per track instead of 576 B through HBM.
#pragma once
#include "common.hpp"

namespace yta {

constexpr double KF_W_POS = 1.0 / 20;    // bytetrack_kf.py:52
constexpr double KF_W_VEL = 1.0 / 160;   // bytetrack_kf.py:53
constexpr int KF_NP = 36;                // packed 8x8 symmetric

__host__ __device__ constexpr int pidx(int i, int j) {
    return i <= j ? i * 8 - (i * (i - 1)) / 2 + (j - i) : j * 8 - (j * (j - 1)) / 2 + (i - j);
}

struct KfState {
    double m[8];
    double p[KF_NP];
};

// bytetrack_kf.py:55-86
__host__ __device__ inline void kf_initiate(const double *z, KfState &s) {
    const double h = z[3];
    double sd[8] = {2 * KF_W_POS * h, 2 * KF_W_POS * h, 1e-2, 2 * KF_W_POS * h,
                    10 * KF_W_VEL * h, 10 * KF_W_VEL * h, 1e-5, 10 * KF_W_VEL * h};
    for (int i = 0; i < 4; ++i) { s.m[i] = z[i]; s.m[i + 4] = 0.0; }
    for (int k = 0; k < KF_NP; ++k) s.p[k] = 0.0;
    for (int i = 0; i < 8; ++i) s.p[pidx(i, i)] = sd[i] * sd[i];
}

// bytetrack_kf.py:155-192 for one track: x' = F x, P' = F P F^T + Q(h), F = [[I, I], [0, I]].
// With F's 0/1 structure every product term NumPy forms is exact, so
//   P'[i][j]     = (P[i][j] + P[i+4][j]) + (P[i][j+4] + P[i+4][j+4])   (i, j < 4)
//   P'[i][j+4]   =  P[i][j+4] + P[i+4][j+4]
//   P'[i+4][j+4] =  P[i+4][j+4]
// then + Q on the diagonal.
__host__ __device__ inline void kf_predict(KfState &s) {
    const double h = s.m[3];
    double sd[8] = {KF_W_POS * h, KF_W_POS * h, 1e-2, KF_W_POS * h,
                    KF_W_VEL * h, KF_W_VEL * h, 1e-5, KF_W_VEL * h};
    double np_[KF_NP];
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j)
            np_[pidx(i, j)] = (s.p[pidx(i, j)] + s.p[pidx(i + 4, j)]) +
                              (s.p[pidx(i, j + 4)] + s.p[pidx(i + 4, j + 4)]);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            np_[pidx(i, j + 4)] = s.p[pidx(i, j + 4)] + s.p[pidx(i + 4, j + 4)];
    for (int i = 4; i < 8; ++i)
        for (int j = i; j < 8; ++j) np_[pidx(i, j)] = s.p[pidx(i, j)];
    for (int i = 0; i < 8; ++i) np_[pidx(i, i)] = np_[pidx(i, i)] + sd[i] * sd[i];
    for (int k = 0; k < KF_NP; ++k) s.p[k] = np_[k];
    for (int i = 0; i < 4; ++i) s.m[i] = s.m[i] + s.m[i + 4];
}

// bytetrack_kf.py:194-226 (+ project :126-153): S = H P H^T + R(h), K = P H^T S^-1 via a 4x4
// Cholesky, x += K (z - Hx), P -= K S K^T.
__host__ __device__ inline void kf_update(KfState &s, const double *z) {
    const double h = s.m[3];
    const double r[4] = {KF_W_POS * h, KF_W_POS * h, 1e-1, KF_W_POS * h};
    double S[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) S[i][j] = s.p[pidx(i, j)];
    for (int i = 0; i < 4; ++i) S[i][i] = S[i][i] + r[i] * r[i];
    // Cholesky S = L L^T
    double L[4][4] = {{0}};
    for (int j = 0; j < 4; ++j) {
        double d = S[j][j];
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
        double ljj = sqrt(d);
        L[j][j] = ljj;
        for (int i = j + 1; i < 4; ++i) {
            double v = S[i][j];
            for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
            L[i][j] = v / ljj;
        }
    }
    // K^T (4x8) = S^-1 (P H^T)^T : solve L Y = B, L^T X = Y for the 8 columns
    double K[8][4];
    for (int c = 0; c < 8; ++c) {
        double y[4];
        for (int i = 0; i < 4; ++i) {
            double v = s.p[pidx(c, i)];
            for (int k = 0; k < i; ++k) v -= L[i][k] * y[k];
            y[i] = v / L[i][i];
        }
        double x[4];
        for (int i = 3; i >= 0; --i) {
            double v = y[i];
            for (int k = i + 1; k < 4; ++k) v -= L[k][i] * x[k];
            x[i] = v / L[i][i];
        }
        for (int i = 0; i < 4; ++i) K[c][i] = x[i];
    }
    double innov[4];
    for (int i = 0; i < 4; ++i) innov[i] = z[i] - s.m[i];
    for (int c = 0; c < 8; ++c) {
        double acc = 0.0;
        for (int i = 0; i < 4; ++i) acc += innov[i] * K[c][i];
        s.m[c] = s.m[c] + acc;
    }
    // KS = K S (8x4), then P -= KS K^T
    double KS[8][4];
    for (int c = 0; c < 8; ++c)
        for (int j = 0; j < 4; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 4; ++k) acc += K[c][k] * S[k][j];
            KS[c][j] = acc;
        }
    for (int i = 0; i < 8; ++i)
        for (int j = i; j < 8; ++j) {
            double acc = 0.0;
            for (int k = 0; k < 4; ++k) acc += KS[i][k] * K[j][k];
            s.p[pidx(i, j)] = s.p[pidx(i, j)] - acc;
        }
}

}  // namespace yta
