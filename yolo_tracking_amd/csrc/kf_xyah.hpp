// Constant-velocity Kalman filters of ByteTrack (state (xc, yc, a, h), bytetrack_kf.py:40-226) and
// BoT-SORT (state (xc, yc, w, h), botsort_kf.py:21-226), float64, one track per thread.  The two
// differ only in their noise terms (template parameter M: KF_XYAH / KF_XYWH):
//   XYAH: every std scales with the height h = mean[3]; the aspect terms are constants
//   XYWH: x / w terms scale with the width w = mean[2], y / h terms with the height
//
// Layout.  initiate() builds a diagonal covariance (:85), Q and R are diagonal (:117, :148) and F
// couples only position i with velocity i+4 (:44-46).  Hence every covariance the reference ever
// forms is exactly zero outside the four 2x2 blocks {i, i+4} (checked on every golden state), and
// each block evolves independently.  A track is stored as 24 doubles (192 B):
//   m[0..7]                 mean
//   c[4i+0..3] (i = 0..3)   P[i][i], P[i][i+4], P[i+4][i], P[i+4][i+4]
// The two off-diagonal entries are kept separately because the reference's products leave them
// one ulp apart.  Every value is computed with the exact operation sequence NumPy / SciPy /
// OpenBLAS perform on the full 8x8 matrices (their extra terms are exact zeros), so predict and
// update are bit-identical to the reference (KAT: tests/test_gpu_kat.py::test_kf_xyah_kat):
//   predict  P'pp = ((pp + vp) + (pv + vv)) + qp,  P'pv = pv + vv,  P'vp = vp + vv,  P'vv = vv + qv
//   update   S = pp + r^2, l = sqrt(S), K = (b * (1/l)) * (1/l)   (dpotrf + OpenBLAS dtrsm with
//            inverted diagonal), x += innov * K, P -= K (S K^T)    (multi_dot order A(BC))
#pragma once
#include "common.hpp"

namespace yta {

constexpr double KF_W_POS = 1.0 / 20;    // bytetrack_kf.py:52
constexpr double KF_W_VEL = 1.0 / 160;   // bytetrack_kf.py:53
constexpr int KF_REC = 24;               // doubles per stored track
constexpr int KF_XYAH = 0, KF_XYWH = 1;   // noise models

// Per-axis standard deviations (before squaring) from a mean / measurement (n = 4 each):
// scale(i) = h for XYAH, (w, h, w, h)[i] for XYWH.
template <int M>
__host__ __device__ __forceinline__ double kf_scale(const double *v, int i) {
    return M == KF_XYWH ? ((i & 1) ? v[3] : v[2]) : v[3];
}

struct KfState {
    double m[8];
    double c[16];
};

// bytetrack_kf.py:55-86 / botsort_kf.py:43-73
template <int M = KF_XYAH>
__host__ __device__ inline void kf_initiate(const double *z, KfState &s) {
    double sp[4], sv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double g = kf_scale<M>(z, i);
        const bool aspect = M == KF_XYAH && i == 2;
        sp[i] = aspect ? 1e-2 : 2 * KF_W_POS * g;
        sv[i] = aspect ? 1e-5 : 10 * KF_W_VEL * g;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        s.m[i] = z[i];
        s.m[i + 4] = 0.0;
        s.c[4 * i + 0] = sp[i] * sp[i];
        s.c[4 * i + 1] = 0.0;
        s.c[4 * i + 2] = 0.0;
        s.c[4 * i + 3] = sv[i] * sv[i];
    }
}

// Predicted mean only (what the association boxes need): x' = F x.
__host__ __device__ inline void kf_predict_mean(const double *m, double *out) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        out[i] = m[i] + m[i + 4];
        out[i + 4] = m[i + 4];
    }
}

// bytetrack_kf.py:155-192 / botsort_kf.py:150-190 (multi_predict) for one track.
template <int M = KF_XYAH>
__host__ __device__ inline void kf_predict(KfState &s) {
    double sp[4], sv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double g = kf_scale<M>(s.m, i);
        const bool aspect = M == KF_XYAH && i == 2;
        sp[i] = aspect ? 1e-2 : KF_W_POS * g;
        sv[i] = aspect ? 1e-5 : KF_W_VEL * g;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double pp = s.c[4 * i], pv = s.c[4 * i + 1], vp = s.c[4 * i + 2], vv = s.c[4 * i + 3];
        s.c[4 * i + 0] = ((pp + vp) + (pv + vv)) + sp[i] * sp[i];
        s.c[4 * i + 1] = pv + vv;
        s.c[4 * i + 2] = vp + vv;
        s.c[4 * i + 3] = vv + sv[i] * sv[i];
        s.m[i] = s.m[i] + s.m[i + 4];
    }
}

// bytetrack_kf.py:194-226 (+ project :126-153) / botsort_kf.py:192-226 (+ project :110-148).
template <int M = KF_XYAH>
__host__ __device__ inline void kf_update(KfState &s, const double *z) {
    double r[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        r[i] = (M == KF_XYAH && i == 2) ? 1e-1 : KF_W_POS * kf_scale<M>(s.m, i);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double pp = s.c[4 * i], pv = s.c[4 * i + 1], vp = s.c[4 * i + 2], vv = s.c[4 * i + 3];
        const double S = pp + r[i] * r[i];
        const double il = 1.0 / sqrt(S);
        const double kp = (pp * il) * il;
        const double kv = (vp * il) * il;
        const double innov = z[i] - s.m[i];
        s.m[i] = s.m[i] + innov * kp;
        s.m[i + 4] = s.m[i + 4] + innov * kv;
        s.c[4 * i + 0] = pp - kp * (S * kp);
        s.c[4 * i + 1] = pv - kp * (S * kv);
        s.c[4 * i + 2] = vp - kv * (S * kp);
        s.c[4 * i + 3] = vv - kv * (S * kv);
    }
}

// Full 8x8 view (parity introspection / KAT entry points).
__host__ __device__ inline void kf_cov_full(const KfState &s, double *P) {
    for (int k = 0; k < 64; ++k) P[k] = 0.0;
    for (int i = 0; i < 4; ++i) {
        P[i * 8 + i] = s.c[4 * i];
        P[i * 8 + i + 4] = s.c[4 * i + 1];
        P[(i + 4) * 8 + i] = s.c[4 * i + 2];
        P[(i + 4) * 8 + i + 4] = s.c[4 * i + 3];
    }
}
__host__ __device__ inline void kf_cov_pack(const double *P, KfState &s) {
    for (int i = 0; i < 4; ++i) {
        s.c[4 * i] = P[i * 8 + i];
        s.c[4 * i + 1] = P[i * 8 + i + 4];
        s.c[4 * i + 2] = P[(i + 4) * 8 + i];
        s.c[4 * i + 3] = P[(i + 4) * 8 + i + 4];
    }
}

}  // namespace yta
