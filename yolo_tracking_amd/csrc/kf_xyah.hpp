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

// ByteTrack's lost list is predicted lazily: a track's stored state is the one of the frame it was
// marked lost, and the k predicts of the frames since (multi_predict zeroes vh first,
// bytetrack_kf.py:41-42; its state is Lost, or Removed for one frame after expiry, the
// removed_stracks quirk :262-265) are replayed where the state is needed, in the same operation
// order, so the result is bit-identical to predicting every frame.
__host__ __device__ inline void kf_predict_lost(KfState &s, int k) {
    for (int j = 0; j < k; ++j) {
        s.m[7] = 0;
        kf_predict<KF_XYAH>(s);
    }
}
// The mean alone (pool / duplicate-removal boxes): kf_predict's mean update with vh = 0.
__host__ __device__ inline void kf_predict_lost_mean(double *m, int k) {
    m[7] = 0;
    for (int j = 0; j < k; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) m[i] = m[i] + m[i + 4];
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

// ---------------------------------------------------------------- BoT-SORT camera-motion warps
// STrack.multi_gmc (bot_sort.py:95-111): mean <- kron(I4, R) mean, mean[:2] += t,
// P <- R8 P R8^T with R8 = kron(I4, R).  R mixes x with y (and w with h, and their velocities),
// so after a warp P is no longer confined to the 2x2 blocks {i, i+4}: it is block-diagonal over
// the two groups {x, y, vx, vy} = {0, 1, 4, 5} and {w, h, vw, vh} = {2, 3, 6, 7} (F, H, Q, R and
// R8 never couple the groups).  A warped track keeps the 8 extra entries of each group in
// x[8g + k] (the pairs of a group whose two indices lie on different axes, XCROSS order below)
// beside its compact record; predict / update then run on each group's dense 4x4 block with the
// reference's product order (the compact formulas above are these with the cross terms zero).
// Local index l of a group g: global 2g + (l & 1) + 4 * (l >> 1); axis l & 1.
__host__ __device__ __forceinline__ int grp_global(int g, int l) { return 2 * g + (l & 1) + 4 * (l >> 1); }
// cross pairs (r, c), axis(r) != axis(c), row-major
__host__ __device__ __forceinline__ void xcross(int k, int &r, int &c) {
    const int R[8] = {0, 0, 1, 1, 2, 2, 3, 3}, C[8] = {1, 3, 0, 2, 1, 3, 0, 2};
    r = R[k];
    c = C[k];
}

// group block P[16] (row-major, local indices) from the compact record + cross terms
__host__ __device__ inline void grp_load(const KfState &s, const double *x, int g, double *P) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if ((r & 1) != (c & 1)) continue;
            const int i = 2 * g + (r & 1);             // the compact block of this axis
            const int k = ((r >> 1) << 1) | (c >> 1);   // 0 pp, 1 pv, 2 vp, 3 vv
            P[4 * r + c] = s.c[4 * i + k];
        }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int r, c;
        xcross(k, r, c);
        P[4 * r + c] = x[8 * g + k];
    }
}
__host__ __device__ inline void grp_store(const double *P, int g, KfState &s, double *x) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if ((r & 1) != (c & 1)) continue;
            const int i = 2 * g + (r & 1);
            const int k = ((r >> 1) << 1) | (c >> 1);
            s.c[4 * i + k] = P[4 * r + c];
        }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int r, c;
        xcross(k, r, c);
        x[8 * g + k] = P[4 * r + c];
    }
}

// multi_gmc on one track: H = [R00 R01 t0; R10 R11 t1] row-major (2x3)
__host__ __device__ inline void kf_gmc(KfState &s, double *x, const double *H) {
    const double R[2][2] = {{H[0], H[1]}, {H[3], H[4]}};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const double a = s.m[2 * p], b = s.m[2 * p + 1];
        s.m[2 * p] = R[0][0] * a + R[0][1] * b;
        s.m[2 * p + 1] = R[1][0] * a + R[1][1] * b;
    }
    s.m[0] += H[2];
    s.m[1] += H[5];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        double P[16], T[16];
        grp_load(s, x, g, P);
#pragma unroll
        for (int r = 0; r < 4; ++r)                     // T = Rg P (Rg = blockdiag(R, R))
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int q = r & ~1;
                T[4 * r + c] = R[r & 1][0] * P[4 * q + c] + R[r & 1][1] * P[4 * (q + 1) + c];
            }
#pragma unroll
        for (int r = 0; r < 4; ++r)                     // P = T Rg^T
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int q = c & ~1;
                P[4 * r + c] = T[4 * r + q] * R[c & 1][0] + T[4 * r + q + 1] * R[c & 1][1];
            }
        grp_store(P, g, s, x);
    }
}

// botsort_kf.py:150-190 for a track carrying cross terms (XYWH noise)
__host__ __device__ inline void kf_predict_x(KfState &s, double *x) {
    double q[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double g = kf_scale<KF_XYWH>(s.m, i);
        q[i] = (KF_W_POS * g) * (KF_W_POS * g);
        q[i + 4] = (KF_W_VEL * g) * (KF_W_VEL * g);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        double P[16], L[16];
        grp_load(s, x, g, P);
#pragma unroll
        for (int r = 0; r < 4; ++r)                     // L = F P
#pragma unroll
            for (int c = 0; c < 4; ++c) L[4 * r + c] = r < 2 ? P[4 * r + c] + P[4 * (r + 2) + c] : P[4 * r + c];
#pragma unroll
        for (int r = 0; r < 4; ++r)                     // P = L F^T + Q
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                double v = c < 2 ? L[4 * r + c] + L[4 * r + c + 2] : L[4 * r + c];
                if (r == c) v = v + q[grp_global(g, r)];
                P[4 * r + c] = v;
            }
        grp_store(P, g, s, x);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) s.m[i] = s.m[i] + s.m[i + 4];
}

// botsort_kf.py:192-226 for a track carrying cross terms: S = H P H^T + R per group (2x2),
// Cholesky, K = P H^T S^-1, x += K innovation, P -= K (S K^T)
__host__ __device__ inline void kf_update_x(KfState &s, double *x, const double *z) {
    double r2[4], innov[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double r = KF_W_POS * kf_scale<KF_XYWH>(s.m, i);
        r2[i] = r * r;
        innov[i] = z[i] - s.m[i];
    }
    double dm[8];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        double P[16], K[8];
        grp_load(s, x, g, P);
        const double S00 = P[0] + r2[2 * g], S10 = P[4], S01 = P[1], S11 = P[5] + r2[2 * g + 1];
        const double l00 = sqrt(S00), i0 = 1.0 / l00;
        const double l10 = S10 * i0;
        const double l11 = sqrt(S11 - l10 * l10), i1 = 1.0 / l11;
#pragma unroll
        for (int r = 0; r < 4; ++r) {                  // row r of K: solve S k = (P_r0, P_r1)
            const double y0 = P[4 * r] * i0;
            const double y1 = (P[4 * r + 1] - l10 * y0) * i1;
            const double k1 = y1 * i1;
            const double k0 = (y0 - l10 * k1) * i0;
            K[2 * r] = k0;
            K[2 * r + 1] = k1;
        }
        const double e0 = innov[2 * g], e1 = innov[2 * g + 1];
#pragma unroll
        for (int r = 0; r < 4; ++r) dm[grp_global(g, r)] = e0 * K[2 * r] + e1 * K[2 * r + 1];
        double M[8];                                    // M = S K^T (2 x 4)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            M[c] = S00 * K[2 * c] + S01 * K[2 * c + 1];
            M[4 + c] = S10 * K[2 * c] + S11 * K[2 * c + 1];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) P[4 * r + c] = P[4 * r + c] - (K[2 * r] * M[c] + K[2 * r + 1] * M[4 + c]);
        grp_store(P, g, s, x);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s.m[i] = s.m[i] + dm[i];
}

__host__ __device__ __forceinline__ bool warp_is_identity(const double *H) {
    return H[0] == 1.0 && H[1] == 0.0 && H[2] == 0.0 && H[3] == 0.0 && H[4] == 1.0 && H[5] == 0.0;
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
