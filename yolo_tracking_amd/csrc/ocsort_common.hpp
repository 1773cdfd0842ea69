// Pieces shared by the OCSORT-family engines (ocsort.hip, deepocsort.hip): launch shape, the
// association cost functions (iou.py:6-212), the padded dense LAP call (association.py:20-28)
// and block reductions.
#pragma once
#include "geometry.hpp"
#include "lap.hpp"
#include "lap_dense.hpp"
#include "lap_rect.hpp"

namespace yta {

constexpr int OC_T = 256;          // threads per stream block
constexpr int OC_DT_MAX = 8;       // delta_t capacity of the observation ring
constexpr int OC_LDS_LAP_N = 1536; // dense LAP work arrays in LDS up to this n

constexpr int OF_OBSERVED = 1;     // KalmanFilter.observed
constexpr int OF_SAVED = 2;        // KalmanFilter.attr_saved is not None
constexpr int OF_VELOCITY = 4;     // velocity is not None
constexpr int ERR_GIOU = 32;       // giou enclosure assert (iou.py:58)

__device__ __forceinline__ double asso_of(int kind, const Box &d, const Box &t, double w, double h) {
    switch (kind) {
        case 0: return iou(d, t);
        case 1: return giou(d, t);
        case 2: return diou(d, t);
        case 3: return ciou(d, t);
        default: return centroid(d, t, w, h);
    }
}

__device__ __forceinline__ Box box5(const double *b) { return Box{b[0], b[1], b[2], b[3]}; }

struct OcShared {
    int wsum[32];
    int cnt[8];
    double red[OC_T / WAVE];
};

// Block max of v (wave reductions, then wave 0).
__device__ __forceinline__ double block_max(double v, OcShared &sh) {
    v = wave_reduce(RED_MAX, v);
    if (lane_id() == 0) sh.red[threadIdx.x / WAVE] = v;
    block_sync();
    double m = -INFINITY;
    for (int w = 0; w < (int)blockDim.x / WAVE; ++w) m = fmax(m, sh.red[w]);
    block_sync();
    return m;
}

// association.py:20-28 on the padded problem M: wave 0 solves, x[r] = column or -1 -> rx.
// The solver is one dependent chain of row reads; the matrix was written by k_oc_cost on every
// XCD, so the whole block first streams it once (coalesced) into this XCD's L2.
__device__ __forceinline__ void padded_lap(const LapMat &M, int *rx, unsigned char *lds,
                                           unsigned char *gws, int *err) {
    const int n = M.na > M.nb ? M.na : M.nb;
    {
        const long long cnt = (long long)M.na * M.nb;
        double acc = 0.0;
        for (long long q = threadIdx.x; q < cnt; q += blockDim.x) acc += M.m[q];
        if (acc == 1.2345e300) rx[0] = -7;   // keeps the loads; never true for cost matrices
        block_sync();
    }
    if (threadIdx.x < WAVE && n > 0) {
        const DenseLapWs w = dense_lap_ws(n <= OC_LDS_LAP_N ? lds : gws, n);
        const int rc = n <= OC_LDS_LAP_N ? lap_dense_wave<true>(n, M, w) : lap_dense_wave<false>(n, M, w);
        if (rc && lane_id() == 0) atomicOr(err, ERR_SOLVER);
        for (int r = lane_id(); r < M.na; r += WAVE) rx[r] = w.x[r] < M.nb ? w.x[r] : -1;
    }
    block_sync();
}

// Dynamic LDS of the association kernels (host launch size and device-side view of it).
__host__ __device__ inline long long oc_lds_bytes(long long CAP, long long MAXD) {
    const long long n = CAP > MAXD ? CAP : MAXD;
    return dense_lap_ws_bytes(n < OC_LDS_LAP_N ? n : OC_LDS_LAP_N);
}

// Rectangular solve (lap_rect.hpp) of R; `tr`: R is the transposed view of an na-row problem, so
// the solver's rows are the caller's columns.  rx[caller row] = caller column or -1.
__device__ __forceinline__ void rect_solve(const RectMat &R, const double *pu, const int *px,
                                           const double *ps2, bool tr, int na, int *rx,
                                           unsigned char *lds, long long lds_bytes,
                                           unsigned char *gws, int *err) {
    __shared__ RectShared rsh;
    const int t = threadIdx.x, nt = blockDim.x;
    unsigned char *base = rect_ws_bytes(R.rows, R.cols) <= lds_bytes ? lds : gws;
    const RectWs w = rect_ws(base, R.rows, R.cols);
    const int rc = lap_rect(R, pu, px, ps2, w, rsh);
    if (rc && t == 0) atomicOr(err, ERR_SOLVER);
    if (!tr) {
        for (int i = t; i < R.rows; i += nt) rx[i] = rc ? -1 : w.x[i];
    } else {
        for (int i = t; i < na; i += nt) rx[i] = -1;
        block_sync();
        if (!rc)
            for (int k = t; k < R.rows; k += nt) rx[w.x[k]] = k;
    }
    block_sync();
}

// First-round solve of association.py:20-28 on the padded problem M (rows = detections, columns =
// trackers).  With trackers >= detections every detection row is matched and the result does not
// depend on lapjv's tie-breaking: the rectangular solver, warm-started by the
// chip-wide row pre-pass (pu / px / ps2, main_lap_pre).  Otherwise the lapjv replay.
__device__ __forceinline__ void main_lap(const LapMat &M, const double *pu, const int *px,
                                         const double *ps2, int *rx, unsigned char *lds,
                                         long long lds_bytes, unsigned char *gws, int *err) {
    if (M.na <= M.nb && M.nb <= RECT_CPT_MAX * (int)blockDim.x)
        rect_solve(RectMat{M.m, M.na, M.nb, M.nb, 1, M.neg}, pu, px, ps2, false, M.na, rx, lds,
                   lds_bytes, gws, err);
    else
        padded_lap(M, rx, lds, gws, err);
}

// Row pre-pass of main_lap for one stream, spread over the blocks of a chip-wide launch.
__device__ __forceinline__ void main_lap_pre(const double *mat, int na, int nb, double *u, int *x,
                                             double *s2) {
    if (na <= 0 || na > nb || nb > RECT_CPT_MAX * OC_T) return;
    const RectMat M{mat, na, nb, nb, 1, false};
    const int nw = blockDim.x / WAVE;
    for (int i = blockIdx.x * nw + threadIdx.x / WAVE; i < na; i += gridDim.x * nw)
        rect_row_pre(M, i, u, x, s2);
}

// The -IoU rounds (BYTE / OCR: association.py:20-28 on -iou): only pairs with IoU >= threshold
// survive and the leftover lists are re-sorted (np.setdiff1d), so any optimal solution gives the
// reference's result: the rectangular solver in whichever orientation has rows <= columns.
__device__ __forceinline__ void iou_lap(const LapMat &M, int *rx, unsigned char *lds,
                                        long long lds_bytes, unsigned char *gws, int *err) {
    const bool tr = M.na > M.nb;
    const int rows = tr ? M.nb : M.na, cols = tr ? M.na : M.nb;
    if (cols > RECT_CPT_MAX * (int)blockDim.x) {
        padded_lap(M, rx, lds, gws, err);
        return;
    }
    const RectMat R = tr ? RectMat{M.m, rows, cols, 1, M.nb, M.neg}
                         : RectMat{M.m, rows, cols, M.nb, 1, M.neg};
    rect_solve(R, nullptr, nullptr, nullptr, tr, M.na, rx, lds, lds_bytes, gws, err);
}

#ifndef YTA_LAP_T
#define YTA_LAP_T 512
#endif
constexpr int LAP_T = YTA_LAP_T;                // threads of the first-round solve kernels
constexpr long long LAP_LDS_MAX = 156 * 1024;   // their dynamic LDS cap (160 KiB - static)

__host__ __device__ inline long long lap_kernel_lds(long long CAP, long long MAXD) {
    const long long b = rect_ws_bytes(MAXD, CAP);
    return b < LAP_LDS_MAX ? b : LAP_LDS_MAX;
}

// First-round solve in its own launch, one LAP_T-thread block per stream (up to 16 columns per
// thread: 8192 trackers, every cost load of a step in flight at once).  When trackers >= detections and
// the fast path (association.py:156-159, `fast_rule`) does not apply, solve with lap_rect
// (warm-started by the row pre-pass) into rx and set *done; the association kernel then skips its
// own first-round solve.  rcnt / ccnt: the per-row / per-column counts of asso > thr (rcnt may
// alias rx: it is read before the solve).
__device__ __forceinline__ void first_round_lap(const double *mat, int na, int nb, const int *rcnt,
                                                const int *ccnt, bool fast_rule, const double *pu,
                                                const int *px, const double *ps2, int *rx,
                                                unsigned char *lds, long long lds_bytes,
                                                unsigned char *gws, int *err, int *done) {
    __shared__ RectShared rsh;
    __shared__ int flags[2];
    const int t = threadIdx.x, nt = blockDim.x;
    bool solve = na > 0 && na <= nb && nb <= 16 * nt;
    if (solve && fast_rule) {
        if (t < 2) flags[t] = 0;
        __syncthreads();
        int over = 0, bad = 0;
        for (int i = t; i < na; i += nt) {
            const int k = rcnt[i];
            over |= k;
            bad |= k > 1;
        }
        for (int j = t; j < nb; j += nt) bad |= ccnt[j] > 1;
        if (over) atomicOr(&flags[0], 1);
        if (bad) atomicOr(&flags[1], 1);
        __syncthreads();
        if (flags[1] == 0 && flags[0]) solve = false;   // the fast path
    }
    if (!solve) {
        if (t == 0) *done = 0;
        return;
    }
    unsigned char *base = rect_ws_bytes(na, nb) <= lds_bytes ? lds : gws;
    const RectWs w = rect_ws(base, na, nb);
    const int rc = lap_rect<LAP_T>(RectMat{mat, na, nb, nb, 1, false}, pu, px, ps2, w, rsh);
    if (rc && t == 0) atomicOr(err, ERR_SOLVER);
    for (int i = t; i < na; i += nt) rx[i] = rc ? -1 : w.x[i];
    if (t == 0) *done = 1;
}

}  // namespace yta
