// Pieces shared by the OCSORT-family engines (ocsort.hip, deepocsort.hip): launch shape, the
// association cost functions (iou.py:6-212), the padded dense LAP call (association.py:20-28)
// and block reductions.
#pragma once
#include "geometry.hpp"
#include "lap.hpp"
#include "lap_dense.hpp"

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

}  // namespace yta
