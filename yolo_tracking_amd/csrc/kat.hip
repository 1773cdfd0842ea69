// Parity / known-answer entry points: the individual association and Kalman primitives on the
// device, synchronous, host buffers in and out.  The tracker engine uses the same device
// functions (geometry.hpp, kf_xyah.hpp, assoc.hip).
#include <vector>

#include "assoc.hpp"
#include "aw.hpp"
#include "grid.hpp"
#include "kf_deep.hpp"
#include "kf_xyah.hpp"
#include "lap_dense.hpp"
#include "lap_dense_block.hpp"
#include "lap_rect.hpp"

using namespace yta;

namespace {

__global__ void k_affinity(int kind, const Box *a, int na, const Box *b, int nb, double w,
                           double h, double *out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)na * nb) return;
    const int i = (int)(idx / nb), j = (int)(idx % nb);
    const Box &p = a[i], &q = b[j];
    double v;
    switch (kind) {
        case YTA_AFF_IOU: v = iou(p, q); break;
        case YTA_AFF_GIOU: v = giou(p, q); break;
        case YTA_AFF_DIOU: v = diou(p, q); break;
        case YTA_AFF_CIOU: v = ciou(p, q); break;
        default: v = centroid(p, q, w, h); break;
    }
    out[idx] = v;
}

__global__ void k_iou_distance(const Box *a, int na, const Box *b, int nb, const double *score,
                               double *out) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)na * nb) return;
    const int i = (int)(idx / nb), j = (int)(idx % nb);
    double d = 1 - iou(a[i], b[j]);
    if (score) d = 1 - (1 - d) * score[j];
    out[idx] = d;
}

__global__ void k_kf(int op, int n, const double *in_vec, double *mean, double *cov) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    KfState s;
    if (op == 0) {
        kf_initiate(in_vec + 4 * i, s);
    } else {
        for (int k = 0; k < 8; ++k) s.m[k] = mean[8 * i + k];
        kf_cov_pack(cov + 64 * i, s);   // the 2x2 blocks {j, j+4}; the rest is zero (kf_xyah.hpp)
        if (op == 1) kf_predict(s);
        else kf_update(s, in_vec + 4 * i);
    }
    for (int k = 0; k < 8; ++k) mean[8 * i + k] = s.m[k];
    kf_cov_full(s, cov + 64 * i);
}

// Dense cost matrix -> CSR of the entries below the limit -> lap_block (one block).  LDS arena
// first, the global one if the problem does not fit (the KAT suite exercises both).
__device__ __forceinline__ bool lap_dense_body(const double *cost, int nr, int nc, double thresh,
                                               int *X, int *Y, int *err, Arena &ar,
                                               const LapSlab &slab, LapShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x;
    int *row_off = ar.alloc_top<int>(nr + 1);
    int *col_deg = ar.alloc_top<int>(nc);
    if (ar.fail) return false;
    for (int j = t; j < nc; j += nt) col_deg[j] = 0;
    int run = 0;
    for (int start = 0; start < nr; start += nt) {
        const int i = start + t;
        int cnt = 0;
        if (i < nr)
            for (int j = 0; j < nc; ++j) cnt += cost[(long long)i * nc + j] < thresh;
        int tot;
        const int pos = block_exclusive_scan(cnt, sh.wsum, &tot);
        if (i < nr) row_off[i] = run + pos;
        run += tot;
    }
    if (t == 0) row_off[nr] = run;
    int *csr_col = ar.alloc_top<int>(run);
    double *csr_cost = ar.alloc_top<double>(run);
    if (ar.fail) return false;
    block_sync();
    for (int i = t; i < nr; i += nt) {
        int k = row_off[i];
        for (int j = 0; j < nc; ++j) {
            const double c = cost[(long long)i * nc + j];
            if (c < thresh) {
                csr_col[k] = j;
                csr_cost[k] = c;
                ++k;
                atomicAdd(&col_deg[j], 1);
            }
        }
    }
    block_sync();
    return lap_block(nr, nc, row_off, csr_col, csr_cost, col_deg, thresh, X, Y, err, ar, slab, sh);
}

__global__ __launch_bounds__(1024) void k_lap_dense(const double *cost, int nr, int nc,
                                                    double thresh, int *X, int *Y, int *err,
                                                    size_t lds_bytes, unsigned char *ws,
                                                    size_t ws_bytes, LapSlab slab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ LapShared sh;
    {
        Arena ar(smem, lds_bytes);
        if (lap_dense_body(cost, nr, nc, thresh, X, Y, err, ar, slab, sh)) return;
    }
    block_sync();
    Arena ag(ws, ws_bytes);
    if (!lap_dense_body(cost, nr, nc, thresh, X, Y, err, ag, slab, sh) && threadIdx.x == 0)
        atomicOr(err, ERR_EDGE_OVERFLOW);
}

// The padded dense solve of association.py:20-28 (lapjv(cost, extend_cost=True)) as the engines
// run it (padded_lap: one 512-thread block, phases 1-2 on wave 0, phase 3 block-wide for large n,
// work arrays placed within `lds_bytes` of LDS).
constexpr long long LAP_PADDED_LDS = 152 * 1024;   // the first-round kernels' LDS cap (LAP_LDS_MAX)
constexpr int LAP_PADDED_T = 512;
__global__ __launch_bounds__(LAP_PADDED_T) void k_lap_padded(const double *cost, int nr, int nc,
                                                             int *X, int *Y, int *err,
                                                             unsigned char *gws,
                                                             long long lds_bytes,
                                                             unsigned char *csr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int n = nr > nc ? nr : nc;
    const LapMat M{cost, nr, nc, false};
    DenseLapWs w;
    const int rc = lap_dense_block(n, M, smem, lds_bytes, gws, w, csr);
    if (rc && threadIdx.x == 0) atomicOr(err, ERR_SOLVER);
    for (int r = threadIdx.x; r < nr; r += blockDim.x) X[r] = w.x[r] < nc ? w.x[r] : -1;
    for (int k = threadIdx.x; k < nc; k += blockDim.x) Y[k] = w.y[k] < nr ? w.y[k] : -1;
}

// Rectangular solver KAT (lap_rect.hpp): rows <= cols solved as given with the chip-wide row
// pre-pass (k_lap_rect_pre, as the first-round association), rows > cols on the transposed view
// with the in-block pre-pass (as the -IoU rounds).  Work arrays in global memory.
__global__ __launch_bounds__(256) void k_lap_rect_pre(const double *cost, int nr, int nc, double *u,
                                                      int *x, double *s2) {
    if (nr > nc) return;
    const RectMat M{cost, nr, nc, nc, 1, false};
    const int nw = blockDim.x / WAVE;
    for (int i = blockIdx.x * nw + threadIdx.x / WAVE; i < nr; i += gridDim.x * nw)
        rect_row_pre(M, i, u, x, s2);
}
__global__ __launch_bounds__(256) void k_lap_rect(const double *cost, int nr, int nc,
                                                  const double *pu, const int *px,
                                                  const double *ps2, int *X, int *Y, int *err,
                                                  unsigned char *ws) {
    __shared__ RectShared sh;
    const bool tr = nr > nc;
    const RectMat R = tr ? RectMat{cost, nc, nr, 1, nc, false} : RectMat{cost, nr, nc, nc, 1, false};
    const RectWs w = rect_ws(ws, R.rows, R.cols);
    const int rc = tr ? lap_rect(R, nullptr, nullptr, nullptr, w, sh) : lap_rect(R, pu, px, ps2, w, sh);
    if (rc && threadIdx.x == 0) atomicOr(err, 1 << (-rc));
    block_sync();
    if (rc) return;
    for (int k = threadIdx.x; k < R.rows; k += blockDim.x) {
        const int c = w.x[k];
        if (!tr) { X[k] = c; Y[c] = k; }
        else { Y[k] = c; X[c] = k; }
    }
}

// One block: grid over b, then every a-box queries it; pairs with 1 - IoU < thresh are written
// (the shape of remove_duplicate_stracks, byte_tracker.py:312-325).
__global__ __launch_bounds__(1024) void k_grid_pairs(const Box *a, int na, const Box *b, int nb,
                                                    double thresh, GridHdr *hdr, int *cell,
                                                    int *ids, Box *boxes, int *big,
                                                    int *pairs, int *n_pairs, int cap) {
    __shared__ int wsum[32];
    __shared__ GridScratch gs;
    const GridView gv{hdr, cell, ids, boxes, nullptr, big};
    grid_build(nb, [&](int q) { return b[q]; }, [](int) { return 1.0; }, gv, gs, wsum);
    const GridHdr h = gs.hdr;
    for (int p = threadIdx.x; p < na; p += blockDim.x) {
        const Box T = a[p];
        auto pair = [&](int q, const Box &lb) {
            if (!intersects(T, lb)) return;
            if (1 - iou(T, lb) < thresh) {
                const int k = atomicAdd(n_pairs, 1);
                if (k < cap) { pairs[2 * k] = p; pairs[2 * k + 1] = q; }
            }
        };
        // thresh < 1: 1 - IoU < thresh needs IoU > 1 - thresh, the corner-window query the
        // duplicate removal uses; thresh >= 1: every intersecting pair (the association query)
        if (thresh < 1.0 && thresh > 0.0)
            grid_query_iou_above(gv, h, T, 1.0 - thresh,
                                 [&](int q, const Box &lb, double) { pair(q, lb); },
                                 [&](int q) { pair(q, b[q]); });
        else
            grid_query(gv, h, T, [&](int q, const Box &lb, double) { pair(q, lb); },
                       [&](int q) { pair(q, b[q]); });
    }
}

// Self-test of the block primitives (DPP scans / reductions) against serial answers.
__device__ __forceinline__ int st_val(int u, int trial) {
    return (int)(((unsigned)u * 2654435761u + (unsigned)trial * 40503u) >> 28) % 5 - (trial == 3);
}
__global__ __launch_bounds__(1024) void k_selftest(int *err) {
    __shared__ int wsum[32];
    __shared__ GridScratch gs;
    const int t = threadIdx.x, nt = blockDim.x;
    for (int trial = 0; trial < 6; ++trial) {
        const int v = st_val(t, trial);
        int tot;
        const int ex = block_exclusive_scan(v, wsum, &tot);
        int e = 0, all = 0, mn = 1 << 30, mx = -(1 << 30);
        for (int u = 0; u < nt; ++u) {
            const int vu = st_val(u, trial);
            if (u < t) e += vu;
            all += vu;
            mn = vu < mn ? vu : mn;
            mx = vu > mx ? vu : mx;
        }
        if (ex != e || tot != all) atomicOr(err, 1);
        double r[6] = {(double)v, (double)v, (double)v, (double)-v, (double)v, 1.0};
        const int ops[6] = {RED_MIN, RED_MAX, RED_SUM, RED_MIN, RED_SUM, RED_SUM};
        block_reduce6(r, ops, gs.red);
        if (r[0] != mn || r[1] != mx || r[2] != all || r[3] != -mx || r[4] != all || r[5] != nt)
            atomicOr(err, 2);
    }
}

// embedding_distance (matching.py:145-167): max(0, cdist(track f32, det f32, 'cosine')), one pair
// per 16-lane row group through the engine's own cosine_dist16 (assoc.hpp)
__global__ __launch_bounds__(256) void k_emb_dist(const float *tf, int n, const float *df, int m,
                                                  int D, double *out) {
    const long long pair = ((long long)blockIdx.x * 256 + threadIdx.x) >> 4;
    const long long np = (long long)n * m;
    const long long p = pair < np ? pair : np - 1;   // whole row groups stay for the DPP reduce
    const int i = (int)(p / m), j = (int)(p - (long long)i * m);
    const float *dv = df + (long long)j * D;
    const double cd = cosine_dist16(tf + (long long)i * D, [&](int k) { return dv[k]; }, D);
    if (pair < np && (threadIdx.x & 15) == 0) out[p] = cd > 0.0 ? cd : 0.0;
}

// compute_aw_max_metric (association.py:79-108): row and column weights from the top two values
// (the DeepOCSORT engine's top2_push / aw_weight, aw.hpp), then ((w * rw) * cw) * emb
__global__ void k_aw_weights(const double *e, int nr, int nc, double bottom, double *rw,
                             double *cw) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double m1 = -INFINITY, m2 = -INFINITY;
    if (t < nr) {
        for (int c = 0; c < nc; ++c) top2_push(e[(long long)t * nc + c], m1, m2);
        rw[t] = aw_weight(m1, m2, bottom, nc);
    } else if (t < nr + nc) {
        const int c = t - nr;
        for (int r = 0; r < nr; ++r) top2_push(e[(long long)r * nc + c], m1, m2);
        cw[c] = aw_weight(m1, m2, bottom, nr);
    }
}
__global__ void k_aw_apply(const double *e, int nr, int nc, double w, const double *rw,
                           const double *cw, double *out) {
    const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= (long long)nr * nc) return;
    const int r = (int)(q / nc), c = (int)(q - (long long)r * nc);
    out[q] = ((w * rw[r]) * cw[c]) * e[q];
}

// Camera-motion correction of n Kalman states (mean 8, full 8 x 8 covariance, in place), with the
// engines' own device functions: kind 0 = BoT-SORT STrack.multi_gmc (bot_sort.py:95-111, kf_gmc
// on the compact record + cross terms), kind 1 = DeepOCSORT's KF correction
// (deepocsort_kf.py:387-407, kf8_affine on the two 4x4 groups).  warps: n row-major 2x3.
__global__ void k_affine(int kind, int n, const double *warps, double *mean, double *cov) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *H = warps + 6LL * i;
    double *m = mean + 8LL * i, *P = cov + 64LL * i;
    if (kind == 0) {
        KfState s;
        double x[16];
        for (int k = 0; k < 8; ++k) s.m[k] = m[k];
        for (int a = 0; a < 4; ++a) {   // compact 2x2 blocks {a, a+4}: pp, pv, vp, vv
            s.c[4 * a + 0] = P[8 * a + a];
            s.c[4 * a + 1] = P[8 * a + a + 4];
            s.c[4 * a + 2] = P[8 * (a + 4) + a];
            s.c[4 * a + 3] = P[8 * (a + 4) + a + 4];
        }
        for (int g = 0; g < 2; ++g)
            for (int k = 0; k < 8; ++k) {
                int r, c;
                xcross(k, r, c);
                x[8 * g + k] = P[8 * grp_global(g, r) + grp_global(g, c)];
            }
        kf_gmc(s, x, H);
        for (int k = 0; k < 8; ++k) m[k] = s.m[k];
        for (int k = 0; k < 64; ++k) P[k] = 0.0;
        for (int g = 0; g < 2; ++g) {
            double B[16];
            grp_load(s, x, g, B);
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) P[8 * grp_global(g, r) + grp_global(g, c)] = B[4 * r + c];
        }
    } else {
        Kf8 s;
        for (int k = 0; k < 8; ++k) s.x[k] = m[k];
        for (int g = 0; g < 2; ++g)
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) s.p[g][4 * r + c] = P[8 * dk_glob(g, r) + dk_glob(g, c)];
        const double mm[4] = {H[0], H[1], H[3], H[4]}, t[2] = {H[2], H[5]};
        kf8_affine(s, mm, t);
        for (int k = 0; k < 8; ++k) m[k] = s.x[k];
        for (int k = 0; k < 64; ++k) P[k] = 0.0;
        for (int g = 0; g < 2; ++g)
            for (int r = 0; r < 4; ++r)
                for (int c = 0; c < 4; ++c) P[8 * dk_glob(g, r) + dk_glob(g, c)] = s.p[g][4 * r + c];
    }
}

struct DevBuf {
    std::vector<void *> ptrs;
    ~DevBuf() {
        for (void *p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    hipError_t get(T **p, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, sizeof(T) * (n ? n : 1));
        if (e == hipSuccess) ptrs.push_back(q);
        *p = (T *)q;
        return e;
    }
};

}  // namespace

extern "C" {

int yta_box_affinity(int device, int kind, const double *a, int na, const double *b, int nb,
                     double img_w, double img_h, double *out) {
    YTA_CHECK(kind >= 0 && kind <= 4, YTA_ERR_INVALID, "unknown affinity kind %d", kind);
    YTA_CHECK(na >= 0 && nb >= 0, YTA_ERR_INVALID, "negative size");
    if ((long long)na * nb == 0) return YTA_OK;
    YTA_CHECK(a && b && out, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    Box *da, *db;
    double *dout;
    const long long n = (long long)na * nb;
    YTA_HIP(m.get(&da, na));
    YTA_HIP(m.get(&db, nb));
    YTA_HIP(m.get(&dout, n));
    YTA_HIP(hipMemcpy(da, a, sizeof(Box) * na, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(db, b, sizeof(Box) * nb, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_affinity, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, kind, da, na,
                       db, nb, img_w, img_h, dout);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost));
    if (kind == YTA_AFF_GIOU) {
        // iou.py:58 asserts a positive enclosure; NaN marks the violation
        for (long long k = 0; k < n; ++k)
            YTA_CHECK(out[k] == out[k], YTA_ERR_INVALID, "giou: degenerate enclosing box");
    }
    return YTA_OK;
}

int yta_iou_distance(int device, const double *a, int na, const double *b, int nb,
                     const double *scores, double *out) {
    YTA_CHECK(na >= 0 && nb >= 0, YTA_ERR_INVALID, "negative size");
    if ((long long)na * nb == 0) return YTA_OK;
    YTA_CHECK(a && b && out, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    Box *da, *db;
    double *dout, *ds = nullptr;
    const long long n = (long long)na * nb;
    YTA_HIP(m.get(&da, na));
    YTA_HIP(m.get(&db, nb));
    YTA_HIP(m.get(&dout, n));
    YTA_HIP(hipMemcpy(da, a, sizeof(Box) * na, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(db, b, sizeof(Box) * nb, hipMemcpyHostToDevice));
    if (scores) {
        YTA_HIP(m.get(&ds, nb));
        YTA_HIP(hipMemcpy(ds, scores, sizeof(double) * nb, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(k_iou_distance, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, da, na,
                       db, nb, ds, dout);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost));
    return YTA_OK;
}

static int kf_call(int device, int op, int n, const double *vec, double *mean, double *cov) {
    YTA_CHECK(n >= 0, YTA_ERR_INVALID, "negative n");
    if (n == 0) return YTA_OK;
    YTA_CHECK(mean && cov && (op == 1 || vec), YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    double *dv = nullptr, *dm, *dc;
    YTA_HIP(m.get(&dm, 8 * (size_t)n));
    YTA_HIP(m.get(&dc, 64 * (size_t)n));
    if (op != 1) {
        YTA_HIP(m.get(&dv, 4 * (size_t)n));
        YTA_HIP(hipMemcpy(dv, vec, sizeof(double) * 4 * n, hipMemcpyHostToDevice));
    }
    if (op != 0) {
        YTA_HIP(hipMemcpy(dm, mean, sizeof(double) * 8 * n, hipMemcpyHostToDevice));
        YTA_HIP(hipMemcpy(dc, cov, sizeof(double) * 64 * n, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(k_kf, dim3((n + 127) / 128), dim3(128), 0, 0, op, n, dv, dm, dc);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(mean, dm, sizeof(double) * 8 * n, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(cov, dc, sizeof(double) * 64 * n, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_affine_apply(int device, int kind, int n, const double *warps, double *mean,
                     double *cov) {
    YTA_CHECK(kind == 0 || kind == 1, YTA_ERR_INVALID, "kind %d: 0 (BoT-SORT multi_gmc) or 1 "
              "(DeepOCSORT)", kind);
    YTA_CHECK(n >= 0, YTA_ERR_INVALID, "negative n");
    if (n == 0) return YTA_OK;
    YTA_CHECK(warps && mean && cov, YTA_ERR_INVALID, "null buffer");
    // the engines keep P block-diagonal over {x, y, x', y'} and {w, h, w', h'} (kf_xyah.hpp,
    // kf_deep.hpp): a covariance coupling the two groups is not a state they can hold
    for (long long q = 0; q < n; ++q)
        for (int r = 0; r < 8; ++r)
            for (int c = 0; c < 8; ++c)
                YTA_CHECK(((r >> 1) & 1) == ((c >> 1) & 1) || cov[64 * q + 8 * r + c] == 0.0,
                          YTA_ERR_INVALID, "track %lld: covariance couples (x, y) with (w, h)", q);
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    double *dw, *dm, *dc;
    YTA_HIP(m.get(&dw, 6 * (size_t)n));
    YTA_HIP(m.get(&dm, 8 * (size_t)n));
    YTA_HIP(m.get(&dc, 64 * (size_t)n));
    YTA_HIP(hipMemcpy(dw, warps, sizeof(double) * 6 * n, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(dm, mean, sizeof(double) * 8 * n, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(dc, cov, sizeof(double) * 64 * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_affine, dim3((n + 63) / 64), dim3(64), 0, 0, kind, n, dw, dm, dc);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(mean, dm, sizeof(double) * 8 * n, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(cov, dc, sizeof(double) * 64 * n, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_kf_xyah_initiate(int device, int n, const double *meas, double *mean, double *cov) {
    return kf_call(device, 0, n, meas, mean, cov);
}
int yta_kf_xyah_predict(int device, int n, double *mean, double *cov) {
    return kf_call(device, 1, n, nullptr, mean, cov);
}
int yta_kf_xyah_update(int device, int n, double *mean, double *cov, const double *z) {
    return kf_call(device, 2, n, z, mean, cov);
}

int yta_grid_pairs(int device, const double *a, int na, const double *b, int nb, double thresh,
                   int *pairs, int cap, int *n_pairs) {
    YTA_CHECK(na >= 0 && nb >= 0 && cap >= 0 && n_pairs, YTA_ERR_INVALID, "bad argument");
    *n_pairs = 0;
    if (na == 0 || nb == 0) return YTA_OK;
    YTA_CHECK(a && b && (cap == 0 || pairs), YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    Box *da, *db, *boxes;
    GridHdr *hdr;
    int *cell, *ids, *big, *dp, *dn;
    YTA_HIP(m.get(&da, na));
    YTA_HIP(m.get(&db, nb));
    YTA_HIP(m.get(&hdr, 1));
    YTA_HIP(m.get(&cell, GRID_MAX_CELLS + 1));
    YTA_HIP(m.get(&ids, nb));
    YTA_HIP(m.get(&boxes, nb));
    YTA_HIP(m.get(&big, nb));
    YTA_HIP(m.get(&dp, 2 * (size_t)(cap > 0 ? cap : 1)));
    YTA_HIP(m.get(&dn, 1));
    YTA_HIP(hipMemcpy(da, a, sizeof(Box) * na, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(db, b, sizeof(Box) * nb, hipMemcpyHostToDevice));
    YTA_HIP(hipMemset(dn, 0, sizeof(int)));
    hipLaunchKernelGGL(k_grid_pairs, dim3(1), dim3(1024), 0, 0, da, na, db, nb, thresh, hdr, cell,
                       ids, boxes, big, dp, dn, cap);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(n_pairs, dn, sizeof(int), hipMemcpyDeviceToHost));
    const int n = *n_pairs < cap ? *n_pairs : cap;
    if (n) YTA_HIP(hipMemcpy(pairs, dp, sizeof(int) * 2 * n, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_selftest(int device) {
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    int *derr;
    YTA_HIP(m.get(&derr, 1));
    YTA_HIP(hipMemset(derr, 0, sizeof(int)));
    for (int threads : {64, 128, 256, 512, 960, 1024})
        hipLaunchKernelGGL(k_selftest, dim3(1), dim3(threads), 0, 0, derr);
    YTA_HIP(hipGetLastError());
    int herr = 0;
    YTA_HIP(hipMemcpy(&herr, derr, sizeof(int), hipMemcpyDeviceToHost));
    YTA_CHECK(herr == 0, YTA_ERR_HIP, "block primitive self-test failed (flags 0x%x)", herr);
    return YTA_OK;
}

int yta_lap_limited(int device, int nr, int nc, const double *cost, double cost_limit, int *x,
                    int *y) {
    YTA_CHECK(nr >= 0 && nc >= 0, YTA_ERR_INVALID, "negative size");
    YTA_CHECK(cost_limit == cost_limit, YTA_ERR_INVALID, "cost_limit is NaN");
    YTA_CHECK((nr == 0 || x) && (nc == 0 || y), YTA_ERR_INVALID, "null buffer");
    for (int i = 0; i < nr; ++i) x[i] = -1;
    for (int j = 0; j < nc; ++j) y[j] = -1;
    if ((long long)nr * nc == 0) return YTA_OK;
    YTA_CHECK(cost, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    const long long n = (long long)nr * nc;
    constexpr int THREADS = 1024, WAVES = THREADS / WAVE;
    constexpr size_t LDS = 64 * 1024;
    double *dcost;
    int *dx, *dy, *derr;
    unsigned char *ws;
    LapSlab slab;
    const size_t ws_bytes = (size_t)(((4LL * (nr + 1) + 4LL * nc + 12 * n) +
                                      4LL * 8 * (nr + nc + 1) + 64 * 16 + 255) & ~255LL);
    slab.R = nr;
    slab.C = nc;
    slab.i_stride = lap_slab_ints(nr, nc);
    slab.d_stride = lap_slab_doubles(nr, nc);
    YTA_HIP(m.get(&dcost, n));
    YTA_HIP(m.get(&dx, nr));
    YTA_HIP(m.get(&dy, nc));
    YTA_HIP(m.get(&derr, 1));
    YTA_HIP(m.get(&ws, ws_bytes));
    YTA_HIP(m.get(&slab.i, WAVES * slab.i_stride));
    YTA_HIP(m.get(&slab.d, WAVES * slab.d_stride));
    YTA_HIP(hipMemset(derr, 0, sizeof(int)));
    YTA_HIP(hipMemcpy(dcost, cost, sizeof(double) * n, hipMemcpyHostToDevice));
    YTA_HIP(hipFuncSetAttribute((const void *)k_lap_dense,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS));
    hipLaunchKernelGGL(k_lap_dense, dim3(1), dim3(THREADS), LDS, 0, dcost, nr, nc, cost_limit, dx,
                       dy, derr, LDS, ws, ws_bytes, slab);
    YTA_HIP(hipGetLastError());
    int herr = 0;
    YTA_HIP(hipMemcpy(x, dx, sizeof(int) * nr, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(y, dy, sizeof(int) * nc, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(&herr, derr, sizeof(int), hipMemcpyDeviceToHost));
    YTA_CHECK(herr == 0, YTA_ERR_HIP, "assignment solver error flags 0x%x", herr);
    return YTA_OK;
}

int yta_lap_padded(int device, int nr, int nc, const double *cost, int *x, int *y) {
    YTA_CHECK(nr >= 0 && nc >= 0, YTA_ERR_INVALID, "negative size");
    YTA_CHECK((nr == 0 || x) && (nc == 0 || y), YTA_ERR_INVALID, "null buffer");
    for (int i = 0; i < nr; ++i) x[i] = -1;
    for (int j = 0; j < nc; ++j) y[j] = -1;
    if (nr == 0 && nc == 0) return YTA_OK;
    YTA_CHECK((long long)nr * nc == 0 || cost, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    const long long n = nr > nc ? nr : nc;
    double *dcost = nullptr;
    int *dx, *dy, *derr;
    unsigned char *gws;
    const size_t ws = (size_t)dense_lap_ws_bytes(n);
    if ((long long)nr * nc) YTA_HIP(m.get(&dcost, (long long)nr * nc));
    YTA_HIP(m.get(&dx, nr > 0 ? nr : 1));
    YTA_HIP(m.get(&dy, nc > 0 ? nc : 1));
    YTA_HIP(m.get(&derr, 1));
    YTA_HIP(m.get(&gws, ws));
    unsigned char *csr = nullptr;   // the sparse sweeps' row entries (lap_dense_block.hpp)
    if (n >= LAPB_MIN_N && lap_sparse_on()) YTA_HIP(m.get(&csr, (size_t)lap_csr_bytes(n)));
    YTA_HIP(hipMemset(derr, 0, sizeof(int)));
    if (dcost)
        YTA_HIP(hipMemcpy(dcost, cost, sizeof(double) * nr * nc, hipMemcpyHostToDevice));
    const long long lds = dense_lap_ws_bytes(n) <= LAP_PADDED_LDS ? dense_lap_ws_bytes(n)
                          : dense_lap_ws_bytes_norow(n) <= LAP_PADDED_LDS ? dense_lap_ws_bytes_norow(n)
                                                                           : 0;
    YTA_HIP(hipFuncSetAttribute((const void *)k_lap_padded,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)LAP_PADDED_LDS));
    hipLaunchKernelGGL(k_lap_padded, dim3(1), dim3(LAP_PADDED_T), (size_t)lds, 0, dcost, nr, nc, dx,
                       dy, derr, gws, lds, csr);
    YTA_HIP(hipGetLastError());
    int herr = 0;
    if (nr) YTA_HIP(hipMemcpy(x, dx, sizeof(int) * nr, hipMemcpyDeviceToHost));
    if (nc) YTA_HIP(hipMemcpy(y, dy, sizeof(int) * nc, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(&herr, derr, sizeof(int), hipMemcpyDeviceToHost));
    YTA_CHECK(herr == 0, YTA_ERR_HIP, "padded assignment solver error flags 0x%x", herr);
    return YTA_OK;
}

int yta_lap_rect(int device, int nr, int nc, const double *cost, int *x, int *y) {
    YTA_CHECK(nr >= 0 && nc >= 0, YTA_ERR_INVALID, "negative size");
    YTA_CHECK((nr == 0 || x) && (nc == 0 || y), YTA_ERR_INVALID, "null buffer");
    for (int i = 0; i < nr; ++i) x[i] = -1;
    for (int j = 0; j < nc; ++j) y[j] = -1;
    if (nr == 0 || nc == 0) return YTA_OK;
    YTA_CHECK(cost, YTA_ERR_INVALID, "null buffer");
    const int rows = nr < nc ? nr : nc, cols = nr < nc ? nc : nr;
    YTA_CHECK(cols <= RECT_CPT_MAX * 256, YTA_ERR_INVALID, "more than %d columns", RECT_CPT_MAX * 256);
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf m;
    double *dcost, *pu, *ps2;
    int *dx, *dy, *derr, *px;
    unsigned char *ws;
    YTA_HIP(m.get(&dcost, (long long)nr * nc));
    YTA_HIP(m.get(&dx, nr));
    YTA_HIP(m.get(&dy, nc));
    YTA_HIP(m.get(&derr, 1));
    YTA_HIP(m.get(&pu, nr));
    YTA_HIP(m.get(&ps2, nr));
    YTA_HIP(m.get(&px, nr));
    YTA_HIP(m.get(&ws, (size_t)rect_ws_bytes(rows, cols)));
    YTA_HIP(hipMemset(derr, 0, sizeof(int)));
    YTA_HIP(hipMemset(dx, 0xFF, sizeof(int) * nr));
    YTA_HIP(hipMemset(dy, 0xFF, sizeof(int) * nc));
    YTA_HIP(hipMemcpy(dcost, cost, sizeof(double) * nr * nc, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_lap_rect_pre, dim3((unsigned)std::min(1024, (nr + 3) / 4)), dim3(256), 0, 0,
                       dcost, nr, nc, pu, px, ps2);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_lap_rect, dim3(1), dim3(256), 0, 0, dcost, nr, nc, pu, px, ps2, dx, dy,
                       derr, ws);
    YTA_HIP(hipGetLastError());
    int herr = 0;
    YTA_HIP(hipMemcpy(x, dx, sizeof(int) * nr, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(y, dy, sizeof(int) * nc, hipMemcpyDeviceToHost));
    YTA_HIP(hipMemcpy(&herr, derr, sizeof(int), hipMemcpyDeviceToHost));
    YTA_CHECK(herr == 0, YTA_ERR_HIP, "rectangular assignment solver error flags 0x%x", herr);
    return YTA_OK;
}

int yta_embedding_distance(int device, const float *track_feats, int n, const float *det_feats,
                           int m, int dim, double *out) {
    YTA_CHECK(n >= 0 && m >= 0 && dim > 0, YTA_ERR_INVALID, "bad sizes (%d, %d, %d)", n, m, dim);
    if ((long long)n * m == 0) return YTA_OK;
    YTA_CHECK(track_feats && det_feats && out, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf mb;
    float *dt, *dd;
    double *dout;
    const long long np = (long long)n * m;
    YTA_HIP(mb.get(&dt, (size_t)n * dim));
    YTA_HIP(mb.get(&dd, (size_t)m * dim));
    YTA_HIP(mb.get(&dout, np));
    YTA_HIP(hipMemcpy(dt, track_feats, sizeof(float) * n * dim, hipMemcpyHostToDevice));
    YTA_HIP(hipMemcpy(dd, det_feats, sizeof(float) * m * dim, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_emb_dist, dim3((unsigned)((np * 16 + 255) / 256)), dim3(256), 0, 0, dt, n,
                       dd, m, dim, dout);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(out, dout, sizeof(double) * np, hipMemcpyDeviceToHost));
    return YTA_OK;
}

int yta_aw_max_metric(int device, const double *emb_cost, int nr, int nc, double w_association_emb,
                      double bottom, double *out) {
    YTA_CHECK(nr >= 0 && nc >= 0, YTA_ERR_INVALID, "negative size");
    const long long q = (long long)nr * nc;
    if (q == 0) return YTA_OK;
    YTA_CHECK(emb_cost && out, YTA_ERR_INVALID, "null buffer");
    int rc = select_device(device);
    if (rc) return rc;
    DevBuf mb;
    double *de, *drw, *dcw, *dout;
    YTA_HIP(mb.get(&de, q));
    YTA_HIP(mb.get(&drw, nr));
    YTA_HIP(mb.get(&dcw, nc));
    YTA_HIP(mb.get(&dout, q));
    YTA_HIP(hipMemcpy(de, emb_cost, sizeof(double) * q, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_aw_weights, dim3((nr + nc + 255) / 256), dim3(256), 0, 0, de, nr, nc,
                       bottom, drw, dcw);
    YTA_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_aw_apply, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, 0, de, nr, nc,
                       w_association_emb, drw, dcw, dout);
    YTA_HIP(hipGetLastError());
    YTA_HIP(hipMemcpy(out, dout, sizeof(double) * q, hipMemcpyDeviceToHost));
    return YTA_OK;
}

}  // extern "C"

#ifdef YTA_STAMPS
// diagnostic build only: this file's stamps (the KATs' solver phases)
extern "C" int yta_kat_debug_stamps(unsigned long long *out) {
    YTA_HIP(hipDeviceSynchronize());
    YTA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), 128 * sizeof(unsigned long long)));
    return YTA_OK;
}
#endif
