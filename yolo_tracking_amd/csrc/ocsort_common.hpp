// Pieces shared by the OCSORT-family engines (ocsort.hip, deepocsort.hip): launch shape, the
// association cost functions (iou.py:6-212), the padded dense LAP call (association.py:20-28)
// and block reductions.
#pragma once
#include "geometry.hpp"
#include "lap.hpp"
#include "lap_dense.hpp"
#include "lap_dense_block.hpp"
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

// Solver counters of a stream, cumulative over frames (yta_*_lap_stats): first-round solves of the
// transposed problem (more detections than trackers), those whose optimum was not certified
// unique, and lapjv replays (padded_lap, any round).
struct LapStats {
    int transposed, uncertified, replays;
    int reduced;   // -IoU rounds solved on their positive part (iou_lap_reduced)
};

// association.py:20-28 on the padded problem M: wave 0 solves, x[r] = column or -1 -> rx.
// The solver is one dependent chain of row reads; the matrix was written by k_oc_cost on every
// XCD, so the whole block first streams it once (coalesced) into this XCD's L2.
// Work arrays: all in LDS when they fit `lds_bytes`; else the arrays in LDS and the two row buffers
// in `gws` when those fit (n <= ~3900 in the 156 KiB of the first-round kernels); else all in gws.
__device__ __forceinline__ void padded_lap(const LapMat &M, int *rx, unsigned char *lds,
                                           long long lds_bytes, unsigned char *gws, int *err,
                                           LapStats *ls, unsigned char *csr = nullptr) {
    const int n = M.na > M.nb ? M.na : M.nb;
    if (threadIdx.x == 0 && n > 0) ls->replays += 1;
    {
        const long long cnt = (long long)M.na * M.nb;
        double acc = 0.0;
        for (long long q = threadIdx.x; q < cnt; q += blockDim.x) acc += M.m[q];
        if (acc == 1.2345e300) rx[0] = -7;   // keeps the loads; never true for cost matrices
        block_sync();
    }
    if (n > 0) {   // the whole block (phase 3 block-wide for large n, lap_dense_block.hpp)
        DenseLapWs w;
        const int rc = lap_dense_block(n, M, lds, lds_bytes, gws, w, csr);
        if (rc && threadIdx.x == 0) atomicOr(err, ERR_SOLVER);
        for (int r = threadIdx.x; r < M.na; r += blockDim.x) rx[r] = w.x[r] < M.nb ? w.x[r] : -1;
    }
    block_sync();
}

#ifndef YTA_LAP_T
#define YTA_LAP_T 512
#endif
constexpr int LAP_T = YTA_LAP_T;                // threads of the first-round solve kernels
constexpr long long LAP_LDS_MAX = 152 * 1024;   // their dynamic LDS cap (160 KiB - static)

// Per-stream solver workspace (engines' lap_ws): the lapjv replay's arrays when they exceed LDS,
// the bidding rounds' arrays (lap_rect.hpp rect_arr), the uniqueness certificate's edges (tws at
// the end).  n = max(CAP, MAXD).
#ifndef YTA_LAP_ARR
#define YTA_LAP_ARR 1
#endif
__host__ __device__ inline long long arr_ws_region(long long n) {   // in-block or chip-wide rounds
    const long long a = arr_ws_bytes(n, n), b = arr_state_bytes(n, n);
    return ((a > b ? a : b) + 255) & ~255LL;
}

// The first-round solve's work arrays, either orientation (first_round_lap transposes the
// problem when detections outnumber trackers).
__host__ __device__ inline long long lap_kernel_lds(long long CAP, long long MAXD) {
    const long long b1 = rect_ws_bytes(MAXD, CAP) + 8 * CAP + 16,   // + the rounds' duals
                    b2 = rect_ws_bytes(CAP, MAXD, true);
    const long long b = b1 > b2 ? b1 : b2;
    return b < LAP_LDS_MAX ? b : LAP_LDS_MAX;
}

// Dynamic LDS of the association kernels (host launch size and device-side view of it).
__host__ __device__ inline long long oc_lds_bytes(long long CAP, long long MAXD) {
    const long long n = CAP > MAXD ? CAP : MAXD;
    return dense_lap_ws_bytes(n < OC_LDS_LAP_N ? n : OC_LDS_LAP_N);
}

// Rectangular solve (lap_rect.hpp) of R; `tr`: R is the transposed view of an na-row problem, so
// the solver's rows are the caller's columns.  rx[caller row] = caller column or -1.
template <int MAXT = 256>
__device__ __forceinline__ void rect_solve(const RectMat &R, const double *pu, const int *px,
                                           const double *ps2, bool tr, int na, int *rx,
                                           unsigned char *lds, long long lds_bytes,
                                           unsigned char *gws, int *err,
                                           unsigned char *tws = nullptr) {
    __shared__ RectShared rsh;
    const int t = threadIdx.x, nt = blockDim.x;
    unsigned char *base = rect_ws_bytes(R.rows, R.cols) <= lds_bytes ? lds : gws;
    RectWs w = rect_ws(base, R.rows, R.cols);
    if (YTA_LAP_ARR && tws) {   // bidding rounds (lap_rect.hpp rect_arr): arrays just below tws
        rect_arr_ws(tws - arr_ws_region(R.rows > R.cols ? R.rows : R.cols), R.rows, R.cols, w);
        const long long wo = (rect_ws_bytes(R.rows, R.cols) + 15) & ~15LL;
        if (base == lds && wo + 8LL * R.cols <= lds_bytes) {
            w.av = reinterpret_cast<double *>(lds + wo);
            w.av_lds = 1;
        }
    }
    const int rc = lap_rect<MAXT>(R, pu, px, ps2, w, rsh);
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
// trackers) when k_*_lap left it (more than 16384 trackers): the rectangular solver with
// trackers >= detections, otherwise the lapjv replay.
// csr: the engine's lap_csr region of the stream (lap_dense_block.hpp sparse sweeps) or nullptr.
__device__ __forceinline__ void main_lap(const LapMat &M, const double *pu, const int *px,
                                         const double *ps2, int *rx, unsigned char *lds,
                                         long long lds_bytes, unsigned char *gws, int *err,
                                         LapStats *ls, unsigned char *csr = nullptr) {
    if (M.na <= M.nb && M.nb <= RECT_CPT_MAX * (int)blockDim.x)
        rect_solve(RectMat{M.m, M.na, M.nb, M.nb, 1, M.neg}, pu, px, ps2, false, M.na, rx, lds,
                   lds_bytes, gws, err);
    else
        padded_lap(M, rx, lds, lds_bytes, gws, err, ls, csr);
}

// Row pre-pass of the first-round solve for one stream, spread over the blocks of a chip-wide
// launch.  na <= nb: the rows of mat (one wave a row).  na > nb: the rows of the transposed
// problem (first_round_lap), i.e. the columns of mat: a block takes 64 tracker columns, lane =
// column (coalesced across the wave), its waves split the detection rows, partials merged in LDS.
__device__ __forceinline__ void main_lap_pre(const double *mat, int na, int nb, double *u, int *x,
                                             double *s2, bool neg = false) {   // neg: costs -mat
    if (na <= 0 || nb <= 0) return;
    const int nw = blockDim.x / WAVE;
    if (na <= nb) {
        if (nb > RECT_CPT_MAX * LAP_T) return;
        const RectMat M{mat, na, nb, nb, 1, neg};
        for (int i = blockIdx.x * nw + threadIdx.x / WAVE; i < na; i += gridDim.x * nw)
            rect_row_pre(M, i, u, x, s2);
        return;
    }
    if (na > RECT_CPT_MAX * LAP_T) return;
    __shared__ double pm1[OC_T], pm2[OC_T];
    __shared__ int pk1[OC_T];
    const int lane = lane_id(), wid = threadIdx.x / WAVE;
    for (int g = blockIdx.x; g * WAVE < nb; g += gridDim.x) {
        const int j = g * WAVE + lane;
        double m1 = INFINITY, m2 = INFINITY;
        int k1 = INT_MAX;
        if (j < nb)
            for (int i = wid; i < na; i += nw) {   // ascending rows: strict < keeps the first
                const double c = neg ? -mat[(long long)i * nb + j] : mat[(long long)i * nb + j];
                if (c < m1) { m2 = m1; m1 = c; k1 = i; }
                else if (c < m2) m2 = c;
            }
        pm1[threadIdx.x] = m1;
        pm2[threadIdx.x] = m2;
        pk1[threadIdx.x] = k1;
        __syncthreads();
        if (wid == 0 && j < nb) {
            for (int w = 1; w < nw; ++w) {
                const double om1 = pm1[w * WAVE + lane], om2 = pm2[w * WAVE + lane];
                const int ok1 = pk1[w * WAVE + lane];
                const bool other = om1 < m1 || (om1 == m1 && ok1 < k1);
                const double lose = other ? m1 : om1;
                const double m2w = other ? om2 : m2;
                m2 = lose < m2w ? lose : m2w;
                m1 = other ? om1 : m1;
                k1 = other ? ok1 : k1;
            }
            u[j] = m1;
            x[j] = k1 == INT_MAX ? 0 : k1;
            s2[j] = m2 - m1;
        }
        __syncthreads();
    }
}

// A -IoU round's matrix (BYTE / OCR: asso(left dets, left trackers), association.py:20-28 input):
// mat[p * nb + k] = asso(dbox(p), tbox(k)), and its maximum.  The na + nb boxes are gathered once
// into LDS (every gather of a thread's batch in flight at once) when they fit `lds_bytes`, so
// the na x nb evaluations read LDS; a gather chain per evaluation (index -> record, ~1 us) made
// the C5 OCR round ~360 us.  Otherwise every evaluation gathers its two boxes.
template <typename DB, typename TB>
__device__ __forceinline__ double asso_matrix(int kind, int na, int nb, DB dbox, TB tbox, double w,
                                              double h, double *mat, unsigned char *lds,
                                              long long lds_bytes, int *err, OcShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x;
    const long long nm = (long long)na * nb;
    double mx = -INFINITY;
    bool bad = false;
    if ((long long)(na + nb) * (long long)sizeof(Box) <= lds_bytes) {
        Box *bd = reinterpret_cast<Box *>(lds), *bt = bd + na;
        batched_for<4>(na, [&](int p) { return dbox(p); }, [&](int p, const Box &b) { bd[p] = b; });
        batched_for<4>(nb, [&](int k) { return tbox(k); }, [&](int k, const Box &b) { bt[k] = b; });
        block_sync();
        for (int p = 0; p < na; ++p) {   // a row at a time: no index division per entry
            const Box dp = bd[p];
            double *row = mat + (long long)p * nb;
            for (int k = t; k < nb; k += nt) {
                const double v = asso_of(kind, dp, bt[k], w, h);
                bad |= kind == 1 && v != v;
                row[k] = v;
                mx = np_max(mx, v);
            }
        }
    } else {
        for (long long q = t; q < nm; q += nt) {
            const int p = (int)(q / nb), k = (int)(q % nb);
            const double v = asso_of(kind, dbox(p), tbox(k), w, h);
            bad |= kind == 1 && v != v;
            mat[q] = v;
            mx = np_max(mx, v);
        }
    }
    if (bad) atomicOr(err, ERR_GIOU);
    block_sync();
    return block_max(mx, sh);
}

// The -IoU round's problem reduced to its positive part.  The padded lapjv the reference runs
// (association.py:20-28, extend_cost: every row may stay unassigned at cost 0) maximises the summed
// IoU, so the positive pairs of any optimum form a maximum-weight matching of the graph of
// positive entries, and conversely; rows and columns with no positive entry only ever hold
// zero-IoU pairs, which the caller drops (IoU < threshold, threshold > 0).  Solving the rows x
// columns that have a positive entry (their zero entries kept) therefore keeps exactly the pairs
// of the full solve whenever the positive part's optimum is unique - the same condition the
// full rectangular solve relies on.  The matrix must hold only values >= 0 (IoU / GIoU as the
// reference computes them are exactly 0 for disjoint boxes: iou.py:6-25, :52-60); anything else,
// a reduction of less than half the entries, or a reduced matrix larger than the `tws` region
// returns false (the caller solves the full matrix).  The OCR rounds of the steady state keep
// ~20 of ~70 rows and a few dozen of ~1200 columns (C5): the searches of the rows that overlap
// nothing - each a block-wide Dijkstra step over every column - disappear.
__host__ __device__ inline long long tight_ws_bytes();   // below: the certificate's edge region
template <int MAXT>
__device__ __noinline__ bool iou_lap_reduced(const LapMat &M, int *rx, unsigned char *lds,
                                             long long lds_bytes, unsigned char *gws, int *err,
                                             unsigned char *tws) {
    __shared__ int wsum[32];
    __shared__ int s_bad;
    const int t = threadIdx.x, nt = blockDim.x;
    const int na = M.na, nb = M.nb;
    if (na <= 0 || nb <= 0 || (long long)na + nb > lds_bytes) return false;
    unsigned char *rf = lds, *cf = lds + na;   // positive-entry flags of rows / columns
    for (int i = t; i < na + nb; i += nt) lds[i] = 0;
    if (t == 0) s_bad = 0;
    block_sync();
    bool bad = false;
    for (int p = 0; p < na; ++p) {   // a row at a time: no index division per entry
        const double *row = M.m + (long long)p * nb;
        bool any = false;
        for (int k = t; k < nb; k += nt) {
            const double v = row[k];
            if (v > 0.0) {
                any = true;
                cf[k] = 1;
            } else if (!(v == 0.0)) {
                bad = true;   // negative or NaN
            }
        }
        if (any) rf[p] = 1;
    }
    if (bad) s_bad = 1;
    block_sync();
    if (s_bad) return false;
    int *ra = reinterpret_cast<int *>(tws), *ca = ra + na;
    const int nr = block_compact(na, wsum, [&](int i) { return rf[i] != 0; },
                                 [&](int i, int pos) { ra[pos] = i; });
    const int nc = block_compact(nb, wsum, [&](int j) { return cf[j] != 0; },
                                 [&](int j, int pos) { ca[pos] = j; });
    int *rxr = ca + nb;
    const long long mo = ((4LL * (na + nb + nr) + 15) & ~15LL);
    if (2LL * nr * nc > (long long)na * nb || mo + 8LL * nr * nc > tight_ws_bytes() ||
        (nr > nc ? nr : nc) > RECT_CPT_MAX * nt)
        return false;
    block_sync();   // ra / ca (other threads' runs) before their reads
    if (nr == 0) {
        for (int p = t; p < na; p += nt) rx[p] = -1;
        block_sync();
        return true;
    }
    double *R = reinterpret_cast<double *>(tws + mo);
    for (int i = 0; i < nr; ++i) {
        const double *row = M.m + (long long)ra[i] * nb;
        for (int j = t; j < nc; j += nt) R[(long long)i * nc + j] = row[ca[j]];
    }
    block_sync();   // R in global memory: every store before the solver's loads
    const bool tr = nr > nc;
    const RectMat Rm = tr ? RectMat{R, nc, nr, 1, nc, true} : RectMat{R, nr, nc, nc, 1, true};
    rect_solve<MAXT>(Rm, nullptr, nullptr, nullptr, tr, nr, rxr, lds, lds_bytes, gws, err);
    for (int p = t; p < na; p += nt) rx[p] = -1;
    block_sync();
    for (int i = t; i < nr; i += nt) {
        const int k = rxr[i];
        rx[ra[i]] = k >= 0 ? ca[k] : -1;
    }
    block_sync();
    return true;
}

// The -IoU rounds (BYTE / OCR: association.py:20-28 on -iou): only pairs with IoU >= threshold
// survive and the leftover lists are re-sorted (np.setdiff1d), so any optimal solution gives the
// reference's result: the rectangular solver in whichever orientation has rows <= columns, on the
// positive part of the matrix when that is much smaller (iou_lap_reduced; needs `tws` and the
// caller's keep threshold thr > 0).
// MAXT > 256: the solver bodies inlined (a kernel that has the registers for them)
// pu / px / ps2: the solved orientation's row pre-pass (main_lap_pre) when a grid kernel ran it,
// else nullptr (the block runs it).
#ifndef YTA_IOU_REDUCE
#define YTA_IOU_REDUCE 1
#endif
template <int MAXT = 256>
__device__ __forceinline__ void iou_lap(const LapMat &M, int *rx, unsigned char *lds,
                                        long long lds_bytes, unsigned char *gws, int *err,
                                        LapStats *ls, unsigned char *tws = nullptr,
                                        const double *pu = nullptr, const int *px = nullptr,
                                        const double *ps2 = nullptr, double thr = 0.0) {
    if (YTA_IOU_REDUCE && tws && thr > 0.0 && M.neg &&
        iou_lap_reduced<MAXT>(M, rx, lds, lds_bytes, gws, err, tws)) {
        if (threadIdx.x == 0) ls->reduced += 1;
        return;
    }
    const bool tr = M.na > M.nb;
    const int rows = tr ? M.nb : M.na, cols = tr ? M.na : M.nb;
    if (cols > RECT_CPT_MAX * (int)blockDim.x) {
        padded_lap(M, rx, lds, lds_bytes, gws, err, ls);
        return;
    }
    const RectMat R = tr ? RectMat{M.m, rows, cols, 1, M.nb, M.neg}
                         : RectMat{M.m, rows, cols, M.nb, 1, M.neg};
    // (no bidding rounds here: on the OCR matrices of the C5 run they cost more than they saved,
    // k_hs_assoc 465 -> 567 us, profiles/r04k_*)
    (void)tws;
    rect_solve<MAXT>(R, pu, px, ps2, tr, M.na, rx, lds, lds_bytes, gws, err);
}

// Is x, the solution of the transposed first-round problem (rows = trackers, all matched;
// columns = detections), its UNIQUE optimum?  With the solver's column duals v (v <= 0, v = 0 on
// unmatched columns) and u_i = c(i, x_i) - v(x_i), (u, v) is dual feasible and tight on x, so by
// complementary slackness every optimum uses tight edges only and matches every column with
// v < 0.  Another optimum differs from x by an alternating cycle of tight edges, or by an
// alternating path of tight edges ending at an unmatched column.  The shortest-path trees of the
// augmentations leave tight non-matching edges behind (a row stays tight to the column it left),
// so the test is structural: collect the tight non-matching edges (reduced cost <= UNIQ_TOL times
// the magnitude of the entry and duals involved, at least 1: a margin over either solver's
// rounding that scales with the costs, so an embedding- or long-term-weighted matrix with larger
// entries is judged as conservatively as a unit-scale one; a looser test only certifies less
// and sends more frames to the exact replay), fail on one into
// an unmatched column, and look for a cycle in the column digraph (x_i -> k for a tight (i, k)),
// by peeling columns without out-edges.  Unique => lapjv (any exact solver) returns x too,
// whatever its tie-breaking.  Block-wide; the edges go to `tws` (TIGHT_CAP), out-degrees to the
// solver's path array (dead after the solve).  Returns 1 = unique; *n_tight = edges found.
constexpr double UNIQ_TOL = 1e-9;
constexpr int TIGHT_CAP = 16384;
__host__ __device__ inline long long tight_ws_bytes() { return 8LL * TIGHT_CAP; }
__host__ __device__ inline long long oc_lap_ws_stride(long long n) {
    return (n > OC_LDS_LAP_N ? ((dense_lap_ws_bytes(n) + 255) & ~255LL) : 256) + arr_ws_region(n) +
           tight_ws_bytes();
}
__device__ __forceinline__ int unique_optimum_tr(const double *mat, int na, int nb, const RectWs &w,
                                                 int2 *tws, int *n_tight) {
    __shared__ int ne, bad, changed[2];
    const int t = threadIdx.x, nt = blockDim.x;
    if (t == 0) { ne = 0; bad = 0; changed[0] = changed[1] = 0; }
    block_sync();
    for (int j0 = 0; j0 < nb; j0 += nt) {
        const int j = j0 + t;
        if (j >= nb) break;
        const int xj = w.x[j];
        const double own = mat[(long long)xj * nb + j] - w.v[xj];
        auto visit = [&](int i, double c) {
            const double r = (c - w.v[i]) - own;
            if (r != r) { bad = 1; return; }
            const double mag = fmax(1.0, fmax(fabs(c), fmax(fabs(w.v[i]), fabs(own))));
            if (i == xj || r > UNIQ_TOL * mag) return;
            if (w.yw[i] < 0) { bad = 1; return; }   // tight into an unmatched column
            const int k = atomicAdd(&ne, 1);
            if (k < TIGHT_CAP) tws[k] = make_int2(xj, i);
            else bad = 1;
        };
        int i = 0;
        for (; i + 4 <= na; i += 4) {
            double c[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = mat[(long long)(i + k) * nb + j];
#pragma unroll
            for (int k = 0; k < 4; ++k) visit(i + k, c[k]);
        }
        for (; i < na; ++i) visit(i, mat[(long long)i * nb + j]);
    }
    block_sync();
    const int m = ne < TIGHT_CAP ? ne : TIGHT_CAP;
    if (n_tight && t == 0) *n_tight = ne;
    if (bad) return 0;
    if (m == 0) return 1;
    int *deg = w.path;
    for (int i = t; i < na; i += nt) deg[i] = 0;
    block_sync();
    for (int e = t; e < m; e += nt) atomicAdd(&deg[tws[e].x], 1);
    block_sync();
    for (int par = 0;; par ^= 1) {   // peel: an edge into a column without out-edges goes
        for (int e = t; e < m; e += nt) {
            const int2 ed = tws[e];
            if (ed.x >= 0 && atomicAdd(&deg[ed.y], 0) == 0) {
                atomicSub(&deg[ed.x], 1);
                tws[e].x = -1;
                changed[par] = 1;
            }
        }
        block_sync();
        const int ch = changed[par];
        if (t == 0) changed[par ^ 1] = 0;
        block_sync();
        if (!ch) break;
    }
    int left = 0;
    for (int e = t; e < m; e += nt) left |= tws[e].x >= 0;
    if (left) bad = 1;   // a cycle of tight edges
    block_sync();
    return bad == 0;
}

constexpr int ARR_SCAN_WPB = 4;       // fr_arr_scan: waves per block
constexpr int ARR_SCAN_BLOCKS = 256;  // blocks per stream (a block per free row, looping beyond)
// Engines solve first rounds this large with the chip-wide rounds (smaller ones in the block)
constexpr int ARR_CHIP_MIN_DETS = 1024;

// Does the first round solve here (first_round_lap), and not take the fast path or leave it to the
// association kernel?  Block-wide (all threads get the answer).
__device__ __forceinline__ bool fr_solves(int na, int nb, const int *rcnt, const int *ccnt,
                                          bool fast_rule) {
    __shared__ int flags[2];
    const int t = threadIdx.x, nt = blockDim.x;
    const int rows = na > nb ? nb : na, cols = na > nb ? na : nb;
    bool solve = rows > 0 && cols <= RECT_CPT_MAX * LAP_T;
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
        __syncthreads();
    }
    return solve;
}

// The chip-wide bidding rounds of a first round solved in the normal orientation (lap_rect.hpp
// ArrState), between the row pre-pass and first_round_lap: fr_arr_round0 (block per stream),
// then ARR_CHIP_ROUNDS x (fr_arr_scan: a wave per free row over the grid, fr_arr_apply: block per
// stream).  The state sits in the bidding region below tws; hdr[2] tells first_round_lap to start
// from it.  Same arguments as first_round_lap.
__device__ __forceinline__ void fr_arr_round0(const double *mat, int na, int nb, const int *rcnt,
                                              const int *ccnt, bool fast_rule, const double *pu,
                                              const int *px, const double *ps2, unsigned char *tws,
                                              int *wsum) {
    const bool ok = YTA_LAP_ARR && na <= nb && fr_solves(na, nb, rcnt, ccnt, fast_rule);
    const ArrState st = arr_state(tws - arr_ws_region(nb), na, nb);
    if (!ok) {
        if (threadIdx.x == 0 && nb > 0) st.hdr[0] = st.hdr[2] = 0;
        return;
    }
    arr_round0(RectMat{mat, na, nb, nb, 1, false}, pu, px, ps2, st, wsum);
}
// block blk of the grid's nblk blocks for this stream: a free row at a time
__device__ __forceinline__ void fr_arr_scan(const double *mat, int na, int nb, unsigned char *tws,
                                            int blk, int nblk) {
    __shared__ ArrTop2 slot[ARR_SCAN_WPB];
    if (na > nb || na <= 0) return;
    const ArrState st = arr_state(tws - arr_ws_region(nb), na, nb);
    if (!st.hdr[0]) return;
    const int n = st.hdr[1];
    const RectMat M{mat, na, nb, nb, 1, false};
    for (int k = blk; k < n; k += nblk) arr_scan_row(M, st, k, slot);
}
__device__ __forceinline__ void fr_arr_apply(const double *mat, int na, int nb, unsigned char *tws,
                                             int *wsum) {
    if (na > nb || na <= 0) return;
    const ArrState st = arr_state(tws - arr_ws_region(nb), na, nb);
    if (!st.hdr[0]) return;
    arr_apply(RectMat{mat, na, nb, nb, 1, false}, st, wsum);
}

// First-round solve in its own launch, one LAP_T-thread block per stream (up to 32 columns per
// thread: 16384 columns, every cost load of a step in flight at once), when the fast path
// (association.py:156-159, `fast_rule`) does not apply; rx and *done = 1 on success, else the
// association kernel solves.  rcnt / ccnt: the per-row / per-column counts of asso > thr (rcnt
// may alias rx: it is read before the solve).
//  * trackers >= detections: lap_rect warm-started by the row pre-pass; every detection row is
//    matched and the outputs do not depend on which optimum is returned.
//  * more detections than trackers (a crowd entering): which detections stay on lapjv's dummy
//    columns sets the order of the unmatched list (association.py:179-199) and so the birth ids;
//    the transposed problem (trackers as rows, every one matched; dummy columns cost 0, so the
//    padded optimum is the rectangular one) is solved, and kept when its optimum is certified
//    unique (unique_optimum_tr).  Otherwise (exact ties: e.g. a tracker without velocity and
//    without overlap has a whole row of exact zeros under IoU) *done = 0 and the association
//    kernel replays lapjv.
__device__ __forceinline__ void first_round_lap(const double *mat, int na, int nb, const int *rcnt,
                                                const int *ccnt, bool fast_rule, const double *pu,
                                                const int *px, const double *ps2, int *rx,
                                                unsigned char *lds, long long lds_bytes,
                                                unsigned char *gws, int *err, int *done,
                                                LapStats *ls, unsigned char *tws,
                                                int *n_tight = nullptr, bool chip = false) {
    __shared__ RectShared rsh;
    const int t = threadIdx.x, nt = blockDim.x;
    const bool tr = na > nb;
    const int rows = tr ? nb : na, cols = tr ? na : nb;
    const bool solve = fr_solves(na, nb, rcnt, ccnt, fast_rule);
    if (!solve) {
        if (t == 0) *done = 0;
        return;
    }
    unsigned char *base = rect_ws_bytes(rows, cols, tr) <= lds_bytes ? lds : gws;
    RectWs w = rect_ws(base, rows, cols, tr);
    unsigned char *aws = tws - arr_ws_region(rows > cols ? rows : cols);
    const ArrState st = arr_state(aws, rows, cols);
    if (YTA_LAP_ARR && chip && !tr && st.hdr[2]) {   // the chip-wide rounds ran: their state
        w.sx = st.ax;
        w.su = st.au;
        w.ss2 = st.as2;
        w.syw = st.ayw;
        w.sv = st.av;
    } else if (YTA_LAP_ARR && !tr) {
        // the bidding rounds in this block: the region just below tws (oc_lap_ws_stride).  Not for
        // the transposed solve: a bid leaves its row tight on two columns, and a tight edge into
        // an unmatched column fails the uniqueness certificate
        rect_arr_ws(aws, rows, cols, w);
        // the column duals of the rounds (read by every bid scan) in LDS after the work arrays
        const long long wo = (rect_ws_bytes(rows, cols) + 15) & ~15LL;
        if (base == lds && wo + 8LL * cols <= lds_bytes) {
            w.av = reinterpret_cast<double *>(lds + wo);
            w.av_lds = 1;
        }
    }
    const RectMat R = tr ? RectMat{mat, rows, cols, 1, nb, false} : RectMat{mat, rows, cols, nb, 1, false};
    const int rc = lap_rect<LAP_T>(R, pu, px, ps2, w, rsh);
    if (rc && t == 0) atomicOr(err, ERR_SOLVER);
    if (!tr) {
        for (int i = t; i < na; i += nt) rx[i] = rc ? -1 : w.x[i];
        if (t == 0) *done = 1;
        return;
    }
    if (t == 0) ls->transposed += 1;
    block_sync();
    const bool uniq = rc == 0 &&
        unique_optimum_tr(mat, na, nb, w, reinterpret_cast<int2 *>(tws), n_tight);
    if (!uniq) {
        if (t == 0) {
            if (rc == 0) ls->uncertified += 1;
            *done = 0;
        }
        return;
    }
    for (int i = t; i < na; i += nt) rx[i] = -1;
    block_sync();
    for (int k = t; k < nb; k += nt) rx[w.x[k]] = k;
    if (t == 0) *done = 1;
}

}  // namespace yta
