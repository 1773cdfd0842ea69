// Uniform-grid binning of a box set, so a track only scores the detections it can intersect.
//
// Exactness.  A pair whose boxes do not intersect has IoU = +-0 (or NaN), hence 1 - IoU >= 1 and
// 1 - (1 - (1 - IoU)) * s >= 1 for every cost threshold the reference uses (< 1): it can never be an
// association candidate (assoc.hpp).  Boxes with a non-positive or non-finite width/height never
// intersect anything and are left out.  The grid only skips pairs that provably do not intersect;
// every visited pair is then scored with the exact float64 expression.
//
//  * cell size g = mean box size; a box goes to the cell of its top-left corner and its box is
//    stored next to its id in cell order (one load per candidate);
//  * boxes larger than 4 g go to a "big" list that every query scans, so the binned boxes have a
//    small maximum width W and height H;
//  * a query box T visits cells x in [cell(T.x1 - W - eps), cell(T.x2)] (same for y): a box D that
//    intersects T has D.x1 < T.x2 and D.x1 = D.x2 - w(D) > T.x1 - W, cell() is monotone, and eps
//    (1e-12 relative) covers the rounding of w(D) and of the subtraction.
#pragma once
#include "common.hpp"
#include "geometry.hpp"
#include "lap.hpp"

namespace yta {

constexpr int GRID_MAX_CELLS = 2048;

// Cell budget for n items: about two cells per item (fewer cells only coarsen the pruning).
__host__ __device__ __forceinline__ int grid_cells_for(int n) {
    const int c = 2 * n + 16;
    return c < GRID_MAX_CELLS ? c : GRID_MAX_CELLS;
}

struct GridHdr {
    double ox, oy, inv_g, maxw, maxh, g;
    int gx, gy, n_big, n_binned;
};

struct GridView {
    GridHdr *hdr;      // optional copy of the header (global)
    int *cell_start;   // GRID_MAX_CELLS + 1
    int *ids;          // binned item ids, in cell order
    Box *boxes;        // their boxes, same order (nullptr: read through by_id)
    double *w;         // optional per-item weight, same order (nullptr: none)
    int *big;          // items scanned by every query
    const Box *by_id = nullptr;   // with boxes == nullptr: every item's box, by item id
    // structure-of-arrays boxes (x1[], y1[], x2[], y2[], cell order) instead of `boxes`: a wave
    // reading the boxes of consecutive positions then reads consecutive 8-B words per component
    // (no LDS bank conflicts), where 32-B records put two lanes on every bank pair it touches
    double *sx = nullptr;         // 4 arrays of n doubles: sx, sx + n, sx + 2 n, sx + 3 n
    int sn = 0;
};

// Box of the binned item at cell-order position k.
__device__ __forceinline__ Box grid_box(const GridView &gv, int k) {
    if (gv.sx) return Box{gv.sx[k], gv.sx[gv.sn + k], gv.sx[2 * gv.sn + k], gv.sx[3 * gv.sn + k]};
    return gv.boxes ? gv.boxes[k] : gv.by_id[gv.ids[k]];
}


__host__ __device__ __forceinline__ bool box_usable(const Box &b) {
    const double w = b.x2 - b.x1, h = b.y2 - b.y1;
    return w > 0.0 && h > 0.0 && isfinite(b.x1) && isfinite(b.y1) && isfinite(b.x2) &&
           isfinite(b.y2) && isfinite(w) && isfinite(h);
}

__device__ __forceinline__ int grid_cell_1d(double x, double o, double inv_g, int n) {
    double f = floor((x - o) * inv_g);
    f = f < 0.0 ? 0.0 : (f > (double)(n - 1) ? (double)(n - 1) : f);
    return (int)f;
}

struct GridScratch {
    double red[8 * 16];
    GridHdr hdr;
    unsigned long long maxw_bits, maxh_bits;   // max binned width / height (positive doubles)
};

// Block-wide reduction of 6 values; op[k]: RED_MIN / RED_MAX / RED_SUM.  Per-wave partials go
// through `red` (>= 8 * 16 doubles); every wave then reduces the partials itself.
__device__ __forceinline__ void block_reduce6(double v[6], const int op[6], double *red) {
    const int wv = threadIdx.x / WAVE, nw = blockDim.x / WAVE, lane = lane_id();
    for (int k = 0; k < 6; ++k) v[k] = wave_reduce(op[k], v[k]);
    if (lane == 0)
        for (int k = 0; k < 6; ++k) red[8 * wv + k] = v[k];
    block_sync();
    for (int k = 0; k < 6; ++k)
        v[k] = wave_reduce(op[k], lane < nw ? red[8 * lane + k] : red_ident(op[k]));
    __syncthreads();   // red is reused
}

// Block-wide build (every thread of the block calls it).  box(i) returns item i's box, wof(i) its
// weight (stored only when gv.w is set).  gv.cell_start needs grid_cells_for(n) + 1 entries,
// gv.ids / gv.boxes / gv.w / gv.big n entries.
//   1. one block reduction over the usable boxes: mean size, extent of the top-left corners
//   2. count per cell (items larger than 4 x mean go to the big list instead); the maximum
//      width / height of the binned items by 64-bit LDS atomicMax on their bit patterns
//   3. one block scan of the cell counts, 4. scatter
template <typename BoxOf, typename WOf>
__device__ __forceinline__ void grid_build(int n, BoxOf box, WOf wof, GridView gv, GridScratch &gs,
                                           int *wsum) {
    const int t = threadIdx.x, nt = blockDim.x;
    YTA_STAMP_ABS(110);
    double v[6] = {0.0, 0.0, INFINITY, INFINITY, -INFINITY, -INFINITY};
    const int ops[6] = {RED_SUM, RED_SUM, RED_MIN, RED_MIN, RED_MAX, RED_MAX};
    for (int i = t; i < n; i += nt) {
        const Box b = box(i);
        if (!box_usable(b)) continue;
        v[0] += fmax(b.x2 - b.x1, b.y2 - b.y1);
        v[1] += 1.0;
        v[2] = fmin(v[2], b.x1);
        v[3] = fmin(v[3], b.y1);
        v[4] = fmax(v[4], b.x1);
        v[5] = fmax(v[5], b.y1);
    }
    if (t == 0) {
        gs.maxw_bits = 0ull;
        gs.maxh_bits = 0ull;
        gs.hdr.n_big = 0;
    }
    block_reduce6(v, ops, gs.red);
    YTA_STAMP_ABS(111);
    const double mean = v[1] > 0 ? v[0] / v[1] : 1.0;
    const double bthr = 4.0 * mean;
    auto binned = [&](const Box &b) {
        return box_usable(b) && !(b.x2 - b.x1 > bthr) && !(b.y2 - b.y1 > bthr);
    };
    GridHdr h;
    if (!(v[4] >= v[2])) {   // nothing usable
        h.ox = h.oy = 0.0;
        h.g = 1.0;
        h.inv_g = 1.0;
        h.gx = h.gy = 1;
    } else {
        double g = mean;
        const double ex = v[4] - v[2], ey = v[5] - v[3];
        double gxf = floor(ex / g) + 1.0, gyf = floor(ey / g) + 1.0;
        const double max_cells = (double)grid_cells_for(n);
        while (gxf * gyf > max_cells) {
            g *= 1.25;
            gxf = floor(ex / g) + 1.0;
            gyf = floor(ey / g) + 1.0;
        }
        h.ox = v[2];
        h.oy = v[3];
        h.g = g;
        h.inv_g = 1.0 / g;
        h.gx = (int)gxf;
        h.gy = (int)gyf;
    }
    const int ncell = h.gx * h.gy;
    int *cs = gv.cell_start;
    for (int c = t; c <= ncell; c += nt) cs[c] = 0;
    block_sync();
    YTA_STAMP_ABS(112);
    auto cell_of = [&](const Box &b) {
        return grid_cell_1d(b.y1, h.oy, h.inv_g, h.gy) * h.gx + grid_cell_1d(b.x1, h.ox, h.inv_g, h.gx);
    };
    // counts land in cs[c + 1]; the exclusive scan leaves start(c) there, and the scatter's cursor
    // increments turn it into end(c) = start(c + 1), so cs[c] = start(c) afterwards
    double mw = 0.0, mh = 0.0;
    for (int i = t; i < n; i += nt) {
        const Box b = box(i);
        if (!box_usable(b)) continue;
        if (!binned(b)) {
            gv.big[atomicAdd(&gs.hdr.n_big, 1)] = i;
            continue;
        }
        mw = fmax(mw, b.x2 - b.x1);
        mh = fmax(mh, b.y2 - b.y1);
        atomicAdd(&cs[cell_of(b) + 1], 1);
    }
    mw = wave_reduce(RED_MAX, mw);
    mh = wave_reduce(RED_MAX, mh);
    if (lane_id() == 0) {
        atomicMax(&gs.maxw_bits, (unsigned long long)__double_as_longlong(mw));
        atomicMax(&gs.maxh_bits, (unsigned long long)__double_as_longlong(mh));
    }
    block_sync();
    YTA_STAMP_ABS(113);
    {   // one scan: every thread owns a contiguous run of cells
        const int per = (ncell + nt - 1) / nt;
        const int c0 = t * per, c1 = c0 + per < ncell ? c0 + per : ncell;
        int mine = 0;
        for (int c = c0; c < c1; ++c) mine += ald(cs + c + 1);
        int tot;
        int run = block_exclusive_scan(mine, wsum, &tot);
        for (int c = c0; c < c1; ++c) {
            const int k = ald(cs + c + 1);
            cs[c + 1] = run;
            run += k;
        }
        if (t == 0) {
            h.n_big = gs.hdr.n_big;
            h.n_binned = tot;
            h.maxw = __longlong_as_double((long long)gs.maxw_bits);
            h.maxh = __longlong_as_double((long long)gs.maxh_bits);
            gs.hdr = h;
            if (gv.hdr) *gv.hdr = h;
        }
    }
    block_sync();
    YTA_STAMP_ABS(115);
    for (int i = t; i < n; i += nt) {
        const Box b = box(i);
        if (!binned(b)) continue;
        const int pos = atomicAdd(&cs[cell_of(b) + 1], 1);
        gv.ids[pos] = i;
        if (gv.boxes) gv.boxes[pos] = b;
        if (gv.sx) {
            gv.sx[pos] = b.x1;
            gv.sx[gv.sn + pos] = b.y1;
            gv.sx[2 * gv.sn + pos] = b.x2;
            gv.sx[3 * gv.sn + pos] = b.y2;
        }
        if (gv.w) gv.w[pos] = wof(i);
    }
    block_sync();
    YTA_STAMP_ABS(116);
}

// grid_scan: every binned item whose box intersects T (exact float64 test): hit(k, id, box, w)
// with k its position in cell order (w = 1 without weights).  Software-pipelined: the next cell
// row's range is loaded while this one is scanned, and two candidates' box / id / weight are
// loaded together before either is tested (one LDS round trip per pair).
// grid_query: the same plus visit_big(id) for every big item (unfiltered).
template <typename Hit>
__device__ __forceinline__ void grid_scan(const GridView &gv, const GridHdr &h, const Box &T,
                                          Hit hit) {
    if (h.n_binned == 0) return;
    if (!(T.x2 > T.x1 && T.y2 > T.y1)) return;   // also false for NaN: intersects nothing
    const double lx = (T.x1 - h.maxw * (1.0 + 1e-12)) - (fabs(T.x1) + h.maxw) * 1e-12;
    const double ly = (T.y1 - h.maxh * (1.0 + 1e-12)) - (fabs(T.y1) + h.maxh) * 1e-12;
    const double fx1 = floor((T.x2 - h.ox) * h.inv_g), fy1 = floor((T.y2 - h.oy) * h.inv_g);
    if (fx1 < 0.0 || fy1 < 0.0) return;
    const int cx0 = grid_cell_1d(lx, h.ox, h.inv_g, h.gx);
    const int cy0 = grid_cell_1d(ly, h.oy, h.inv_g, h.gy);
    const int cx1 = fx1 > (double)(h.gx - 1) ? h.gx - 1 : (int)fx1;
    const int cy1 = fy1 > (double)(h.gy - 1) ? h.gy - 1 : (int)fy1;
    auto wt = [&](int k) { return gv.w ? gv.w[k] : 1.0; };
    int b = ald(gv.cell_start + cy0 * h.gx + cx0), e = ald(gv.cell_start + cy0 * h.gx + cx1 + 1);
    for (int cy = cy0; cy <= cy1; ++cy) {
        int nb = 0, ne = 0;
        if (cy < cy1) {
            const int base = (cy + 1) * h.gx;
            nb = ald(gv.cell_start + base + cx0);
            ne = ald(gv.cell_start + base + cx1 + 1);
        }
        int k = b;
        for (; k + 1 < e; k += 2) {   // the cells of a grid row are contiguous
            const Box b0 = grid_box(gv, k), b1 = grid_box(gv, k + 1);
            const int i0 = gv.ids[k], i1 = gv.ids[k + 1];
            const double w0 = wt(k), w1 = wt(k + 1);
            if (intersects(T, b0)) hit(k, i0, b0, w0);
            if (intersects(T, b1)) hit(k + 1, i1, b1, w1);
        }
        if (k < e) {
            const Box b0 = grid_box(gv, k);
            if (intersects(T, b0)) hit(k, gv.ids[k], b0, wt(k));
        }
        b = nb;
        e = ne;
    }
}

// The cell window grid_scan visits for query box T: false when it visits nothing.
__device__ __forceinline__ bool grid_scan_window(const GridHdr &h, const Box &T, int &cx0, int &cx1,
                                                 int &cy0, int &cy1) {
    if (h.n_binned == 0) return false;
    if (!(T.x2 > T.x1 && T.y2 > T.y1)) return false;   // also false for NaN: intersects nothing
    const double lx = (T.x1 - h.maxw * (1.0 + 1e-12)) - (fabs(T.x1) + h.maxw) * 1e-12;
    const double ly = (T.y1 - h.maxh * (1.0 + 1e-12)) - (fabs(T.y1) + h.maxh) * 1e-12;
    const double fx1 = floor((T.x2 - h.ox) * h.inv_g), fy1 = floor((T.y2 - h.oy) * h.inv_g);
    if (fx1 < 0.0 || fy1 < 0.0) return false;
    cx0 = grid_cell_1d(lx, h.ox, h.inv_g, h.gx);
    cy0 = grid_cell_1d(ly, h.oy, h.inv_g, h.gy);
    cx1 = fx1 > (double)(h.gx - 1) ? h.gx - 1 : (int)fx1;
    cy1 = fy1 > (double)(h.gy - 1) ? h.gy - 1 : (int)fy1;
    return true;
}

// Binned items whose top-left corner lies in [lx, hx] x [ly, hy] (a superset: whole cells):
// hit(k, id, box, w).  Same pipelining as grid_scan.
template <typename Hit>
__device__ __forceinline__ void grid_scan_corner(const GridView &gv, const GridHdr &h, double lx,
                                                 double hx, double ly, double hy, Hit hit) {
    if (h.n_binned == 0) return;
    if (!(hx >= lx && hy >= ly)) return;   // also false for NaN
    const double fx1 = floor((hx - h.ox) * h.inv_g), fy1 = floor((hy - h.oy) * h.inv_g);
    if (fx1 < 0.0 || fy1 < 0.0) return;
    const int cx0 = grid_cell_1d(lx, h.ox, h.inv_g, h.gx);
    const int cy0 = grid_cell_1d(ly, h.oy, h.inv_g, h.gy);
    const int cx1 = fx1 > (double)(h.gx - 1) ? h.gx - 1 : (int)fx1;
    const int cy1 = fy1 > (double)(h.gy - 1) ? h.gy - 1 : (int)fy1;
    auto wt = [&](int k) { return gv.w ? gv.w[k] : 1.0; };
    int b = ald(gv.cell_start + cy0 * h.gx + cx0), e = ald(gv.cell_start + cy0 * h.gx + cx1 + 1);
    for (int cy = cy0; cy <= cy1; ++cy) {
        int nb = 0, ne = 0;
        if (cy < cy1) {
            const int base = (cy + 1) * h.gx;
            nb = ald(gv.cell_start + base + cx0);
            ne = ald(gv.cell_start + base + cx1 + 1);
        }
        int k = b;
        for (; k + 1 < e; k += 2) {
            const Box b0 = grid_box(gv, k), b1 = grid_box(gv, k + 1);
            const int i0 = gv.ids[k], i1 = gv.ids[k + 1];
            const double w0 = wt(k), w1 = wt(k + 1);
            hit(k, i0, b0, w0);
            hit(k + 1, i1, b1, w1);
        }
        if (k < e) hit(k, gv.ids[k], grid_box(gv, k), wt(k));
        b = nb;
        e = ne;
    }
}

// Every binned item that can have IoU(T, item) > t (0 < t < 1), plus every big item: IoU > t
// needs the intersection width > t * max(w_T, w_item), so the corners differ by less than
// (1 - t) / t * w_T in x (likewise in y); a relative 1e-6 plus an absolute slack covers the
// rounding of the bound.  visit(id, box, w) then decides exactly.
template <typename Visit, typename VisitBig>
__device__ __forceinline__ void grid_query_iou_above(const GridView &gv, const GridHdr &h,
                                                     const Box &T, double t, Visit visit,
                                                     VisitBig visit_big) {
    for (int k = 0; k < h.n_big; ++k) visit_big(gv.big[k]);
    if (!(T.x2 > T.x1 && T.y2 > T.y1)) return;   // intersects nothing (also NaN)
    const double r = (1.0 - t) / t * (1.0 + 1e-6);
    const double mx = (T.x2 - T.x1) * r + (fabs(T.x1) + 1.0) * 1e-9;
    const double my = (T.y2 - T.y1) * r + (fabs(T.y1) + 1.0) * 1e-9;
    grid_scan_corner(gv, h, T.x1 - mx, T.x1 + mx, T.y1 - my, T.y1 + my,
                     [&](int, int id, const Box &b, double w) { visit(id, b, w); });
}

// ---- float boxes with exact pre-tests (the duplicate-removal grid, k_finish)
// A box rounded outward to float: the float box contains the double one (x1 / y1 rounded down,
// x2 / y2 up; NaN stays NaN).  16 B instead of 32 in LDS.
__device__ __forceinline__ float4 box_outer_f32(const Box &b) {
    auto dn = [](double x) {
        const float f = (float)x;
        return (double)f > x ? nextafterf(f, -INFINITY) : f;
    };
    auto up = [](double x) {
        const float f = (float)x;
        return (double)f < x ? nextafterf(f, INFINITY) : f;
    };
    return make_float4(dn(b.x1), dn(b.y1), up(b.x2), up(b.y2));
}

__device__ __forceinline__ Box box_of_f4(const float4 &f) {
    return Box{(double)f.x, (double)f.y, (double)f.z, (double)f.w};
}

// Conservative pre-test of IoU(T, L) > t for a box L known only by its outward-rounded float box
// Lo: the exact L lies between Lo and the inner box one float step inside it, so
// IoU(T, L) <= I(T, Lo) / (A(T) + A(inner) - I(T, Lo)) (IoU grows with the intersection, falls
// with the other area).  Float values and their products are exact in double; the remaining
// double roundings (~1e-16 relative) are covered by the 1e-6 slack.  false => IoU(T, L) <= t
// (1 - 1e-6): the pair can be skipped; NaN boxes intersect nothing.
__device__ __forceinline__ bool iou_may_exceed(const Box &T, const float4 &Lo, double t) {
    const double iw = fmin(T.x2, (double)Lo.z) - fmax(T.x1, (double)Lo.x);
    const double ih = fmin(T.y2, (double)Lo.w) - fmax(T.y1, (double)Lo.y);
    if (!(iw > 0.0 && ih > 0.0)) return false;   // the outer boxes do not meet: neither do L, T
    const double I = iw * ih;
    const double bw = (double)nextafterf(Lo.z, -INFINITY) - (double)nextafterf(Lo.x, INFINITY);
    const double bh = (double)nextafterf(Lo.w, -INFINITY) - (double)nextafterf(Lo.y, INFINITY);
    const double B = fmax(bw, 0.0) * fmax(bh, 0.0);
    const double den = (T.x2 - T.x1) * (T.y2 - T.y1) + B - I;
    return !(den > 0.0) || I > t * (1.0 - 1e-6) * den;
}

// grid_query_iou_above over a grid whose items' boxes are outward-rounded float boxes lc[id]
// (grid built on box_of_f4(lc[id])): the corner window is widened by the float rounding of the
// corners (<= 2^-23 relative); visit(id, lc[id]) / visit_big(id) then decide.
template <typename Visit, typename VisitBig>
__device__ __forceinline__ void grid_query_iou_above_f4(const GridView &gv, const GridHdr &h,
                                                        const float4 *lc, const Box &T, double t,
                                                        Visit visit, VisitBig visit_big) {
    for (int k = 0; k < h.n_big; ++k) visit_big(gv.big[k]);
    if (!(T.x2 > T.x1 && T.y2 > T.y1)) return;   // intersects nothing (also NaN)
    if (h.n_binned == 0) return;
    const double r = (1.0 - t) / t * (1.0 + 1e-6);
    double mx = (T.x2 - T.x1) * r + (fabs(T.x1) + 1.0) * 1e-9;
    double my = (T.y2 - T.y1) * r + (fabs(T.y1) + 1.0) * 1e-9;
    mx += (fabs(T.x1) + mx + 1.0) * 2.5e-7;
    my += (fabs(T.y1) + my + 1.0) * 2.5e-7;
    const double lx = T.x1 - mx, hx = T.x1 + mx, ly = T.y1 - my, hy = T.y1 + my;
    const double fx1 = floor((hx - h.ox) * h.inv_g), fy1 = floor((hy - h.oy) * h.inv_g);
    if (fx1 < 0.0 || fy1 < 0.0) return;
    const int cx0 = grid_cell_1d(lx, h.ox, h.inv_g, h.gx);
    const int cy0 = grid_cell_1d(ly, h.oy, h.inv_g, h.gy);
    const int cx1 = fx1 > (double)(h.gx - 1) ? h.gx - 1 : (int)fx1;
    const int cy1 = fy1 > (double)(h.gy - 1) ? h.gy - 1 : (int)fy1;
    for (int cy = cy0; cy <= cy1; ++cy) {
        const int b = ald(gv.cell_start + cy * h.gx + cx0);
        const int e = ald(gv.cell_start + cy * h.gx + cx1 + 1);
        int k = b;
        for (; k + 1 < e; k += 2) {
            const int i0 = gv.ids[k], i1 = gv.ids[k + 1];
            const float4 b0 = lc[i0], b1 = lc[i1];
            visit(i0, b0);
            visit(i1, b1);
        }
        if (k < e) {
            const int i0 = gv.ids[k];
            visit(i0, lc[i0]);
        }
    }
}

template <typename Visit, typename VisitBig>
__device__ __forceinline__ void grid_query(const GridView &gv, const GridHdr &h, const Box &T,
                                           Visit visit, VisitBig visit_big) {
    for (int k = 0; k < h.n_big; ++k) visit_big(gv.big[k]);
    grid_scan(gv, h, T, [&](int, int id, const Box &b, double w) { visit(id, b, w); });
}

}  // namespace yta
