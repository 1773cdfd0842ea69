// Association on gfx950: candidate edges + exact sparse linear assignment with lapx's cost_limit
// semantics, as one block-level step of a per-stream kernel.
//
// Why sparse is exact.  lap.lapjv(cost, extend_cost=True, cost_limit=t) (matching.py:64) solves the
// (R+C)^2 problem whose off-diagonal blocks cost t/2 and whose dummy block costs 0, i.e. it
// minimises  sum_{matched (i,j)} (c_ij - t)  + const.  A pair with c_ij >= t never improves that
// objective (swapping it for two dummies changes the cost by t - c_ij <= 0), so only "edges"
// c_ij < t matter: the problem is a maximum-weight bipartite matching with weights t - c_ij > 0 on
// a graph that, for tracking, has ~1 edge per row.  Its connected components are independent and
// solved by lap_block (lap.hpp).
//
// Candidate edges.  A pair whose boxes do not intersect has cost >= 1 >= t for the thresholds
// ByteTrack uses (t <= 1), so a uniform grid over the column boxes (grid.hpp) yields every
// candidate; t > 1 falls back to all pairs.  Each candidate is scored with the reference's float64
// expression (1 - IoU, matching.py:117; fused 1 - (1 - d) * score, matching.py:216-220) and kept
// iff cost < t.  The CSR is built in two passes over the rows (count, block scan, fill) straight
// into the arena: no edge list, no global atomics.
//
// Results equal lapx's whenever the optimum is unique (tie-free); lapx's own tie-breaking is
// unpinned (not installed), see DESIGN.md.
#pragma once
#include "common.hpp"
#include "geometry.hpp"
#include "grid.hpp"
#include "lap.hpp"

namespace yta {

struct AssocShared {     // static LDS of a kernel that calls assoc_block
    GridScratch gs;
    LapShared lap;
};

// Arena bytes that suffice for one assoc_block with <= R rows, <= C columns and <= E edges (the
// global-memory fallback arena is sized with this and E = R * C).
__host__ __device__ inline long long assoc_arena_bytes(long long R, long long C, long long E) {
    const long long grid = 4 * (GRID_MAX_CELLS + 1) + C * (4 + 32 + 8 + 4) + 5 * 16 +
                           1024 * 20 + 2 * 16;   // + overflow list
    const long long top = 4 * (R + 1) + 4 * C + 12 * E + 3 * 16;
    const long long lap = 4 * (R + C) * 3 + 4 * 5 * (R + C + 1) + 8 * 16;
    return (grid > lap ? grid : lap) + top + 256;
}

// The first KC candidate edges of a row, kept in registers between the counting pass and the
// CSR fill (compile-time slots: no scratch).
constexpr int KC = 2;
struct EdgeCache {
    int n;
    int c0, c1;
    double w0, w1;
    __device__ __forceinline__ void push(int c, double w) {
        if (n == 0) { c0 = c; w0 = w; }
        else if (n == 1) { c1 = c; w1 = w; }
        ++n;
    }
};

// One association problem of the calling block.  rowbox(i) / colbox(j): boxes; colscore(j): the
// fuse_score weight (only called when `fused`).  X[nr] / Y[nc] receive the assignment, edge count
// in *n_edges (thread 0).  Returns false if the arena is exhausted.
//
//   grid over the columns (boxes staged once into the arena when it has room)
//   pass 1: every row queries the grid and counts its edges; the first KC stay in registers
//           (rows of the first two row-chunks), the rest go to an LDS overflow list with their
//           position in the row; block scan per chunk -> CSR row offsets
//   pass 2: rows write their cached edges, the overflow list is scattered; rows query again
//           only when that list overflowed
//   lap_block on the CSR
template <typename RowBox, typename ColBox, typename ColScore>
__device__ __forceinline__ bool assoc_block(int nr, RowBox rowbox, int nc, ColBox colbox,
                                            bool fused, ColScore colscore, double thresh, int *X,
                                            int *Y, int *err, int *n_edges, Arena &ar,
                                            const LapSlab &slab, AssocShared &sh,
                                            const Box *ext_cbox = nullptr,
                                            const double *ext_cw = nullptr) {
    const int t = threadIdx.x, nt = blockDim.x;
    const bool use_grid = thresh <= 1.0 && nr > 0 && nc > 0;
    const size_t lo0 = ar.lo;
    GridView gv{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    if (use_grid) {
        gv.cell_start = ar.alloc<int>(grid_cells_for(nc) + 1);
        gv.ids = ar.alloc<int>(nc);
        gv.boxes = ar.alloc<Box>(nc);
        gv.w = fused ? ar.alloc<double>(nc) : nullptr;
        gv.big = ar.alloc<int>(nc);
    }
    int *row_off = ar.alloc_top<int>(nr + 1);
    int *col_deg = ar.alloc_top<int>(nc);
    if (ar.fail) return false;
    const size_t hi0 = ar.hi;
    // column boxes / weights staged in the arena: by the caller (ext_*), else here if room
    const bool ext = ext_cbox && (!fused || ext_cw);
    Box *ccache = ext ? nullptr : (use_grid ? ar.try_alloc_top<Box>(nc) : nullptr);
    double *wcache = nullptr;
    if (ccache && fused) {
        wcache = ar.try_alloc_top<double>(nc);
        if (!wcache) {
            ccache = nullptr;
            ar.hi = hi0;
        }
    }
    for (int j = t; j < nc; j += nt) {
        col_deg[j] = 0;
        if (ccache) {
            ccache[j] = colbox(j);
            if (wcache) wcache[j] = colscore(j);
        }
    }
    const Box *cb_src = ext ? ext_cbox : ccache;
    const double *cw_src = ext ? ext_cw : wcache;
    if (use_grid) {
        block_sync();
        if (cb_src)
            grid_build(
                nc, [&](int j) { return cb_src[j]; },
                [&](int j) { return cw_src ? cw_src[j] : 1.0; }, gv, sh.gs, sh.lap.wsum);
        else
            grid_build(
                nc, [&](int j) { return colbox(j); },
                [&](int j) { return fused ? colscore(j) : 1.0; }, gv, sh.gs, sh.lap.wsum);
    }
    ar.hi = hi0;   // the column cache is dead
    const GridHdr gh = sh.gs.hdr;
    YTA_STAMP(5);

    // every candidate (j, cost) of row box rb with cost < thresh
    auto cost_of = [&](const Box &rb, const Box &cb, double w) {
        const double dist = 1 - iou(rb, cb);                              // matching.py:117
        return fused ? 1 - (1 - dist) * w : dist;                         // matching.py:216-220
    };
    auto for_each_edge = [&](const Box &rb, auto &&f) {
        if (!use_grid) {
            for (int j = 0; j < nc; ++j) {
                const double c = cost_of(rb, colbox(j), fused ? colscore(j) : 1.0);
                if (c < thresh) f(j, c);
            }
            return;
        }
        grid_query(
            gv, gh, rb,
            [&](int j, const Box &cb, double w) {
                const double c = cost_of(rb, cb, w);
                if (c < thresh) f(j, c);
            },
            [&](int j) {
                const Box cb = colbox(j);
                if (!intersects(rb, cb)) return;
                const double c = cost_of(rb, cb, fused ? colscore(j) : 1.0);
                if (c < thresh) f(j, c);
            });
    };
    // pass 1: edges per row (rows strided over the threads, chunk by chunk) -> row offsets.  The
    // first KC edges of a row in the first two chunks stay in registers; every other edge goes
    // to an overflow list with its position in the row (so no lane re-queries in pass 2 unless
    // the list itself overflows: then rows not fully captured query again).
    const int ovf_cap = nr > 0 && nc > 0 ? (nr < 448 ? 2 * nr + 128 : 1024) : 0;
    int *ovf_i = ovf_cap ? ar.try_alloc<int>(3 * ovf_cap) : nullptr;
    double *ovf_c = ovf_i ? ar.try_alloc<double>(ovf_cap) : nullptr;
    const int ovf_n_cap = ovf_c ? ovf_cap : 0;
    if (t == 0) { sh.lap.cnt[2] = 0; sh.lap.cnt[3] = 0; }
    block_sync();
    EdgeCache ea, eb;
    ea.n = eb.n = 0;
    int run = 0;
    for (int start = 0, chunk = 0; start < nr; start += nt, ++chunk) {
        const int i = start + t;
        EdgeCache ec;
        ec.n = 0;
        if (i < nr && nc > 0)
            for_each_edge(rowbox(i), [&](int j, double c) {
                if (chunk < 2 && ec.n < KC) {
                    ec.push(j, c);
                    return;
                }
                const int p = atomicAdd(&sh.lap.cnt[2], 1);
                if (p < ovf_n_cap) {
                    ovf_i[3 * p] = i;
                    ovf_i[3 * p + 1] = ec.n;
                    ovf_i[3 * p + 2] = j;
                    ovf_c[p] = c;
                } else {
                    sh.lap.cnt[3] = 1;
                }
                ++ec.n;
            });
        if (chunk == 0) ea = ec;
        else if (chunk == 1) eb = ec;
        int tot;
        const int pos = block_exclusive_scan(ec.n, sh.lap.wsum, &tot);
        if (i < nr) row_off[i] = run + pos;
        run += tot;
    }
    const int E = run;
    if (t == 0) {
        row_off[nr] = E;
        *n_edges = E;
    }
    int *csr_col = ar.alloc_top<int>(E);
    double *csr_cost = ar.alloc_top<double>(E);
    if (ar.fail) return false;
    block_sync();
    const bool lost = sh.lap.cnt[3] != 0;
    const int n_ovf = lost ? 0 : sh.lap.cnt[2];
    YTA_STAMP(6);
    // pass 2: fill from registers and the overflow list
    if (E > 0) {
        for (int start = 0, chunk = 0; start < nr; start += nt, ++chunk) {
            const int i = start + t;
            if (i >= nr) continue;
            int k = row_off[i];
            auto put = [&](int j, double cost) {
                csr_col[k] = j;
                csr_cost[k] = cost;
                ++k;
                atomicAdd(&col_deg[j], 1);
            };
            const EdgeCache ec = chunk == 0 ? ea : eb;
            const bool captured = chunk < 2 && ec.n <= KC;
            if (captured || !lost) {
                if (chunk < 2 && ec.n > 0) put(ec.c0, ec.w0);
                if (chunk < 2 && ec.n > 1) put(ec.c1, ec.w1);
            } else {
                for_each_edge(rowbox(i), put);   // the overflow list was not enough
            }
        }
        for (int p = t; p < n_ovf; p += nt) {
            const int j = ovf_i[3 * p + 2];
            const int k = row_off[ovf_i[3 * p]] + ovf_i[3 * p + 1];
            csr_col[k] = j;
            csr_cost[k] = ovf_c[p];
            atomicAdd(&col_deg[j], 1);
        }
    }
    block_sync();
    YTA_STAMP(7);
    ar.lo = lo0;   // the grid is dead: the solver's node arrays reuse its space
    return lap_block(nr, nc, row_off, csr_col, csr_cost, col_deg, thresh, X, Y, err, ar, slab,
                     sh.lap);
}

}  // namespace yta
