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
    const long long grid = 4 * (GRID_MAX_CELLS + 1) + C * (4 + 32 + 4) + 4 * 16;
    const long long top = 4 * (R + 1) + 4 * C + 12 * E + 3 * 16;
    const long long lap = 4 * (R + C) * 3 + 4 * 5 * (R + C + 1) + 8 * 16;
    return (grid > lap ? grid : lap) + top + 256;
}

// One association problem of the calling block.  rowbox(i) / colbox(j): boxes; colscore(j): the
// fuse_score weight (only called when `fused`).  X[nr] / Y[nc] receive the assignment, edge count
// in *n_edges (thread 0).  Returns false if the arena is exhausted.
template <typename RowBox, typename ColBox, typename ColScore>
__device__ __forceinline__ bool assoc_block(int nr, RowBox rowbox, int nc, ColBox colbox,
                                            bool fused, ColScore colscore, double thresh, int *X,
                                            int *Y, int *err, int *n_edges, Arena &ar,
                                            const LapSlab &slab, AssocShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x;
    const bool use_grid = thresh <= 1.0;
    const size_t lo0 = ar.lo;
    GridView gv{nullptr, nullptr, nullptr, nullptr, nullptr};
    if (use_grid && nr > 0 && nc > 0) {
        gv.cell_start = ar.alloc<int>(GRID_MAX_CELLS + 1);
        gv.ids = ar.alloc<int>(nc);
        gv.boxes = ar.alloc<Box>(nc);
        gv.big = ar.alloc<int>(nc);
    }
    int *row_off = ar.alloc_top<int>(nr + 1);
    int *col_deg = ar.alloc_top<int>(nc);
    if (ar.fail) return false;
    for (int j = t; j < nc; j += nt) col_deg[j] = 0;
    if (use_grid && nr > 0 && nc > 0) grid_build(nc, colbox, gv, sh.gs, sh.lap.wsum);
    const GridHdr gh = sh.gs.hdr;

    // every candidate (j, cost) of row box rb with cost < thresh
    auto for_each_edge = [&](const Box &rb, auto &&f) {
        auto score = [&](const Box &cb, int j) {
            const double dist = 1 - iou(rb, cb);
            const double cost = fused ? 1 - (1 - dist) * colscore(j) : dist;
            if (cost < thresh) f(j, cost);
        };
        if (use_grid) {
            grid_query(
                gv, gh, rb,
                [&](int j, const Box &cb) {
                    if (intersects(rb, cb)) score(cb, j);
                },
                [&](int j) {
                    const Box cb = colbox(j);
                    if (intersects(rb, cb)) score(cb, j);
                });
        } else {
            for (int j = 0; j < nc; ++j) score(colbox(j), j);
        }
    };
    // pass 1: edges per row -> row offsets
    int run = 0;
    for (int start = 0; start < nr; start += nt) {
        const int i = start + t;
        int cnt = 0;
        if (i < nr && nc > 0) for_each_edge(rowbox(i), [&](int, double) { ++cnt; });
        int tot;
        const int pos = block_exclusive_scan(cnt, sh.lap.wsum, &tot);
        if (i < nr) row_off[i] = run + pos;
        run += tot;
    }
    if (t == 0) {
        row_off[nr] = run;
        *n_edges = run;
    }
    const int E = run;
    int *csr_col = ar.alloc_top<int>(E);
    double *csr_cost = ar.alloc_top<double>(E);
    if (ar.fail) return false;
    block_sync();
    // pass 2: fill (same rows per thread, same candidate set)
    if (E > 0) {
        for (int i = t; i < nr; i += nt) {
            int k = row_off[i];
            for_each_edge(rowbox(i), [&](int j, double cost) {
                csr_col[k] = j;
                csr_cost[k] = cost;
                ++k;
                atomicAdd(&col_deg[j], 1);
            });
        }
    }
    block_sync();
    ar.lo = lo0;   // the grid is dead: the solver's node arrays reuse its space
    return lap_block(nr, nc, row_off, csr_col, csr_cost, col_deg, thresh, X, Y, err, ar, slab,
                     sh.lap);
}

}  // namespace yta
