// Association on gfx950: sparse candidate-edge extraction + exact sparse linear assignment with
// lapx's cost_limit semantics.
//
// Why sparse is exact.  lap.lapjv(cost, extend_cost=True, cost_limit=t) (matching.py:64) solves the
// (R+C)^2 problem whose off-diagonal blocks cost t/2 and whose dummy block costs 0, i.e. it
// minimises  sum_{matched (i,j)} (c_ij - t)  + const.  A pair with c_ij >= t never improves that
// objective (swapping it for two dummies changes the cost by t - c_ij <= 0), so only "edges"
// c_ij < t matter: the problem is a maximum-weight bipartite matching with weights t - c_ij > 0 on
// a graph that, for tracking, has ~1 edge per row.  Its connected components are independent:
//   * a component that is a single edge is matched outright;
//   * every other component is solved exactly by successive shortest augmenting paths (Dijkstra
//     with potentials, rows in ascending order) where each row owns a private zero-cost dummy
//     column ("stay unmatched"): one wavefront per component, its state in registers (one column
//     per lane) when the component has <= 64 columns + dummies, else in a global-memory slab.
// Candidate edges come from a uniform grid over the column boxes (grid.hpp): only intersecting
// pairs can have c < t for the thresholds ByteTrack uses (t <= 1); t > 1 falls back to all pairs.
// Results equal lapx's whenever the optimum is unique (tie-free); lapx's own tie-breaking is
// unpinned (not installed), see DESIGN.md.
#pragma once
#include "common.hpp"
#include "geometry.hpp"
#include "grid.hpp"

namespace yta {

struct Edge {
    int row;
    int col;
    double cost;
};

// A batch of independent problems of one kind (problem p = stream p).  Every count lives on the
// device; the host only knows capacities.
struct ProblemSet {
    const Box *rows;
    long long rows_stride;
    const int *n_rows;
    int n_rows_stride;          // in ints
    const Box *cols;
    long long cols_stride;
    const double *col_score;    // fuse_score weights (nullptr: plain 1 - IoU)
    long long score_stride;
    const int *n_cols;
    int n_cols_stride;
    // optional grid over an item set; item ids map to columns through remap (nullptr: identity)
    GridHdr *ghdr;              // stride 1 GridHdr per problem
    int *gcell;
    long long gcell_stride;
    int *gitems;
    Box *gboxes;
    int *gbig;
    long long gitems_stride;    // for gitems, gboxes and gbig
    const int *remap;
    long long remap_stride;
    double thresh;
    // edge pool
    Edge *edges;
    long long edges_stride;
    long long edge_cap;
    int *n_edges;
    int n_edges_stride;
    int *err;
    int err_stride;
    // solver workspace + results
    int *ws;
    long long ws_stride;
    double *wsd;
    long long wsd_stride;
    int max_rows, max_cols;
    int *x;                     // row -> col or -1
    long long x_stride;
    int *y;                     // col -> row or -1
    long long y_stride;
};

constexpr int ERR_EDGE_OVERFLOW = 1;
constexpr int ERR_SOLVER = 2;
constexpr int ERR_TRACK_CAPACITY = 4;
constexpr int ERR_DET_CAPACITY = 8;

long long lap_ws_ints(int max_rows, int max_cols, long long edge_cap);
long long lap_ws_doubles(int max_rows, int max_cols, long long edge_cap);

// Launch over one or two problem sets (b may be null): blocks [0, na) solve a, [na, na+nb) b.
hipError_t launch_edges(const ProblemSet &a, int na, const ProblemSet *b, int nb, int max_rows,
                        hipStream_t stream);
hipError_t launch_lap(const ProblemSet &a, int na, const ProblemSet *b, int nb, hipStream_t stream);

}  // namespace yta
