// Association on gfx950: sparse candidate-edge extraction + exact sparse linear assignment with
// lapx's cost_limit semantics.
//
// Why sparse is exact.  lap.lapjv(cost, extend_cost=True, cost_limit=t) (matching.py:64) solves the
// (R+C)^2 problem whose off-diagonal blocks cost t/2 and whose dummy block costs 0, i.e. it
// minimises  sum_{matched (i,j)} (c_ij - t)  + const.  A pair with c_ij >= t never improves that
// objective (swapping it for two dummies changes the cost by t - c_ij <= 0), so only "edges"
// c_ij < t matter: the problem is a maximum-weight bipartite matching with weights t - c_ij > 0 on
// a graph that, for tracking, has ~1 edge per row.  Components of that graph are independent:
//   * a component that is a single edge is matched outright;
//   * every other component is solved exactly by successive shortest augmenting paths (Dijkstra
//     with potentials, rows in ascending order) where each row owns a private zero-cost dummy
//     column ("stay unmatched"), one wavefront per component, state in LDS.
// Results equal lapx's whenever the optimum is unique (tie-free); lapx's own tie-breaking is
// unpinned (not installed), see DESIGN.md.
#pragma once
#include "common.hpp"
#include "geometry.hpp"

namespace yta {

struct Edge {
    int row;
    int col;
    double cost;
};

// Where a batch of independent association problems lives (problem p = blockIdx.y for the edge
// kernel, blockIdx.x for the solver).  Counts are read on the device: the host only knows upper
// bounds.
struct ProblemSet {
    // rows (tracks) and columns (detections) as xyxy boxes
    const Box *rows;
    long long rows_stride;
    const int *n_rows;
    int n_rows_stride;  // in ints
    const Box *cols;
    long long cols_stride;
    const double *col_score;  // fuse_score weights, nullptr for plain 1 - IoU
    long long score_stride;
    const int *n_cols;
    int n_cols_stride;
    double thresh;
    // edge pool
    Edge *edges;
    long long edges_stride;
    long long edge_cap;
    int *n_edges;  // one per problem (stride n_edges_stride ints)
    int n_edges_stride;
    int *err;      // one per problem (bit flags)
    int err_stride;
    // solver workspace + results
    int *ws;            // int workspace per problem
    long long ws_stride;
    double *wsd;        // double workspace per problem (csr costs, big-component slabs)
    long long wsd_stride;
    int max_rows, max_cols;   // capacities used to carve the workspace
    int *x;             // per problem: row -> col or -1
    long long x_stride;
    int *y;             // per problem: col -> row or -1
    long long y_stride;
};

constexpr int ERR_EDGE_OVERFLOW = 1;
constexpr int ERR_SOLVER = 2;
constexpr int ERR_TRACK_CAPACITY = 4;
constexpr int ERR_DET_CAPACITY = 8;

// Per-problem workspace sizes (ints / doubles) for the solver.
long long lap_ws_ints(int max_rows, int max_cols, long long edge_cap);
long long lap_ws_doubles(int max_rows, int max_cols, long long edge_cap);

// Launchers (async on `stream`).
hipError_t launch_edges(const ProblemSet &ps, int n_problems, int max_rows, hipStream_t stream);
hipError_t launch_lap(const ProblemSet &ps, int n_problems, hipStream_t stream);

}  // namespace yta
