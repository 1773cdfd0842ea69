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

namespace yta {

// ------------------------------------------------------------------ IoU + appearance (BoT-SORT)
// Cosine distance of two float32 feature rows in float64 (scipy cdist 'cosine':
// 1 - u.v / (|u| |v|)), by one 16-lane row group: every lane accumulates a strided share, the
// row group reduces with DPP.  Returns the value on every lane of the group.
template <int CB = 16, typename ColElem>   // CB: elements per lane loaded before any is used
__device__ __forceinline__ double cosine_dist16(const float *u, ColElem v, int D) {
    const int l16 = lane_id() & 15;
    double d = 0.0, nu = 0.0, nv = 0.0;
    int k = l16;
    for (; k + 16 * (CB - 1) < D; k += 16 * CB) {
        float ua[CB], va[CB];
#pragma unroll
        for (int j = 0; j < CB; ++j) ua[j] = u[k + 16 * j];
#pragma unroll
        for (int j = 0; j < CB; ++j) va[j] = v(k + 16 * j);
#pragma unroll
        for (int j = 0; j < CB; ++j) {   // the same order of operations as the scalar loop
            const double a = (double)ua[j], b = (double)va[j];
            d += a * b;
            nu += a * a;
            nv += b * b;
        }
    }
    for (; k < D; k += 16) {
        const double a = (double)u[k], b = (double)v(k);
        d += a * b;
        nu += a * a;
        nv += b * b;
    }
    d = row_allreduce(RED_SUM, d);
    nu = row_allreduce(RED_SUM, nu);
    nv = row_allreduce(RED_SUM, nv);
    return 1 - d / (sqrt(nu) * sqrt(nv));
}

// One association problem whose cost is BoT-SORT's min(iou cost, gated appearance cost)
// (bot_sort.py:307-322, :355-370):
//   iou_d = 1 - IoU; mask = iou_d > prox; c = fused ? 1 - (1 - iou_d) * score : iou_d
//   emb = max(0, cosine) / 2; emb > app -> 1; masked -> 1; cost = min(c, emb); edge iff < thresh
// With prox < 1 and thresh <= 1 only intersecting pairs can be edges (emb needs iou_d <= prox),
// so candidates come from the column grid (else every pair is visited).  Pass A (a thread per
// row) records direct edges (masked pairs whose IoU cost alone is below thresh) and pending pairs
// (the appearance cost is needed); pass B computes the pending pairs' cosine distances, one
// 16-lane group per pair.  Edges are collected in a list at the arena's top end, then laid out
// as CSR where the grid and the pending list were, each row sorted by column (run-to-run
// deterministic whatever order the atomics produced).
// Arena: the lists take what the grid leaves (LDS), or every pair (the global fallback arena,
// sized by assoc_emb_arena_bytes).
// rowfeat(i) -> const float* (smoothed track feature row); colfeat(j) -> accessor whose (k) is
// the k-th element of column j's (normalised) feature.
__host__ __device__ inline long long assoc_emb_arena_bytes(long long R, long long C) {
    const long long P = R * C;
    const long long grid = 4 * (GRID_MAX_CELLS + 1) + C * (4 + 32 + 8 + 4) + 5 * 16;
    const long long lists = 8 * P + 16 * P + 2 * 16;
    const long long lap = 12 * P + 4 * (R + C) * 3 + 4 * 5 * (R + C + 1) + 10 * 16;
    return (grid + lists > lap + 16 * P ? grid + lists : lap + 16 * P) + 4 * (R + 1) + 4 * C +
           512;
}

constexpr int EMB_PAIRS_SMALL = 4096;   // assoc_block_emb: every pair tested up to this many

template <typename RowBox, typename ColBox, typename ColScore, typename RowFeat, typename ColFeat>
__device__ __forceinline__ bool assoc_block_emb(int nr, RowBox rowbox, int nc, ColBox colbox,
                                                bool fused, ColScore colscore, RowFeat rowfeat,
                                                ColFeat colfeat, int D, double prox, double app,
                                                double thresh, int *X, int *Y, int *err,
                                                int *n_edges, Arena &ar, const LapSlab &slab,
                                                AssocShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x;
    bool use_grid = prox < 1.0 && thresh <= 1.0 && nr > 0 && nc > 0;
    const size_t lo0 = ar.lo;
    // few pairs (prox < 1, thresh <= 1): every pair tested, pairs over the threads, from row and
    // column boxes staged in the arena - one round of loads instead of a grid's five passes
    Box *rst = nullptr, *cst = nullptr;
    double *wst = nullptr;
    if (use_grid && (long long)nr * nc <= EMB_PAIRS_SMALL) {
        rst = ar.try_alloc<Box>(nr);
        cst = ar.try_alloc<Box>(nc);
        wst = ar.try_alloc<double>(nc);
        if (!rst || !cst || !wst) {
            ar.lo = lo0;
            rst = cst = nullptr;
            wst = nullptr;
        } else {
            use_grid = false;
        }
    }
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
    const size_t hi_rows = ar.hi;
    const long long pairs = (long long)nr * nc;
    const long long avail = (long long)ar.hi - (long long)ar.lo - 64;
    long long pcap = avail > 0 ? avail / 24 : 0;
    pcap = pcap < pairs ? pcap : pairs;
    long long ecap = avail > 0 ? (avail - 8 * pcap) / 16 : 0;
    ecap = ecap < pairs ? ecap : pairs;
    int2 *pend = ar.alloc<int2>(pcap);
    int2 *edge = ar.alloc_top<int2>(ecap);
    double *edge_c = ar.alloc_top<double>(ecap);
    if (ar.fail) return false;
    for (int i = t; i <= nr; i += nt) {
        row_off[i] = 0;
        if (rst && i < nr) rst[i] = rowbox(i);
    }
    for (int j = t; j < nc; j += nt) {
        col_deg[j] = 0;
        if (cst) {
            cst[j] = colbox(j);
            wst[j] = fused ? colscore(j) : 1.0;
        }
    }
    if (t == 0) { sh.lap.cnt[0] = 0; sh.lap.cnt[1] = 0; sh.lap.cnt[2] = 0; }
    if (use_grid) {
        block_sync();
        grid_build(
            nc, colbox, [&](int j) { return fused ? colscore(j) : 1.0; }, gv, sh.gs, sh.lap.wsum);
    }
    block_sync();
    YTA_STAMP(1);
    const GridHdr gh = sh.gs.hdr;
    auto push_edge = [&](int i, int j, double c) {
        const int p = atomicAdd(&sh.lap.cnt[1], 1);
        if (p < ecap) {
            edge[p] = make_int2(i, j);
            edge_c[p] = c;
            atomicAdd(&row_off[i + 1], 1);
            atomicAdd(&col_deg[j], 1);
        } else {
            sh.lap.cnt[2] = 1;   // overflow: the caller redoes the frame over the global arena
        }
    };
    auto iou_cost = [&](const Box &rb, const Box &cb, double w, double &d) {
        d = 1 - iou(rb, cb);                                        // matching.py:117
        return fused ? 1 - (1 - d) * w : d;                         // matching.py:216-220
    };
    auto pair = [&](int i, const Box &rb, int j, const Box &cb, double w) {
        double d;
        const double c = iou_cost(rb, cb, w, d);
        if (d > prox) {                                             // emb masked to 1 (:319)
            const double m = np_min(c, 1.0);
            if (m < thresh) push_edge(i, j, m);
        } else {
            const int p = atomicAdd(&sh.lap.cnt[0], 1);
            if (p < pcap) pend[p] = make_int2(i, j);
            else sh.lap.cnt[2] = 1;
        }
    };
    // pass A
    if (rst) {   // a disjoint pair is masked at cost 1 (prox < 1, thresh <= 1): no candidate
        for (int q = t; q < nr * nc; q += nt) {
            const int i = q / nc, j = q - (q / nc) * nc;
            const Box rb = rst[i], cb = cst[j];
            if (intersects(rb, cb)) pair(i, rb, j, cb, wst[j]);
        }
    }
    for (int i = t; i < nr && !rst; i += nt) {
        const Box rb = rowbox(i);
        if (use_grid) {
            grid_query(
                gv, gh, rb, [&](int j, const Box &cb, double w) { pair(i, rb, j, cb, w); },
                [&](int j) {
                    const Box cb = colbox(j);
                    if (intersects(rb, cb)) pair(i, rb, j, cb, fused ? colscore(j) : 1.0);
                });
        } else {
            for (int j = 0; j < nc; ++j) pair(i, rb, j, colbox(j), fused ? colscore(j) : 1.0);
        }
    }
    block_sync();
    YTA_STAMP(2);
    if (sh.lap.cnt[2]) return false;
    const int n_pend = sh.lap.cnt[0];
    // pass B: appearance cost of the pending pairs, one 16-lane group each.  The feature rows'
    // addresses (index chains through the stream's lists) are resolved for every pair first, a
    // thread per pair, where the pending list's reserved span has room
    {
        using CF = decltype(colfeat(0));
        struct RC {
            const float *r;
            CF c;
        };
        // after the pending list's used entries, inside its reserved span
        RC *rcs = reinterpret_cast<RC *>(((uintptr_t)(pend + n_pend) + 15) & ~(uintptr_t)15);
        const bool pre = (uintptr_t)(rcs + n_pend) <= (uintptr_t)(pend + pcap);
        if (pre) {
            batched_for<4>(
                n_pend,
                [&](int p) {
                    const int2 ij = pend[p];
                    return RC{rowfeat(ij.x), colfeat(ij.y)};
                },
                [&](int p, const RC &v) { rcs[p] = v; });
            block_sync();
        }
        const int groups = nt / 16, g = t / 16;
        for (int p = g; p < n_pend; p += groups) {
            const int2 ij = pend[p];
            const RC rc = pre ? rcs[p] : RC{rowfeat(ij.x), colfeat(ij.y)};
            const auto &cf = rc.c;
            const double cd = cosine_dist16<32>(rc.r, cf, D);   // D = 512: one round trip
            if ((lane_id() & 15) == 0) {
                double emb = np_max(0.0, cd) / 2.0;                 // matching.py:164-166
                if (emb > app) emb = 1.0;                           // bot_sort.py:318
                double d;
                const double c = iou_cost(rowbox(ij.x), colbox(ij.y),
                                          fused ? colscore(ij.y) : 1.0, d);
                const double cost = np_min(c, emb);                 // bot_sort.py:320
                if (cost < thresh) push_edge(ij.x, ij.y, cost);
            }
        }
    }
    block_sync();
    YTA_STAMP(3);
    if (sh.lap.cnt[2]) return false;
    const int E = sh.lap.cnt[1];
    if (t == 0) *n_edges = E;
    // row starts: exclusive scan of the counts (per-thread runs of rows)
    {
        const int per = (nr + nt - 1) / nt;
        const int r0 = t * per < nr ? t * per : nr, r1 = r0 + per < nr ? r0 + per : nr;
        int mine = 0;
        for (int r = r0; r < r1; ++r) mine += ald(row_off + r + 1);
        int tot;
        int run = block_exclusive_scan(mine, sh.lap.wsum, &tot);
        block_sync();
        for (int r = r0; r < r1; ++r) {
            const int k = ald(row_off + r + 1);
            row_off[r + 1] = run;   // start of row r: the cursor, its end after the scatter
            run += k;
        }
    }
    ar.lo = lo0;   // the grid and the pending list are dead
    int *csr_col = ar.alloc<int>(E);
    double *csr_cost = ar.alloc<double>(E);
    if (ar.fail) return false;
    block_sync();
    for (int e = t; e < E; e += nt) {
        const int2 ij = edge[e];
        const int k = atomicAdd(&row_off[ij.x + 1], 1);
        csr_col[k] = ij.y;
        csr_cost[k] = edge_c[e];
    }
    block_sync();
    // the row ends came from atomics (L2): drop any stale L1 lines before plain loads of them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ar.hi = hi_rows;   // the edge list is dead
    for (int r = t; r < nr; r += nt) {   // rows in column order (insertion sort, ~1 edge/row)
        const int b = r == 0 ? 0 : ald(row_off + r), en = ald(row_off + r + 1);
        for (int k = b + 1; k < en; ++k) {
            const int cj = csr_col[k];
            const double cc = csr_cost[k];
            int q = k - 1;
            while (q >= b && csr_col[q] > cj) {
                csr_col[q + 1] = csr_col[q];
                csr_cost[q + 1] = csr_cost[q];
                --q;
            }
            csr_col[q + 1] = cj;
            csr_cost[q + 1] = cc;
        }
    }
    block_sync();
    return lap_block(nr, nc, row_off, csr_col, csr_cost, col_deg, thresh, X, Y, err, ar, slab,
                     sh.lap);
}

}  // namespace yta
