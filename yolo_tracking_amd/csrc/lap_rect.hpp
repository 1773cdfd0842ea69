// Dense rectangular linear assignment on one block: the exact optimum of
//   boxmot/utils/association.py:20-28  lap.lapjv(cost, extend_cost=True)
// for a zero-padded problem whose real block has rows <= cols (every row is matched; the padding
// rows take the columns left over at cost 0, so the padded optimum restricted to the real rows is
// the rectangular optimum).  Used where the padded solve's result does not depend on how lapjv
// breaks exact ties: the OCSORT-family first round when trackers >= detections,
// and the -IoU rounds (BYTE / OCR), whose surviving pairs are filtered by IoU >= threshold and
// re-sorted (np.setdiff1d).  Everything else keeps the lapjv replay of lap_dense.hpp.
//
// Algorithm (shortest augmenting paths with a warm start, duals u / v, v = 0 on free columns):
//   1. row pre-pass (chip-wide kernel, or this block for small problems): u_i = min_j c_ij, its
//      first column, and s2_i = second minimum - minimum (a lower bound of row i's reduced costs
//      off its own column);
//   2. every row claims its argmin column; the lowest claiming row keeps it (tight, feasible);
//      with the bidding arrays (RectWs::av, the OCSORT-family first round): rounds of bids instead
//      (rect_arr below), the first from the pre-pass, which leave fewer free rows and shorter
//      searches;
//   3. every other row is augmented by Dijkstra over the columns, one block-wide step per row
//      relaxation.  Pruning: the row of an assigned column j is only relaxed while
//      spc_j + s2_row < B, B = the cheapest free column reached so far; any other row can only
//      produce distances >= B and cannot change the result.  The search stops when no prunable
//      column is left below B; every column below B gets the usual dual update.  s2 stays a valid
//      lower bound through the dual updates (u_i += d  =>  s2_i -= d) and is reset to 0 on the
//      augmenting path (refreshed exactly whenever the row is relaxed).
// Each thread owns the columns j = t + q * blockDim (q < CPT): distance, price, owner row and
// bound live in registers; a step is one coalesced row read + one block argmin (one barrier).
#pragma once
#include <float.h>
#include <limits.h>

#include "common.hpp"

namespace yta {

// The solver's view of the cost matrix: element (i, j) at m[i * rs + j * cs] (a transposed view
// swaps the strides), negated when `neg`.
struct RectMat {
    const double *m;
    int rows, cols;
    long long rs, cs;
    bool neg;
    __device__ __forceinline__ double at(int i, int j) const {
        const double v = ((const __attribute__((address_space(1))) double *)m)[i * rs + j * cs];
        return neg ? -v : v;
    }
};

// Work arrays (LDS or global): rect_ws_bytes(rows, cols, duals) bytes, 8-aligned.  `duals`: keep
// the column duals on return (the transposed first round's uniqueness certificate); they cost 8 B
// a column, which would push a 4096 x 4096 problem's arrays out of LDS.
struct RectWs {
    double *u;          // rows
    float *s2;          // rows: the bound, rounded down (still a lower bound)
    double *v;          // cols: the column duals on return (<= 0, 0 on free columns), or nullptr
    int *x, *fl;        // rows: assigned column, free-row list
    int *path, *yw;     // cols: predecessor row, owner row (authoritative copy)
    // bidding rounds before the searches (rect_arr; nullptr: the claims only), global memory:
    double *av = nullptr;               // cols: column duals during the rounds (LDS when it fits)
    unsigned long long *abid = nullptr; // cols: the largest bid of the round
    int *atgt = nullptr;                // rows: the column a free row bids for
    double *adel = nullptr;             // rows: its bid (second minimum - minimum)
    int av_lds = 0;                     // av is in LDS
    // the state left by the chip-wide bidding rounds (ArrState) to start the searches from
    const int *sx = nullptr, *syw = nullptr;
    const double *su = nullptr, *sv = nullptr;
    const float *ss2 = nullptr;
};
// The bidding rounds' arrays (rect_arr_ws), 16-B aligned pieces.
__host__ __device__ inline long long arr_ws_bytes(long long rows, long long cols) {
    return cols * 16 + rows * 12 + 64;
}
__host__ __device__ inline void rect_arr_ws(unsigned char *base, int rows, int cols, RectWs &w) {
    w.av = reinterpret_cast<double *>(base);
    w.abid = reinterpret_cast<unsigned long long *>(w.av + cols);
    w.adel = reinterpret_cast<double *>(w.abid + cols);
    w.atgt = reinterpret_cast<int *>(w.adel + rows);
}
__host__ __device__ inline long long rect_ws_bytes(long long rows, long long cols,
                                                   bool duals = false) {
    return rows * 20 + cols * (duals ? 16 : 8) + 64;
}
__host__ __device__ inline RectWs rect_ws(unsigned char *base, int rows, int cols,
                                          bool duals = false) {
    RectWs w;
    w.u = reinterpret_cast<double *>(base);
    w.x = reinterpret_cast<int *>(w.u + rows);
    w.fl = w.x + rows;
    w.s2 = reinterpret_cast<float *>(w.fl + rows);
    w.path = reinterpret_cast<int *>(w.s2 + rows);
    w.yw = w.path + cols;
    // 8-aligned: 20 * rows + 8 * cols bytes precede it (+ 4 when rows is odd)
    const size_t vo = ((size_t)20 * rows + (size_t)8 * cols + 7) & ~(size_t)7;
    w.v = duals ? reinterpret_cast<double *>(base + vo) : nullptr;
    return w;
}
constexpr int RECT_CPT_MAX = 32;

// One wave: minimum of row i (first column on ties), and second minimum - minimum (a float s2:
// rounded down, so still a lower bound).
__device__ __forceinline__ void store_s2(double *s2, int i, double d) { s2[i] = d; }
__device__ __forceinline__ void store_s2(float *s2, int i, double d) { s2[i] = __double2float_rd(d); }
template <typename S2T>
__device__ __forceinline__ void rect_row_pre(const RectMat M, int i, double *u, int *x, S2T *s2) {
    const int lane = lane_id();
    double m1 = INFINITY, m2 = INFINITY;
    int k1 = INT_MAX;
    for (int j = lane; j < M.cols; j += WAVE) {
        const double c = M.at(i, j);
        if (c < m1) { m2 = m1; m1 = c; k1 = j; }
        else if (c < m2) m2 = c;
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const double om1 = __shfl_xor(m1, s), om2 = __shfl_xor(m2, s);
        const int ok1 = __shfl_xor(k1, s);
        const bool other = om1 < m1 || (om1 == m1 && ok1 < k1);
        const double lose = other ? m1 : om1;
        const double m2w = other ? om2 : m2;
        m2 = lose < m2w ? lose : m2w;
        m1 = other ? om1 : m1;
        k1 = other ? ok1 : k1;
    }
    if (lane == 0) {
        u[i] = m1;
        x[i] = k1 == INT_MAX ? 0 : k1;
        store_s2(s2, i, m2 - m1);
    }
}

struct RectRed {
    double b, ma, mo;
    int sink, key;   // key = ja << 16 | ya (columns, rows < 32768)
};
struct RectShared {
    RectRed slot[2][16];
    int wsum[32];
};

__device__ __forceinline__ void rect_lex_min(double &v, int &k, double ov, int ok) {
    if (ov < v || (ov == v && ok < k)) { v = ov; k = ok; }
}
template <int CTRL>
__device__ __forceinline__ void dpp_lex_min(double &v, int &k) {
    const double ov = dpp_f64<CTRL>(v);
    const int ok = dpp_i32<CTRL>(k);
    rect_lex_min(v, k, ov, ok);
}
template <int CTRL>
__device__ __forceinline__ void dpp_fmin(double &v) {
    const double ov = dpp_f64<CTRL>(v);
    v = ov < v ? ov : v;
}
// Wave-uniform lexicographic minima of (a, ka), (b, kb) and the minimum of m: DPP within each
// 16-lane row (quad_perm, row_ror), then the four row results by readlane.
__device__ __forceinline__ void wave_rect_reduce(double &a, int &ka, double &b, int &kb, double &m) {
    dpp_lex_min<0xB1>(a, ka); dpp_lex_min<0xB1>(b, kb); dpp_fmin<0xB1>(m);
    dpp_lex_min<0x4E>(a, ka); dpp_lex_min<0x4E>(b, kb); dpp_fmin<0x4E>(m);
    dpp_lex_min<0x124>(a, ka); dpp_lex_min<0x124>(b, kb); dpp_fmin<0x124>(m);
    dpp_lex_min<0x128>(a, ka); dpp_lex_min<0x128>(b, kb); dpp_fmin<0x128>(m);
    double ra = readlane_f64(a, 0), rb = readlane_f64(b, 0), rm = readlane_f64(m, 0);
    int rka = __builtin_amdgcn_readlane(ka, 0), rkb = __builtin_amdgcn_readlane(kb, 0);
#pragma unroll
    for (int L = 16; L < WAVE; L += 16) {
        rect_lex_min(ra, rka, readlane_f64(a, L), __builtin_amdgcn_readlane(ka, L));
        rect_lex_min(rb, rkb, readlane_f64(b, L), __builtin_amdgcn_readlane(kb, L));
        const double om = readlane_f64(m, L);
        rm = om < rm ? om : rm;
    }
    a = ra; ka = rka; b = rb; kb = rkb; m = rm;
}

// ---- bidding rounds (augmenting row reduction, all free rows at once)
// A free row i bids for the column j1 of its smallest reduced cost c_ij - v_j with
// delta = (second smallest) - (smallest); each column goes to its largest bid (lowest row on equal
// bids), whose column dual drops by that delta: the winner is then tight on j1 and on its second
// column (u_i = c_ij1 - v_j1, s2_i = 0), every dual stays feasible (v only decreases, so every
// other row's reduced costs only grow), and a displaced owner becomes free with its old u_i, still
// a lower bound of its reduced costs.  So after any number of rounds the state is what the searches
// start from (duals feasible, every assigned edge tight, v = 0 on unassigned columns: a column
// once taken stays taken), and the searches finish an optimum.  Round 1 takes the bids from the
// row pre-pass (v = 0); later rounds rescan the free rows, one wave a row.  On the OCSORT-family
// first rounds the rounds leave 2-10x fewer rows and row scans to the searches
// (tools/sim_lap_parallel.py).  Rounds stop when a round frees no row (bids that only displace).
constexpr int ARR_ROUNDS = 24;

__device__ __forceinline__ unsigned long long arr_key(double d) {
    return (unsigned long long)__double_as_longlong(d) + 1ull;   // d >= 0: bit order = order
}
__device__ __forceinline__ void top2_push(double c, int j, double &m1, int &k1, double &m2, int &k2) {
    if (c < m1) { m2 = m1; k2 = k1; m1 = c; k1 = j; }
    else if (c < m2) { m2 = c; k2 = j; }
}
// One wave: the smallest and second smallest reduced cost c_ij - v_j of row i and their columns
// (lowest column on ties); wave-uniform results.
// Loads are unconditional (index clamped, value masked): a load under `j < cols` becomes a branch
// per element with its own wait, one round trip per element.  AS: address space of v (3 = LDS).
// Merge of two (smallest, second smallest) pairs with their columns, lexicographic (value, column).
__device__ __forceinline__ void top2_merge(double &m1, int &k1, double &m2, int &k2, double o1, int q1,
                                           double o2, int q2) {
    if (o1 < m1 || (o1 == m1 && q1 < k1)) {          // the other's first wins
        if (m1 < o2 || (m1 == o2 && k1 < q2)) { m2 = m1; k2 = k1; }
        else { m2 = o2; k2 = q2; }
        m1 = o1; k1 = q1;
    } else if (o1 < m2 || (o1 == m2 && q1 < k2)) {
        m2 = o1; k2 = q1;
    }
}
// Columns [jb, je) of row i, lanes strided; wave-uniform results.
template <int AS>
__device__ __forceinline__ void rect_row_bid_range(const RectMat M, int i, const double *v, int jb,
                                                   int je, double &u1, int &j1, double &u2, int &j2) {
    typedef const __attribute__((address_space(AS))) double *VP;
    const VP vp = (VP)v;
    const int lane = lane_id();
    constexpr int CH = 16;
    double m1 = INFINITY, m2 = INFINITY;
    int k1 = INT_MAX, k2 = INT_MAX;
    for (int j0 = jb; j0 < je; j0 += CH * WAVE) {
        double c[CH], vv[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int j = j0 + k * WAVE + lane, jc = j < je ? j : je - 1;
            c[k] = M.at(i, jc);
            vv[k] = vp[jc];
        }
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int j = j0 + k * WAVE + lane;
            top2_push(j < je ? c[k] - vv[k] : INFINITY, j, m1, k1, m2, k2);
        }
    }
#pragma unroll
    for (int s = 1; s < WAVE; s <<= 1) {
        const double o1 = __shfl_xor(m1, s), o2 = __shfl_xor(m2, s);
        const int q1 = __shfl_xor(k1, s), q2 = __shfl_xor(k2, s);
        top2_merge(m1, k1, m2, k2, o1, q1, o2, q2);
    }
    u1 = m1; j1 = k1; u2 = m2; j2 = k2;
}
template <int AS>
__device__ __forceinline__ void rect_row_bid(const RectMat M, int i, const double *v, double &u1,
                                             int &j1, double &u2, int &j2) {
    rect_row_bid_range<AS>(M, i, v, 0, M.cols, u1, j1, u2, j2);
}

// Block-wide; the rows' pre-pass in pu / px / ps2.  On return: w.x, w.u, w.s2, w.yw and w.av
// describe a feasible partial assignment (w.path = INT_MAX on every column).
template <typename S2T>
__device__ __noinline__ void rect_arr(const RectMat M, const double *pu, const int *px,
                                      const S2T *ps2, RectWs w, RectShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x, wid = t / WAVE, nw = nt / WAVE;
    const int rows = M.rows, cols = M.cols;
    for (int j = t; j < cols; j += nt) {
        w.abid[j] = 0ull;
        w.path[j] = INT_MAX;
        w.yw[j] = -1;
        w.av[j] = 0.0;
    }
    for (int i = t; i < rows; i += nt) {   // pu / px / ps2 may be w.u / w.x / w.s2: read first
        const double d = (double)ps2[i], ui = pu[i];
        const int xi = px[i];
        w.x[i] = -1;
        w.u[i] = ui;
        w.s2[i] = 0.0f;
        w.atgt[i] = xi;
        w.adel[i] = d < INFINITY ? d : 0.0;
    }
    block_sync();
    int nbid = rows;
    for (int round = 0; round < ARR_ROUNDS; ++round) {
        YTA_COUNT(106);
        if (round > 0) {   // the free rows bid under the current duals
            for (int k = wid; k < nbid; k += nw) {
                const int i = w.fl[k];
                double u1, u2;
                int j1, j2;
                if (w.av_lds) rect_row_bid<3>(M, i, w.av, u1, j1, u2, j2);
                else rect_row_bid<1>(M, i, w.av, u1, j1, u2, j2);
                double d = u2 - u1;
                if (!(d < INFINITY) || j1 == INT_MAX) d = 0.0;
                int tg = j1 == INT_MAX ? 0 : j1;
                // a tie on an owned column: the other tight column when it is free
                if (d == 0.0 && j2 != INT_MAX && w.yw[tg] >= 0 && w.yw[j2] < 0) tg = j2;
                if (lane_id() == 0) {
                    w.u[i] = u1;
                    w.atgt[i] = tg;
                    w.adel[i] = d;
                }
            }
            block_sync();
        }
        for (int k = t; k < nbid; k += nt) {
            const int i = round ? w.fl[k] : k;
            atomicMax(&w.abid[w.atgt[i]], arr_key(w.adel[i]));
        }
        block_sync();
        for (int k = t; k < nbid; k += nt) {
            const int i = round ? w.fl[k] : k;
            const int j = w.atgt[i];
            if (w.abid[j] == arr_key(w.adel[i])) atomicMin(&w.path[j], i);
        }
        block_sync();
        for (int k = t; k < nbid; k += nt) {   // one winner per column; bidders own nothing
            const int i = round ? w.fl[k] : k;
            const int j = w.atgt[i];
            if (w.path[j] != i) continue;
            const int old = w.yw[j];
            if (old >= 0) w.x[old] = -1;
            w.yw[j] = i;
            w.x[i] = j;
            const double vj = w.av[j] - w.adel[i];
            w.av[j] = vj;
            w.u[i] = M.at(i, j) - vj;
            w.s2[i] = 0.0f;
        }
        block_sync();
        for (int k = t; k < nbid; k += nt) {
            const int j = w.atgt[round ? w.fl[k] : k];
            w.abid[j] = 0ull;
            w.path[j] = INT_MAX;
        }
        block_sync();
        const int nf = block_compact(rows, sh.wsum, [&](int i) { return w.x[i] < 0; },
                                     [&](int i, int pos) { w.fl[pos] = i; });
        block_sync();
        if (nf == 0 || (round > 0 && nf >= nbid)) break;
        nbid = nf;
    }
}

// ---- the same rounds chip-wide (large first rounds: C4 / C5).  In one block, 8 waves rescan the
// free rows (~100 per C5 frame) one after another; here every free row's wave runs at once on its
// own CU.  One round = arr_scan (grid: each free row's bid, atomicMax into its column) + arr_apply
// (block per stream: winners, displaced owners, the new free list); arr_round0 (block) takes the
// first round's bids from the row pre-pass.  The state lives in global memory (ArrState) and
// lap_rect_body starts its searches from it (RectWs::sx ...).  A bid is one 64-bit key: the bid
// rounded down to float in the high half (any winner rule keeps the duals feasible, as the winner
// pays its own exact bid), the complement of the row in the low half (lowest row on equal keys).
struct ArrState {
    int *hdr;                   // [0] rounds on, [1] free rows, [2] state valid, [3] rounds run
    double *av, *au, *adel;     // cols: duals; rows: u, bid
    unsigned long long *abid;   // cols: the round's largest key
    int *ayw, *ax, *afl, *atgt; // cols: owner; rows: column, free list, bid column
    float *as2;                 // rows: bound
};
__host__ __device__ inline long long arr_state_bytes(long long rows, long long cols) {
    return 64 + cols * 20 + rows * 32 + 64;
}
__device__ __forceinline__ ArrState arr_state(unsigned char *base, int rows, int cols) {
    ArrState st;
    st.hdr = reinterpret_cast<int *>(base);
    st.av = reinterpret_cast<double *>(base + 64);
    st.abid = reinterpret_cast<unsigned long long *>(st.av + cols);
    st.au = reinterpret_cast<double *>(st.abid + cols);
    st.adel = st.au + rows;
    st.ayw = reinterpret_cast<int *>(st.adel + rows);
    st.ax = st.ayw + cols;
    st.afl = st.ax + rows;
    st.atgt = st.afl + rows;
    st.as2 = reinterpret_cast<float *>(st.atgt + rows);
    return st;
}
__device__ __forceinline__ unsigned long long arr_bid_key(double d, int i) {
    return ((unsigned long long)__float_as_uint(__double2float_rd(d)) << 32) | (unsigned)(~i);
}
constexpr int ARR_CHIP_ROUNDS = 8;   // rounds launched after round 0 (idle ones return at once)

// Winners of the bids of rows list[0..n) (list == nullptr: rows 0..n), then the new free list.
// Block-wide.  Returns the number of free rows.
__device__ __forceinline__ int arr_settle(const RectMat M, const ArrState &st, const int *list, int n,
                                         int *wsum) {
    const int t = threadIdx.x, nt = blockDim.x;
    for (int k = t; k < n; k += nt) {   // one winner per column; bidders own nothing
        const int i = list ? list[k] : k;
        const int j = st.atgt[i];
        if (st.abid[j] != arr_bid_key(st.adel[i], i)) continue;
        const int old = st.ayw[j];
        if (old >= 0) st.ax[old] = -1;
        st.ayw[j] = i;
        st.ax[i] = j;
        const double vj = st.av[j] - st.adel[i];
        st.av[j] = vj;
        st.au[i] = M.at(i, j) - vj;
        st.as2[i] = 0.0f;
    }
    block_sync();
    for (int k = t; k < n; k += nt) st.abid[st.atgt[list ? list[k] : k]] = 0ull;
    block_sync();
    // the list is read above; the compaction may overwrite it (it is st.afl)
    const int nf = block_compact(M.rows, wsum, [&](int i) { return st.ax[i] < 0; },
                                 [&](int i, int pos) { st.afl[pos] = i; });
    block_sync();
    return nf;
}

// Round 0, block per stream: state from the row pre-pass, every row bids for its argmin column.
__device__ __forceinline__ void arr_round0(const RectMat M, const double *pu, const int *px,
                                           const double *ps2, const ArrState &st, int *wsum) {
    const int t = threadIdx.x, nt = blockDim.x;
    for (int j = t; j < M.cols; j += nt) {
        st.av[j] = 0.0;
        st.abid[j] = 0ull;
        st.ayw[j] = -1;
    }
    for (int i = t; i < M.rows; i += nt) {
        const double d = ps2[i];
        st.ax[i] = -1;
        st.au[i] = pu[i];
        st.as2[i] = 0.0f;
        st.atgt[i] = px[i];
        st.adel[i] = d >= 0.0 && d < INFINITY ? d : 0.0;
    }
    block_sync();
    for (int i = t; i < M.rows; i += nt) atomicMax(&st.abid[st.atgt[i]], arr_bid_key(st.adel[i], i));
    block_sync();
    const int nf = arr_settle(M, st, nullptr, M.rows, wsum);
    if (t == 0) {
        st.hdr[0] = nf > 0;
        st.hdr[1] = nf;
        st.hdr[2] = 1;
        st.hdr[3] = 1;
    }
}

// One block: the bid of free-list entry k, each wave over its share of the columns (one or two
// chunks of loads in flight per lane instead of five for a whole C5 row on one wave).
struct ArrTop2 {
    double m1, m2;
    int k1, k2;
};
__device__ __forceinline__ void arr_scan_row(const RectMat M, const ArrState &st, int k,
                                             ArrTop2 *slot) {
    const int nw = blockDim.x / WAVE, wid = threadIdx.x / WAVE;
    const int i = st.afl[k];
    const int per = (M.cols + nw - 1) / nw;
    const int jb = wid * per < M.cols ? wid * per : M.cols;
    const int je = jb + per < M.cols ? jb + per : M.cols;
    double u1, u2;
    int j1, j2;
    rect_row_bid_range<1>(M, i, st.av, jb, je, u1, j1, u2, j2);
    if (lane_id() == 0) slot[wid] = ArrTop2{u1, u2, j1, j2};
    __syncthreads();
    if (threadIdx.x == 0) {
        double m1 = INFINITY, m2 = INFINITY;
        int k1 = INT_MAX, k2 = INT_MAX;
        for (int w = 0; w < nw; ++w) top2_merge(m1, k1, m2, k2, slot[w].m1, slot[w].k1, slot[w].m2, slot[w].k2);
        double d = m2 - m1;
        if (!(d >= 0.0 && d < INFINITY) || k1 == INT_MAX) d = 0.0;
        int tg = k1 == INT_MAX ? 0 : k1;
        if (d == 0.0 && k2 != INT_MAX && st.ayw[tg] >= 0 && st.ayw[k2] < 0) tg = k2;
        st.au[i] = m1;
        st.atgt[i] = tg;
        st.adel[i] = d;
        atomicMax(&st.abid[tg], arr_bid_key(d, i));
    }
    __syncthreads();   // the slots are reused by the block's next row
}

// Block per stream after arr_scan: settle the round; stop when it freed no row.
__device__ __forceinline__ void arr_apply(const RectMat M, const ArrState &st, int *wsum) {
    const int n = st.hdr[1];
    block_sync();   // every thread read the header
    const int nf = arr_settle(M, st, st.afl, n, wsum);
    if (threadIdx.x == 0) {
        st.hdr[0] = nf > 0 && nf < n;
        st.hdr[1] = nf;
        st.hdr[3] += 1;
    }
}

// Solve.  pre_u / pre_x / pre_s2: the row pre-pass (global, or nullptr: computed here).  Returns 0,
// or -2 if a row cannot reach a free column (rows > cols, or NaN costs).  On return w.x[i] is the
// column of row i.  All threads of the block must call it; blockDim.x * CPT >= M.cols.
template <int CPT>
__device__ __forceinline__ int lap_rect_body(const RectMat M, const double *pre_u, const int *pre_x,
                                           const double *pre_s2, RectWs w, RectShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x, wid = t / WAVE, nw = nt / WAVE;
    constexpr int CH = CPT <= 16 ? CPT : 8;   // loads in flight per chunk
    const int rows = M.rows, cols = M.cols;
    if (rows <= 0) return 0;
    if (rows > cols) return -2;
    // ---- 1. row pre-pass (when not supplied) and 2. claims
    const bool chip = w.sx != nullptr;   // start from the chip-wide rounds' state (ArrState)
    const bool own_pre = !chip && pre_u == nullptr;   // the bounds then already in w.s2 (floats)
    if (own_pre) {
        for (int i = wid; i < rows; i += nw) rect_row_pre(M, i, w.u, w.x, w.s2);
        pre_u = w.u; pre_x = w.x;
        block_sync();
    }
    const bool arr = !chip && w.av != nullptr;
    if (chip) {
        for (int i = t; i < rows; i += nt) {
            w.x[i] = w.sx[i];
            w.u[i] = w.su[i];
            w.s2[i] = w.ss2[i];
        }
        for (int j = t; j < cols; j += nt) w.yw[j] = w.syw[j];
    } else if (arr) {
#ifdef YTA_STAMPS
        const unsigned long long ta = wall_clock64();
#endif
        if (own_pre) rect_arr(M, pre_u, pre_x, (const float *)w.s2, w, sh);
        else rect_arr(M, pre_u, pre_x, pre_s2, w, sh);
#ifdef YTA_STAMPS
        if (blockIdx.x == 0 && t == 0) g_stamps[107] += wall_clock64() - ta;
#endif
    } else {   // claims: every row its argmin column, the lowest row keeps it
        for (int j = t; j < cols; j += nt) w.path[j] = INT_MAX;
        block_sync();
        for (int i = t; i < rows; i += nt) atomicMin(&w.path[pre_x[i]], i);
        block_sync();
        for (int i = t; i < rows; i += nt) {
            const int xi = pre_x[i];
            const double ui = pre_u[i];
            const bool won = w.path[xi] == i;
            w.u[i] = ui;
            if (!own_pre) w.s2[i] = __double2float_rd(pre_s2[i]);
            w.x[i] = won ? xi : -1;
        }
    }
    block_sync();
    // s2c: the bound of each column's row, as a float rounded down (still a lower bound)
    double v[CPT], spc[CPT];
    float s2c[CPT];
    int y[CPT];
    unsigned rel = 0u;
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const int j = t + q * nt;
        v[q] = 0.0;
        y[q] = -1;
        s2c[q] = 0.0f;
        if (j < cols) {
            if (chip) {
                v[q] = w.sv[j];
                y[q] = w.syw[j];
            } else if (arr) {
                v[q] = w.av[j];
                y[q] = w.yw[j];
            } else {
                const int r = w.path[j];
                y[q] = r == INT_MAX ? -1 : r;
                w.yw[j] = y[q];
            }
            if (y[q] >= 0) s2c[q] = w.s2[y[q]];
        }
    }
    YTA_STAMP_ABS(104);
    const int nfree = block_compact(rows, sh.wsum, [&](int i) { return w.x[i] < 0; },
                                    [&](int i, int pos) { w.fl[pos] = i; });
    block_sync();
    int par = 0;
    // ---- 3. augment the free rows
    for (int f = 0; f < nfree; ++f) {
        const int cur = w.fl[f];
        YTA_COUNT(100);
#pragma unroll
        for (int q = 0; q < CPT; ++q) spc[q] = INFINITY;
        rel = 0u;
        int i = cur, xi = -1;
        double base = 0.0, ui = w.u[cur], bprev = INFINITY, B = INFINITY;
        int sink = -1;
        bool done = false;
        for (int guard = 0; guard <= rows && !done; ++guard) {
            YTA_COUNT(101);
#ifdef YTA_STAMPS
            const unsigned long long ts0 = wall_clock64();
#endif
            double lb = INFINITY, lma = INFINITY, lmo = INFINITY;
            int lsink = INT_MAX, lja = INT_MAX, lya = -1;
            // row costs in chunks of 8 columns (loads of a chunk in flight together)
#pragma unroll
            for (int q0 = 0; q0 < CPT; q0 += CH) {
                double c[CH];
#pragma unroll
                for (int k = 0; k < CH; ++k) {   // unconditional loads (see rect_row_bid)
                    const int j = t + (q0 + k) * nt;
                    c[k] = M.at(i, j < cols ? j : cols - 1);
                }
#pragma unroll
                for (int k = 0; k < CH; ++k) {
                    const int q = q0 + k;
                    const int j = t + q * nt;
                    if (j >= cols) continue;
                    const double rc = c[k] - ui - v[q];
                    if (j != xi) lmo = rc < lmo ? rc : lmo;
                    if ((rel >> q) & 1u) continue;
                    const double r = base + rc;
                    if (r < spc[q]) {
                        spc[q] = r;
                        w.path[j] = i;
                    }
                    if (y[q] < 0) {
                        if (spc[q] < lb) { lb = spc[q]; lsink = j; }
                    } else if (spc[q] + (double)s2c[q] < bprev && spc[q] < lma) {
                        lma = spc[q]; lja = j; lya = y[q];
                    }
                }
            }
#ifdef YTA_STAMPS
            const unsigned long long ts1 = wall_clock64();
            if (blockIdx.x == 0 && t == 0) g_stamps[102] += ts1 - ts0;
#endif
            // wave (DPP), then block: lexicographic (B, sink), (ma, ja) with ya packed into the
            // key, min mo; one barrier (the slots alternate between steps)
            int lkey = lja == INT_MAX ? INT_MAX : ((lja << 16) | lya);
            wave_rect_reduce(lb, lsink, lma, lkey, lmo);
            if (lane_id() == 0) sh.slot[par][wid] = RectRed{lb, lma, lmo, lsink, lkey};
            __syncthreads();
            B = INFINITY;
            sink = INT_MAX;
            double ma = INFINITY, mo = INFINITY;
            int key = INT_MAX;
            for (int k = 0; k < nw; ++k) {
                const RectRed r = sh.slot[par][k];
                rect_lex_min(B, sink, r.b, r.sink);
                rect_lex_min(ma, key, r.ma, r.key);
                mo = r.mo < mo ? r.mo : mo;
            }
            const int ja = key == INT_MAX ? INT_MAX : key >> 16, ya = key & 0xFFFF;
            par ^= 1;
#ifdef YTA_STAMPS
            if (blockIdx.x == 0 && t == 0) g_stamps[103] += wall_clock64() - ts1;
#endif
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                const int j = t + q * nt;
                if (j == xi) s2c[q] = __double2float_rd(mo);   // exact for the current duals
                if (ma < B && j == ja) rel |= 1u << q;
            }
            if (!(ma < B)) { done = true; break; }
            i = ya;
            xi = ja;
            base = ma;
            bprev = B;
            ui = w.u[ya];
        }
        if (!done || !(B < INFINITY) || sink == INT_MAX) return -2;
        // dual update of every column below B (and of its row)
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int j = t + q * nt;
            if (j < cols && y[q] >= 0 && spc[q] < B) {
                const double dl = B - spc[q];
                w.u[y[q]] += dl;
                s2c[q] = __double2float_rd((double)s2c[q] - dl);
                v[q] -= dl;
            }
        }
        if (t == 0) w.u[cur] += B;
        block_sync();
        if (t == 0) {   // flip the alternating path back to the source row
            int j = sink;
            for (int steps = 0; steps <= rows; ++steps) {
                const int r = w.path[j];
                w.yw[j] = r;
                const int nx = w.x[r];
                w.x[r] = j;
                if (r == cur) break;
                j = nx;
            }
        }
        block_sync();
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int j = t + q * nt;
            if (j < cols) {
                const int ny = w.yw[j];
                if (ny != y[q]) { y[q] = ny; s2c[q] = 0.0f; }
            }
        }
    }
    YTA_STAMP_ABS(105);
    if (w.v)
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int j = t + q * nt;
            if (j < cols) w.v[j] = v[q];
        }
    return 0;
}

template <int CPT>
__device__ __noinline__ int lap_rect_block(const RectMat M, const double *pre_u, const int *pre_x,
                                           const double *pre_s2, RectWs w, RectShared &sh) {
    return lap_rect_body<CPT>(M, pre_u, pre_x, pre_s2, w, sh);
}

// Dispatch on the columns per thread (blockDim.x <= MAXT).  Returns -3 when cols exceeds the
// register tiles.
template <int MAXT = 256>
__device__ __forceinline__ int lap_rect(const RectMat M, const double *pre_u, const int *pre_x,
                                        const double *pre_s2, RectWs w, RectShared &sh) {
    const int nt = blockDim.x;
    if (MAXT > 256) {   // the solve kernels: inlined, registers allocated for these bodies, no calls
        if (M.cols <= 2 * nt) return lap_rect_body<2>(M, pre_u, pre_x, pre_s2, w, sh);
        if (M.cols <= 8 * nt) return lap_rect_body<8>(M, pre_u, pre_x, pre_s2, w, sh);
        if (M.cols <= 16 * nt) return lap_rect_body<16>(M, pre_u, pre_x, pre_s2, w, sh);
        // > 8192 columns (rare): not inlined, so its spills do not touch the common bodies
        if (M.cols <= RECT_CPT_MAX * nt) return lap_rect_block<RECT_CPT_MAX>(M, pre_u, pre_x, pre_s2, w, sh);
        return -3;
    }
    if (M.cols <= 2 * nt) return lap_rect_block<2>(M, pre_u, pre_x, pre_s2, w, sh);
    if (M.cols <= 8 * nt) return lap_rect_block<8>(M, pre_u, pre_x, pre_s2, w, sh);
    if (M.cols <= RECT_CPT_MAX * nt) return lap_rect_block<RECT_CPT_MAX>(M, pre_u, pre_x, pre_s2, w, sh);
    return -3;
}

}  // namespace yta
