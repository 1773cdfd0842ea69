// Dense linear assignment on one wavefront: the lapx `lapjv` algorithm (Jonker-Volgenant, dense
// form) with exactly the operation and tie-breaking sequence of oracle/lapjv.c, for the calls
//   boxmot/utils/association.py:20-28  lap.lapjv(cost, extend_cost=True)   (OCSORT family)
// whose cost matrices are dense (every pair has a finite cost, no cost_limit), so the sparse
// component solver of lap.hpp does not apply.
//
// Each phase keeps the sequential semantics of the C code; the work inside a step is spread over
// the 64 lanes:
//   column reduction   columns over lanes (first row wins: strict <), rows unrolled so that many
//                      loads are in flight; the zero rows / columns of the padding need no loads.
//                      Winner bookkeeping by per-row atomicMax (the highest column a row wins is
//                      the one it keeps, as the downward walk does) and counts (solo rows)
//   reduction transfer solo rows in ascending order (each reads the prices earlier rows lowered);
//                      the next row's costs are fetched while the current one is reduced
//   row reduction      the free-row loop as written; each row's best / second-best reduced cost is
//                      a lane-parallel two-minimum with first-index ties
//   augmentation       Dijkstra over the column permutation `cols`: the min-gather and the relax
//                      sweep evaluate every position in parallel (each position is visited once
//                      and its distance only changes at its own visit), then lane 0 replays the
//                      swaps of the qualifying positions in position order, and the sweep stops at
//                      the first position that reaches a free column at the current minimum.  The
//                      scanned row is staged in an LDS row buffer; the next scanned row is fetched
//                      into registers while the current one is relaxed.
// Latency, not bandwidth, bounds this solver (one dependent chain per problem): each step costs an
// LDS round trip or two, the cost rows come from L2 behind the current step.
#pragma once
#include <float.h>

#include "common.hpp"

namespace yta {

// The padded problem: real block na x nb of a row-major matrix (leading dimension nb), entries
// negated when `neg`; everything outside it is 0.
struct LapMat {
    const double *m;
    int na, nb;
    bool neg;
    __device__ __forceinline__ double real(int r, int k) const {
        // global_load (not FLAT): FLAT loads count against the LDS counter too, and the solver's
        // LDS-only waits must not wait for row prefetches
        const double v = ((const __attribute__((address_space(1))) double *)m)[(long long)r * nb + k];
        return neg ? -v : v;
    }
    __device__ __forceinline__ double at(int r, int k) const {
        return r < na && k < nb ? real(r, k) : 0.0;
    }
};

struct DenseLapWs {
    int *x, *y, *free_rows, *cols, *pred;
    double *v, *d;
    int *aux;      // n ints: per-row winner column / counts / solo list
    double *row;   // 2 x n: row buffers
};

__host__ __device__ inline long long dense_lap_ws_bytes(long long n) {
    return n * (6 * 4 + 4 * 8) + 64;
}

// the work arrays without the two row buffers (those then live in global memory)
__host__ __device__ inline long long dense_lap_ws_bytes_norow(long long n) {
    return n * (6 * 4 + 2 * 8) + 64;
}

// carve a DenseLapWs out of `base` (dense_lap_ws_bytes(n) bytes, 8-aligned)
__host__ __device__ inline DenseLapWs dense_lap_ws(unsigned char *base, int n) {
    DenseLapWs w;
    w.v = reinterpret_cast<double *>(base);
    w.d = w.v + n;
    w.row = w.d + n;
    w.x = reinterpret_cast<int *>(w.row + 2 * n);
    w.y = w.x + n;
    w.free_rows = w.y + n;
    w.cols = w.free_rows + n;
    w.pred = w.cols + n;
    w.aux = w.pred + n;
    return w;
}

// the same with the row buffers (2 n doubles) at `rows` instead (LDS arrays, global rows)
__host__ __device__ inline DenseLapWs dense_lap_ws_split(unsigned char *base, unsigned char *rows,
                                                        int n) {
    DenseLapWs w;
    w.v = reinterpret_cast<double *>(base);
    w.d = w.v + n;
    w.x = reinterpret_cast<int *>(w.d + n);
    w.y = w.x + n;
    w.free_rows = w.y + n;
    w.cols = w.free_rows + n;
    w.pred = w.cols + n;
    w.aux = w.pred + n;
    w.row = reinterpret_cast<double *>(rows);
    return w;
}

constexpr double LAP_BIG = DBL_MAX;

// Work-array pointers of one instantiation: LDS (address space 3, ds_* instructions) or global.
// The caller's workspace pointer is generic (it picks LDS or global at run time), so the solver
// casts it back explicitly instead of leaving every access to the FLAT path.
template <bool LDS, typename T>
struct WsPtr {
    using type = T *;
};
template <typename T>
struct WsPtr<true, T> {
    using type = __attribute__((address_space(3))) T *;
};
template <bool LDS, typename T>
__device__ __forceinline__ typename WsPtr<LDS, T>::type ws_ptr(T *p) {
    return (typename WsPtr<LDS, T>::type)p;
}
constexpr int LAP_PF_MAX = 24;   // registers per lane: positions / columns up to 64 * PF

// (value, index) lexicographic "less": smaller value, then smaller index
__device__ __forceinline__ bool lex_less(double a, int ia, double b, int ib) {
    return a < b || (a == b && ia < ib);
}

// First and second lexicographic minima of (s_k, k) over the wave's columns (k1: first index of
// the minimum; k2: first index of the minimum over k != k1 among values < LAP_BIG, else -1) - the
// result of lapjv.c's sequential two-minimum scan.
__device__ __forceinline__ void wave_two_min(double &m1, int &k1, double &m2, int &k2) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const double om1 = __shfl_xor(m1, s), om2 = __shfl_xor(m2, s);
        const int ok1 = __shfl_xor(k1, s), ok2 = __shfl_xor(k2, s);
        const bool other_wins = ok1 >= 0 && (k1 < 0 || lex_less(om1, ok1, m1, k1));
        double wm1 = other_wins ? om1 : m1, wm2 = other_wins ? om2 : m2;
        int wk1 = other_wins ? ok1 : k1, wk2 = other_wins ? ok2 : k2;
        const double lm1 = other_wins ? m1 : om1;
        const int lk1 = other_wins ? k1 : ok1;
        if (lk1 >= 0 && lm1 < LAP_BIG && (wk2 < 0 || lex_less(lm1, lk1, wm2, wk2))) {
            wm2 = lm1;
            wk2 = lk1;
        }
        m1 = wm1; k1 = wk1; m2 = wm2; k2 = wk2;
    }
}

// Row prefetch: lane l holds columns l, l+64, ... (up to LAP_PF of them) in registers.
template <int PF>
struct RowPf {
    double v[PF];
};
template <int PF>
__device__ __forceinline__ void row_issue(const LapMat M, int r, int n, RowPf<PF> &pf) {
    const int lane = lane_id();
    const bool real = r >= 0 && r < M.na;
#pragma unroll
    for (int j = 0; j < PF; ++j) {
        const int k = lane + WAVE * j;
        pf.v[j] = (real && k < M.nb && k < n) ? M.real(r, k) : 0.0;
    }
}
// Stage row r (prefetched in pf) into an LDS / workspace row buffer; columns beyond the
// prefetch registers are loaded here.
template <int PF, typename DP>
__device__ __forceinline__ void row_store(const LapMat M, int r, int n, const RowPf<PF> &pf,
                                          DP buf) {
    const int lane = lane_id();
#pragma unroll
    for (int j = 0; j < PF; ++j) {
        const int k = lane + WAVE * j;
        if (k < n) buf[k] = pf.v[j];
    }
    for (int k = lane + WAVE * PF; k < n; k += WAVE) buf[k] = M.at(r, k);
}

// Inclusive prefix minimum over the 64 lanes (DPP row shifts / broadcasts, as wave_inclusive_scan).
__device__ __forceinline__ double wave_incl_min(double x) {
    const int l = lane_id(), rl = l & 15;
    double t;
    t = dpp_f64<0x111>(x); if (rl >= 1) x = t < x ? t : x;
    t = dpp_f64<0x112>(x); if (rl >= 2) x = t < x ? t : x;
    t = dpp_f64<0x114>(x); if (rl >= 4) x = t < x ? t : x;
    t = dpp_f64<0x118>(x); if (rl >= 8) x = t < x ? t : x;
    t = dpp_f64<0x142>(x); if ((l & 31) >= 16) x = t < x ? t : x;
    t = dpp_f64<0x143>(x); if (l >= 32) x = t < x ? t : x;
    return x;
}

// Memory ordering between the lanes of the solving wave.  With the work arrays in LDS (in-order per
// wave) it is enough to wait for the LDS counter, so cost-row prefetches stay in flight across it;
// a global-memory workspace needs the vector-memory counter too.
template <bool LDS_WS>
__device__ __forceinline__ void lap_sync() {
    if (LDS_WS) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// gather_min (lapjv.c) with every position of [lo+1, n) held in registers (n - lo - 1 <=
// 64 * LAP_PF): per-chunk prefix minima decide which positions qualify (<= the running minimum of
// all earlier ones; a reset where strictly smaller); lane 0 replays the swaps in position order.
// Returns the new hi.
template <bool LDS_WS, int LAP_PF, typename DP, typename IP>
__device__ __forceinline__ int gather_min_reg(int n, int lo, DP d, IP cols) {
    const int lane = lane_id();
    const int b0 = lo + 1;
    double e[LAP_PF];
    int ck[LAP_PF];
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        const int t = b0 + WAVE * j + lane;
        ck[j] = cols[t < n ? t : n - 1];
    }
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        const int t = b0 + WAVE * j + lane;
        const double x = d[ck[j]];
        e[j] = t < n ? x : LAP_BIG;
    }
    double run = d[cols[lo]];
    unsigned long long qb[LAP_PF], rb[LAP_PF];
    bool any = false;
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        qb[j] = rb[j] = 0ull;
        if (b0 + WAVE * j < n) {
            const double pm = wave_incl_min(e[j]);
            double excl = __shfl_up(pm, 1);
            if (lane == 0) excl = LAP_BIG;
            const double before = excl < run ? excl : run;
            const bool q = b0 + WAVE * j + lane < n && e[j] <= before;
            qb[j] = __ballot(q);
            rb[j] = __ballot(q && e[j] < before);
            any |= qb[j] != 0ull;
            const double cm = readlane_f64(pm, WAVE - 1);
            run = cm < run ? cm : run;
        }
    }
    int hi = lo + 1;
    if (any) {
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < LAP_PF; ++j) {
                unsigned long long m = qb[j];
                while (m) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const int tt = b0 + WAVE * j + l;
                    if ((rb[j] >> l) & 1ull) hi = lo;
                    const int kk = cols[tt];
                    cols[tt] = cols[hi];
                    cols[hi] = kk;
                    ++hi;
                }
            }
        }
        hi = __shfl(hi, 0);
        lap_sync<LDS_WS>();
    }
    return hi;
}

// One relax sweep of relax_scan (lapjv.c) for the scanned column's row r (costs in `rowbuf`, or
// all zero for a padding row) over positions [shi, n) held in registers: every position's new
// distance is computed at once; the first position that reaches a free column at the current
// minimum ends the sweep (positions after it are not visited); lane 0 replays the swaps of the
// other minimum-distance positions before it.  Returns that free column or -1; `shi` advances.
template <bool LDS_WS, int LAP_PF, typename RP, typename DP, typename IP>
__device__ __forceinline__ int relax_reg(int n, int &shi, int r, double h, double dk, bool real_row,
                                         RP rowbuf, DP d, DP v, IP pred, IP cols, IP y) {
    const int lane = lane_id();
    const int b0 = shi;
    int kk[LAP_PF];
    double nd[LAP_PF];
    unsigned long long fb[LAP_PF], hb[LAP_PF];
    unsigned imp_bits = 0u;
    // branch-free: every chunk's loads are issued before any is consumed (out-of-range positions
    // read a clamped valid entry and are masked)
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        const int t = b0 + WAVE * j + lane;
        kk[j] = cols[t < n ? t : n - 1];
    }
    double rc[LAP_PF], vv[LAP_PF], dd[LAP_PF];
    int yy[LAP_PF];
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        rc[j] = rowbuf[kk[j]];
        vv[j] = v[kk[j]];
        dd[j] = d[kk[j]];
        yy[j] = y[kk[j]];
    }
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        const bool valid = b0 + WAVE * j + lane < n;
        nd[j] = (real_row ? rc[j] : 0.0) - vv[j] - h;
        const bool imp = valid && nd[j] < dd[j];
        const bool hit = imp && nd[j] == dk;
        const bool fin = hit && yy[j] < 0;
        imp_bits |= (imp ? 1u : 0u) << j;
        fb[j] = __ballot(fin);
        hb[j] = __ballot(hit && !fin);
        if (!valid) kk[j] = -1;
    }
    int jstar = LAP_PF, lstar = WAVE;
#pragma unroll
    for (int j = LAP_PF - 1; j >= 0; --j)
        if (fb[j]) { jstar = j; lstar = __builtin_ctzll(fb[j]); }
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) {
        const bool allowed = j < jstar || (j == jstar && lane <= lstar);
        if (((imp_bits >> j) & 1u) && allowed) {
            d[kk[j]] = nd[j];
            pred[kk[j]] = r;
        }
        if (j > jstar) hb[j] = 0ull;
        else if (j == jstar) hb[j] &= lstar >= WAVE ? ~0ull : ((1ull << lstar) - 1ull);
    }
    bool anyhit = false;
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j) anyhit |= hb[j] != 0ull;
    if (anyhit) {
        lap_sync<LDS_WS>();
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < LAP_PF; ++j) {
                unsigned long long m = hb[j];
                while (m) {
                    const int l = __builtin_ctzll(m);
                    m &= m - 1;
                    const int tt = b0 + WAVE * j + l;
                    const int q = cols[tt];
                    cols[tt] = cols[shi];
                    cols[shi] = q;
                    ++shi;
                }
            }
        }
        shi = __shfl(shi, 0);
    }
    int ret = -1;
#pragma unroll
    for (int j = 0; j < LAP_PF; ++j)
        if (j == jstar) ret = __shfl(kk[j], lstar);
    lap_sync<LDS_WS>();
    return ret;
}

// Square dense solve of the padded n x n problem M by the calling wave (all 64 lanes).  x[row] =
// col, y[col] = row.  Returns 0, or -2 if an augmenting path could not be traced (corrupt input).
// LDS_WS: the work arrays of `w` are in LDS.
// ROW_LDS: the two row buffers are in LDS too (else in global memory, the other arrays in LDS
// when LDS_WS).
// P3 = false: stop after phase 2 and return the number of free rows left (w.free_rows), for a
// block-wide phase 3 (lap_dense_block.hpp).
template <bool LDS_WS, bool ROW_LDS, int LAP_PF, bool P3 = true>
__device__ __noinline__ int lap_dense_wave_pf(int n, const LapMat M, const DenseLapWs w) {
    const int lane = lane_id();
    auto x = ws_ptr<LDS_WS>(w.x), y = ws_ptr<LDS_WS>(w.y), fr = ws_ptr<LDS_WS>(w.free_rows);
    auto cols = ws_ptr<LDS_WS>(w.cols), pred = ws_ptr<LDS_WS>(w.pred), aux = ws_ptr<LDS_WS>(w.aux);
    auto v = ws_ptr<LDS_WS>(w.v), d = ws_ptr<LDS_WS>(w.d);
    if (n <= 0) return 0;
    const int na = M.na < n ? M.na : n;
    // ---------------- phase 1: column reduction ----------------
    for (int k = lane; k < n; k += WAVE) {
        x[k] = -1;
        aux[k] = -1;
        pred[k] = 0;   // per-row win counts
        double best = LAP_BIG;
        int br = 0;
        if (k < M.nb) {
            int r = 0;
            for (; r + 8 <= na; r += 8) {
                double c[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) c[u] = M.real(r + u, k);
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (c[u] < best) { best = c[u]; br = r + u; }
            }
            for (; r < na; ++r) {
                const double c = M.real(r, k);
                if (c < best) { best = c; br = r; }
            }
            if (na < n && 0.0 < best) { best = 0.0; br = na; }   // first padding row
        } else {
            best = 0.0;   // padding column: every row costs 0, row 0 wins
            br = 0;
        }
        v[k] = best;
        y[k] = br;
    }
    lap_sync<LDS_WS>();
    for (int k = lane; k < n; k += WAVE) {
        // the downward walk keeps the highest column a row wins
        __hip_atomic_fetch_max(&aux[y[k]], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&pred[y[k]], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    lap_sync<LDS_WS>();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (int k = lane; k < n; k += WAVE) {
        const int r = y[k];
        if (aux[r] != k) y[k] = -1;
    }
    for (int r = lane; r < n; r += WAVE) x[r] = aux[r];
    lap_sync<LDS_WS>();
    // free rows (ascending); solo rows (ascending) into aux
    int nfree = 0, nsolo = 0;
    for (int base = 0; base < n; base += WAVE) {
        const int r = base + lane;
        const bool f = r < n && x[r] < 0;
        const bool so = r < n && x[r] >= 0 && pred[r] == 1;
        const unsigned long long bf = __ballot(f), bs = __ballot(so);
        const unsigned long long below = (1ull << lane) - 1;
        if (f) fr[nfree + __popcll(bf & below)] = r;
        if (so) aux[nsolo + __popcll(bs & below)] = r;
        nfree += __popcll(bf);
        nsolo += __popcll(bs);
    }
    lap_sync<LDS_WS>();
    YTA_STAMP(20);
    // reduction transfer, solo rows ascending; the next solo row is fetched during the current
    // (two register sets used in turn, so no copy waits on a load in flight)
    {
        auto transfer = [&](int r, const RowPf<LAP_PF> &pf) {
            const int own = x[r];
            double best = LAP_BIG;
#pragma unroll
            for (int j = 0; j < LAP_PF; ++j) {
                const int k = lane + WAVE * j;
                if (k < n && k != own) {
                    const double s = pf.v[j] - v[k];
                    if (s < best) best = s;
                }
            }
            for (int k = lane + WAVE * LAP_PF; k < n; k += WAVE)
                if (k != own) {
                    const double s = M.at(r, k) - v[k];
                    if (s < best) best = s;
                }
            best = wave_reduce(RED_MIN, best);
            if (lane == 0) v[own] -= best;
            lap_sync<LDS_WS>();
        };
        RowPf<LAP_PF> pa, pb;
        if (nsolo > 0) row_issue(M, aux[0], n, pa);
        for (int q = 0; q < nsolo; q += 2) {
            const int ra = aux[q];
            const int rb = q + 1 < nsolo ? aux[q + 1] : -1;
            if (rb >= 0) row_issue(M, rb, n, pb);
            transfer(ra, pa);
            if (rb >= 0) {
                if (q + 2 < nsolo) row_issue(M, aux[q + 2], n, pa);
                transfer(rb, pb);
            }
        }
    }
    YTA_STAMP(21);
    // ---------------- phase 2: augmenting row reduction (at most twice) ----------------
    for (int pass = 0; nfree > 0 && pass < 2; ++pass) {
        int pos = 0, out = 0;
        unsigned long long iters = 0;
        while (pos < nfree) {
            ++iters;
            YTA_COUNT(120);
            const int r = fr[pos++];
            RowPf<LAP_PF> cur;
            row_issue(M, r, n, cur);
            double m1 = LAP_BIG, m2 = LAP_BIG;
            int k1 = -1, k2 = -1;
            auto visit = [&](int k, double c) {   // this lane's columns, ascending
                const double s = c - v[k];
                if (k1 < 0) { m1 = s; k1 = k; return; }
                if (s < m2) {
                    if (s >= m1) { m2 = s; k2 = k; }
                    else { m2 = m1; k2 = k1; m1 = s; k1 = k; }
                }
            };
#pragma unroll
            for (int j = 0; j < LAP_PF; ++j) {
                const int k = lane + WAVE * j;
                if (k < n) visit(k, cur.v[j]);
            }
            for (int k = lane + WAVE * LAP_PF; k < n; k += WAVE) visit(k, M.at(r, k));
            wave_two_min(m1, k1, m2, k2);
            int displaced = y[k1];
            const double vk1 = v[k1];
            const double lowered = vk1 - (m2 - m1);
            const bool can_lower = lowered < vk1;
            if (iters < (unsigned long long)pos * (unsigned long long)n) {
                if (can_lower) {
                    if (lane == 0) v[k1] = lowered;
                } else if (displaced >= 0 && k2 >= 0) {
                    k1 = k2;
                    displaced = y[k2];
                }
                if (displaced >= 0) {
                    if (can_lower) {
                        --pos;
                        if (lane == 0) fr[pos] = displaced;
                    } else {
                        if (lane == 0) fr[out] = displaced;
                        ++out;
                    }
                }
            } else if (displaced >= 0) {
                if (lane == 0) fr[out] = displaced;
                ++out;
            }
            if (lane == 0) {
                x[r] = k1;
                y[k1] = r;
            }
            lap_sync<LDS_WS>();
        }
        nfree = out;
    }
    YTA_STAMP(22);
    if (!P3) return nfree;
    // ---------------- phase 3: shortest augmenting paths ----------------
#ifdef YTA_STAMPS
    unsigned long long acc_store = 0, acc_relax = 0, acc_gather = 0, acc_init = 0;
#endif
    auto rowA = ws_ptr<ROW_LDS>(w.row), rowB = ws_ptr<ROW_LDS>(w.row + n);
    constexpr bool ROW_SYNC_LDS = LDS_WS && ROW_LDS;   // a staged row is visible after an LDS wait
    for (int f = 0; f < nfree; ++f) {
        const int src = fr[f];
        YTA_COUNT(121);
        {
            RowPf<LAP_PF> cur;
            row_issue(M, src, n, cur);
#pragma unroll
            for (int j = 0; j < LAP_PF; ++j) {
                const int k = lane + WAVE * j;
                if (k < n) {
                    cols[k] = k;
                    pred[k] = src;
                    d[k] = cur.v[j] - v[k];
                }
            }
            for (int k = lane + WAVE * LAP_PF; k < n; k += WAVE) {
                cols[k] = k;
                pred[k] = src;
                d[k] = M.at(src, k) - v[k];
            }
        }
        lap_sync<LDS_WS>();
        int lo = 0, hi = 0, ready = 0, end = -1;
        while (end < 0) {
            if (lo == hi) {
                // gather_min: positions lo.. n-1; qualifying positions are those whose value is
                // <= the running minimum of the earlier ones (resets where strictly smaller)
                ready = lo;
#ifdef YTA_STAMPS
                const unsigned long long tg0 = wall_clock64();
#endif
                YTA_COUNT(122);
                if (n - lo - 1 <= WAVE * LAP_PF) {
                    hi = gather_min_reg<LDS_WS, LAP_PF>(n, lo, d, cols);
                } else {
                double run = d[cols[lo]];
                hi = lo + 1;
                for (int base = lo + 1; base < n; base += WAVE) {
                    const int t = base + lane;
                    const double e = t < n ? d[cols[t]] : LAP_BIG;
                    double pm = e;   // inclusive prefix min within the chunk
#pragma unroll
                    for (int s = 1; s < WAVE; s <<= 1) {
                        const double o = __shfl_up(pm, s);
                        if (lane >= s) pm = pm < o ? pm : o;
                    }
                    double excl = __shfl_up(pm, 1);
                    if (lane == 0) excl = LAP_BIG;
                    const double before = excl < run ? excl : run;
                    const bool q = t < n && e <= before;
                    const bool reset = q && e < before;
                    unsigned long long qb = __ballot(q), rb = __ballot(reset);
                    if (qb) {
                        if (lane == 0) {   // replay the swaps in position order
                            while (qb) {
                                const int l = __builtin_ctzll(qb);
                                qb &= qb - 1;
                                const int tt = base + l;
                                if ((rb >> l) & 1ull) hi = lo;
                                const int kk = cols[tt];
                                cols[tt] = cols[hi];
                                cols[hi] = kk;
                                ++hi;
                            }
                        }
                        hi = __shfl(hi, 0);
                        lap_sync<LDS_WS>();
                    }
                    const double cm = __shfl(pm, WAVE - 1);
                    run = cm < run ? cm : run;
                }
                }
                // the last free column of the gathered set
                int e_last = -1;
                for (int t = lo + lane; t < hi; t += WAVE)
                    if (y[cols[t]] < 0) e_last = t;
#pragma unroll
                for (int s = 32; s >= 1; s >>= 1) {
                    const int o = __shfl_xor(e_last, s);
                    e_last = o > e_last ? o : e_last;
                }
                if (e_last >= 0) end = cols[e_last];
#ifdef YTA_STAMPS
                acc_gather += wall_clock64() - tg0;
#endif
            }
            if (end < 0) {
                // relax_scan from the scan set [lo, hi); the row of the next scanned column is
                // fetched while the current one is relaxed
                int slo = lo, shi = hi, ret = -1;
                RowPf<LAP_PF> nxt;
                int r_next = slo < shi ? y[cols[slo]] : -1;
                row_issue(M, r_next, n, nxt);
                while (slo != shi && ret < 0) {
                    const int k = cols[slo++];
                    YTA_COUNT(123);
                    const int r = r_next;
                    auto rowbuf = (slo & 1) ? rowA : rowB;
                    const bool real_row = r < M.na;
#ifdef YTA_STAMPS
                    unsigned long long t0 = wall_clock64();
#endif
                    if (real_row) row_store(M, r, n, nxt, rowbuf);
                    r_next = slo < shi ? y[cols[slo]] : -1;
                    if (r_next >= 0) row_issue(M, r_next, n, nxt);
                    lap_sync<ROW_SYNC_LDS>();
                    const double dk = d[k];
                    const double h = (real_row ? rowbuf[k] : 0.0) - v[k] - dk;
#ifdef YTA_STAMPS
                    unsigned long long t1 = wall_clock64();
                    acc_store += t1 - t0;
#endif
                    if (n - shi <= WAVE * LAP_PF) {
                        YTA_COUNT(124);
                        ret = relax_reg<LDS_WS, LAP_PF>(n, shi, r, h, dk, real_row, rowbuf, d, v, pred, cols, y);
#ifdef YTA_STAMPS
                        acc_relax += wall_clock64() - t1;
#endif
                    } else
                    for (int base = shi; base < n && ret < 0; base += WAVE) {
                        const int t = base + lane;
                        int kk = -1;
                        double nd = 0.0;
                        bool imp = false;
                        if (t < n) {
                            kk = cols[t];
                            nd = (real_row ? rowbuf[kk] : 0.0) - v[kk] - h;
                            imp = nd < d[kk];
                        }
                        const bool hit = imp && nd == dk;
                        const bool fin = hit && y[kk] < 0;
                        const unsigned long long fb = __ballot(fin);
                        const int first_fin = fb ? __builtin_ctzll(fb) : WAVE;
                        // positions up to the first free hit are visited; later ones are not
                        if (imp && lane <= first_fin) {
                            d[kk] = nd;
                            pred[kk] = r;
                        }
                        unsigned long long hb = __ballot(hit && !fin) &
                                                (first_fin >= WAVE ? ~0ull : ((1ull << first_fin) - 1));
                        if (hb) {
                            lap_sync<LDS_WS>();
                            if (lane == 0) {
                                while (hb) {
                                    const int l = __builtin_ctzll(hb);
                                    hb &= hb - 1;
                                    const int tt = base + l;
                                    const int q = cols[tt];
                                    cols[tt] = cols[shi];
                                    cols[shi] = q;
                                    ++shi;
                                }
                            }
                            shi = __shfl(shi, 0);
                        }
                        lap_sync<LDS_WS>();
                        if (first_fin < WAVE) ret = __shfl(kk, first_fin);
                    }
                    // the scan set may have grown past the prefetched row's column
                    if (ret < 0 && r_next < 0 && slo < shi) {
                        r_next = y[cols[slo]];
                        row_issue(M, r_next, n, nxt);
                    }
                }
                if (ret >= 0) {
                    end = ret;   // lo / hi keep their values (early return)
                } else {
                    lo = slo;
                    hi = shi;
                }
            }
        }
        const double m = d[cols[lo]];
        for (int t = lane; t < ready; t += WAVE) {
            const int k = cols[t];
            v[k] += d[k] - m;
        }
        lap_sync<LDS_WS>();
        if (lane == 0) {   // flip the alternating path back to the source row
            int k = end, r = -1, steps = 0;
            while (r != src) {
                r = pred[k];
                y[k] = r;
                const int prev = x[r];
                x[r] = k;
                k = prev;
                if (++steps > n) { aux[0] = -2; break; }
            }
        }
        lap_sync<LDS_WS>();
        if (aux[0] == -2) return -2;
    }
    YTA_STAMP(23);
#ifdef YTA_STAMPS
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        g_stamps[110] += acc_store;
        g_stamps[111] += acc_relax;
        g_stamps[112] += acc_gather;
    }
#endif
    return 0;
}

// Dispatch on the problem size: 8 registers per lane up to n = 512, 24 beyond.
template <bool LDS_WS, bool ROW_LDS = LDS_WS, bool P3 = true>
__device__ __forceinline__ int lap_dense_wave(int n, const LapMat M, const DenseLapWs w) {
    if (n <= WAVE * 8) return lap_dense_wave_pf<LDS_WS, ROW_LDS, 8, P3>(n, M, w);
    return lap_dense_wave_pf<LDS_WS, ROW_LDS, LAP_PF_MAX, P3>(n, M, w);
}

}  // namespace yta

namespace yta {
// The padded solve with its work arrays placed by size: all in LDS (dense_lap_ws_bytes(n) <=
// lds_bytes); else the arrays in LDS and the two row buffers in `gws`
// (dense_lap_ws_bytes_norow(n) <= lds_bytes: n <= ~3900 in 156 KiB); else all in `gws`.  `w`
// receives the layout used (the caller reads w.x / w.y).
__device__ __forceinline__ int lap_dense_placed(int n, const LapMat M, unsigned char *lds,
                                                long long lds_bytes, unsigned char *gws,
                                                DenseLapWs &w) {
    if (dense_lap_ws_bytes(n) <= lds_bytes) {
        w = dense_lap_ws(lds, n);
        return lap_dense_wave<true>(n, M, w);
    }
    if (dense_lap_ws_bytes_norow(n) <= lds_bytes) {
        w = dense_lap_ws_split(lds, gws, n);
        return lap_dense_wave<true, false>(n, M, w);
    }
    w = dense_lap_ws(gws, n);
    return lap_dense_wave<false>(n, M, w);
}
}  // namespace yta
