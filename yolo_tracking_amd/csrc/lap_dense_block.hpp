// Phase 3 of the lapjv replay (shortest augmenting paths, oracle/lapjv.c shortest_path /
// gather_min / relax_scan) run by a whole block instead of one wave, with the same operation and
// tie-breaking sequence.  Phases 1-2 (column reduction, reduction transfer, augmenting row
// reduction) stay on wave 0 (lap_dense.hpp, P3 = false); a large replay (a crowd surge under
// GIoU) spends its time here, in row scans over every remaining column.
//
// relax_scan: a row's sweep over the positions [hi, n) visits each position once in position
// order and stops at the first free column reached at the current minimum; its distance updates
// touch distinct columns, and its hits (columns reached at the minimum) are swapped to the front
// in position order.  So the block evaluates every position at once: the first free hit is a
// block minimum of positions, the updates up to it are independent, and thread 0 replays the
// hits' swaps from a position bitmap in order.  gather_min: a position qualifies when its
// distance is <= the running minimum of the earlier ones; a block prefix-minimum over contiguous
// position ranges marks them, and thread 0 replays their swaps (with the resets) in order.
//
// Sparse sweeps (tools/lapjv_sparse_proto.c): a sweep from scanned column k (row
// r, h = c[r][k] - v[k] - d[k]) relaxes a zero entry kk only if -h < d[kk] + v[kk], and d[kk] +
// v[kk] <= c[src][kk] <= cmax (the search's source row maximum) for the whole search.  When
// -h >= cmax only the row's nonzero entries can change anything, and the columns not yet visited
// keep their positions during a sweep, so wave 0 visits just those entries, in position order
// (pos: the inverse of cols), and runs such sweeps back to back without block barriers; a sweep
// that needs the dense form (or a row with more than LAPS_K nonzero entries) goes to the block.
// The rows' nonzero entries are collected once per replay into `csr_ws` (lap_csr_bytes).
#pragma once
#include <cstdlib>

#include "lap_dense.hpp"

namespace yta {

constexpr int LAPS_K = 16;   // nonzero entries per row kept for the sparse sweeps
__host__ __device__ inline long long lap_csr_bytes(long long n) { return 16 * n * LAPS_K; }
// the sparse sweeps are on unless YTA_LAP_SPARSE=0 (host: engines' workspace, the KAT)
inline bool lap_sparse_on() {
    const char *v = getenv("YTA_LAP_SPARSE");
    return !v || atoi(v) != 0;
}
// Row r's entries at ent[r * LAPS_K + i], ascending columns: (value, bits(count << 32 | column)),
// every entry of the row carrying the row's count of nonzero entries (-1: more than LAPS_K;
// entry 0 holds it also when the row has none), so one 16-B load per lane brings a sweep its row.
struct LapCsr {
    double2 *ent;
};
__device__ __forceinline__ LapCsr lap_csr(unsigned char *base, int) {
    return LapCsr{reinterpret_cast<double2 *>(base)};
}
__device__ __forceinline__ double2 lap_csr_entry(double val, int col, int cnt) {
    return make_double2(val, __longlong_as_double(((long long)cnt << 32) | (unsigned)col));
}

constexpr int LAPB_MAX_N = 8192;    // positions covered by the sweep bitmap (1 KiB of LDS)
constexpr int LAPB_MIN_N = 768;     // below this the one-wave replay is as fast

#ifdef YTA_STAMPS
// diagnostic build: block 0 thread 0 accumulates ticks / counts into g_stamps[k]
#define LAPB_ADD(k, v)                                                         \
    do {                                                                       \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[(k)] += (v);          \
    } while (0)
#define LAPB_T0() const unsigned long long lapb_t0 = wall_clock64()
#define LAPB_DT(k) LAPB_ADD(k, wall_clock64() - lapb_t0)
#else
#define LAPB_ADD(k, v) do { } while (0)
#define LAPB_T0() do { } while (0)
#define LAPB_DT(k) do { } while (0)
#endif

struct LapBShared {
    unsigned bits[LAPB_MAX_N / 32];
    int wrank[LAPB_MAX_N / 32];   // exclusive prefix of the bitmap words' popcounts
    int wsum[32];
    double red[2][32];            // alternating reduction slots (one barrier per reduction)
    double pre[32];               // gather_min's per-wave prefix minima
    int lo, hi, end, ready;
};

// lapjv.c's swap-to-front (for each marked position p, ascending: swap(cols[p], cols[h]); ++h,
// from h = h0) done by the block.  The result in closed form: the marked elements land at h0,
// h0 + 1, ... in position order; the unmarked elements of the window [h0, h0 + m) move, in
// position order, to the marked positions beyond the window (in order); nothing else moves.
// bits: the marks over positions [h0, h0 + 32 nwords) (nwords <= blockDim.x).  hitpos (n ints)
// and tmp (2 n ints) are scratch.  Returns m.
template <typename IP, typename HP, typename TP>
__device__ int lapb_swap_front(int h0, int nwords, IP cols, HP hitpos, TP tmp, LapBShared &sh,
                               IP pos = nullptr) {
    const int t = threadIdx.x, nt = blockDim.x;
    LAPB_T0();
    const unsigned wbits = t < nwords ? sh.bits[t] : 0u;
    int m = 0;
    const int wr = block_exclusive_scan(__popc(wbits), sh.wsum, &m);
    if (m == 0) return 0;   // (every thread read its bitmap word before the scan's barriers)
    if (t < nwords) sh.wrank[t] = wr;
    {
        unsigned b = wbits;
        int r = wr;
        while (b) {
            hitpos[r++] = h0 + t * 32 + __builtin_ctz(b);
            b &= b - 1u;
        }
    }
    block_sync();
    auto rank_before = [&](int q) -> int {   // marked positions in [h0, q)
        const int o = q - h0, wi = o >> 5;
        if (wi >= nwords) return m;
        return sh.wrank[wi] + (int)__popc(sh.bits[wi] & ((1u << (o & 31)) - 1u));
    };
    const int k = rank_before(h0 + m);   // marked positions inside the window
    for (int i = t; i < m; i += nt) tmp[i] = cols[hitpos[i]];
    for (int q = h0 + t; q < h0 + m; q += nt) {
        const int o = q - h0;
        const bool marked = (o >> 5) < nwords && ((sh.bits[o >> 5] >> (o & 31)) & 1u);
        if (!marked) tmp[m + (o - rank_before(q))] = cols[q];
    }
    block_sync();
    for (int i = t; i < m; i += nt) {
        const int c = tmp[i];
        cols[h0 + i] = c;
        if (pos) pos[c] = h0 + i;
    }
    for (int r = t; r < m - k; r += nt) {
        const int q = hitpos[k + r], c = tmp[m + r];
        cols[q] = c;
        if (pos) pos[c] = q;
    }
    block_sync();
    LAPB_DT(66);
    LAPB_ADD(67, m);
    return m;
}

// block-uniform minimum / maximum of a double (all threads get it).  The slots alternate between
// calls (par: block-uniform, a register of every thread), so one barrier suffices: a slot is
// rewritten two reductions later, after the other reduction's barrier.
__device__ __forceinline__ double lapb_reduce(bool is_min, double v, LapBShared &sh, int &par) {
    v = wave_reduce(is_min ? RED_MIN : RED_MAX, v);
    const int nw = blockDim.x / WAVE, wv = threadIdx.x / WAVE;
    double *red = sh.red[par];
    par ^= 1;
    if (lane_id() == 0) red[wv] = v;
    block_sync();
    double r = red[0];
    for (int k = 1; k < nw; ++k) r = is_min ? (red[k] < r ? red[k] : r) : (red[k] > r ? red[k] : r);
    return r;
}

// One relax_scan sweep of row r over positions [base, n) with RP >= (n - base) / blockDim
// positions per thread: the cols / cost loads of all of them issued at once (unconditional,
// clamped index: a guarded load becomes a branch and a wait per position), the first free column
// reached at the minimum found, then the updates from the kept values.  Returns that position.
template <int RP, typename DP, typename IP>
__device__ __forceinline__ int lapb_relax_regs(int n, const LapMat &M, int base, int r, double dk,
                                               double hh, DP d, DP v, IP cols, IP pred, IP y,
                                               LapBShared &sh, int &par) {
    const int t = threadIdx.x, nt = blockDim.x;
    int kkr[RP];
    double ndr[RP];
#pragma unroll
    for (int q = 0; q < RP; ++q) {
        const int p = base + t + q * nt;
        kkr[q] = cols[p < n ? p : n - 1];
    }
    double cr[RP];
#pragma unroll
    for (int q = 0; q < RP; ++q) cr[q] = M.at(r, kkr[q]);
    int my_fin = INT_MAX;
#pragma unroll
    for (int q = 0; q < RP; ++q) {
        const int p = base + t + q * nt, kk = kkr[q];
        ndr[q] = cr[q] - v[kk] - hh;
        if (my_fin == INT_MAX && p < n && ndr[q] < d[kk] && ndr[q] == dk && y[kk] < 0) my_fin = p;
    }
    const double ff = lapb_reduce(true, my_fin == INT_MAX ? 1e300 : (double)my_fin, sh, par);
    const int ffin = ff >= 1e300 ? INT_MAX : (int)ff;
#pragma unroll
    for (int q = 0; q < RP; ++q) {
        const int p = base + t + q * nt, kk = kkr[q];
        const double nd = ndr[q];
        if (p < n && p <= ffin && nd < d[kk]) {
            d[kk] = nd;
            pred[kk] = r;
            if (nd == dk && p < ffin) atomicOr(&sh.bits[(p - base) >> 5], 1u << ((p - base) & 31));
        }
    }
    return ffin;
}

// Sparse sweeps by wave 0 (the header's argument): from position l while l != h, as long as the
// scanned row has <= LAPS_K nonzero entries and -h >= cmax.  Returns a free column reached at the
// minimum (l / h then as the caller passed them, as lapjv.c's early return), else -1 with l / h
// advanced over the sweeps done.  Stores of one lane are read by others after lap_sync<false>.
template <typename DP, typename IP>
__device__ int lapb_sparse_sweeps(int &l, int &h, DP d, DP v, IP cols, IP pred, IP y, IP pos,
                                  const LapCsr &cs, double cmax) {
    const int lane = lane_id();
    int ll = l, hh = h;
    while (ll != hh) {
        const int k = cols[ll];
        const int r = y[k];
        const double dk = d[k], vk = v[k];
        double2 en = make_double2(0.0, 0.0);
        if (lane < LAPS_K) en = cs.ent[(long long)r * LAPS_K + lane];
        const long long bits = __double_as_longlong(en.y);
        const int cnt = __shfl((int)(bits >> 32), 0);
        if (cnt < 0) break;   // a row with more entries: the block's sweep
        const bool in = lane < cnt;
        const int kk = in ? (int)(unsigned)bits : -1;
        const double cv = in ? en.x : 0.0;
        const unsigned long long mk = __ballot(in && kk == k);
        const double crk = mk ? __shfl(cv, __ffsll((long long)mk) - 1) : 0.0;
        const double hr = crk - vk - dk;
        if (!(-hr >= cmax)) break;   // a zero entry may relax: the block's sweep
        ++ll;
        // the entry columns' position, price, distance and row in one round trip
        const int ks = in ? kk : k;
        const int p0 = pos[ks], yk = y[ks];
        const double vkk = v[ks], dkk = d[ks];
        const int p = in ? p0 : -1;
        double nd = 0.0;
        bool upd = false;
        if (in && p >= hh) {
            nd = cv - vkk - hr;
            upd = nd < dkk;
        }
        const bool eq = upd && nd == dk;
        const bool fr = eq && yk < 0;
        int pf = INT_MAX;   // the first free hit's position (a reduction only when there is one)
        if (__ballot(fr)) {
            const double pfd = wave_reduce(RED_MIN, fr ? (double)p : 1e300);
            pf = (int)pfd;
        }
        if (upd && p <= pf) {   // the updates up to the first free hit (inclusive)
            d[kk] = nd;
            pred[kk] = r;
        }
        if (pf != INT_MAX) {
            lap_sync<false>();
            const unsigned long long mf = __ballot(fr && p == pf);
            return __shfl(kk, __ffsll((long long)mf) - 1);
        }
        // the hits to the front, in position order
        bool pend = eq;
        while (__ballot(pend)) {
            const double pm = wave_reduce(RED_MIN, pend ? (double)p : 1e300);
            lap_sync<false>();
            if (pend && (double)p == pm) {
                const int c = cols[hh];
                cols[p] = c;
                pos[c] = p;
                cols[hh] = kk;
                pos[kk] = hh;
                pend = false;
            }
            ++hh;
        }
        lap_sync<false>();
    }
    l = ll;
    h = hh;
    return -1;
}

// relax_scan (lapjv.c) by the block.  Returns a free column reached at the minimum distance
// (lo / hi left as they were, as the C code's early return leaves *plo / *phi), or -1 with
// lo / hi advanced.  cs: the rows' nonzero entries (sparse sweeps by wave 0 where they apply, pos
// maintained), or nullptr.
template <typename DP, typename IP, typename HP, typename TP>
__device__ int lapb_relax_scan(int n, const LapMat &M, int &lo, int &hi, DP d, DP v, IP cols,
                               IP pred, IP y, HP hitpos, TP tmp, LapBShared &sh, int &par,
                               IP pos = nullptr, const LapCsr *cs = nullptr, double cmax = 0.0) {
    const int t = threadIdx.x, nt = blockDim.x;
    int l = lo, h = hi;
    while (l != h) {
        if (cs) {
            if (t < WAVE) {
                LAPB_T0();
                int ls = l, hs = h;
                const int e = lapb_sparse_sweeps(ls, hs, d, v, cols, pred, y, pos, *cs, cmax);
                if (t == 0) {
                    sh.lo = ls;
                    sh.hi = hs;
                    sh.end = e;
                }
                LAPB_DT(69);
                LAPB_ADD(68, ls - l + (e >= 0));
            }
            block_sync();
            const int e = sh.end;
            l = sh.lo;
            h = sh.hi;
            block_sync();
            if (e >= 0) return e;
            if (l == h) break;
        }
        LAPB_ADD(63, 1);
        LAPB_T0();
        const int k = cols[l++];
        const int r = y[k];
        const double dk = d[k];
        const double hh = M.at(r, k) - v[k] - dk;
        const int base = h, cnt = n - h;
        for (int q = t; q < (cnt + 31) / 32; q += nt) sh.bits[q] = 0u;
        // the first free column reached at the minimum (in position order), then every position
        // up to it: distance updates, hits into the bitmap.  Up to 8 positions per thread go
        // through lapb_relax_regs (the row's entries of all of them loaded at once, kept for the
        // update pass); larger problems loop
        int ffin;
        const int m = (cnt + nt - 1) / nt;   // positions per thread, block-uniform
        if (m <= 2) ffin = lapb_relax_regs<2>(n, M, base, r, dk, hh, d, v, cols, pred, y, sh, par);
        else if (m <= 4) ffin = lapb_relax_regs<4>(n, M, base, r, dk, hh, d, v, cols, pred, y, sh, par);
        else if (m <= 8) ffin = lapb_relax_regs<8>(n, M, base, r, dk, hh, d, v, cols, pred, y, sh, par);
        else {
            int my_fin = INT_MAX;
            for (int p = base + t; p < n; p += nt) {
                const int kk = cols[p];
                const double nd = M.at(r, kk) - v[kk] - hh;
                if (nd < d[kk] && nd == dk && y[kk] < 0) {
                    my_fin = p;
                    break;
                }
            }
            const double ff = lapb_reduce(true, my_fin == INT_MAX ? 1e300 : (double)my_fin, sh, par);
            ffin = ff >= 1e300 ? INT_MAX : (int)ff;
            for (int p = base + t; p < n && p <= ffin; p += nt) {
                const int kk = cols[p];
                const double nd = M.at(r, kk) - v[kk] - hh;
                if (nd < d[kk]) {
                    d[kk] = nd;
                    pred[kk] = r;
                    if (nd == dk && p < ffin)
                        atomicOr(&sh.bits[(p - base) >> 5], 1u << ((p - base) & 31));
                }
            }
        }
        block_sync();
        const int last = ffin < n ? ffin - base : cnt;
        h += lapb_swap_front(base, (last + 31) / 32, cols, hitpos, tmp, sh, pos);
        const int end = ffin < n ? cols[ffin] : -1;   // ffin is beyond every moved position
        LAPB_DT(64);
        if (end >= 0) return end;
    }
    lo = l;
    hi = h;
    return -1;
}

// gather_min (lapjv.c) by the block: returns the new hi.  A position qualifies when its distance
// is <= the running minimum of the earlier ones (starting from m0 = d[cols[lo]]); a strictly
// smaller one resets the front.  With m* the minimum over [lo, n): if m0 == m*, the qualifying
// positions are exactly the ties to m0 and the whole gather is one swap-to-front from lo + 1;
// otherwise the qualifying positions before the first occurrence q* of m* are replayed in order
// by thread 0 (with their resets), then q* and the later ties to m* are one swap-to-front from lo.
template <typename DP, typename IP, typename HP, typename TP>
__device__ int lapb_gather_min(int n, int lo, DP d, IP cols, HP hitpos, TP tmp, LapBShared &sh,
                               int &par, IP pos = nullptr) {
    const int t = threadIdx.x, nt = blockDim.x, lane = lane_id(), wv = t / WAVE;
    LAPB_ADD(65, 1);
    const double m0 = d[cols[lo]];
    const int first = lo + 1, cnt = n - first;
    double lmin = LAP_BIG;
    for (int q = first + t; q < n; q += nt) {
        const double e = d[cols[q]];
        lmin = e < lmin ? e : lmin;
    }
    const double gmin = lapb_reduce(true, lmin, sh, par);
    if (!(gmin < m0)) {   // no reset: the ties to m0, one swap-to-front from lo + 1
        for (int q = t; q < (cnt + 31) / 32; q += nt) sh.bits[q] = 0u;
        block_sync();
        for (int q = first + t; q < n; q += nt)
            if (d[cols[q]] == m0) atomicOr(&sh.bits[(q - first) >> 5], 1u << ((q - first) & 31));
        block_sync();
        return first + lapb_swap_front(first, (cnt + 31) / 32, cols, hitpos, tmp, sh, pos);
    }
    // q*: the first position holding the minimum
    double fq = 1e300;
    for (int q = first + t; q < n; q += nt)
        if (d[cols[q]] == gmin) {
            fq = (double)q;
            break;
        }
    const int qs = (int)lapb_reduce(true, fq, sh, par);
    // the qualifying positions in (lo, q*): prefix minima over contiguous ranges
    const int pc = qs - first;
    const int per = (pc + nt - 1) / nt;
    const int a = first + t * per, b = min(qs, a + per);
    double rmin = LAP_BIG;
    for (int q = a; q < b; ++q) {
        const double e = d[cols[q]];
        rmin = e < rmin ? e : rmin;
    }
    for (int q = t; q < (cnt + 31) / 32; q += nt) sh.bits[q] = 0u;
    const double incl = wave_incl_min(rmin);
    double excl = __shfl_up(incl, 1);
    if (lane == 0) excl = LAP_BIG;
    if (lane == WAVE - 1) sh.pre[wv] = incl;
    block_sync();
    for (int k = 0; k < wv; ++k) excl = sh.pre[k] < excl ? sh.pre[k] : excl;
    double run = m0 < excl ? m0 : excl;
    for (int q = a; q < b; ++q) {
        const double e = d[cols[q]];
        if (e <= run) {
            atomicOr(&sh.bits[(q - first) >> 5], 1u << ((q - first) & 31));
            run = e < run ? e : run;
        }
    }
    block_sync();
    if (t == 0) {   // their swaps (and resets) in position order
        int hi = lo + 1;
        double m = m0;
        for (int q = 0; q < (pc + 31) / 32; ++q) {
            unsigned bb = sh.bits[q];
            while (bb) {
                const int p = first + q * 32 + __builtin_ctz(bb);
                bb &= bb - 1u;
                const int k = cols[p];
                const double e = d[k];
                if (e < m) {
                    hi = lo;
                    m = e;
                }
                const int c = cols[hi];
                cols[p] = c;
                cols[hi] = k;
                if (pos) {
                    pos[c] = p;
                    pos[k] = hi;
                }
                ++hi;
            }
        }
    }
    block_sync();
    // the reset at q* and the ties after it: one swap-to-front from lo
    const int cnt2 = n - lo;
    for (int q = t; q < (cnt2 + 31) / 32; q += nt) sh.bits[q] = 0u;
    block_sync();
    for (int q = qs + t; q < n; q += nt)
        if (d[cols[q]] == gmin) atomicOr(&sh.bits[(q - lo) >> 5], 1u << ((q - lo) & 31));
    block_sync();
    return lo + lapb_swap_front(lo, (cnt2 + 31) / 32, cols, hitpos, tmp, sh, pos);
}

// Phase 3 for the free rows w.free_rows[0 .. nfree) left by phases 1-2 (all threads of the block).
// Returns 0, or -2 when an augmenting path does not close.
// The rows' nonzero entries (M.at != 0, ascending columns, up to LAPS_K; more: cnt -1), one wave
// per row, columns over the lanes.
__device__ __forceinline__ void lap_csr_build(int n, const LapMat &M, const LapCsr &cs) {
    const int lane = lane_id(), nw = blockDim.x / WAVE;
    for (int r = threadIdx.x / WAVE; r < n; r += nw) {
        int c = 0;   // the row's nonzero entries (counted first: each kept entry carries it)
        if (r < M.na)
            for (int k0 = 0; k0 < M.nb && c <= LAPS_K; k0 += WAVE) {
                const int k = k0 + lane;
                c += __popcll(__ballot(k < M.nb && M.real(r, k) != 0.0));
            }
        const int cnt = c <= LAPS_K ? c : -1;
        if (cnt <= 0) {
            if (lane == 0) cs.ent[(long long)r * LAPS_K] = lap_csr_entry(0.0, 0, cnt);
            continue;
        }
        int w = 0;
        for (int k0 = 0; k0 < M.nb && w < cnt; k0 += WAVE) {
            const int k = k0 + lane;
            const double e = k < M.nb ? M.real(r, k) : 0.0;
            const bool nz = k < M.nb && e != 0.0;
            const unsigned long long b = __ballot(nz);
            if (nz) cs.ent[(long long)r * LAPS_K + w + __popcll(b & ((1ull << lane) - 1ull))] =
                lap_csr_entry(e, k, cnt);
            w += __popcll(b);
        }
    }
}

// sh: the caller's (one static LDS instance for every instantiation).
template <bool LDS_WS, bool SPARSE>
__device__ int lap_dense_block_p3(int n, const LapMat M, const DenseLapWs w, int nfree,
                                  unsigned char *csr_ws, LapBShared &sh) {
    const int t = threadIdx.x, nt = blockDim.x;
    auto x = ws_ptr<LDS_WS>(w.x), y = ws_ptr<LDS_WS>(w.y), fr = ws_ptr<LDS_WS>(w.free_rows);
    auto cols = ws_ptr<LDS_WS>(w.cols), pred = ws_ptr<LDS_WS>(w.pred);
    auto v = ws_ptr<LDS_WS>(w.v), d = ws_ptr<LDS_WS>(w.d);
    // scratch of the swap-to-front: aux (n ints) and the unused row buffers (2 n doubles); with
    // the sparse sweeps aux holds the inverse permutation of cols and the hit positions go to the
    // row buffers' second half
    int *tmp = reinterpret_cast<int *>(w.row);
    constexpr bool sparse = SPARSE;
    auto hitpos = [&] {
        if constexpr (SPARSE) return tmp + 2 * n;
        else return ws_ptr<LDS_WS>(w.aux);
    }();
    decltype(ws_ptr<LDS_WS>(w.aux)) pos = SPARSE ? ws_ptr<LDS_WS>(w.aux) : nullptr;
    LapCsr cs{};
    if (sparse) {
        cs = lap_csr(csr_ws, n);
        lap_csr_build(n, M, cs);
        block_sync();
    }
    int par = 0;
    for (int f = 0; f < nfree; ++f) {
        const int src = fr[f];
        double lmax = -LAP_BIG;
        for (int k = t; k < n; k += nt) {
            const double c = M.at(src, k);
            cols[k] = k;
            if (sparse) pos[k] = k;
            pred[k] = src;
            d[k] = c - v[k];
            lmax = c > lmax ? c : lmax;
        }
        // the source row's maximum (bounds d + v of every column during this search)
        const double cmax = sparse ? lapb_reduce(false, lmax, sh, par) : 0.0;
        block_sync();
        int lo = 0, hi = 0, ready = 0, end = -1;
        while (end < 0) {
            if (lo == hi) {
                ready = lo;
                hi = lapb_gather_min(n, lo, d, cols, hitpos, tmp, sh, par, pos);
                // the last free column of the gathered set
                double e = -1.0;
                for (int q = lo + t; q < hi; q += nt)
                    if (y[cols[q]] < 0) e = (double)q;
                e = lapb_reduce(false, e, sh, par);
                if (e >= 0.0) end = cols[(int)e];
            }
            if (end < 0)
                end = lapb_relax_scan(n, M, lo, hi, d, v, cols, pred, y, hitpos, tmp, sh, par, pos,
                                      sparse ? &cs : nullptr, cmax);
        }
        const double m = d[cols[lo]];
        for (int q = t; q < ready; q += nt) {
            const int k = cols[q];
            v[k] += d[k] - m;
        }
        block_sync();
        if (t == 0) {   // flip the alternating path back to the source row
            int k = end, r = -1, steps = 0;
            sh.end = 0;
            while (r != src) {
                r = pred[k];
                y[k] = r;
                const int prev = x[r];
                x[r] = k;
                k = prev;
                if (++steps > n) {
                    sh.end = -2;
                    break;
                }
            }
        }
        block_sync();
        if (sh.end == -2) return -2;
        block_sync();
    }
    return 0;
}

// The whole replay on a block: phases 1-2 on wave 0, phase 3 block-wide when n is large enough,
// work arrays in LDS (without the row buffers, which phase 3 does not use) when they fit.  Every
// thread of the block calls it; `w` receives the layout (w.x: the assignment).  Returns the
// solver's rc (0 on success).
__device__ __forceinline__ int lap_dense_block(int n, const LapMat M, unsigned char *lds,
                                               long long lds_bytes, unsigned char *gws,
                                               DenseLapWs &w, unsigned char *csr_ws = nullptr) {
    __shared__ int s_rc;
    if (n < LAPB_MIN_N || n > LAPB_MAX_N || blockDim.x < 256) {
        if (threadIdx.x < WAVE) {
            const int rc = lap_dense_placed(n, M, lds, lds_bytes, gws, w);
            if (lane_id() == 0) s_rc = rc;
        } else {   // the layout lap_dense_placed picks, for the other threads' reads of w.x
            w = dense_lap_ws_bytes(n) <= lds_bytes ? dense_lap_ws(lds, n)
                : dense_lap_ws_bytes_norow(n) <= lds_bytes ? dense_lap_ws_split(lds, gws, n)
                                                           : dense_lap_ws(gws, n);
        }
        block_sync();
        return s_rc;
    }
    const bool in_lds = dense_lap_ws_bytes_norow(n) <= lds_bytes;
    w = in_lds ? dense_lap_ws_split(lds, gws, n) : dense_lap_ws(gws, n);
    YTA_STAMP_ABS(60);
    if (threadIdx.x < WAVE) {
        const int nf = in_lds ? lap_dense_wave<true, false, false>(n, M, w)
                              : lap_dense_wave<false, false, false>(n, M, w);
        if (lane_id() == 0) s_rc = nf;
    }
    block_sync();
    const int nfree = s_rc;
    block_sync();
    YTA_STAMP_ABS(61);
    if (nfree < 0) return nfree;
    __shared__ LapBShared sh;
    int rc;
    if (csr_ws) rc = in_lds ? lap_dense_block_p3<true, true>(n, M, w, nfree, csr_ws, sh)
                            : lap_dense_block_p3<false, true>(n, M, w, nfree, csr_ws, sh);
    else rc = in_lds ? lap_dense_block_p3<true, false>(n, M, w, nfree, nullptr, sh)
                     : lap_dense_block_p3<false, false>(n, M, w, nfree, nullptr, sh);
    YTA_STAMP_ABS(62);
    return rc;
}

}  // namespace yta
