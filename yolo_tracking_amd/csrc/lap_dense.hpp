// Dense linear assignment on one wavefront: the lapx `lapjv` algorithm (Jonker-Volgenant, dense
// form) with exactly the operation and tie-breaking sequence of oracle/lapjv.c, for the calls
//   boxmot/utils/association.py:20-28  lap.lapjv(cost, extend_cost=True)   (OCSORT family)
// whose cost matrices are dense (every pair has a finite cost, no cost_limit), so the sparse
// component solver of lap.hpp does not apply.
//
// Each phase keeps the sequential semantics of the C code; the work inside a step is spread over
// the 64 lanes:
//   column reduction   columns over lanes (first row wins: strict <); winner bookkeeping by
//                      per-row atomicMax (the highest column a row wins is the one it keeps, as the
//                      downward walk does) and counts (solo rows)
//   reduction transfer solo rows in ascending order (each reads the prices earlier rows lowered);
//                      the row scan is a lane-parallel min
//   row reduction      the free-row loop as written; each row's best / second-best reduced cost is
//                      a lane-parallel two-minimum with first-index ties
//   augmentation       Dijkstra over the column permutation `cols`: the min-gather and the relax
//                      sweep evaluate every position in parallel (each position is visited once
//                      and its distance only changes at its own visit), then lane 0 replays the
//                      swaps of the qualifying positions in position order, and the sweep stops at
//                      the first position that reaches a free column at the current minimum.
// The cost matrix is read through an accessor cost(r, c) (n x n, padded by the caller).  Work
// arrays (n ints x 5, n doubles x 2) are wave-private; `solo` n bytes.
#pragma once
#include <float.h>

#include "common.hpp"

namespace yta {

struct DenseLapWs {
    int *x, *y, *free_rows, *cols, *pred;
    double *v, *d;
    int *aux;   // n ints: per-row winner column / count scratch
};

__host__ __device__ inline long long dense_lap_ws_bytes(long long n) {
    return n * (6 * 4 + 2 * 8) + 64;
}

constexpr double LAP_BIG = DBL_MAX;

// (value, index) lexicographic "less": smaller value, then smaller index
__device__ __forceinline__ bool lex_less(double a, int ia, double b, int ib) {
    return a < b || (a == b && ia < ib);
}

// Wave all-reduce of the first minimum (value, lowest index); an index of -1 means "none" and
// loses to any real entry.
__device__ __forceinline__ void wave_argmin(double &m, int &k) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const double om = __shfl_xor(m, s);
        const int ok = __shfl_xor(k, s);
        const bool take = ok >= 0 && (k < 0 || lex_less(om, ok, m, k));
        if (take) { m = om; k = ok; }
    }
}

// First and second lexicographic minima of (s_k, k) over the wave's columns (k1: first index of
// the minimum; k2: first index of the minimum over k != k1 among values < LAP_BIG, else -1) - the
// result of lapjv.c's sequential two-minimum scan.
__device__ __forceinline__ void wave_two_min(double &m1, int &k1, double &m2, int &k2) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const double om1 = __shfl_xor(m1, s), om2 = __shfl_xor(m2, s);
        const int ok1 = __shfl_xor(k1, s), ok2 = __shfl_xor(k2, s);
        // winner W / loser L by first minimum
        const bool other_wins = ok1 >= 0 && (k1 < 0 || lex_less(om1, ok1, m1, k1));
        double wm1 = other_wins ? om1 : m1, wm2 = other_wins ? om2 : m2;
        int wk1 = other_wins ? ok1 : k1, wk2 = other_wins ? ok2 : k2;
        const double lm1 = other_wins ? m1 : om1;
        const int lk1 = other_wins ? k1 : ok1;
        // second = lexmin(W.second, L.first) (L.first only if < BIG)
        if (lk1 >= 0 && lm1 < LAP_BIG && (wk2 < 0 || lex_less(lm1, lk1, wm2, wk2))) {
            wm2 = lm1;
            wk2 = lk1;
        }
        m1 = wm1; k1 = wk1; m2 = wm2; k2 = wk2;
    }
}

// Square dense solve of n x n costs by the calling wave (all 64 lanes).  x[row] = col,
// y[col] = row.  Returns 0, or -2 if an augmenting path could not be traced (corrupt input).
template <typename Cost>
__device__ int lap_dense_wave(int n, Cost cost, const DenseLapWs &w) {
    const int lane = lane_id();
    int *x = w.x, *y = w.y, *fr = w.free_rows, *cols = w.cols, *pred = w.pred, *aux = w.aux;
    double *v = w.v, *d = w.d;
    if (n <= 0) return 0;
    // ---------------- phase 1: column reduction ----------------
    for (int k = lane; k < n; k += WAVE) {
        x[k] = -1;
        aux[k] = -1;
        double best = LAP_BIG;
        int br = 0;
        for (int r = 0; r < n; ++r) {
            const double c = cost(r, k);
            if (c < best) { best = c; br = r; }
        }
        v[k] = best;
        y[k] = br;
        pred[k] = 0;   // per-row win counts
    }
    wave_mem_sync();
    for (int k = lane; k < n; k += WAVE) {
        atomicMax(&aux[y[k]], k);   // the downward walk keeps the highest column a row wins
        atomicAdd(&pred[y[k]], 1);
    }
    wave_mem_sync();
    for (int k = lane; k < n; k += WAVE) {
        const int r = y[k];
        if (aux[r] != k) y[k] = -1;
    }
    for (int r = lane; r < n; r += WAVE) x[r] = aux[r];
    wave_mem_sync();
    // free rows (ascending) and solo rows' reduction transfer (ascending, sequential)
    int nfree = 0;
    for (int base = 0; base < n; base += WAVE) {
        const int r = base + lane;
        const bool f = r < n && x[r] < 0;
        const unsigned long long b = __ballot(f);
        if (f) fr[nfree + __popcll(b & ((1ull << lane) - 1))] = r;
        nfree += __popcll(b);
    }
    for (int r = 0; r < n; ++r) {
        const int own = x[r];
        if (own < 0 || pred[r] != 1) continue;   // free, or won several columns
        double best = LAP_BIG;
        for (int k = lane; k < n; k += WAVE)
            if (k != own) {
                const double s = cost(r, k) - v[k];
                if (s < best) best = s;
            }
        best = wave_reduce(RED_MIN, best);
        if (lane == 0) v[own] -= best;
        wave_mem_sync();
    }
    wave_mem_sync();
    // ---------------- phase 2: augmenting row reduction (at most twice) ----------------
    for (int pass = 0; nfree > 0 && pass < 2; ++pass) {
        int pos = 0, out = 0;
        unsigned long long iters = 0;
        while (pos < nfree) {
            ++iters;
            const int r = fr[pos++];
            double m1 = LAP_BIG, m2 = LAP_BIG;
            int k1 = -1, k2 = -1;
            for (int k = lane; k < n; k += WAVE) {   // this lane's columns, ascending
                const double s = cost(r, k) - v[k];
                if (k1 < 0) { m1 = s; k1 = k; continue; }
                if (s < m2) {
                    if (s >= m1) { m2 = s; k2 = k; }
                    else { m2 = m1; k2 = k1; m1 = s; k1 = k; }
                }
            }
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
            wave_mem_sync();
        }
        nfree = out;
    }
    // ---------------- phase 3: shortest augmenting paths ----------------
    for (int f = 0; f < nfree; ++f) {
        const int src = fr[f];
        for (int k = lane; k < n; k += WAVE) {
            cols[k] = k;
            pred[k] = src;
            d[k] = cost(src, k) - v[k];
        }
        wave_mem_sync();
        int lo = 0, hi = 0, ready = 0, end = -1;
        while (end < 0) {
            if (lo == hi) {
                // gather_min: positions lo.. n-1; qualifying positions are those whose value is
                // <= the running minimum of the earlier ones (resets where strictly smaller)
                ready = lo;
                const double m0 = d[cols[lo]];
                double run = m0;   // running min carried across chunks
                hi = lo + 1;
                for (int base = lo + 1; base < n; base += WAVE) {
                    const int t = base + lane;
                    const double e = t < n ? d[cols[t]] : LAP_BIG;
                    // exclusive prefix min within the chunk
                    double pm = e;
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
                    // lane 0 replays the swaps in position order
                    if (lane == 0) {
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
                    const double cm = __shfl(pm, WAVE - 1);
                    run = cm < run ? cm : run;
                    wave_mem_sync();
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
            }
            if (end < 0) {
                // relax_scan from the scan set [lo, hi)
                int slo = lo, shi = hi, ret = -1;
                while (slo != shi && ret < 0) {
                    const int k = cols[slo++];
                    const int r = y[k];
                    const double dk = d[k];
                    const double h = cost(r, k) - v[k] - dk;
                    for (int base = shi; base < n && ret < 0; base += WAVE) {
                        const int t = base + lane;
                        int kk = -1;
                        double nd = 0.0;
                        bool imp = false;
                        if (t < n) {
                            kk = cols[t];
                            nd = cost(r, kk) - v[kk] - h;
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
                        wave_mem_sync();
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
                        wave_mem_sync();
                        if (first_fin < WAVE) ret = __shfl(kk, first_fin);
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
        wave_mem_sync();
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
        wave_mem_sync();
        if (aux[0] == -2) return -2;
    }
    return 0;
}

}  // namespace yta
