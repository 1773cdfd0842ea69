// Block-level exact sparse linear assignment with lapx's cost_limit semantics (see assoc.hpp for
// why only edges c < t matter).  Called by the fused per-stream kernels (bytetrack.hip) and the
// KAT entry (kat.hip) on a CSR graph that the caller built:
//
//   row_off[nr+1], csr_col[E], csr_cost[E]  rows' candidate edges (any order within a row)
//   col_deg[nc]                             number of edges per column
//
// Phases (one block, every thread calls lap_block):
//   P1  every row with one edge whose column has one edge is matched outright; every other edge
//       unites its row and column (lock-free union-find)
//   P2  complex nodes (unmatched, with edges) get their root (full path compression); count
//   P3  complex nodes and component roots listed in node order
//   P4  components gathered by counting sort (rows then columns, ascending)
//   P5  one-row components take their cheapest edge (lowest cost, then lowest column: what the
//       shortest-augmenting-path solve gives); components of <= 3 rows and <= 3 columns with a
//       unique optimum are enumerated by one thread (solve_small); the rest are solved exactly by
//       successive shortest
//       augmenting paths with one private zero-cost dummy column per row: 16-lane segments (four
//       components per wave), one wave (<= 64 columns + dummies), or a global-memory slab.
//
// Memory comes from an Arena: the caller instantiates the fused kernel twice, once with the arena
// over LDS and once over the stream's global workspace (a frame whose problem does not fit in LDS
// is redone in the global instantiation).  All pointers are plain C++ pointers; after inlining the
// compiler knows their address space, so the LDS instantiation issues ds_* instructions.
#pragma once
#include <climits>

#include "common.hpp"

namespace yta {

constexpr int ERR_EDGE_OVERFLOW = 1;   // workspace too small for the frame (capacity)
constexpr int ERR_SOLVER = 2;
constexpr int ERR_TRACK_CAPACITY = 4;
constexpr int ERR_DET_CAPACITY = 8;
constexpr int ERR_CLS_HIST = 16;       // a BoT-SORT track voted over more than CLS_K classes

__device__ __forceinline__ int ald(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double aldd(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wave_mem_sync() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// Two-ended bump allocator over one region (LDS or global).  Every thread of the block performs
// the same allocations, so `fail` is block-uniform.
struct Arena {
    unsigned char *base;
    size_t lo, hi, cap;
    bool fail;
    __device__ __forceinline__ Arena(void *b, size_t c)
        : base((unsigned char *)b), lo(0), hi(c), cap(c), fail(false) {}
    __device__ __forceinline__ void reset() { lo = 0; hi = cap; fail = false; }
    __device__ __forceinline__ static size_t round(long long n, size_t sz) {
        return ((size_t)(n > 0 ? n : 1) * sz + 15) & ~(size_t)15;
    }
    template <typename T>
    __device__ __forceinline__ T *alloc(long long n) {
        const size_t b = round(n, sizeof(T));
        if (fail || b > hi - lo) { fail = true; return (T *)base; }
        T *p = (T *)(base + lo);
        lo += b;
        return p;
    }
    // optional caches: nullptr (and no failure) when the space is not there
    template <typename T>
    __device__ __forceinline__ T *try_alloc(long long n) {
        const size_t b = round(n, sizeof(T));
        if (fail || b > hi - lo) return nullptr;
        T *p = (T *)(base + lo);
        lo += b;
        return p;
    }
    template <typename T>
    __device__ __forceinline__ T *try_alloc_top(long long n) {
        const size_t b = round(n, sizeof(T));
        if (fail || b > hi - lo) return nullptr;
        hi -= b;
        return (T *)(base + hi);
    }
    template <typename T>
    __device__ __forceinline__ T *alloc_top(long long n) {
        const size_t b = round(n, sizeof(T));
        if (fail || b > hi - lo) { fail = true; return (T *)base; }
        hi -= b;
        return (T *)(base + hi);
    }
};

// Global-memory state of the large-component solver: one slab per wave.
struct LapSlab {
    int *i;               // per wave: y[V] pred[V] vis[V] x[R] rowg[R] colg[C] col_local[C]
    double *d;            // per wave: d[V] v[V] u[R]
    long long i_stride, d_stride;
    int R, C;             // capacities (V = R + C)
};

__host__ __device__ inline long long lap_slab_ints(int R, int C) {
    return 3LL * (R + C) + 2LL * R + 2LL * C;
}
__host__ __device__ inline long long lap_slab_doubles(int R, int C) {
    return 2LL * (R + C) + R;
}

// Exact solve of one component with V = l + k <= W columns (+ dummies), on a W-lane segment of the
// wave (W = 16 or 64): one column per lane, rows on lanes < k.  rows_in / cols_in: ascending
// global ids.  Control flow is uniform within a segment and every shuffle stays inside it.
template <int W>
__device__ __forceinline__ void solve_seg(int k, int l, const int *rows_in, const int *cols_in,
                                          const int *row_off, const int *csr_col,
                                          const double *csr_cost, double thresh, int *X, int *Y,
                                          int *err) {
    const int lane = lane_id() & (W - 1);
    const int base = lane_id() & ~(W - 1);
    const unsigned long long segmask = (W == 64) ? ~0ull : (((1ull << W) - 1) << base);
    const int V = l + k;
    const int rowg = lane < k ? rows_in[lane] : -1;
    const int colg = lane < l ? cols_in[lane] : -1;
    double v = 0.0, u = 0.0;
    int y = -1, x = -1;
    for (int cur = 0; cur < k; ++cur) {
        double d = INFINITY;
        bool vis = false;
        int pred = -1;
        double minval = 0.0;
        int i = cur, sink = -1;
        for (int guard = 0; guard <= V; ++guard) {
            const int gi = __shfl(rowg, i, W);
            const double ui = __shfl(u, i, W);
            const int beg = row_off[gi], end = row_off[gi + 1];
            for (int e = beg; e < end; ++e) {
                const int c = csr_col[e];
                const double w = csr_cost[e];
                const unsigned long long mm = __ballot(lane < l && colg == c) & segmask;
                const int j = (int)__ffsll((long long)mm) - 1 - base;
                if (lane == j && !vis) {
                    const double r = minval + (w - thresh) - ui - v;
                    if (r < d) { d = r; pred = i; }
                }
            }
            if (lane == l + i && !vis) {
                const double r = minval + 0.0 - ui - v;
                if (r < d) { d = r; pred = i; }
            }
            // argmin: lower distance, then a free column, then the lower lane
            double bd = (lane < V && !vis) ? d : INFINITY;
            bd = W == 16 ? row_allreduce(RED_MIN, bd) : wave_reduce(RED_MIN, bd);
            if (!(bd < INFINITY)) { if (lane == 0) atomicOr(err, ERR_SOLVER); return; }
            const bool cand = lane < V && !vis && d == bd;
            const unsigned long long mfree = __ballot(cand && y < 0) & segmask;
            const unsigned long long many = __ballot(cand) & segmask;
            const int jstar = (int)__ffsll((long long)(mfree ? mfree : many)) - 1 - base;
            minval = bd;
            if (lane == jstar) vis = true;
            const int owner = __shfl(y, jstar, W);
            if (owner < 0) { sink = jstar; break; }
            i = owner;
        }
        if (sink < 0) { if (lane == 0) atomicOr(err, ERR_SOLVER); return; }
        // duals: rows entered during the search own the visited non-sink columns
        const bool upd = lane < V && vis && lane != sink;
        const double delta = minval - d;
        const int jr = x >= 0 ? x : 0;
        const double dj = __shfl(delta, jr, W);
        const int vj = __shfl(upd ? 1 : 0, jr, W);
        if (lane < k && x >= 0 && vj) u += dj;
        if (upd) v -= delta;
        if (lane == cur) u += minval;
        // augment along pred
        int j = sink;
        for (int guard = 0; guard <= V; ++guard) {
            const int r = __shfl(pred, j, W);
            if (lane == j) y = r;
            const int prev = __shfl(x, r, W);
            if (lane == r) x = j;
            j = prev;
            if (r == cur) break;
        }
    }
    const int cg = __shfl(colg, (x >= 0 && x < l) ? x : 0, W);
    if (lane < k) {
        if (x >= 0 && x < l) {
            X[rowg] = cg;
            Y[cg] = rowg;
        } else {
            X[rowg] = -1;
        }
    }
}

// Same algorithm for components beyond one wavefront, state in a global-memory slab (one lane
// per column, strided).  Rare: only dense clutter produces them.
__device__ __noinline__ void solve_large(int *bi, double *bd, int R, int C, const int *rows_in,
                                         int k, const int *cols_in, int l, const int *row_off,
                                         const int *csr_col, const double *csr_cost, double thresh,
                                         int *X, int *Y, int *err) {
    const long long V0 = (long long)R + C;
    int *sy = bi, *spred = bi + V0, *svis = bi + 2 * V0, *sx = bi + 3 * V0;
    int *srowg = sx + R, *scolg = srowg + R, *scol_local = scolg + C;
    double *sd = bd, *sv = bd + V0, *su = bd + 2 * V0;
    const int lane = lane_id();
    const int V = l + k;
    for (int a = lane; a < k; a += WAVE) srowg[a] = rows_in[a];
    for (int a = lane; a < l; a += WAVE) {
        scolg[a] = cols_in[a];
        scol_local[cols_in[a]] = a;
    }
    for (int j = lane; j < V; j += WAVE) { sv[j] = 0.0; sy[j] = -1; }
    for (int q = lane; q < k; q += WAVE) { su[q] = 0.0; sx[q] = -1; }
    wave_mem_sync();
    for (int cur = 0; cur < k; ++cur) {
        for (int j = lane; j < V; j += WAVE) { sd[j] = INFINITY; svis[j] = 0; }
        wave_mem_sync();
        double minval = 0.0;
        int i = cur, sink = -1;
        for (int guard = 0; guard <= V; ++guard) {
            const int gi = ald(srowg + i);
            const double ui = aldd(su + i);
            const int beg = row_off[gi], end = row_off[gi + 1];
            for (int e = beg + lane; e < end; e += WAVE) {
                const int j = ald(scol_local + csr_col[e]);
                if (!ald(svis + j)) {
                    const double r = minval + (csr_cost[e] - thresh) - ui - aldd(sv + j);
                    if (r < aldd(sd + j)) { sd[j] = r; spred[j] = i; }
                }
            }
            if (lane == 0) {
                const int j = l + i;
                if (!ald(svis + j)) {
                    const double r = minval + 0.0 - ui - aldd(sv + j);
                    if (r < aldd(sd + j)) { sd[j] = r; spred[j] = i; }
                }
            }
            wave_mem_sync();
            double bdist = INFINITY;
            int bk = INT_MAX;
            for (int j = lane; j < V; j += WAVE) {
                if (!ald(svis + j)) {
                    const double dj = aldd(sd + j);
                    const int kj = ((ald(sy + j) >= 0) << 30) | j;
                    if (dj < bdist || (dj == bdist && kj < bk)) { bdist = dj; bk = kj; }
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const double od = __shfl_xor(bdist, off);
                const int ok = __shfl_xor(bk, off);
                if (od < bdist || (od == bdist && ok < bk)) { bdist = od; bk = ok; }
            }
            if (!(bdist < INFINITY)) { if (lane == 0) atomicOr(err, ERR_SOLVER); return; }
            const int jstar = bk & ((1 << 30) - 1);
            minval = bdist;
            if (lane == 0) svis[jstar] = 1;
            const int owner = ald(sy + jstar);
            wave_mem_sync();
            if (owner < 0) { sink = jstar; break; }
            i = owner;
        }
        if (sink < 0) { if (lane == 0) atomicOr(err, ERR_SOLVER); return; }
        for (int j = lane; j < V; j += WAVE) {
            if (ald(svis + j) && j != sink) {
                const double delta = minval - aldd(sd + j);
                su[ald(sy + j)] += delta;   // distinct rows per visited column
                sv[j] -= delta;
            }
        }
        wave_mem_sync();
        if (lane == 0) {
            su[cur] += minval;
            int j = sink;
            for (int guard = 0; guard <= V; ++guard) {
                const int r = ald(spred + j);
                sy[j] = r;
                const int prev = ald(sx + r);
                sx[r] = j;
                j = prev;
                if (r == cur) break;
            }
        }
        wave_mem_sync();
    }
    for (int q = lane; q < k; q += WAVE) {
        const int j = ald(sx + q);
        const int g = ald(srowg + q);
        if (j >= 0 && j < l) {
            const int cg = ald(scolg + j);
            X[g] = cg;
            Y[cg] = g;
        } else {
            X[g] = -1;
        }
    }
    wave_mem_sync();
}

// Components with k <= 3 rows and l <= 3 columns, solved by one thread that enumerates every
// matching (<= 64).  The objective is sum(c - thresh) over the matched edges (assoc.hpp), summed in
// row order.  When the best matching beats every other one by more than a rounding margin it is
// the unique optimum, which every exact solver returns (solve_seg and lapx included); on a
// (near-)tie this returns false and the component goes to solve_seg, whose tie-breaking the
// goldens were checked against.  Every index below is a compile-time constant after unrolling,
// so the 3x3 cost block stays in registers.
constexpr double SMALL_TIE_MARGIN = 1e-12;
__device__ __forceinline__ bool solve_small(int k, int l, const int *rows, const int *cols,
                                            const int *row_off, const int *csr_col,
                                            const double *csr_cost, double thresh, int *X,
                                            int *Y) {
    double C[3][3];
    bool has[3][3];
    int rg[3], cg[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        rg[a] = a < k ? rows[a] : -1;
        cg[a] = a < l ? cols[a] : -1;
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            C[a][b] = 0.0;
            has[a][b] = false;
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (a >= k) continue;
        const int e0 = row_off[rg[a]], e1 = row_off[rg[a] + 1];
#pragma unroll
        for (int q = 0; q < 3; ++q) {   // a row's edges all lead to the component's <= 3 columns
            if (e0 + q >= e1) continue;
            const int col = csr_col[e0 + q];
            const double w = csr_cost[e0 + q] - thresh;
#pragma unroll
            for (int b = 0; b < 3; ++b)
                if (col == cg[b]) {
                    C[a][b] = w;
                    has[a][b] = true;
                }
        }
    }
    double best = INFINITY, second = INFINITY;
    int best_code = -1;
#pragma unroll
    for (int x0 = -1; x0 < 3; ++x0)
#pragma unroll
        for (int x1 = -1; x1 < 3; ++x1)
#pragma unroll
            for (int x2 = -1; x2 < 3; ++x2) {
                if ((x1 >= 0 && x1 == x0) || (x2 >= 0 && (x2 == x0 || x2 == x1))) continue;
                bool ok = (x0 < 0 || (k > 0 && has[0][x0 < 0 ? 0 : x0])) &&
                          (x1 < 0 || (k > 1 && has[1][x1 < 0 ? 0 : x1])) &&
                          (x2 < 0 || (k > 2 && has[2][x2 < 0 ? 0 : x2]));
                if (!ok) continue;
                double o = 0.0;
                if (x0 >= 0) o = o + C[0][x0 < 0 ? 0 : x0];
                if (x1 >= 0) o = o + C[1][x1 < 0 ? 0 : x1];
                if (x2 >= 0) o = o + C[2][x2 < 0 ? 0 : x2];
                if (o < best) {
                    second = best;
                    best = o;
                    best_code = (x0 + 1) | ((x1 + 1) << 2) | ((x2 + 1) << 4);
                } else if (o < second) {
                    second = o;
                }
            }
    if (!(second - best > SMALL_TIE_MARGIN)) return false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (a >= k) continue;
        const int x = ((best_code >> (2 * a)) & 3) - 1;
        int colg = -1;
#pragma unroll
        for (int b = 0; b < 3; ++b)
            if (x == b) colg = cg[b];
        X[rg[a]] = colg;
        if (colg >= 0) Y[colg] = rg[a];
    }
    return true;
}

// Reads of arrays that other threads modify with atomics go through ald(): on global memory they
// bypass the CU's L1 (the atomics execute in L2); on LDS they are plain ds_read.
__device__ __forceinline__ int uf_find(const int *parent, int a) {
    int p = ald(parent + a);
    while (p != a) { a = p; p = ald(parent + a); }
    return a;
}

// Lock-free union by lower root (roots only ever point to a smaller root).
__device__ __forceinline__ void uf_union(int *parent, int a, int b) {
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) { const int t = a; a = b; b = t; }
        if (atomicCAS(parent + a, a, b) == a) return;
    }
}

struct LapShared {       // static LDS of the calling kernel
    int wsum[32];
    int cnt[4];
};

// Solve one problem.  X[nr], Y[nc] (global) receive the assignment.  Arrays come from `ar`
// (lo end); returns false if the arena is exhausted (X / Y then hold garbage; the caller redoes
// the frame with a larger arena or reports capacity).  Every thread of the block calls it.
// init_xy false: the caller already set X / Y (-1, or pairs of components it matched itself and
// left out of the graph); only matched pairs are written.
__device__ __forceinline__ bool lap_block(int nr, int nc, const int *row_off, const int *csr_col,
                                          const double *csr_cost, const int *col_deg,
                                          double thresh, int *X, int *Y, int *err, Arena &ar,
                                          const LapSlab &slab, LapShared &sh, bool init_xy = true) {
    const int t = threadIdx.x, nt = blockDim.x;
    const int N = nr + nc;
    if (init_xy) {
        for (int i = t; i < nr; i += nt) X[i] = -1;
        for (int j = t; j < nc; j += nt) Y[j] = -1;
    }
    const int E = nr > 0 ? row_off[nr] : 0;
    if (E == 0) {
        block_sync();
        return true;
    }
    int *parent = ar.alloc<int>(N);
    if (ar.fail) return false;
    for (int n = t; n < N; n += nt) parent[n] = n;
    if (t == 0) { sh.cnt[0] = 0; sh.cnt[1] = 0; }
    block_sync();
    YTA_STAMP(8);
    // P1: single-edge components matched outright, every other edge united
    for (int i = t; i < nr; i += nt) {
        const int b = row_off[i], e = row_off[i + 1];
        for (int k = b; k < e; ++k) {
            const int c = csr_col[k];
            if (e - b == 1 && ald(col_deg + c) == 1) {
                X[i] = c;
                Y[c] = i;
            } else {
                uf_union(parent, i, nr + c);
            }
        }
    }
    block_sync();
    YTA_STAMP(9);
    // P2: roots of the complex nodes (full path compression: a concurrent find only ever sees a
    // parent replaced by one of its ancestors), counts of complex nodes and of components
    auto complex_node = [&](int n) {
        return n < nr ? (row_off[n + 1] > row_off[n] && ald(X + n) < 0)
                      : (ald(col_deg + n - nr) > 0 && ald(Y + n - nr) < 0);
    };
    for (int start = 0; start < N; start += nt) {
        const int n = start + t;
        bool cx = false, rt = false;
        if (n < N && complex_node(n)) {
            cx = true;
            const int r = uf_find(parent, n);
            rt = r == n;
            if (!rt) parent[n] = r;
        }
        const unsigned long long bc = __ballot(cx), br = __ballot(rt);
        if (lane_id() == 0 && bc) {
            atomicAdd(&sh.cnt[0], __popcll(bc));
            atomicAdd(&sh.cnt[1], __popcll(br));
        }
    }
    block_sync();
    YTA_STAMP(10);
    const int ncx = sh.cnt[0], ncomp = sh.cnt[1];
    if (ncomp == 0) return true;
    int *cnodes = ar.alloc<int>(ncx);
    int *roots = ar.alloc<int>(ncomp);
    int *kc = ar.alloc<int>(ncomp + 1);
    int *lc = ar.alloc<int>(ncomp + 1);
    int *moff = ar.alloc<int>(ncomp + 1);
    int *members = ar.alloc<int>(ncx);
    int *queue = ar.alloc<int>(ncomp);
    int *big_q = ar.alloc<int>(ncomp);
    if (ar.fail) return false;
    // P3: complex nodes and roots in node order (each thread a contiguous run of nodes, one block
    // scan of the packed counts)
    for (int base = 0; base < N; base += 32 * nt) {
        const int m = N - base < 32 * nt ? N - base : 32 * nt;
        const int per = (m + nt - 1) / nt;
        const int lo = base + t * per;
        const int hi = lo + per < base + m ? lo + per : base + m;
        unsigned bc = 0, br = 0;
        for (int n = lo; n < hi; ++n) {
            if (!complex_node(n)) continue;
            bc |= 1u << (n - lo);
            if (ald(parent + n) == n) br |= 1u << (n - lo);
        }
        int tot;
        const int ex = block_exclusive_scan(__popc(bc) | (__popc(br) << 16), sh.wsum, &tot);
        int pc = (base == 0 ? 0 : sh.cnt[2]) + (ex & 0xFFFF);
        int pr = (base == 0 ? 0 : sh.cnt[3]) + (ex >> 16);
        while (bc) {
            const int k = __ffs(bc) - 1;
            bc &= bc - 1;
            cnodes[pc++] = lo + k;
            if ((br >> k) & 1u) roots[pr++] = lo + k;
        }
        block_sync();
        if (t == 0) {
            sh.cnt[2] = (base == 0 ? 0 : sh.cnt[2]) + (tot & 0xFFFF);
            sh.cnt[3] = (base == 0 ? 0 : sh.cnt[3]) + (tot >> 16);
        }
        block_sync();
    }
    for (int c = t; c < ncomp; c += nt) { kc[c] = 0; lc[c] = 0; }
    block_sync();
    YTA_STAMP(11);
    // P4: per-component row / column counts, offsets, members (roots are ascending: binary search)
    auto comp_of = [&](int n) {
        const int r = ald(parent + n);
        int lo = 0, hi = ncomp - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (roots[mid] < r) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    for (int q = t; q < ncx; q += nt) {
        const int n = cnodes[q];
        atomicAdd(n < nr ? kc + comp_of(n) : lc + comp_of(n), 1);
    }
    block_sync();
    {
        int run = 0;
        for (int start = 0; start < ncomp; start += nt) {
            const int c = start + t;
            const int sz = c < ncomp ? ald(kc + c) + ald(lc + c) : 0;
            int tot;
            const int pos = block_exclusive_scan(sz, sh.wsum, &tot);
            if (c < ncomp) {
                moff[c] = run + pos;
                lc[c] = run + pos + ald(kc + c);   // column cursor
                kc[c] = run + pos;           // row cursor
            }
            run += tot;
        }
        if (t == 0) moff[ncomp] = run;
    }
    block_sync();
    for (int q = t; q < ncx; q += nt) {
        const int n = cnodes[q];
        const int c = comp_of(n);
        const int pos = atomicAdd(n < nr ? kc + c : lc + c, 1);
        members[pos] = n < nr ? n : n - nr;
    }
    if (t == 0) { sh.cnt[0] = 0; sh.cnt[1] = 0; sh.cnt[2] = 0; }
    block_sync();
    YTA_STAMP(12);
    // P5: classify and solve.  After the gather kc[c] = end of rows, lc[c] = end of columns.  The
    // members of a component are in ascending order within rows and within columns only after a
    // sort: atomics scattered them, so each component sorts its (few) members first.
    for (int c = t; c < ncomp; c += nt) {
        const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
        // insertion sort rows [m0, mr) and columns [mr, me) (components are tiny)
        for (int a = m0 + 1; a < mr; ++a) {
            const int v = members[a];
            int b = a - 1;
            while (b >= m0 && members[b] > v) { members[b + 1] = members[b]; --b; }
            members[b + 1] = v;
        }
        for (int a = mr + 1; a < me; ++a) {
            const int v = members[a];
            int b = a - 1;
            while (b >= mr && members[b] > v) { members[b + 1] = members[b]; --b; }
            members[b + 1] = v;
        }
        const int k = mr - m0, l = me - mr;
        if (k == 1) {
            const int r = members[m0];
            int bestc = -1;
            double bestw = INFINITY;
            for (int e = row_off[r]; e < row_off[r + 1]; ++e) {
                const double w = csr_cost[e];
                const int col = csr_col[e];
                if (w < bestw || (w == bestw && col < bestc)) { bestw = w; bestc = col; }
            }
            X[r] = bestc;
            Y[bestc] = r;
        } else if (k <= 3 && l <= 3 &&
                   solve_small(k, l, members + m0, members + mr, row_off, csr_col, csr_cost,
                               thresh, X, Y)) {
            // unique optimum of a small component
        } else if (k + l <= 16) {
#ifdef YTA_STAMPS
            if (blockIdx.x == 0) {   // component shapes (tools/diag_s1.py)
                const int bkt = l == 1 ? (k == 2 ? 0 : 1)
                                       : (k == 2 && l == 2 ? 2 : (k == 2 ? 3 : (k == 3 && l == 2 ? 4 : (k + l <= 6 ? 5 : 6))));
                atomicAdd(&g_stamps[117 + bkt], 1ull);
            }
#endif
            queue[atomicAdd(&sh.cnt[0], 1)] = c;
        } else if (k + l <= 64) {
            queue[ncomp - 1 - atomicAdd(&sh.cnt[1], 1)] = c;
        } else {
            big_q[atomicAdd(&sh.cnt[2], 1)] = c;
        }
    }
    block_sync();
    YTA_STAMP(13);
    const int n16 = sh.cnt[0], n64 = sh.cnt[1], nbig = sh.cnt[2];
#ifdef YTA_STAMPS
    if (blockIdx.x == 0 && t == 0) {
        g_stamps[g_stamp_off + 15] = n16;
        g_stamps[g_stamp_off + 16] = n64;
        g_stamps[g_stamp_off + 17] = nbig;
        g_stamps[g_stamp_off + 18] = E;
        g_stamps[g_stamp_off + 19] = ncx;
    }
#endif
    const int wave = t / WAVE, lane = lane_id(), nwaves = nt / WAVE;
    for (int q = wave * 4 + (lane >> 4); q - (lane >> 4) < n16; q += nwaves * 4) {
        if (q < n16) {
            const int c = queue[q];
            const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
            solve_seg<16>(mr - m0, me - mr, members + m0, members + mr, row_off, csr_col, csr_cost,
                          thresh, X, Y, err);
        }
    }
    for (int q = wave; q < n64; q += nwaves) {
        const int c = queue[ncomp - 1 - q];
        const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
        solve_seg<64>(mr - m0, me - mr, members + m0, members + mr, row_off, csr_col, csr_cost,
                      thresh, X, Y, err);
    }
    for (int q = wave; q < nbig; q += nwaves) {
        const int c = big_q[q];
        const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
        if (nr > slab.R || nc > slab.C) {
            if (lane == 0) atomicOr(err, ERR_EDGE_OVERFLOW);
            continue;
        }
        solve_large(slab.i + wave * slab.i_stride, slab.d + wave * slab.d_stride, slab.R, slab.C,
                    members + m0, mr - m0, members + mr, me - mr, row_off, csr_col, csr_cost,
                    thresh, X, Y, err);
    }
    block_sync();
    YTA_STAMP(14);
    return true;
}

}  // namespace yta
