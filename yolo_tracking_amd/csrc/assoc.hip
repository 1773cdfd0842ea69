// Association kernels for gfx950: candidate edges + exact sparse assignment (see assoc.hpp).
#include <climits>
#include <cmath>

#include "assoc.hpp"

namespace yta {

namespace {

constexpr int EDGE_THREADS = 256;
constexpr int EDGE_SBUF = 1024;        // block-local edge staging (LDS)

constexpr int LAP_THREADS = 1024;
constexpr int LAP_WAVES = LAP_THREADS / WAVE;
constexpr int LAP_LDS_NODES = 3200;    // node arrays in LDS when rows + cols capacity fits
constexpr int LAP_LDS_EDGES = 2048;    // CSR in LDS when the frame's edge count fits

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

__device__ __forceinline__ const ProblemSet &pick(const ProblemSet &a, int na, const ProblemSet &b,
                                                  int p, int &local) {
    if (p < na) { local = p; return a; }
    local = p - na;
    return b;
}

// ------------------------------------------------------------------------------ edge extraction
// One thread per track row.  Candidates come from the column grid (or all columns when the
// threshold admits non-intersecting pairs); each candidate is scored with the reference's
// float64 expression and kept iff cost < thresh.  Edges are staged in LDS and appended to the
// problem's pool with one atomic per block.
__global__ __launch_bounds__(EDGE_THREADS) void edges_kernel(ProblemSet A, int na, ProblemSet B) {
    __shared__ Edge sbuf[EDGE_SBUF];
    __shared__ int s_n, s_base;
    int p;
    const ProblemSet &ps = pick(A, na, B, blockIdx.y, p);
    const int nr = ps.n_rows[(long long)p * ps.n_rows_stride];
    const int nc = ps.n_cols[(long long)p * ps.n_cols_stride];
    if ((int)(blockIdx.x * EDGE_THREADS) >= nr || nc <= 0) return;   // block-uniform
    const int t = threadIdx.x;
    const int row = blockIdx.x * EDGE_THREADS + t;
    if (t == 0) s_n = 0;
    block_sync();
    Edge *edges = ps.edges + p * ps.edges_stride;
    int *n_edges = ps.n_edges + (long long)p * ps.n_edges_stride;
    int *err = ps.err + (long long)p * ps.err_stride;
    const Box *cols = ps.cols + p * ps.cols_stride;
    const double *colw = ps.col_score ? ps.col_score + p * ps.score_stride : nullptr;
    const double thresh = ps.thresh;

    auto emit = [&](int r, int c, double cost) {
        int pos = atomicAdd(&s_n, 1);
        Edge e;
        e.row = r;
        e.col = c;
        e.cost = cost;
        if (pos < EDGE_SBUF) {
            sbuf[pos] = e;
        } else {
            long long g = atomicAdd(n_edges, 1);
            if (g < ps.edge_cap) edges[g] = e;
            else atomicOr(err, ERR_EDGE_OVERFLOW);
        }
    };
    auto score = [&](const Box &rb, const Box &cb, int c) {
        const double dist = 1 - iou(rb, cb);                             // matching.py:117
        const double cost = colw ? 1 - (1 - dist) * colw[c] : dist;      // matching.py:216-220
        if (cost < thresh) emit(row, c, cost);
    };

    if (row < nr) {
        const Box rb = ps.rows[p * ps.rows_stride + row];
        if (ps.ghdr && thresh <= 1.0) {
            const GridView gv{ps.ghdr + p, ps.gcell + p * ps.gcell_stride,
                              ps.gitems + p * ps.gitems_stride, ps.gboxes + p * ps.gitems_stride,
                              ps.gbig + p * ps.gitems_stride};
            const GridHdr h = *gv.hdr;
            const int *remap = ps.remap ? ps.remap + p * ps.remap_stride : nullptr;
            grid_query(
                gv, h, rb,
                [&](int item, const Box &cb) {
                    if (!intersects(rb, cb)) return;
                    const int c = remap ? remap[item] : item;
                    if (c >= 0) score(rb, cb, c);
                },
                [&](int item) {
                    const int c = remap ? remap[item] : item;
                    if (c < 0) return;
                    const Box cb = cols[c];
                    if (intersects(rb, cb)) score(rb, cb, c);
                });
        } else {
            // thresholds above 1 admit non-intersecting pairs: score every column
            for (int c = 0; c < nc; ++c) {
                const Box cb = cols[c];
                if (thresh > 1.0 || intersects(rb, cb)) score(rb, cb, c);
            }
        }
    }
    block_sync();
    const int n = s_n < EDGE_SBUF ? s_n : EDGE_SBUF;
    if (t == 0) s_base = n ? atomicAdd(n_edges, n) : 0;
    block_sync();
    for (int k = t; k < n; k += EDGE_THREADS) {
        long long g = (long long)s_base + k;
        if (g < ps.edge_cap) edges[g] = sbuf[k];
        else atomicOr(err, ERR_EDGE_OVERFLOW);
    }
}

// ------------------------------------------------------------------------------ solver
// Global workspace (per problem) used when the node arrays do not fit in LDS, plus the
// global-memory slabs of the large-component fallback.
struct LapWs {
    int *parent, *deg, *row_off, *cnodes, *croot, *roots, *comp_of, *members, *queue, *big_q;
    int *csr_col;
    double *csr_cost;
    int *big_i;       // per wave: y[V] pred[V] vis[V] x[R] rowg[R] colg[C] col_local[C]
    double *big_d;    // per wave: d[V] v[V] u[R]
    long long big_i_stride, big_d_stride;
};

__host__ __device__ inline LapWs carve(int *wi, double *wd, int R, int C, long long E) {
    LapWs w;
    const long long N = (long long)R + C, V = N;
    int *q = wi;
    w.parent = q; q += N;
    w.deg = q; q += N;
    w.row_off = q; q += R + 1;
    w.cnodes = q; q += N;
    w.croot = q; q += N;
    w.roots = q; q += N;
    w.comp_of = q; q += N;
    w.members = q; q += N;
    w.queue = q; q += N / 2 + 1;
    w.big_q = q; q += N / 2 + 1;
    w.csr_col = q; q += E;
    w.big_i = q;
    w.big_i_stride = 3 * V + 2LL * R + 2LL * C;
    w.csr_cost = wd;
    w.big_d = wd + E;
    w.big_d_stride = 2 * V + R;
    return w;
}

// Exact solve of one component with V = l + k <= W columns (+ dummies), on a W-lane segment of the
// wave (W = 16 or 64): one column per lane, rows on lanes < k.  rows_in / cols_in: ascending
// global ids (the segment's own copies).  Every segment of a wave runs its own component; control
// flow is uniform within a segment and every shuffle stays inside it.
template <int W>
__device__ void solve_seg(int k, int l, const int *rows_in, const int *cols_in, const int *row_off,
                          const int *csr_col, const double *csr_cost, double thresh, int *X, int *Y,
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
#pragma unroll
            for (int off = W / 2; off > 0; off >>= 1) bd = fmin(bd, __shfl_xor(bd, off, W));
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

struct Slab {
    double *d, *v, *u;
    int *y, *pred, *vis, *x, *rowg, *colg, *col_local;
};

// Same algorithm for large components, state in a global-memory slab (one lane per column,
// strided).  Rare: only dense clutter produces components beyond one wavefront.
__device__ void solve_large(Slab s, const int *rows_in, int k, const int *cols_in, int l,
                            const int *row_off, const int *csr_col, const double *csr_cost,
                            double thresh, int *X, int *Y, int *err) {
    const int lane = lane_id();
    const int V = l + k;
    for (int a = lane; a < k; a += WAVE) s.rowg[a] = rows_in[a];
    for (int a = lane; a < l; a += WAVE) {
        s.colg[a] = cols_in[a];
        s.col_local[cols_in[a]] = a;
    }
    for (int j = lane; j < V; j += WAVE) { s.v[j] = 0.0; s.y[j] = -1; }
    for (int q = lane; q < k; q += WAVE) { s.u[q] = 0.0; s.x[q] = -1; }
    wave_mem_sync();
    for (int cur = 0; cur < k; ++cur) {
        for (int j = lane; j < V; j += WAVE) { s.d[j] = INFINITY; s.vis[j] = 0; }
        wave_mem_sync();
        double minval = 0.0;
        int i = cur, sink = -1;
        for (int guard = 0; guard <= V; ++guard) {
            const int gi = s.rowg[i];
            const double ui = s.u[i];
            const int beg = ald(row_off + gi), end = ald(row_off + gi + 1);
            for (int e = beg + lane; e < end; e += WAVE) {
                const int j = s.col_local[ald(csr_col + e)];
                if (!s.vis[j]) {
                    const double r = minval + (aldd(csr_cost + e) - thresh) - ui - s.v[j];
                    if (r < s.d[j]) { s.d[j] = r; s.pred[j] = i; }
                }
            }
            if (lane == 0) {
                const int j = l + i;
                if (!s.vis[j]) {
                    const double r = minval + 0.0 - ui - s.v[j];
                    if (r < s.d[j]) { s.d[j] = r; s.pred[j] = i; }
                }
            }
            wave_mem_sync();
            double bd = INFINITY;
            int bk = INT_MAX;
            for (int j = lane; j < V; j += WAVE) {
                if (!s.vis[j]) {
                    const double dj = s.d[j];
                    const int kj = ((s.y[j] >= 0) << 30) | j;
                    if (dj < bd || (dj == bd && kj < bk)) { bd = dj; bk = kj; }
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                const double od = __shfl_xor(bd, off);
                const int ok = __shfl_xor(bk, off);
                if (od < bd || (od == bd && ok < bk)) { bd = od; bk = ok; }
            }
            if (!(bd < INFINITY)) { if (lane == 0) atomicOr(err, ERR_SOLVER); return; }
            const int jstar = bk & ((1 << 30) - 1);
            minval = bd;
            if (lane == 0) s.vis[jstar] = 1;
            const int owner = s.y[jstar];
            wave_mem_sync();
            if (owner < 0) { sink = jstar; break; }
            i = owner;
        }
        if (sink < 0) { if (lane == 0) atomicOr(err, ERR_SOLVER); return; }
        for (int j = lane; j < V; j += WAVE) {
            if (s.vis[j] && j != sink) {
                const double delta = minval - s.d[j];
                s.u[s.y[j]] += delta;
                s.v[j] -= delta;
            }
        }
        if (lane == 0) s.u[cur] += minval;
        wave_mem_sync();
        if (lane == 0) {
            int j = sink;
            for (int guard = 0; guard <= V; ++guard) {
                const int r = s.pred[j];
                s.y[j] = r;
                const int prev = s.x[r];
                s.x[r] = j;
                j = prev;
                if (r == cur) break;
            }
        }
        wave_mem_sync();
    }
    for (int q = lane; q < k; q += WAVE) {
        const int j = s.x[q];
        const int g = s.rowg[q];
        if (j >= 0 && j < l) {
            X[g] = s.colg[j];
            Y[s.colg[j]] = g;
        } else {
            X[g] = -1;
        }
    }
    wave_mem_sync();
}

__device__ int uf_find(int *parent, int a) {
    int p = ald(parent + a);
    while (p != a) { a = p; p = ald(parent + a); }
    return a;
}

__device__ void uf_union(int *parent, int a, int b) {
    for (;;) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a < b) { const int t = a; a = b; b = t; }
        if (atomicCAS(parent + a, a, b) == a) return;
    }
}

#ifdef YTA_STAMPS
// diagnostic build only: per-phase s_memrealtime stamps (100 MHz) of block 0 of the last launch
__device__ unsigned long long g_lap_stamps[16];
#define STAMP(k)                                                                  \
    do {                                                                          \
        if (blockIdx.x == 0 && threadIdx.x == 0 && (int)gridDim.x == na) g_lap_stamps[k] = wall_clock64(); \
    } while (0)
#else
#define STAMP(k) \
    do {         \
    } while (0)
#endif

template <bool NODES_LDS>
__global__ __launch_bounds__(LAP_THREADS) void lap_kernel(ProblemSet A, int na, ProblemSet B) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int wsum[32];
    __shared__ int s_cnt[3];

    int p;
    const ProblemSet &ps = pick(A, na, B, blockIdx.x, p);
    const int t = threadIdx.x, nt = LAP_THREADS;
    const int nr = ps.n_rows[(long long)p * ps.n_rows_stride];
    const int nc = ps.n_cols[(long long)p * ps.n_cols_stride];
    const int N = nr + nc;
    int *err = ps.err + (long long)p * ps.err_stride;
    int *X = ps.x + p * ps.x_stride;
    int *Y = ps.y + p * ps.y_stride;
    const int R = ps.max_rows, C = ps.max_cols;
    long long E = ps.n_edges[(long long)p * ps.n_edges_stride];
    if (E > ps.edge_cap) E = ps.edge_cap;
    const Edge *edges = ps.edges + p * ps.edges_stride;
    LapWs w = carve(ps.ws + p * ps.ws_stride, ps.wsd + p * ps.wsd_stride, R, C, ps.edge_cap);
    int *parent = w.parent, *deg = w.deg, *row_off = w.row_off;
    int *cnodes = w.cnodes, *croot = w.croot, *roots = w.roots, *comp_of = w.comp_of;
    int *members = w.members, *queue = w.queue, *big_q = w.big_q;
    int *csr_col = w.csr_col;
    double *csr_cost = w.csr_cost;
    {
        const int NL = R + C;
        unsigned char *q = smem;
        if (NODES_LDS) {
            parent = (int *)q; q += 4 * NL;
            deg = (int *)q; q += 4 * NL;
            row_off = (int *)q; q += 4 * (NL + 1);
            cnodes = (int *)q; q += 4 * NL;
            croot = (int *)q; q += 4 * NL;
            roots = (int *)q; q += 4 * NL;
            comp_of = (int *)q; q += 4 * NL;
            members = (int *)q; q += 4 * NL;
            queue = (int *)q; q += 4 * (NL / 2 + 1);
            big_q = (int *)q; q += 4 * (NL / 2 + 1);
            q = smem + ((q - smem + 15) & ~15);
        }
        if (E <= LAP_LDS_EDGES) {
            csr_cost = (double *)q; q += 8 * LAP_LDS_EDGES;
            csr_col = (int *)q;
        }
    }
    STAMP(0);
    // P0: init
    for (int n = t; n < N; n += nt) { parent[n] = n; deg[n] = 0; }
    for (int i = t; i < nr; i += nt) X[i] = -1;
    for (int j = t; j < nc; j += nt) Y[j] = -1;
    block_sync();
    STAMP(1);
    if (E == 0) return;
    // P1: degrees
    for (long long e = t; e < E; e += nt) {
        const Edge ed = edges[e];
        atomicAdd(deg + ed.row, 1);
        atomicAdd(deg + nr + ed.col, 1);
    }
    block_sync();
    STAMP(2);
    // P2: CSR row offsets (row degrees then double as scatter cursors)
    {
        int run = 0;
        for (int start = 0; start < nr; start += nt) {
            const int i = start + t;
            const int dg = i < nr ? ald(deg + i) : 0;
            int tot;
            const int pos = block_exclusive_scan(dg, wsum, &tot);
            if (i < nr) { row_off[i] = run + pos; deg[i] = 0; }
            run += tot;
        }
        if (t == 0) row_off[nr] = run;
    }
    block_sync();
    STAMP(3);
    // P3: scatter; single-edge components are matched outright, the rest are united
    for (long long e = t; e < E; e += nt) {
        const Edge ed = edges[e];
        const int b = row_off[ed.row];
        const int rdeg = row_off[ed.row + 1] - b;
        const int pos = b + atomicAdd(deg + ed.row, 1);
        csr_col[pos] = ed.col;
        csr_cost[pos] = ed.cost;
        if (rdeg == 1 && ald(deg + nr + ed.col) == 1) {
            X[ed.row] = ed.col;
            Y[ed.col] = ed.row;
        } else {
            uf_union(parent, ed.row, nr + ed.col);
        }
    }
    block_sync();
    STAMP(4);
    // P4: complex nodes (with their root) in node order, and the component roots in node order
    {
        int run = 0, runr = 0;
        for (int start = 0; start < N; start += nt) {
            const int n = start + t;
            int root = -1;
            if (n < N) {
                const bool cx = n < nr ? (row_off[n + 1] > row_off[n] && X[n] < 0)
                                       : (ald(deg + n) > 0 && Y[n - nr] < 0);
                if (cx) root = uf_find(parent, n);
            }
            int tot, totr;
            const int pos = block_exclusive_scan(root >= 0 ? 1 : 0, wsum, &tot);
            const int posr = block_exclusive_scan(root == n ? 1 : 0, wsum, &totr);
            if (root >= 0) { cnodes[run + pos] = n; croot[run + pos] = root; }
            if (root == n) { roots[runr + posr] = n; comp_of[n] = runr + posr; }
            run += tot;
            runr += totr;
        }
        if (t == 0) { s_cnt[0] = run; s_cnt[1] = runr; }
    }
    block_sync();
    STAMP(5);
    const int ncx = s_cnt[0], ncomp = s_cnt[1];
    if (ncomp == 0) return;
    // P5: per-component row / column counts (parent and deg are free from here on)
    int *kc = deg, *lc = deg + (N >> 1) + 1, *moff = parent;
    for (int c = t; c < ncomp; c += nt) { kc[c] = 0; lc[c] = 0; }
    block_sync();
    for (int q = t; q < ncx; q += nt) {
        const int c = comp_of[croot[q]];
        atomicAdd(cnodes[q] < nr ? kc + c : lc + c, 1);
    }
    block_sync();
    {   // member offsets (rows then columns of each component), then counts become cursors
        int run = 0;
        for (int start = 0; start < ncomp; start += nt) {
            const int c = start + t;
            const int sz = c < ncomp ? ald(kc + c) + ald(lc + c) : 0;
            int tot;
            const int pos = block_exclusive_scan(sz, wsum, &tot);
            if (c < ncomp) moff[c] = run + pos;
            run += tot;
        }
        if (t == 0) moff[ncomp] = run;
    }
    block_sync();
    for (int c = t; c < ncomp; c += nt) { lc[c] = moff[c] + ald(kc + c); kc[c] = moff[c]; }
    block_sync();
    for (int q = t; q < ncx; q += nt) {
        const int n = cnodes[q];
        const int c = comp_of[croot[q]];
        const int pos = atomicAdd(n < nr ? kc + c : lc + c, 1);
        members[pos] = n < nr ? n : n - nr;
    }
    block_sync();
    STAMP(6);
    // P6: classify.  One-row components: the row takes its cheapest edge (what the shortest-path
    // solve gives: lowest distance, ties to the lower column).  Others by size: 16-lane segments,
    // one wave, or the global-memory solver.
    if (t == 0) { s_cnt[0] = 0; s_cnt[1] = 0; s_cnt[2] = 0; }
    block_sync();
    for (int c = t; c < ncomp; c += nt) {
        // after the scatter: kc[c] = end of rows = start of columns, lc[c] = end of columns
        const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
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
        } else if (k + l <= 16) {
            queue[atomicAdd(&s_cnt[0], 1)] = c;
        } else if (k + l <= 64) {
            queue[ncomp - 1 - atomicAdd(&s_cnt[1], 1)] = c;
        } else {
            big_q[atomicAdd(&s_cnt[2], 1)] = c;
        }
    }
    block_sync();
    STAMP(7);
    const int n16 = s_cnt[0], n64 = s_cnt[1], nbig = s_cnt[2];
    const int wave = t / WAVE, lane = lane_id();
    // P7a: components with <= 16 columns + dummies, four per wave at a time
    for (int q = wave * 4 + (lane >> 4); q - (lane >> 4) < n16; q += LAP_WAVES * 4) {
        if (q < n16) {
            const int c = queue[q];
            const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
            solve_seg<16>(mr - m0, me - mr, members + m0, members + mr, row_off, csr_col, csr_cost,
                          ps.thresh, X, Y, err);
        }
    }
    // P7b: up to 64, one per wave
    for (int q = wave; q < n64; q += LAP_WAVES) {
        const int c = queue[ncomp - 1 - q];
        const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
        solve_seg<64>(mr - m0, me - mr, members + m0, members + mr, row_off, csr_col, csr_cost,
                      ps.thresh, X, Y, err);
    }
    // P7c: larger components, state in a global-memory slab
    for (int q = wave; q < nbig; q += LAP_WAVES) {
        const int c = big_q[q];
        const int m0 = moff[c], mr = ald(kc + c), me = ald(lc + c);
        const long long V = (long long)R + C;
        int *bi = w.big_i + wave * w.big_i_stride;
        double *bd = w.big_d + wave * w.big_d_stride;
        Slab s;
        s.y = bi; s.pred = bi + V; s.vis = bi + 2 * V; s.x = bi + 3 * V;
        s.rowg = bi + 3 * V + R; s.colg = bi + 3 * V + 2 * R;
        s.col_local = bi + 3 * V + 2 * R + C;
        s.d = bd; s.v = bd + V; s.u = bd + 2 * V;
        solve_large(s, members + m0, mr - m0, members + mr, me - mr, row_off, csr_col, csr_cost,
                    ps.thresh, X, Y, err);
    }
#ifdef YTA_STAMPS
    block_sync();
    STAMP(8);
    if (blockIdx.x == 0 && threadIdx.x == 0 && (int)gridDim.x == na) {
        g_lap_stamps[10] = ncomp;
        g_lap_stamps[11] = ncx;
        g_lap_stamps[12] = E;
        g_lap_stamps[13] = n16;
        g_lap_stamps[14] = n64;
        g_lap_stamps[15] = nbig;
    }
#endif
}

size_t lap_lds_bytes(int R, int C, bool nodes_lds) {
    size_t b = 0;
    if (nodes_lds) b = 4 * (size_t)(8 * (R + C) + 1 + 2 * ((R + C) / 2 + 1));
    b = (b + 15) & ~(size_t)15;
    return b + 12 * (size_t)LAP_LDS_EDGES;
}

}  // namespace

long long lap_ws_ints(int R, int C, long long E) {
    const long long N = (long long)R + C, V = N;
    return 8 * N + 1 + 2 * (N / 2 + 1) + E + LAP_WAVES * (3 * V + 2LL * R + 2LL * C);
}

long long lap_ws_doubles(int R, int C, long long E) {
    const long long V = (long long)R + C;
    return E + LAP_WAVES * (2 * V + R);
}

hipError_t launch_edges(const ProblemSet &a, int na, const ProblemSet *b, int nb, int max_rows,
                        hipStream_t stream) {
    if (na + nb <= 0 || max_rows <= 0) return hipSuccess;
    dim3 grid((max_rows + EDGE_THREADS - 1) / EDGE_THREADS, na + nb);
    hipLaunchKernelGGL(edges_kernel, grid, dim3(EDGE_THREADS), 0, stream, a, na, b ? *b : a);
    return hipGetLastError();
}

hipError_t launch_lap(const ProblemSet &a, int na, const ProblemSet *b, int nb, hipStream_t stream) {
    if (na + nb <= 0) return hipSuccess;
    const bool nodes_lds = a.max_rows + a.max_cols <= LAP_LDS_NODES &&
                           (!b || b->max_rows + b->max_cols <= LAP_LDS_NODES);
    const int R = b ? (a.max_rows > b->max_rows ? a.max_rows : b->max_rows) : a.max_rows;
    const int C = b ? (a.max_cols > b->max_cols ? a.max_cols : b->max_cols) : a.max_cols;
    const size_t lds = lap_lds_bytes(R, C, nodes_lds);
    if (nodes_lds) {
        hipError_t e = hipFuncSetAttribute((const void *)lap_kernel<true>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(lap_kernel<true>, dim3(na + nb), dim3(LAP_THREADS), lds, stream, a, na,
                           b ? *b : a);
    } else {
        hipError_t e = hipFuncSetAttribute((const void *)lap_kernel<false>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(lap_kernel<false>, dim3(na + nb), dim3(LAP_THREADS), lds, stream, a, na,
                           b ? *b : a);
    }
    return hipGetLastError();
}

}  // namespace yta

#ifdef YTA_STAMPS
extern "C" int yta_debug_lap_stamps(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(yta::g_lap_stamps), sizeof(unsigned long long) * 16) ==
                   hipSuccess
               ? 0
               : -2;
}
#endif
