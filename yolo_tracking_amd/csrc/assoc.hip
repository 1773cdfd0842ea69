// Association kernels for gfx950: candidate edges + exact sparse assignment (see assoc.hpp).
#include <climits>
#include <cmath>

#include "assoc.hpp"

namespace yta {

namespace {

constexpr int EDGE_THREADS = 256;
constexpr int EDGE_ROWS_PER_WAVE = 4;
constexpr int EDGE_ROWS_PER_BLOCK = (EDGE_THREADS / WAVE) * EDGE_ROWS_PER_WAVE;

constexpr int LAP_THREADS = 512;
constexpr int LAP_WAVES = LAP_THREADS / WAVE;
constexpr int SLAB_V = 256;   // LDS slab: columns (real + one dummy per row)
constexpr int SLAB_K = 128;   // LDS slab: rows

__device__ __forceinline__ int ald(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wave_mem_sync() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------------------ edge extraction
// One wave scores EDGE_ROWS_PER_WAVE track rows against every detection column, 64 columns per
// step; only pairs whose boxes intersect pay for the float64 division.  Edges are appended to the
// problem's pool with one atomic per (wave, step) that found any.
template <bool FUSED>
__global__ __launch_bounds__(EDGE_THREADS) void edges_kernel(ProblemSet ps) {
    const int p = blockIdx.y;
    const int nr = ps.n_rows[(long long)p * ps.n_rows_stride];
    const int nc = ps.n_cols[(long long)p * ps.n_cols_stride];
    const int lane = lane_id();
    const int wave = threadIdx.x / WAVE;
    const int row0 = blockIdx.x * EDGE_ROWS_PER_BLOCK + wave * EDGE_ROWS_PER_WAVE;
    if (row0 >= nr || nc <= 0) return;
    const Box *rows = ps.rows + p * ps.rows_stride;
    const Box *cols = ps.cols + p * ps.cols_stride;
    const double *score = FUSED ? ps.col_score + p * ps.score_stride : nullptr;
    Edge *edges = ps.edges + p * ps.edges_stride;
    int *n_edges = ps.n_edges + (long long)p * ps.n_edges_stride;
    const double thresh = ps.thresh;
    const bool all_pairs = !(thresh <= 1.0);  // non-intersecting pairs cost exactly 1

    Box rb[EDGE_ROWS_PER_WAVE];
    bool rv[EDGE_ROWS_PER_WAVE];
#pragma unroll
    for (int r = 0; r < EDGE_ROWS_PER_WAVE; ++r) {
        rv[r] = row0 + r < nr;
        rb[r] = rows[rv[r] ? row0 + r : row0];
    }
    for (int c0 = 0; c0 < nc; c0 += WAVE) {
        const int c = c0 + lane;
        const bool cv = c < nc;
        Box cb = cols[cv ? c : 0];
        double sc = FUSED ? score[cv ? c : 0] : 0.0;
#pragma unroll
        for (int r = 0; r < EDGE_ROWS_PER_WAVE; ++r) {
            bool e = false;
            double cost = 0.0;
            if (cv && rv[r] && (all_pairs || intersects(rb[r], cb))) {
                double dist = 1 - iou(rb[r], cb);     // matching.py:117
                cost = FUSED ? 1 - (1 - dist) * sc : dist;   // matching.py:216-220
                e = cost < thresh;
            }
            unsigned long long m = __ballot(e);
            if (m) {
                const int cnt = __popcll(m);
                int base = 0;
                if (lane == 0) base = atomicAdd(n_edges, cnt);
                base = __shfl(base, 0);
                if (e) {
                    long long pos = (long long)base + __popcll(m & lanemask_lt());
                    if (pos < ps.edge_cap) {
                        Edge ed;
                        ed.row = row0 + r;
                        ed.col = c;
                        ed.cost = cost;
                        edges[pos] = ed;
                    }
                }
                if (lane == 0 && (long long)base + cnt > ps.edge_cap)
                    atomicOr(ps.err + (long long)p * ps.err_stride, ERR_EDGE_OVERFLOW);
            }
        }
    }
}

// ------------------------------------------------------------------------------ solver workspace
struct LapWs {
    int *row_deg, *row_off, *row_cur, *col_deg, *parent, *comp_id;
    int *comp_rcnt, *comp_ccnt, *comp_roff, *comp_coff, *comp_rcur, *comp_ccur;
    int *comp_rows, *comp_cols, *col_local, *csr_col, *misc;
    int *big_i;        // per wave: y[V] pred[V] vis[V] x[R] rowg[R] colg[C]
    double *csr_cost;
    double *big_d;     // per wave: d[V] v[V] u[R]
    long long big_i_stride, big_d_stride;
};

__host__ __device__ inline LapWs carve(int *wi, double *wd, int R, int C, long long E) {
    LapWs w;
    int *q = wi;
    w.row_deg = q; q += R;
    w.row_off = q; q += R + 1;
    w.row_cur = q; q += R;
    w.col_deg = q; q += C;
    w.parent = q; q += R + C;
    w.comp_id = q; q += R + C;
    w.comp_rcnt = q; q += R;
    w.comp_ccnt = q; q += R;
    w.comp_roff = q; q += R + 1;
    w.comp_coff = q; q += R + 1;
    w.comp_rcur = q; q += R;
    w.comp_ccur = q; q += R;
    w.comp_rows = q; q += R;
    w.comp_cols = q; q += C;
    w.col_local = q; q += C;
    w.misc = q; q += 16;
    w.csr_col = q; q += E;
    w.big_i = q;
    const long long V = (long long)R + C;
    w.big_i_stride = 3 * V + 2LL * R + C;
    w.csr_cost = wd;
    w.big_d = wd + E;
    w.big_d_stride = 2 * V + R;
    return w;
}

struct Slab {
    double *d, *v, *u;
    int *y, *pred, *vis, *x, *rowg, *colg;
};

// Wave-level exact solve of one component (k rows, l real columns, one private dummy per row).
// Successive shortest augmenting paths with potentials (Dijkstra over the component's columns),
// rows in ascending global order; ties prefer lower distance, then a free column, then the
// lower local column index.
__device__ void solve_component(const LapWs &w, Slab s, const int *rows_in, int k,
                                const int *cols_in, int l, double thresh, int *X, int *Y,
                                int *err) {
    const int lane = lane_id();
    const int V = l + k;
    // sorted member lists (rank sort: deterministic regardless of the atomic gather order)
    for (int a = lane; a < k; a += WAVE) {
        int g = rows_in[a], rank = 0;
        for (int b = 0; b < k; ++b) rank += rows_in[b] < g;
        s.rowg[rank] = g;
    }
    for (int a = lane; a < l; a += WAVE) {
        int g = cols_in[a], rank = 0;
        for (int b = 0; b < l; ++b) rank += cols_in[b] < g;
        s.colg[rank] = g;
        w.col_local[g] = rank;
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
            // relax the edges of local row i (+ its private dummy column l + i)
            const int gi = s.rowg[i];
            const double ui = s.u[i];
            const int beg = w.row_off[gi], end = w.row_off[gi + 1];
            for (int e = beg + lane; e < end; e += WAVE) {
                int j = w.col_local[w.csr_col[e]];
                if (!s.vis[j]) {
                    double r = minval + (w.csr_cost[e] - thresh) - ui - s.v[j];
                    if (r < s.d[j]) { s.d[j] = r; s.pred[j] = i; }
                }
            }
            if (lane == 0) {
                int j = l + i;
                if (!s.vis[j]) {
                    double r = minval + 0.0 - ui - s.v[j];
                    if (r < s.d[j]) { s.d[j] = r; s.pred[j] = i; }
                }
            }
            wave_mem_sync();
            // argmin over unvisited columns
            double bd = INFINITY;
            int bk = INT_MAX;   // (occupied << 30) | index
            for (int j = lane; j < V; j += WAVE) {
                if (!s.vis[j]) {
                    double dj = s.d[j];
                    int kj = ((s.y[j] >= 0) << 30) | j;
                    if (dj < bd || (dj == bd && kj < bk)) { bd = dj; bk = kj; }
                }
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                double od = __shfl_xor(bd, off);
                int ok = __shfl_xor(bk, off);
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
        // dual update (visited rows are the owners of visited non-sink columns)
        for (int j = lane; j < V; j += WAVE) {
            if (s.vis[j] && j != sink) {
                double delta = minval - s.d[j];
                s.u[s.y[j]] += delta;
                s.v[j] -= delta;
            }
        }
        if (lane == 0) s.u[cur] += minval;
        wave_mem_sync();
        // augment along pred
        if (lane == 0) {
            int j = sink;
            for (int guard = 0; guard <= V; ++guard) {
                int r = s.pred[j];
                s.y[j] = r;
                int prev = s.x[r];
                s.x[r] = j;
                j = prev;
                if (r == cur) break;
            }
        }
        wave_mem_sync();
    }
    for (int q = lane; q < k; q += WAVE) {
        int j = s.x[q];
        int g = s.rowg[q];
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
        if (a < b) { int t = a; a = b; b = t; }
        if (atomicCAS(parent + a, a, b) == a) return;
    }
}

__global__ __launch_bounds__(LAP_THREADS) void lap_kernel(ProblemSet ps) {
    __shared__ int wsum[32];
    __shared__ double sl_d[LAP_WAVES][SLAB_V], sl_v[LAP_WAVES][SLAB_V], sl_u[LAP_WAVES][SLAB_K];
    __shared__ int sl_y[LAP_WAVES][SLAB_V], sl_pred[LAP_WAVES][SLAB_V], sl_vis[LAP_WAVES][SLAB_V];
    __shared__ int sl_x[LAP_WAVES][SLAB_K], sl_rowg[LAP_WAVES][SLAB_K], sl_colg[LAP_WAVES][SLAB_V];
    __shared__ int s_ncomp;

    const int p = blockIdx.x;
    const int t = threadIdx.x, nt = blockDim.x;
    const int nr = ps.n_rows[(long long)p * ps.n_rows_stride];
    const int nc = ps.n_cols[(long long)p * ps.n_cols_stride];
    int *err = ps.err + (long long)p * ps.err_stride;
    int *X = ps.x + p * ps.x_stride;
    int *Y = ps.y + p * ps.y_stride;
    const int R = ps.max_rows, C = ps.max_cols;
    long long E = ps.n_edges[(long long)p * ps.n_edges_stride];
    if (E > ps.edge_cap) E = ps.edge_cap;
    const Edge *edges = ps.edges + p * ps.edges_stride;
    LapWs w = carve(ps.ws + p * ps.ws_stride, ps.wsd + p * ps.wsd_stride, R, C, ps.edge_cap);

    // 0. init
    for (int i = t; i < nr; i += nt) { w.row_deg[i] = 0; w.row_cur[i] = 0; X[i] = -1; }
    for (int j = t; j < nc; j += nt) { w.col_deg[j] = 0; Y[j] = -1; }
    for (int n = t; n < nr + nc; n += nt) w.parent[n] = n;
    __syncthreads();
    if (E == 0) return;
    // 1. degrees
    for (long long e = t; e < E; e += nt) {
        atomicAdd(w.row_deg + edges[e].row, 1);
        atomicAdd(w.col_deg + edges[e].col, 1);
    }
    __syncthreads();
    // 2. CSR offsets
    {
        int run = 0;
        for (int start = 0; start < nr; start += nt) {
            int i = start + t;
            int dg = i < nr ? ald(w.row_deg + i) : 0;
            int tot;
            int pos = block_exclusive_scan(dg, wsum, &tot);
            if (i < nr) w.row_off[i] = run + pos;
            run += tot;
        }
        if (t == 0) w.row_off[nr] = run;
    }
    __syncthreads();
    // 3. scatter + isolated edges + union of the rest
    for (long long e = t; e < E; e += nt) {
        Edge ed = edges[e];
        int pos = atomicAdd(w.row_cur + ed.row, 1);
        w.csr_col[w.row_off[ed.row] + pos] = ed.col;
        w.csr_cost[w.row_off[ed.row] + pos] = ed.cost;
        if (ald(w.row_deg + ed.row) == 1 && ald(w.col_deg + ed.col) == 1) {
            X[ed.row] = ed.col;     // a component that is one edge: always matched
            Y[ed.col] = ed.row;
        } else {
            uf_union(w.parent, ed.row, nr + ed.col);
        }
    }
    __syncthreads();
    // 4. compress; flag complex nodes
    for (int n = t; n < nr + nc; n += nt) {
        int root = uf_find(w.parent, n);
        bool complex_node = n < nr ? (ald(w.row_deg + n) > 0 && X[n] < 0)
                                   : (ald(w.col_deg + (n - nr)) > 0 && Y[n - nr] < 0);
        w.comp_id[n] = complex_node ? root : -1;
    }
    __syncthreads();
    // 5. number the components by root order
    {
        int run = 0;
        for (int start = 0; start < nr + nc; start += nt) {
            int n = start + t;
            bool is_root = n < nr + nc && w.comp_id[n] == n;
            int tot;
            int pos = block_exclusive_scan(is_root ? 1 : 0, wsum, &tot);
            if (is_root) {
                int c = run + pos;
                w.comp_rcnt[c] = 0;
                w.comp_ccnt[c] = 0;
                w.comp_rcur[c] = 0;
                w.comp_ccur[c] = 0;
                ast(w.parent + n, -1 - c);   // parent slot reused: root -> encoded component index
            }
            run += tot;
        }
        if (t == 0) s_ncomp = run;
    }
    __syncthreads();
    const int ncomp = s_ncomp;
    if (ncomp == 0) return;
    // 6. member counts
    for (int n = t; n < nr + nc; n += nt) {
        int root = w.comp_id[n];
        if (root < 0) continue;
        int c = -1 - ald(w.parent + root);
        w.comp_id[n] = c;
        atomicAdd(n < nr ? w.comp_rcnt + c : w.comp_ccnt + c, 1);
    }
    __syncthreads();
    // 7. member offsets
    {
        int runr = 0, runc = 0;
        for (int start = 0; start < ncomp; start += nt) {
            int c = start + t;
            int rc = c < ncomp ? ald(w.comp_rcnt + c) : 0;
            int cc = c < ncomp ? ald(w.comp_ccnt + c) : 0;
            int totr, totc;
            int pr = block_exclusive_scan(rc, wsum, &totr);
            int pc = block_exclusive_scan(cc, wsum, &totc);
            if (c < ncomp) { w.comp_roff[c] = runr + pr; w.comp_coff[c] = runc + pc; }
            runr += totr;
            runc += totc;
        }
        if (t == 0) { w.comp_roff[ncomp] = runr; w.comp_coff[ncomp] = runc; }
    }
    __syncthreads();
    // 8. gather members (any order: the solving wave sorts them)
    for (int n = t; n < nr + nc; n += nt) {
        int c = w.comp_id[n];
        if (c < 0) continue;
        if (n < nr) w.comp_rows[w.comp_roff[c] + atomicAdd(w.comp_rcur + c, 1)] = n;
        else w.comp_cols[w.comp_coff[c] + atomicAdd(w.comp_ccur + c, 1)] = n - nr;
    }
    __syncthreads();
    // 9. one wave per component
    const int wave = t / WAVE;
    for (int c = wave; c < ncomp; c += LAP_WAVES) {
        const int r0 = w.comp_roff[c], k = w.comp_roff[c + 1] - r0;
        const int c0 = w.comp_coff[c], l = w.comp_coff[c + 1] - c0;
        Slab s;
        if (k + l <= SLAB_V && k <= SLAB_K) {
            s.d = sl_d[wave]; s.v = sl_v[wave]; s.u = sl_u[wave];
            s.y = sl_y[wave]; s.pred = sl_pred[wave]; s.vis = sl_vis[wave];
            s.x = sl_x[wave]; s.rowg = sl_rowg[wave]; s.colg = sl_colg[wave];
        } else {
            const long long V = (long long)R + C;
            int *bi = w.big_i + wave * w.big_i_stride;
            double *bd = w.big_d + wave * w.big_d_stride;
            s.y = bi; s.pred = bi + V; s.vis = bi + 2 * V; s.x = bi + 3 * V;
            s.rowg = bi + 3 * V + R; s.colg = bi + 3 * V + 2 * R;
            s.d = bd; s.v = bd + V; s.u = bd + 2 * V;
        }
        solve_component(w, s, w.comp_rows + r0, k, w.comp_cols + c0, l, ps.thresh, X, Y, err);
    }
}

}  // namespace

long long lap_ws_ints(int R, int C, long long E) {
    long long V = (long long)R + C;
    long long fixed = 0;
    fixed += R + (R + 1) + R + C + (R + C) + (R + C);
    fixed += R + R + (R + 1) + (R + 1) + R + R + R + C + C + 16;
    fixed += E;
    return fixed + (long long)LAP_WAVES * (3 * V + 2LL * R + C);
}

long long lap_ws_doubles(int R, int C, long long E) {
    long long V = (long long)R + C;
    return E + (long long)LAP_WAVES * (2 * V + R);
}

hipError_t launch_edges(const ProblemSet &ps, int n_problems, int max_rows, hipStream_t stream) {
    if (n_problems <= 0 || max_rows <= 0) return hipSuccess;
    dim3 grid((max_rows + EDGE_ROWS_PER_BLOCK - 1) / EDGE_ROWS_PER_BLOCK, n_problems);
    if (ps.col_score)
        hipLaunchKernelGGL(edges_kernel<true>, grid, dim3(EDGE_THREADS), 0, stream, ps);
    else
        hipLaunchKernelGGL(edges_kernel<false>, grid, dim3(EDGE_THREADS), 0, stream, ps);
    return hipGetLastError();
}

hipError_t launch_lap(const ProblemSet &ps, int n_problems, hipStream_t stream) {
    if (n_problems <= 0) return hipSuccess;
    hipLaunchKernelGGL(lap_kernel, dim3(n_problems), dim3(LAP_THREADS), 0, stream, ps);
    return hipGetLastError();
}

}  // namespace yta
