/*
 * Prototype (tools, not the product; not the oracle): the dense lapjv of the reference's
 * extend_cost calls (association.py:20-28 -> lapx lapjv) with phase 3's relax sweeps restricted to
 * a row's nonzero entries whenever no zero entry can be relaxed - the same operation and
 * tie-breaking sequence as the dense sweep, checked against oracle/lapjv.c by
 * tools/lapjv_sparse_check.py.
 *
 * Why it is the same sequence.  A sweep from scanned column k (row r = y[k], distance dk, h =
 * c[r][k] - v[k] - dk) relaxes todo column kk to nd = c[r][kk] - v[kk] - h when nd < d[kk].  For an
 * entry c[r][kk] == 0 that needs -h < d[kk] + v[kk]; during one search v is fixed and d only
 * decreases from its start c[src][kk] - v[kk], so d[kk] + v[kk] <= max_k c[src][k] = cmax.  When
 * -h >= cmax no zero entry relaxes, the dense sweep changes nothing at them (no distance, no pred,
 * no swap), and the columns not yet visited keep their positions during a sweep (a swap moves the
 * relaxed column to `hi` and the column at `hi`, already visited, to the current position).  So
 * visiting only the row's nonzero todo entries in position order replays the sweep exactly.
 * Otherwise the dense sweep runs.  `pos` (the inverse of `cols`) is kept for the position order.
 *
 * Build: gcc -O2 -shared -fPIC tools/lapjv_sparse_proto.c -o tools/liblapjv_sparse_proto.so
 */
#include <float.h>
#include <stdlib.h>
#include <string.h>

#define BIG DBL_MAX

static int col_reduce(int n, const double *c, int *free_rows, int *x, int *y, double *v)
{
    for (int k = 0; k < n; ++k) { x[k] = -1; v[k] = BIG; y[k] = 0; }
    for (int r = 0; r < n; ++r) {
        const double *row = c + (size_t)r * n;
        for (int k = 0; k < n; ++k)
            if (row[k] < v[k]) { v[k] = row[k]; y[k] = r; }
    }
    unsigned char *solo = (unsigned char *)malloc((size_t)n);
    memset(solo, 1, (size_t)n);
    for (int k = n - 1; k >= 0; --k) {
        int r = y[k];
        if (x[r] < 0) x[r] = k;
        else { solo[r] = 0; y[k] = -1; }
    }
    int nfree = 0;
    for (int r = 0; r < n; ++r) {
        if (x[r] < 0) { free_rows[nfree++] = r; continue; }
        if (!solo[r]) continue;
        const double *row = c + (size_t)r * n;
        int own = x[r];
        double best = BIG;
        for (int k = 0; k < n; ++k) {
            if (k == own) continue;
            double s = row[k] - v[k];
            if (s < best) best = s;
        }
        v[own] -= best;
    }
    free(solo);
    return nfree;
}

static int row_reduce(int n, const double *c, int nfree, int *free_rows, int *x, int *y, double *v)
{
    int pos = 0, out = 0;
    unsigned long long iters = 0;
    while (pos < nfree) {
        ++iters;
        int r = free_rows[pos++];
        const double *row = c + (size_t)r * n;
        int k1 = 0, k2 = -1;
        double m1 = row[0] - v[0], m2 = BIG;
        for (int k = 1; k < n; ++k) {
            double s = row[k] - v[k];
            if (s < m2) {
                if (s >= m1) { m2 = s; k2 = k; }
                else { m2 = m1; k2 = k1; m1 = s; k1 = k; }
            }
        }
        int displaced = y[k1];
        double lowered = v[k1] - (m2 - m1);
        int can_lower = lowered < v[k1];
        if (iters < (unsigned long long)pos * (unsigned long long)n) {
            if (can_lower) v[k1] = lowered;
            else if (displaced >= 0 && k2 >= 0) { k1 = k2; displaced = y[k2]; }
            if (displaced >= 0) {
                if (can_lower) free_rows[--pos] = displaced;
                else free_rows[out++] = displaced;
            }
        } else if (displaced >= 0) {
            free_rows[out++] = displaced;
        }
        x[r] = k1;
        y[k1] = r;
    }
    return out;
}

struct Csr {
    const int *start, *col;
    const double *val;
};

static inline void put(int *cols, int *pos, int p, int k) { cols[p] = k; pos[k] = p; }

static int gather_min(int n, int lo, const double *d, int *cols, int *pos)
{
    int hi = lo + 1;
    double m = d[cols[lo]];
    for (int t = hi; t < n; ++t) {
        int k = cols[t];
        if (d[k] <= m) {
            if (d[k] < m) { hi = lo; m = d[k]; }
            put(cols, pos, t, cols[hi]);
            put(cols, pos, hi++, k);
        }
    }
    return hi;
}

static int cmp_pos_ctx_n;
static const int *cmp_pos_ctx;
static int by_pos(const void *a, const void *b)
{
    int pa = cmp_pos_ctx[*(const int *)a], pb = cmp_pos_ctx[*(const int *)b];
    return (pa > pb) - (pa < pb);
}

static int relax_scan(int n, const double *c, const struct Csr *S, double cmax, int *plo, int *phi,
                      double *d, int *cols, int *pos, int *pred, const int *y, const double *v,
                      int *buf, long long *st)
{
    int lo = *plo, hi = *phi;
    while (lo != hi) {
        int k = cols[lo++];
        int r = y[k];
        double dk = d[k];
        const double *row = c + (size_t)r * n;
        double h = row[k] - v[k] - dk;
        if (-h >= cmax) {   /* no zero entry can relax: the row's nonzero todo entries only */
            st[0]++;
            int m = 0;
            for (int e = S->start[r]; e < S->start[r + 1]; ++e)
                if (pos[S->col[e]] >= hi) buf[m++] = S->col[e];
            cmp_pos_ctx = pos;
            qsort(buf, (size_t)m, sizeof(int), by_pos);
            for (int q = 0; q < m; ++q) {
                int kk = buf[q];
                int t = pos[kk];
                double nd = row[kk] - v[kk] - h;
                if (nd < d[kk]) {
                    d[kk] = nd;
                    pred[kk] = r;
                    if (nd == dk) {
                        if (y[kk] < 0) return kk;   /* lo / hi as before the sweeps (as lapjv.c) */
                        put(cols, pos, t, cols[hi]);
                        put(cols, pos, hi++, kk);
                    }
                }
            }
            continue;
        }
        st[1]++;
        for (int t = hi; t < n; ++t) {
            int kk = cols[t];
            double nd = row[kk] - v[kk] - h;
            if (nd < d[kk]) {
                d[kk] = nd;
                pred[kk] = r;
                if (nd == dk) {
                    if (y[kk] < 0) return kk;   /* lo / hi as before the sweeps (as lapjv.c) */
                    put(cols, pos, t, cols[hi]);
                    put(cols, pos, hi++, kk);
                }
            }
        }
    }
    *plo = lo;
    *phi = hi;
    return -1;
}

static int shortest_path(int n, const double *c, const struct Csr *S, int src, const int *y,
                         double *v, int *pred, int *cols, int *pos, double *d, int *buf,
                         long long *st)
{
    const double *row = c + (size_t)src * n;
    double cmax = -BIG;
    for (int k = 0; k < n; ++k) {
        cols[k] = k;
        pos[k] = k;
        pred[k] = src;
        d[k] = row[k] - v[k];
        if (row[k] > cmax) cmax = row[k];
    }
    int lo = 0, hi = 0, ready = 0, end = -1;
    while (end < 0) {
        if (lo == hi) {
            st[2]++;
            ready = lo;
            hi = gather_min(n, lo, d, cols, pos);
            for (int t = lo; t < hi; ++t)
                if (y[cols[t]] < 0) end = cols[t];
        }
        if (end < 0) end = relax_scan(n, c, S, cmax, &lo, &hi, d, cols, pos, pred, y, v, buf, st);
    }
    double m = d[cols[lo]];
    for (int t = 0; t < ready; ++t) v[cols[t]] += d[cols[t]] - m;
    return end;
}

/* Square dense solve with the sparse phase-3 sweeps.  st: [sparse sweeps, dense sweeps, gathers] */
int proto_lapjv_square(int n, const double *c, int *x, int *y, double *vout, long long *st)
{
    st[0] = st[1] = st[2] = 0;
    if (n <= 0) return 0;
    int *free_rows = malloc(sizeof(int) * (size_t)n);
    double *v = malloc(sizeof(double) * (size_t)n);
    int nfree = col_reduce(n, c, free_rows, x, y, v);
    for (int pass = 0; nfree > 0 && pass < 2; ++pass) nfree = row_reduce(n, c, nfree, free_rows, x, y, v);
    if (nfree > 0) {
        int *start = malloc(sizeof(int) * (size_t)(n + 1));
        int nnz = 0;
        for (int r = 0; r < n; ++r) {
            start[r] = nnz;
            for (int k = 0; k < n; ++k) nnz += c[(size_t)r * n + k] != 0.0;
        }
        start[n] = nnz;
        int *col = malloc(sizeof(int) * (size_t)(nnz + 1));
        double *val = malloc(sizeof(double) * (size_t)(nnz + 1));
        for (int r = 0, e = 0; r < n; ++r)
            for (int k = 0; k < n; ++k)
                if (c[(size_t)r * n + k] != 0.0) { col[e] = k; val[e++] = c[(size_t)r * n + k]; }
        struct Csr S = {start, col, val};
        int *pred = malloc(sizeof(int) * (size_t)n), *cols = malloc(sizeof(int) * (size_t)n);
        int *pos = malloc(sizeof(int) * (size_t)n), *buf = malloc(sizeof(int) * (size_t)n);
        double *d = malloc(sizeof(double) * (size_t)n);
        for (int f = 0; f < nfree; ++f) {
            int src = free_rows[f];
            int k = shortest_path(n, c, &S, src, y, v, pred, cols, pos, d, buf, st);
            int r = -1;
            while (r != src) {
                r = pred[k];
                y[k] = r;
                int prev = x[r];
                x[r] = k;
                k = prev;
            }
        }
        free(start); free(col); free(val); free(pred); free(cols); free(pos); free(buf); free(d);
    }
    if (vout) memcpy(vout, v, sizeof(double) * (size_t)n);
    free(free_rows);
    free(v);
    return 0;
}
