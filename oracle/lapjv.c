/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Never linked into the product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this.
 *
 * CPU restatement of the linear-assignment solver the reference's hot path calls:
 *   boxmot/utils/matching.py:64      lap.lapjv(cost, extend_cost=True, cost_limit=thresh)
 *   boxmot/utils/association.py:23   lap.lapjv(cost_matrix, extend_cost=True)
 *   boxmot/trackers/hybridsort/association.py:300-311 (same call as association.py)
 *
 * The solver itself lives in the third-party wheel `lapx` (requirements.txt:8, `lapx>=0.5.4`,
 * un-pinned; lapx 0.5.x re-packages gatagat/lap 0.4's `lapjv`), which is NOT installed in this
 * image.  What is restated here is its published algorithm (Jonker & Volgenant 1987, "A shortest
 * augmenting path algorithm for dense and sparse linear assignment problems", in the dense-matrix
 * form that `lap` ships):
 *   1. column reduction + reduction transfer  (every column's cheapest row; unique winners keep
 *      their column and transfer slack to the column price),
 *   2. augmenting row reduction, run at most twice over the free rows,
 *   3. shortest augmenting path (Dijkstra over columns with lazy "ready / scan / todo" sets) for
 *      every row still free, with price updates for the ready set.
 * and the Python wrapper's problem extension:
 *   - cost_limit < inf : solve the (R+C)x(R+C) matrix whose real block is `cost`, whose two
 *                        off-diagonal blocks are cost_limit/2 and whose dummy/dummy block is 0;
 *   - extend_cost only : zero-pad to max(R,C) square;
 *   then map indices >= C (rows) / >= R (cols) to -1 and truncate to R / C entries.
 *
 * Ties are resolved by the scan order below (rows ascending in reduction, columns ascending in
 * the Dijkstra sweeps, last-index-wins in column reduction as lap does by scanning j downwards).
 * Because the wheel is absent, this tie behaviour is "parity unpinned" against lapx itself;
 * every golden used for parity is checked tie-free (tests/golden/make_goldens.py).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define BIG DBL_MAX

/* ---------------- phase 1: column reduction + reduction transfer ---------------- */
static int col_reduce(int n, const double *c, int *free_rows, int *x, int *y, double *v)
{
    for (int k = 0; k < n; ++k) { x[k] = -1; v[k] = BIG; y[k] = 0; }
    /* every column remembers its cheapest row (first row wins on ties: strict <) */
    for (int r = 0; r < n; ++r) {
        const double *row = c + (size_t)r * n;
        for (int k = 0; k < n; ++k)
            if (row[k] < v[k]) { v[k] = row[k]; y[k] = r; }
    }
    unsigned char *solo = (unsigned char *)malloc((size_t)n);
    memset(solo, 1, (size_t)n);
    /* walk the columns from the last one; a row keeps the first (highest) column it wins */
    for (int k = n - 1; k >= 0; --k) {
        int r = y[k];
        if (x[r] < 0) x[r] = k;
        else { solo[r] = 0; y[k] = -1; }
    }
    int nfree = 0;
    for (int r = 0; r < n; ++r) {
        if (x[r] < 0) { free_rows[nfree++] = r; continue; }
        if (!solo[r]) continue;
        /* reduction transfer: lower the price of the row's column by its second-best slack */
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

/* ---------------- phase 2: augmenting row reduction ---------------- */
static int row_reduce(int n, const double *c, int nfree, int *free_rows, int *x, int *y, double *v)
{
    int pos = 0, out = 0;
    unsigned long long iters = 0;
    while (pos < nfree) {
        ++iters;
        int r = free_rows[pos++];
        const double *row = c + (size_t)r * n;
        /* best and second-best reduced cost in this row */
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
                if (can_lower) free_rows[--pos] = displaced;   /* retry the evicted row at once */
                else free_rows[out++] = displaced;             /* defer it to the next phase   */
            }
        } else if (displaced >= 0) {
            free_rows[out++] = displaced;
        }
        x[r] = k1;
        y[k1] = r;
    }
    return out;
}

/* ---------------- phase 3: shortest augmenting paths ---------------- */
/* Move every column of todo[lo..n) whose distance equals the minimum to the front [lo, hi). */
static int gather_min(int n, int lo, const double *d, int *cols)
{
    int hi = lo + 1;
    double m = d[cols[lo]];
    for (int t = hi; t < n; ++t) {
        int k = cols[t];
        if (d[k] <= m) {
            if (d[k] < m) { hi = lo; m = d[k]; }
            cols[t] = cols[hi];
            cols[hi++] = k;
        }
    }
    return hi;
}

/* Relax from the rows assigned to the scan set; returns a free column reached at the minimum
 * distance, or -1. */
static int relax_scan(int n, const double *c, int *plo, int *phi, double *d, int *cols, int *pred,
                      const int *y, const double *v)
{
    int lo = *plo, hi = *phi;
    while (lo != hi) {
        int k = cols[lo++];
        int r = y[k];
        double dk = d[k];
        const double *row = c + (size_t)r * n;
        double h = row[k] - v[k] - dk;
        for (int t = hi; t < n; ++t) {
            int kk = cols[t];
            double nd = row[kk] - v[kk] - h;
            if (nd < d[kk]) {
                d[kk] = nd;
                pred[kk] = r;
                if (nd == dk) {
                    if (y[kk] < 0) return kk;
                    cols[t] = cols[hi];
                    cols[hi++] = kk;
                }
            }
        }
    }
    *plo = lo;
    *phi = hi;
    return -1;
}

static int shortest_path(int n, const double *c, int src, const int *y, double *v, int *pred,
                         int *cols, double *d)
{
    const double *row = c + (size_t)src * n;
    for (int k = 0; k < n; ++k) { cols[k] = k; pred[k] = src; d[k] = row[k] - v[k]; }
    int lo = 0, hi = 0, ready = 0, end = -1;
    while (end < 0) {
        if (lo == hi) {
            ready = lo;
            hi = gather_min(n, lo, d, cols);
            for (int t = lo; t < hi; ++t)
                if (y[cols[t]] < 0) end = cols[t];
        }
        if (end < 0) end = relax_scan(n, c, &lo, &hi, d, cols, pred, y, v);
    }
    double m = d[cols[lo]];
    for (int t = 0; t < ready; ++t) v[cols[t]] += d[cols[t]] - m;
    return end;
}

static int augment_all(int n, const double *c, int nfree, const int *free_rows, int *x, int *y,
                       double *v)
{
    int *pred = (int *)malloc(sizeof(int) * (size_t)n);
    int *cols = (int *)malloc(sizeof(int) * (size_t)n);
    double *d = (double *)malloc(sizeof(double) * (size_t)n);
    if (!pred || !cols || !d) { free(pred); free(cols); free(d); return -1; }
    for (int f = 0; f < nfree; ++f) {
        int src = free_rows[f];
        int k = shortest_path(n, c, src, y, v, pred, cols, d);
        int r = -1, steps = 0;
        while (r != src) {          /* flip the alternating path back to the source row */
            r = pred[k];
            y[k] = r;
            int prev = x[r];
            x[r] = k;
            k = prev;
            if (++steps > n) { free(pred); free(cols); free(d); return -2; }
        }
    }
    free(pred); free(cols); free(d);
    return 0;
}

/* Square dense solve.  cost: n*n row-major.  x[row] = col, y[col] = row. */
int oracle_lapjv_square(int n, const double *cost, int *x, int *y)
{
    if (n <= 0) return 0;
    int *free_rows = (int *)malloc(sizeof(int) * (size_t)n);
    double *v = (double *)malloc(sizeof(double) * (size_t)n);
    if (!free_rows || !v) { free(free_rows); free(v); return -1; }
    int nfree = col_reduce(n, cost, free_rows, x, y, v);
    for (int pass = 0; nfree > 0 && pass < 2; ++pass)
        nfree = row_reduce(n, cost, nfree, free_rows, x, y, v);
    int rc = 0;
    if (nfree > 0) rc = augment_all(n, cost, nfree, free_rows, x, y, v);
    free(free_rows); free(v);
    return rc;
}

/* lapx-style wrapper: rectangular `cost` (nr x nc, row-major), extend / cost_limit semantics.
 * x: nr entries (col or -1), y: nc entries (row or -1).  *opt = sum of matched real costs. */
int oracle_lapjv(int nr, int nc, const double *cost, int extend_cost, double cost_limit,
                 int *x, int *y, double *opt)
{
    if (nr < 0 || nc < 0) return -3;
    if (nr != nc && !extend_cost && !(cost_limit < INFINITY)) return -3;
    int limited = cost_limit < INFINITY;
    int n = limited ? nr + nc : (nr > nc ? nr : nc);
    int extended = limited || extend_cost;
    if (opt) *opt = 0.0;
    if (n == 0) return 0;
    double *m = (double *)malloc(sizeof(double) * (size_t)n * (size_t)n);
    int *xx = (int *)malloc(sizeof(int) * (size_t)n);
    int *yy = (int *)malloc(sizeof(int) * (size_t)n);
    if (!m || !xx || !yy) { free(m); free(xx); free(yy); return -1; }
    double fill = limited ? cost_limit / 2.0 : 0.0;
    for (int r = 0; r < n; ++r)
        for (int k = 0; k < n; ++k) {
            double val;
            if (r < nr && k < nc) val = cost[(size_t)r * nc + k];
            else if (limited && r >= nr && k >= nc) val = 0.0;
            else val = fill;
            m[(size_t)r * n + k] = val;
        }
    int rc = oracle_lapjv_square(n, m, xx, yy);
    if (rc == 0) {
        double s = 0.0;
        for (int r = 0; r < nr; ++r) {
            int k = xx[r];
            if (extended && k >= nc) k = -1;
            x[r] = k;
            if (k >= 0) s += cost[(size_t)r * nc + k];
        }
        for (int k = 0; k < nc; ++k) {
            int r = yy[k];
            if (extended && r >= nr) r = -1;
            y[k] = r;
        }
        if (opt) *opt = s;
    }
    free(m); free(xx); free(yy);
    return rc;
}
